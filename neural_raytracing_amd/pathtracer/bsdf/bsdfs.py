"""BSDFs on the hot path (bsdf/bsdfs.py).  ``ComposeSpatialVarying`` of ``NeuralBSDF`` /
``Diffuse`` / ``Conductor`` evaluates inside the fused shading kernel ``nrt_shade_direct``."""
import ctypes
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import _lib
from .._handles import _Handle, _cache, mlp_handle
from ..neural_blocks import SkipConnMLP, activation_code


def identity(x):
    return x


def identity_div_pi(x):
    return x / math.pi


class BSDF(nn.Module):
    """General BSDF interface (bsdfs.py:63-72)."""

    def __init__(self):
        super().__init__()

    def sample(self, it, sampler, active=True):
        raise NotImplementedError()

    def eval_and_pdf(self, it, wo, active=True):
        raise NotImplementedError()

    def joint_eval_pdf(self, it, wo, active=True):
        spectrum, pdf = self.eval_and_pdf(it, wo, active)
        return torch.cat([spectrum, pdf.reshape(spectrum.shape[:-1] + (1,))], dim=-1)

    def eval(self, it, wo, active=True):
        return self.eval_and_pdf(it, wo, active)[0]

    def pdf(self, it, wo, active=True):
        return self.eval_and_pdf(it, wo, active)[1]


class Diffuse(BSDF):
    """Diffuse (bsdfs.py:78-118)."""

    def __init__(self, reflectance=[0.25, 0.2, 0.7], preprocess=identity_div_pi, device="cuda"):
        super().__init__()
        if type(reflectance) == list:
            self.reflectance = torch.tensor(reflectance, device=device, requires_grad=True)
        else:
            self.reflectance = reflectance
        self.preproc = preprocess

    def parameters(self):
        return [self.reflectance]

    def random(self):
        self.reflectance = torch.rand_like(self.reflectance, requires_grad=True)
        return self

    def _component(self):
        if self.preproc is identity_div_pi:
            act = _lib.ACT["none"]
        else:
            act = _lib.ACT[activation_code(self.preproc)]
        refl = self.reflectance.detach().float().cpu().tolist()
        return (_lib.NRT_BSDF_DIFFUSE, None, act, refl + [0.0])


class Conductor(BSDF):
    """Conductor (bsdfs.py:345-388)."""

    def __init__(self, specular=[1., 1., 1.], eta: float = 1.3, k: float = 1, device="cuda",
                 activation=torch.sigmoid):
        super().__init__()
        self.eta = torch.tensor(eta, requires_grad=True, dtype=torch.float)
        self.k = torch.tensor(k, requires_grad=True, dtype=torch.float)
        if type(specular) == list:
            self.specular = torch.tensor(specular, device=device, requires_grad=True)
        else:
            self.specular = specular
        self.act = activation

    def parameters(self):
        return [self.eta, self.k, self.specular]

    def random(self):
        self.specular = torch.rand_like(self.specular, requires_grad=True)
        return self

    def _component(self):
        eta = float(F.softplus(self.eta.detach().float()))
        spec = self.specular.detach().float().cpu().tolist()
        return (_lib.NRT_BSDF_CONDUCTOR, None, _lib.ACT[activation_code(self.act)], spec + [eta])


class NeuralBSDF(BSDF):
    """act(SkipConnMLP_6x96,F=64(param_rusin2(it.wi, wo))), pdf 1 (bsdfs.py:613-637)."""

    def __init__(self, activation=torch.sigmoid, device="cuda"):
        super().__init__()
        self.mlp = SkipConnMLP(in_size=3, out=3, num_layers=6, hidden_size=96, freqs=64,
                               device=device).to(device)
        self.act = activation

    def parameters(self):
        return self.mlp.parameters()

    def random(self):
        return self

    def _component(self):
        return (_lib.NRT_BSDF_NEURAL, mlp_handle(self.mlp), _lib.ACT[activation_code(self.act)],
                [0.0, 0.0, 0.0, 0.0])

    def eval_and_pdf(self, it, wo, active=True):
        raise _lib.NrtError("NeuralBSDF evaluates inside Direct.sample's fused shading kernel "
                            "(nrt_shade_direct)")


class ComposeSpatialVarying(BSDF):
    """Spatially varying mixture sum_j sigmoid(sp_var(p))_j f_j (bsdfs.py:482-536)."""

    def __init__(self, bsdfs, spatial_varying_fn=None, device="cuda"):
        super().__init__()
        self.bsdfs = bsdfs
        if spatial_varying_fn is None:
            self.sp_var_fn = SkipConnMLP(num_layers=16, hidden_size=256, freqs=128, sigma=2 << 6,
                                         in_size=3, out=len(bsdfs), device=device,
                                         xavier_init=True).to(device)
        else:
            self.sp_var_fn = spatial_varying_fn
        self.preprocess = identity

    def parameters(self):
        from itertools import chain
        own = self.sp_var_fn.parameters() if self.sp_var_fn is not None else []
        return chain(own, *[b.parameters() for b in self.bsdfs])

    def nrt(self):
        """nrt_bsdf handle (rebuilt when any component's parameters change)."""
        comps = [b._component() for b in self.bsdfs]
        sp = self.sp_var_fn
        sph = mlp_handle(sp) if isinstance(sp, SkipConnMLP) else None
        if sp is not None and sph is None:
            raise _lib.NrtError("spatial_varying_fn must be a SkipConnMLP on the HIP path")
        def build():
            arr = (_lib.BsdfComponent * len(comps))()
            for i, (kind, mh, act, params) in enumerate(comps):
                arr[i].kind = kind
                arr[i].mlp = mh.value if mh is not None else None
                arr[i].activation = act
                for q in range(4):
                    arr[i].params[q] = float(params[q])
            out = ctypes.c_void_p()
            _lib.check(_lib.load().nrt_bsdf_create(len(comps), arr, sph.value if sph else None,
                                                   ctypes.byref(out)), "nrt_bsdf_create")
            deps = [c[1] for c in comps if c[1] is not None] + ([sph] if sph else [])
            return _Handle(out, "nrt_bsdf_destroy", deps)

        cached = getattr(self, "_nrt_bsdf", None)
        key = tuple((c[0], c[2], tuple(c[3]), id(c[1])) for c in comps) + (id(sph),)
        if cached is None or cached[0] != key:
            object.__setattr__(self, "_nrt_bsdf", (key, build()))
        return self._nrt_bsdf[1].value

    def eval_and_pdf(self, it, wo, active=True):
        raise _lib.NrtError("ComposeSpatialVarying evaluates inside Direct.sample's fused "
                            "shading kernel (nrt_shade_direct); standalone eval_and_pdf is not "
                            "on the HIP path yet")

    def normalized_weights(self, p, it):
        w = self.sp_var_fn(self.preprocess(p)).reshape(p.shape[:-1] + (len(self.bsdfs),))
        setattr(it, "nonnormalized_weights", w)
        return w.sigmoid()


# ---- reference BSDFs outside the hot path (import surface of scripts/*.py) ----------------------
# The drivers import Phong, Plastic and Bidirectional (nerf_synthetic.py:10-12, dtu.py:11-13,
# colocate.py:10-12) without rendering them.  Their constructors and parameters() follow
# bsdfs.py:132-149, 238-270 and the Bidirectional wrapper; shading with them is not on the HIP path
# and raises NrtError, as any unrecognised BSDF does.

class _Unsupported(BSDF):
    def _component(self):
        raise _lib.NrtError(f"BSDF {type(self).__name__} has no HIP implementation (supported: "
                            "NeuralBSDF, Diffuse, Conductor, ComposeSpatialVarying)")

    def eval_and_pdf(self, it, wo, active=True):
        self._component()

    def sample(self, it, sampler, active=True):
        self._component()


class Phong(_Unsupported):
    """bsdfs.py:132-189 (constructor, parameters, random)."""

    def __init__(self, diffuse=[0.6, 0.5, 0.7], specular=[0.8, 0.8, 0.8], min_spec=1, device="cuda"):
        super().__init__()
        self.diffuse = torch.tensor(diffuse, device=device, requires_grad=True) \
            if type(diffuse) == list else diffuse
        self.specular = torch.tensor(specular, device=device, requires_grad=True) \
            if type(specular) == list else specular
        self.shine = torch.tensor(40., dtype=torch.float, device=device, requires_grad=True)
        self.min_spec = min_spec

    def parameters(self):
        return [self.specular, self.diffuse, self.shine]

    def random(self):
        self.shine = torch.rand_like(self.shine, requires_grad=True)
        self.specular = torch.rand_like(self.specular, requires_grad=True)
        self.diffuse = torch.rand_like(self.diffuse, requires_grad=True)
        return self


def fresnel_diff_refl(eta):
    """bsdfs.py:220-235 (Mitsuba's diffuse Fresnel reflectance fit)."""
    if eta < 1:
        return -1.4399 * (eta * eta) + 0.7099 * eta + 0.6681 + 0.0636 / eta
    inv = 1 / eta
    return 0.919317 - 3.4793 * inv + 6.75335 * inv ** 2 - 7.80989 * inv ** 3 + \
        4.98554 * inv ** 4 - 1.36881 * inv ** 5


class Plastic(_Unsupported):
    """bsdfs.py:238-270 (constructor, parameters, random)."""

    def __init__(self, diffuse=[0.5, 0.5, 0.5], specular=[1., 1., 1.], int_ior: float = 1.49,
                 ext_ior: float = 1.000277, device="cuda"):
        super().__init__()
        self.diffuse = torch.tensor(diffuse, device=device, requires_grad=True) \
            if type(diffuse) == list else diffuse
        self.specular = torch.tensor(specular, device=device, requires_grad=True) \
            if type(specular) == list else specular
        assert int_ior > 0 and ext_ior > 0
        self.eta = int_ior / ext_ior
        self.inv_eta_2 = 1 / (self.eta * self.eta)
        self.fdr_int = fresnel_diff_refl(1 / self.eta)
        self.fdr_ext = fresnel_diff_refl(self.eta)

    def spec_sample_weight(self):
        d = self.diffuse.mean()
        s = self.specular.mean()
        return s / (d + s)

    def parameters(self):
        return [self.diffuse, self.specular]

    def random(self):
        self.specular = torch.rand_like(self.specular, requires_grad=True)
        self.diffuse = torch.rand_like(self.diffuse, requires_grad=True)
        return self


class Bidirectional(_Unsupported):
    """bsdfs.py:409-440: front BSDF for cos(theta_i) > 0, back (default: the front one) with z
    inverted below the surface."""

    def __init__(self, front, back=None):
        super().__init__()
        self.front = front
        self.back = front if back is None else back

    def parameters(self):
        from itertools import chain
        return chain(self.front.parameters(), self.back.parameters())
