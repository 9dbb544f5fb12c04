"""SDF shapes (shapes/sdfs.py): the sphere-tracing march, the 128-step coarse scan and the
normals run in ``nrt_sdf_intersect``; ``SphereSDF`` / ``SkipConnMLP`` SDFs evaluate in
``nrt_sdf_eval``.  Any other SDF callable (a warp or displacement around a packed SDF,
edit_dtu.py:86-100) is evaluated by the caller between the HIP march / scan / shadow steps
(``nrt_*_callable_step``), with autograd normals through the callable as sdfs.py:184-197."""
import ctypes
import random

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import _lib
from .._handles import _Handle, _cache, _host, mlp_handle, train_handle
from ..interaction import MixedInteraction
from ..differentiable import coordinate_system, needs_grad, sdf_gradient, sdf_value
from ..neural_blocks import SkipConnMLP


def SPHERE_SDF(p):
    """Default unit sphere SDF (sdfs.py:13)."""
    return torch.norm(p, dim=-1) - 1


class SphereSDF(nn.Module):
    """Spheres smooth-min-ed together plus a residual MLP (sdfs.py:16-44)."""

    def __init__(self, n=2 << 6, device="cuda"):
        super().__init__()
        self.centers = nn.Parameter(0.3 * torch.rand(n, 3, device=device, requires_grad=True) - 0.15)
        self.radii = nn.Parameter(0.2 * torch.rand(n, device=device, requires_grad=True) - 0.1)
        self.tfs = nn.Parameter(torch.zeros(n, 3, 3, device=device, requires_grad=True))
        self.shift = SkipConnMLP(num_layers=8, hidden_size=128, in_size=3, out=1, device=device,
                                 freqs=32, activation=F.softplus, zero_init=True).to(device)

    def set_center(self, at):
        self.centers = nn.Parameter(at.expand_as(self.centers).clone().detach())

    def transform(self, p):
        tfs = self.tfs + torch.eye(3, device=p.device).unsqueeze(0)
        return torch.einsum("ijk,ibk->ibj", tfs, p.expand(tfs.shape[0], -1, -1))

    def forward(self, p):
        if torch.is_grad_enabled() and (p.requires_grad or needs_grad(self)):
            # inside an SDF callable (a warp) under autograd: the normals of the callable march
            # differentiate through it (sphere part in torch, shift MLP on the HIP backward)
            return sdf_value(self, p)
        return sdf_eval(self, p)


_UNIT = {}


def sdf_handle(sdf):
    """nrt_sdf for a recognised SDF callable (TorchScript modules through script_modules views)."""
    from ..script_modules import resolve
    sdf = resolve(sdf)
    if sdf is SPHERE_SDF:
        if "h" not in _UNIT:
            lib = _lib.load()
            out = ctypes.c_void_p()
            _lib.check(lib.nrt_sdf_create_unit_sphere(ctypes.byref(out)), "nrt_sdf_create_unit_sphere")
            _UNIT["h"] = _Handle(out, "nrt_sdf_destroy")
        return _UNIT["h"].value
    if isinstance(sdf, SkipConnMLP):
        mh = mlp_handle(sdf)
        params = [sdf.basis_p] + list(sdf.parameters())

        def build():
            out = ctypes.c_void_p()
            _lib.check(_lib.load().nrt_sdf_create_mlp(mh.value, ctypes.byref(out)), "nrt_sdf_create_mlp")
            return _Handle(out, "nrt_sdf_destroy", [mh])
        return _cache(sdf, [*params, torch.empty(0)], build).value
    if isinstance(sdf, SphereSDF) or _looks_like_sphere_sdf(sdf):
        shift = getattr(sdf, "shift", None)
        mh = mlp_handle(shift) if shift is not None else None
        params = [sdf.centers, sdf.radii, sdf.tfs] + ([shift.basis_p] + list(shift.parameters()) if shift is not None else [])

        def build():
            c, r, t = _host(sdf.centers), _host(sdf.radii), _host(sdf.tfs)
            out = ctypes.c_void_p()
            _lib.check(_lib.load().nrt_sdf_create_sphere_blob(
                c.shape[0], c.data_ptr(), r.data_ptr(), t.data_ptr(), 32.0,
                mh.value if mh is not None else None, ctypes.byref(out)), "nrt_sdf_create_sphere_blob")
            return _Handle(out, "nrt_sdf_destroy", [mh] if mh is not None else [])
        return _cache(sdf, params, build).value
    raise _lib.NrtError(f"SDF callable {getattr(sdf, '__name__', type(sdf).__name__)} has no HIP "
                        "implementation (supported: SPHERE_SDF, SphereSDF, SkipConnMLP and their "
                        "TorchScript modules)")


def train_sdf_handle(sdf):
    """nrt_sdf for the training loop's march: built over the SDF MLP's training handle
    (``train_handle``: re-packed on the device by nrt_mlp_refresh after each optimiser step) and,
    for a SphereSDF, a sphere table rewritten on the device (nrt_sdf_refresh_spheres) when its
    tensors change -- where ``sdf_handle`` would copy every weight to the host and pack it again
    each step.  The refresh re-rounds the FP16 ring stream too (round 4), so every precision
    marches on it."""
    from ..script_modules import resolve
    s = resolve(sdf)
    if isinstance(s, SkipConnMLP):
        th = train_handle(s)
        cached = getattr(s, "_nrt_train_sdf", None)
        if cached is None or cached[0] is not th:
            out = ctypes.c_void_p()
            _lib.check(_lib.load().nrt_sdf_create_mlp(th.value, ctypes.byref(out)), "nrt_sdf_create_mlp")
            cached = (th, _Handle(out, "nrt_sdf_destroy", [th]))
            object.__setattr__(s, "_nrt_train_sdf", cached)
        return cached[1].value
    if _is_sphere_sdf(s) and getattr(s, "shift", None) is not None:
        sph = (s.centers, s.radii, s.tfs)
        if not all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in sph):
            return sdf_handle(sdf)
        th = train_handle(s.shift)
        shapes = tuple((t.data_ptr(), tuple(t.shape)) for t in sph)
        vers = tuple(t._version for t in sph)
        cached = getattr(s, "_nrt_train_sdf", None)
        if cached is None or cached[0] is not th or cached[2] != shapes:
            c, r, t = _host(s.centers), _host(s.radii), _host(s.tfs)
            out = ctypes.c_void_p()
            _lib.check(_lib.load().nrt_sdf_create_sphere_blob(
                c.shape[0], c.data_ptr(), r.data_ptr(), t.data_ptr(), 32.0, th.value,
                ctypes.byref(out)), "nrt_sdf_create_sphere_blob")
            cached = [th, _Handle(out, "nrt_sdf_destroy", [th]), shapes, vers]
            object.__setattr__(s, "_nrt_train_sdf", cached)
        elif cached[3] != vers:
            _lib.call("nrt_sdf_refresh_spheres", cached[1].value, _lib.ptr(s.centers.detach()),
                      _lib.ptr(s.radii.detach()), _lib.ptr(s.tfs.detach()), _lib.stream())
            cached[3] = vers
        return cached[1].value
    return sdf_handle(sdf)


def march_handle(sdf):
    """The SDF handle a march uses: the training one while the SDF's parameters take
    gradients (the training loop), else the host-packed render handle."""
    return train_sdf_handle(sdf) if needs_grad(sdf) else sdf_handle(sdf)


def is_hip_sdf(sdf):
    """True for the SDFs nrt_sdf packs (SPHERE_SDF, SphereSDF, SkipConnMLP and their TorchScript
    modules); anything else is a callable the march evaluates between its HIP steps."""
    from ..script_modules import resolve
    try:
        s = resolve(sdf)
    except _lib.NrtError:
        return False
    return s is SPHERE_SDF or isinstance(s, SkipConnMLP) or _is_sphere_sdf(s)


def _looks_like_sphere_sdf(m):
    return all(hasattr(m, a) for a in ("centers", "radii", "tfs", "shift"))


def _is_sphere_sdf(m):
    return isinstance(m, SphereSDF) or _looks_like_sphere_sdf(m)


def sdf_eval(sdf, p):
    flat = p.reshape(-1, 3).float().contiguous()
    out = torch.empty(flat.shape[0], device=p.device)
    _lib.call("nrt_sdf_eval", sdf_handle(sdf), _lib.ptr(flat), flat.shape[0], _lib.ptr(out),
              _lib.precision_code(), _lib.stream())
    return out.reshape(p.shape[:-1])


class HipInteraction(MixedInteraction):
    """MixedInteraction produced by nrt_sdf_intersect.  ``raw_normals`` (the un-normalised
    gradients of the hit points, in hit-mask order, sdfs.py:154-155) is materialised on
    first access; it is None when nothing was hit, like the reference's missing attribute."""

    @property
    def raw_normals(self):
        if getattr(self, "_nrt_train", False):
            return self._nrt_raw_train
        if not hasattr(self, "_nrt_raw"):
            return None
        hit = self._nrt_hit_mask.reshape(-1)
        if not bool(hit.any()):
            return None
        return self._nrt_raw[hit]

    # ComposeSpatialVarying.eval_and_pdf / normalized_weights (bsdfs.py:515-536) set these on
    # the interaction for every ray of the tile, misses included; Direct.sample returns before
    # shading (and sets neither) when nothing was hit (integrators.py:171).  The fused path
    # evaluates them on first access: sp_var_fn(preprocess(p)) on the HIP MLP kernel.
    def _spatial_raw(self):
        d = self.__dict__
        if "nonnormalized_weights" in d:
            return d["nonnormalized_weights"]
        bsdf = d.get("_nrt_spatial")
        sp = getattr(bsdf, "sp_var_fn", None)
        if sp is None or not bool(self._nrt_hit_mask.any()):
            raise AttributeError("nonnormalized_weights")
        p = self.p
        w = sp(bsdf.preprocess(p)).reshape(p.shape[:-1] + (len(bsdf.bsdfs),))
        d["nonnormalized_weights"] = w
        return w

    @property
    def nonnormalized_weights(self):
        return self._spatial_raw()

    @nonnormalized_weights.setter
    def nonnormalized_weights(self, v):
        self.__dict__["nonnormalized_weights"] = v

    @property
    def normalized_weights(self):
        d = self.__dict__
        if "normalized_weights" not in d:
            d["normalized_weights"] = self._spatial_raw().sigmoid()
        return d["normalized_weights"]

    @normalized_weights.setter
    def normalized_weights(self, v):
        self.__dict__["normalized_weights"] = v


class SDF:
    """A general SDF shape with sphere-tracing intersection (sdfs.py:89-277)."""

    def __init__(self, device="cuda", sdf=SPHERE_SDF, epsilon=1e-3, max_steps=32, dist=2.2,
                 **kwargs):
        self.device = torch.device(device)
        self.sdf = sdf
        self.epsilon = epsilon
        self.max_steps = max_steps
        self.dist = dist

    def __len__(self):
        return 1

    def parameters(self):
        return self.sdf.parameters()

    def intersect(self, rays, max_t=10, active=True, primary: bool = True):
        """sdfs.py:111-160 on the HIP path.  ``primary`` draws ``random.random()`` for the
        coarse-scan jitter exactly like SDF.throughput (sdfs.py:236)."""
        if not is_hip_sdf(self.sdf):
            return self._intersect_callable(rays, max_t, primary)
        dev = rays.device
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        h = march_handle(self.sdf)
        t = torch.empty(P, device=dev)
        hit = torch.empty(P, dtype=torch.uint8, device=dev)
        p = torch.empty(P, 3, device=dev)
        n = torch.empty(P, 3, device=dev)
        raw = torch.empty(P, 3, device=dev)
        wi = torch.empty(P, 3, device=dev)
        thr = torch.empty(P, device=dev) if primary else None
        hit_idx = torch.empty(max(P, 1), dtype=torch.int32, device=dev)
        hit_count = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.load(require_device=True)
        ws_bytes = lib.nrt_intersect_workspace_bytes(h, P)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        scan_max_t = 0.0
        if primary:
            dist = getattr(self, "dist", 2.2)
            scan_max_t = dist + random.random() * (2 / 128)
        # training (sdfs.py:133-158 with autograd on): the march stays gradient-free; the scan
        # reports its argmin so sdf(best_pos) and the normals are recomputed with gradients
        train = needs_grad(self.sdf)
        scan_idx = torch.empty(P, dtype=torch.int32, device=dev) if (train and primary) else None
        mp = _lib.MarchParams(int(self.max_steps), float(self.epsilon), float(max_t), int(bool(primary)),
                              float(scan_max_t), _lib.precision_code(),
                              None if scan_idx is None else scan_idx.data_ptr())
        _lib.call("nrt_sdf_intersect", h, _lib.ptr(flat), P, ctypes.byref(mp), _lib.ptr(t),
                  _lib.ptr(hit), _lib.ptr(p), _lib.ptr(n), _lib.ptr(raw), _lib.ptr(wi),
                  _lib.ptr(thr), _lib.ptr(hit_idx), _lib.ptr(hit_count), _lib.ptr(ws), _lib.stream())
        hit_b = hit.bool().reshape(lead)
        if train:
            return self._differentiable(flat, t, hit_b.reshape(-1), scan_idx, scan_max_t, lead,
                                        (hit_idx, hit_count, flat)), hit_b
        throughput = thr.reshape(lead) if primary else 0
        si = HipInteraction(p=p.reshape(lead + (3,)), t=t.reshape(lead).squeeze(), obj=self,
                            throughput=throughput)
        si.n = n.reshape(lead + (3,))
        frame = torch.empty(P, 9, device=dev)
        _lib.call("nrt_frames", None, _lib.ptr(n), P, _lib.ptr(frame), None, _lib.stream())
        si.frame = frame.reshape(lead + (3, 3))
        si.wi = wi.reshape(lead + (3,))
        si._nrt_hits = (hit_idx, hit_count, flat)
        si._nrt_raw = raw
        si._nrt_hit_mask = hit_b
        return si, hit_b

    def _differentiable(self, flat, t, hit, scan_idx, scan_max_t, lead, hits):
        """The parts of sdfs.py:133-158 that carry gradients, at the march's and the scan's
        points: throughput = -1000 sdf(best_pos), raw normals (create_graph), p += 5 eps n,
        frames and wi."""
        o, d = flat[:, :3], flat[:, 3:]
        p0 = o + t.unsqueeze(-1) * d
        throughput = 0
        if scan_idx is not None:
            step = scan_max_t / 128
            best = o + scan_idx.long().unsqueeze(-1) * step * d
            throughput = (-1000 * sdf_value(self.sdf, best)).reshape(lead)
        n = torch.zeros_like(p0)
        p = p0
        raw = None
        # the march's compacted hit list, sorted (= hit-mask order, as p0[hit]): one host sync
        # for its length instead of one per boolean-mask gather / scatter and their backwards
        hit_idx, hit_count, _ = hits
        cnt = int(hit_count.item())
        if cnt > 0:
            idx = hit_idx[:cnt].long().sort().values
            ph = p0.index_select(0, idx)
            raw = sdf_gradient(self.sdf, ph)
            nh = F.normalize(raw, eps=1e-6, dim=-1)
            n = n.index_put((idx,), nh)
            p = p0.index_put((idx,), ph + nh * self.epsilon * 5)
        frame = coordinate_system(n)
        si = HipInteraction(p=p.reshape(lead + (3,)), t=t.reshape(lead).squeeze(), obj=self,
                            throughput=throughput)
        si.n = n.reshape(lead + (3,))
        si.frame = frame.reshape(lead + (3, 3))
        si.wi = si.to_local(-d.reshape(lead + (3,)))
        si._nrt_hits = hits
        si._nrt_train = True
        si._nrt_raw_train = raw
        si._nrt_hit_mask = hit.reshape(lead)
        return si

    def intersect_test(self, rays, max_t=10, active=True):
        """sdfs.py:162-181 via nrt_sdf_occlusion (a callable SDF: nrt_occlusion_callable_step)."""
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        mt = torch.as_tensor(max_t, dtype=torch.float32, device=rays.device)
        mt = mt.expand(lead + (1,)).reshape(P).contiguous() if mt.dim() > 0 else mt.expand(P).contiguous()
        vis = torch.empty(P, dtype=torch.uint8, device=rays.device)
        if not is_hip_sdf(self.sdf):
            self._occlusion_callable(flat, lead, mt, vis)
            return vis.bool().reshape(lead)
        _lib.call("nrt_sdf_occlusion", march_handle(self.sdf), _lib.ptr(flat), P, _lib.ptr(mt),
                  int(self.max_steps), float(self.epsilon), _lib.ptr(vis), _lib.precision_code(),
                  _lib.stream())
        return vis.bool().reshape(lead)

    # ---- SDF callables: the callable between HIP steps ------------------------------------------

    def _eval_callable(self, q, lead):
        """self.sdf on the query points in the rays' shape (what the reference passes), flattened
        to one f32 distance per ray."""
        P = q.shape[0]
        d = self.sdf(q.reshape(lead + (3,)))
        if not torch.is_tensor(d) or d.numel() != P:
            raise _lib.NrtError(f"SDF callable returned {tuple(getattr(d, 'shape', ()))} for "
                                f"{tuple(lead)} points (one distance per point expected)")
        return d.detach().reshape(P).float().contiguous()

    def _intersect_callable(self, rays, max_t, primary):
        """sdfs.py:111-160 for an SDF callable: max_steps evaluations of the callable on every
        ray (as the reference) with the depth / remaining / hit update and the next points in
        nrt_march_callable_step; the 129-point coarse scan with nrt_scan_callable_step; then
        throughput = -1000 sdf(best_pos) and the autograd normals through the callable."""
        dev = rays.device
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        t = torch.empty(P, device=dev)
        rem = torch.empty(P, dtype=torch.uint8, device=dev)
        hit = torch.empty(P, dtype=torch.uint8, device=dev)
        q = torch.empty(P, 3, device=dev)
        steps, eps = int(self.max_steps), float(self.epsilon)

        def march(d, prep):
            _lib.call("nrt_march_callable_step", _lib.ptr(flat), P, _lib.ptr(d), eps, float(max_t),
                      prep, _lib.ptr(t), _lib.ptr(rem), _lib.ptr(hit), _lib.ptr(q), _lib.stream())
        with torch.no_grad():
            march(None, 1 if steps > 0 else 0)
            for i in range(steps):
                march(self._eval_callable(q, lead), 1 if i + 1 < steps else 0)
        p0 = q  # r_o + depth r_d (sdfs.py:133)
        throughput = 0
        if primary:
            dist = getattr(self, "dist", 2.2)
            step = (dist + random.random() * (2 / 128)) / 128
            best = flat[:, :3].contiguous()
            cmin = torch.empty(P, device=dev)
            idx = torch.empty(P, dtype=torch.int32, device=dev)
            with torch.no_grad():
                for j in range(129):
                    sd = self._eval_callable(best, lead)
                    _lib.call("nrt_scan_callable_step", _lib.ptr(flat), P, _lib.ptr(sd), j, step,
                              1 if j < 128 else 2, _lib.ptr(cmin), _lib.ptr(idx), _lib.ptr(best),
                              _lib.stream())
            # sdf(best_pos) outside no_grad (sdfs.py:249): differentiable through the callable
            throughput = -1000 * self.sdf(best.reshape(lead + (3,)))
        hit_b = hit.bool()
        n = torch.zeros(P, 3, device=dev)
        p = p0.clone()
        raw = None
        graph = False
        if bool(hit_b.any()):
            # create_graph only when the normals can carry gradients: grad mode on and the
            # callable's output depends on a parameter that requires one (a render with grad
            # mode on over frozen weights -- edit_dtu.py's bend around a loaded SDF -- keeps
            # first-order normals, which every HIP MLP supports)
            graph = self._callable_needs_graph(p0[hit_b])
            raw = self._callable_normals(p0[hit_b], create_graph=graph)
            nh = F.normalize(raw, eps=1e-6, dim=-1)
            n = n.index_put((hit_b,), nh)
            p = p.index_put((hit_b,), p0[hit_b] + nh * self.epsilon * 5)
        si = HipInteraction(p=p.reshape(lead + (3,)), t=t.reshape(lead).squeeze(), obj=self,
                            throughput=throughput)
        si.n = n.reshape(lead + (3,))
        if raw is not None and raw.requires_grad:
            # normals with a graph: frame and wi differentiable as in _differentiable
            si.frame = coordinate_system(n).reshape(lead + (3, 3))
            si.wi = si.to_local(-flat[:, 3:].reshape(lead + (3,)))
        else:
            frame = torch.empty(P, 9, device=dev)
            wi = torch.empty(P, 3, device=dev)
            _lib.call("nrt_frames", _lib.ptr(flat), _lib.ptr(n.contiguous()), P, _lib.ptr(frame),
                      _lib.ptr(wi), _lib.stream())
            si.frame = frame.reshape(lead + (3, 3))
            si.wi = wi.reshape(lead + (3,))
        hit_idx = torch.nonzero(hit_b).reshape(-1).to(torch.int32)
        hit_count = torch.tensor([hit_idx.numel()], dtype=torch.int32, device=dev)
        si._nrt_hits = (hit_idx if hit_idx.numel() else torch.zeros(1, dtype=torch.int32, device=dev),
                        hit_count, flat)
        raw_full = torch.zeros(P, 3, device=dev)
        if raw is not None:
            raw_full[hit_b] = raw.detach()
        si._nrt_raw = raw_full
        si._nrt_hit_mask = hit_b.reshape(lead)
        if raw is not None and raw.requires_grad:
            si._nrt_train = True  # raw_normals keeps its graph (the eikonal term)
            si._nrt_raw_train = raw
        return si, hit_b.reshape(lead)

    def _callable_needs_graph(self, p):
        """True when grad mode is on and sdf(p) requires grad for points that do not: some
        parameter the callable closes over takes gradients."""
        if not torch.is_grad_enabled():
            return False
        with torch.enable_grad():
            out = self.sdf(p.detach())
        return torch.is_tensor(out) and out.requires_grad

    def _callable_normals(self, p, create_graph=True):
        """SDF.autograd_diff (sdfs.py:184-197) through the callable: create_graph, so the normal
        carries gradients for whatever parameters the callable closes over (a render under
        no_grad takes the same values without the graph)."""
        from ..neural_blocks import diff_points
        with torch.enable_grad():
            q = diff_points(p)  # the point leaf (not a trainable input of the callable)
            out = self.sdf(q)
            (g,) = torch.autograd.grad(out, q, torch.ones_like(out), create_graph=create_graph)
        return g if create_graph else g.detach()

    def _occlusion_callable(self, flat, lead, mt, vis):
        P = flat.shape[0]
        dev = flat.device
        depth = torch.empty(P, device=dev)
        rem = torch.empty(P, dtype=torch.uint8, device=dev)
        q = torch.empty(P, 3, device=dev)
        steps, eps = int(self.max_steps), float(self.epsilon)
        t0 = 1e2 * self.epsilon  # zeros(...) + 1e2 * epsilon (sdfs.py:165-166)

        def step(d, phase):
            _lib.call("nrt_occlusion_callable_step", _lib.ptr(flat), P, _lib.ptr(d), eps, t0,
                      _lib.ptr(mt), phase, _lib.ptr(depth), _lib.ptr(rem), _lib.ptr(q),
                      _lib.ptr(vis), _lib.stream())
        with torch.no_grad():
            step(None, 0)
            if steps == 0:
                # no step taken: visible = depth >= max_t | remaining (all remaining)
                vis.fill_(1)
                return
            for i in range(steps):
                step(self._eval_callable(q, lead), 2 if i + 1 == steps else 1)

    def autograd_diff(self, p):
        """Normal direction d sdf / dp (sdfs.py:184-197) from the f32 backward kernel; with
        autograd on and trainable SDF parameters the result is differentiable
        (create_graph=True, nrt_mlp_grad_backward).  A callable SDF: autograd through it."""
        if not is_hip_sdf(self.sdf):
            return self._callable_normals(p.reshape(-1, 3),
                                          create_graph=torch.is_grad_enabled()).reshape(p.shape)
        if needs_grad(self.sdf):
            return sdf_gradient(self.sdf, p)
        flat = p.reshape(-1, 3).float().contiguous()
        g = torch.empty_like(flat)
        _lib.call("nrt_sdf_grad", sdf_handle(self.sdf), _lib.ptr(flat), flat.shape[0], _lib.ptr(g),
                  _lib.stream())
        return g.reshape(p.shape)


class RoundBoxSDF(nn.Module):
    """Rounded boxes smooth-min-ed together (sdfs.py:48-68): import-resolvable for the drivers
    (nerf_synthetic.py:14-16, dtu.py:18-20); constructor and RNG order as the reference.  Not a
    HIP SDF kind: SDF(sdf=RoundBoxSDF()) raises NrtError when it is marched."""

    def __init__(self, n=2 << 4, device="cuda"):
        super().__init__()
        self.centers = nn.Parameter(0.3 * torch.rand(n, 3, device=device, requires_grad=True) - 0.15)
        self.b = nn.Parameter(0.2 * torch.rand_like(self.centers, requires_grad=True))
        self.radii = nn.Parameter(0.2 * torch.rand(n, device=device, requires_grad=True) - 0.1)
        self.tfs = nn.Parameter(torch.zeros(n, 3, 3, device=device, requires_grad=True))

    def forward(self, p):
        raise _lib.NrtError("RoundBoxSDF has no HIP implementation (supported SDFs: SPHERE_SDF, "
                            "SphereSDF, SkipConnMLP)")


class CapsuleSDF(nn.Module):
    """Capsules smooth-min-ed together (sdfs.py:72-86): import-resolvable, like RoundBoxSDF."""

    def __init__(self, n=2 << 5, device="cuda"):
        super().__init__()
        self.a = nn.Parameter(0.1 * torch.rand(n, 3, device=device, requires_grad=True) - 0.05)
        self.b = nn.Parameter(0.1 * torch.rand_like(self.a, requires_grad=True) - 0.05)
        self.radii = nn.Parameter(0.1 * torch.rand(n, device=device, requires_grad=True) - 0.05)

    def forward(self, p):
        raise _lib.NrtError("CapsuleSDF has no HIP implementation (supported SDFs: SPHERE_SDF, "
                            "SphereSDF, SkipConnMLP)")
