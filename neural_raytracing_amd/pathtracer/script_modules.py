"""TorchScript SDF modules on the HIP path (the SDF-callable protocol).

The drivers pass ``torch.jit.load``-ed modules straight into ``SDF(sdf=...)``: a scripted
``SphereSDF`` (nerf_synthetic.py:63, dtu.py:93, edit_dtu.py:83) and, by the same protocol, a
scripted ``SkipConnMLP``.  They keep using the ScriptModule afterwards -- its ``parameters()`` feed
the optimiser (nerf_synthetic.py:82) and ``torch.jit.save(density_field.sdf, ...)`` writes it back
(:119) -- so the SDF must stay that object.  The HIP path therefore reads it through *views*:

* ``MlpView`` -- a ``SkipConnMLP`` whose ``init`` / ``layers`` / ``out`` / ``basis_p`` are the
  ScriptModule's own tensors, read live (an optimiser step on the ScriptModule is seen by the next
  pack, and autograd through the HIP MLP kernels accumulates into the ScriptModule's parameters).
  The activation is not an attribute of a scripted module (TorchScript compiles the function
  into ``forward``), so it is read from the compiled code: ``torch.softplus`` / ``leaky_relu`` /
  ``relu`` / ``sigmoid``.
* ``SphereView`` -- ``centers`` / ``radii`` / ``tfs`` of a scripted SphereSDF plus an ``MlpView`` of
  its ``shift``.

Nothing of the ScriptModule is executed; a scripted module of any other layout raises NrtError.
"""
import re
import weakref

import torch
import torch.nn as nn

from .. import _lib
from .neural_blocks import SkipConnMLP, activation_code

_VIEWS = weakref.WeakKeyDictionary()

_ACT_PATTERNS = [("leaky_relu", "leaky_relu"), ("softplus", "softplus"), ("sigmoid", "sigmoid"),
                 ("relu", "relu")]


def _code(sm):
    try:
        return sm.code
    except Exception:  # noqa: BLE001 -- a module without a compiled forward
        return ""


def scripted_activation(sm):
    """The activation a scripted SkipConnMLP applies, from its compiled forward."""
    code = _code(sm)
    found = []
    rest = code
    for pat, name in _ACT_PATTERNS:
        if re.search(r"\b" + pat + r"_?\(", rest):
            found.append(name)
            rest = re.sub(r"\b" + pat + r"_?\(", "(", rest)
    if len(found) != 1:
        raise _lib.NrtError("scripted SkipConnMLP: cannot identify its activation from the "
                            f"compiled forward (found {found or 'none'})")
    return {"leaky_relu": torch.nn.functional.leaky_relu, "softplus": torch.nn.functional.softplus,
            "sigmoid": torch.sigmoid, "relu": torch.relu}[found[0]]


class _LinearView:
    """An nn.Linear of a ScriptModule seen through its live weight / bias tensors."""

    def __init__(self, lin):
        self._lin = lin

    @property
    def weight(self):
        return self._lin.weight

    @property
    def bias(self):
        return self._lin.bias

    @property
    def out_features(self):
        return self._lin.weight.shape[0]

    @property
    def in_features(self):
        return self._lin.weight.shape[1]


class MlpView(SkipConnMLP):
    """A scripted SkipConnMLP (neural_blocks.py:12-86) for the HIP MLP kernels."""

    def __init__(self, sm, activation=None):
        nn.Module.__init__(self)
        object.__setattr__(self, "_sm", sm)
        self.in_size = int(sm.in_size)
        self.skip = int(sm.skip)
        self.latent_size = int(getattr(sm, "latent_size", 0) or 0)
        self.activation = activation if activation is not None else scripted_activation(sm)
        activation_code(self.activation)  # supported on the HIP path
        self.init = _LinearView(sm.init)
        # a loaded ScriptModule's ModuleList does not iterate; its children are named "0", "1", ...
        kids = sorted(sm.layers.named_children(), key=lambda kv: int(kv[0]))
        self.layers = [_LinearView(lin) for _, lin in kids]
        self.out = _LinearView(sm.out)
        self.dim_p = self.init.in_features

    @property
    def basis_p(self):
        return self._sm.basis_p

    def _apply(self, fn, *args, **kwargs):
        raise _lib.NrtError("move the ScriptModule itself (torch.jit.load(path, device))")

    def parameters(self, recurse=True):
        return self._sm.parameters()


class SphereView(nn.Module):
    """A scripted SphereSDF (sdfs.py:16-44): its tensors and an MlpView of the shift MLP."""

    def __init__(self, sm):
        super().__init__()
        object.__setattr__(self, "_sm", sm)
        shift = getattr(sm, "shift", None)
        # SphereSDF.shift is SkipConnMLP(..., activation=F.softplus) (sdfs.py:23-31)
        self.shift = None if shift is None else (
            shift if isinstance(shift, SkipConnMLP) else MlpView(shift, torch.nn.functional.softplus))

    centers = property(lambda self: self._sm.centers)
    radii = property(lambda self: self._sm.radii)
    tfs = property(lambda self: self._sm.tfs)

    def parameters(self, recurse=True):
        return self._sm.parameters()


def _has(sm, *names):
    return all(hasattr(sm, n) for n in names)


def resolve(sdf):
    """The object the HIP path packs for an SDF callable: ScriptModules become (cached) views,
    everything else is returned unchanged."""
    if not isinstance(sdf, torch.jit.ScriptModule):
        return sdf
    v = _VIEWS.get(sdf)
    if v is None:
        if _has(sdf, "centers", "radii", "tfs", "shift"):
            v = SphereView(sdf)
        elif _has(sdf, "init", "layers", "out", "basis_p", "in_size", "skip"):
            v = MlpView(sdf)
        else:
            raise _lib.NrtError(f"scripted SDF {getattr(sdf, 'original_name', '?')} has no HIP "
                                "implementation (supported: SphereSDF, SkipConnMLP)")
        _VIEWS[sdf] = v
    return v
