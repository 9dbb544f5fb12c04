"""Packed-weight handles: nn.Module parameters -> nrt_mlp / nrt_sdf / nrt_light / nrt_bsdf.

A handle is rebuilt when any parameter's storage or version counter changes, so a module that
is edited between renders is re-packed; packing copies the weights to the host once.
"""
import ctypes
import weakref

import torch

from .. import _lib


def _key(tensors):
    return tuple((t.data_ptr(), t._version, tuple(t.shape)) for t in tensors)


class _Handle:
    """Owns one C handle and destroys it with ``destroy_fn`` when dropped."""

    def __init__(self, value, destroy_fn, deps=()):
        self.value = value
        self.deps = list(deps)  # keep child handles alive
        self._fin = weakref.finalize(self, _destroy, destroy_fn, value)


def _destroy(fn, value):
    try:
        lib = _lib.load()
        getattr(lib, fn)(value)
    except Exception:
        pass


def _host(t):
    return t.detach().to("cpu", torch.float32).contiguous()


def _cache(owner, tensors, build, extra=()):
    key = (_key(tensors), tuple(extra))
    cached = getattr(owner, "_nrt_cache", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    h = build()
    object.__setattr__(owner, "_nrt_cache", (key, h))
    return h


def mlp_handle(mlp):
    """nrt_mlp for a SkipConnMLP-shaped module (init / layers / out / basis_p)."""
    params = [mlp.basis_p] + [p for lin in mlp._linears() for p in (lin.weight, lin.bias)]

    def build():
        lib = _lib.load()
        desc = _lib.MlpDesc(mlp.in_size, mlp.init.out_features, len(mlp.layers),
                            mlp.out.out_features, mlp.basis_p.shape[1], mlp.skip, mlp.latent_size,
                            _lib.ACT[mlp.activation_code()])
        basis = _host(mlp.basis_p)
        ws = [_host(lin.weight) for lin in mlp._linears()]
        bs = [_host(lin.bias) for lin in mlp._linears()]
        wp = (ctypes.c_void_p * len(ws))(*[w.data_ptr() for w in ws])
        bp = (ctypes.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
        out = ctypes.c_void_p()
        _lib.check(lib.nrt_mlp_create(ctypes.byref(desc), basis.data_ptr(), wp, bp,
                                      ctypes.byref(out)), "nrt_mlp_create")
        return _Handle(out, "nrt_mlp_destroy")

    # the activation is packed too (and folded into the FP16 ring stream): re-pack on a change
    return _cache(mlp, params, build, extra=(mlp.activation_code(),))


def train_handle(mlp):
    """The nrt_mlp the training kernels read (nrt_mlp_forward / _backward / _grad_backward):
    packed on the host once, then re-packed on the device by nrt_mlp_refresh whenever an
    optimiser step has changed the weights -- no host round trip per step.  Rendering keeps
    using ``mlp_handle`` (a refreshed handle does not serve the FP16 ring / program kernels)."""
    lins = mlp._linears()
    ws = [lin.weight for lin in lins]
    bs = [lin.bias for lin in lins]
    shape_key = (mlp.basis_p.data_ptr(), mlp.basis_p._version, mlp.activation_code(),
                 tuple((w.data_ptr(), tuple(w.shape)) for w in ws + bs))
    vers = tuple(t._version for t in ws + bs)
    th = getattr(mlp, "_nrt_train", None)
    if th is None or th[0] != shape_key or not all(
            t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() for t in ws + bs):
        h = _TrainBuild(mlp)
        object.__setattr__(mlp, "_nrt_train", (shape_key, vers, h))
        return h
    if th[1] != vers:
        wp = (ctypes.c_void_p * len(ws))(*[w.data_ptr() for w in ws])
        bp = (ctypes.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
        _lib.call("nrt_mlp_refresh", th[2].value, wp, bp, _lib.stream())
        object.__setattr__(mlp, "_nrt_train", (shape_key, vers, th[2]))
    return th[2]


def _TrainBuild(mlp):
    """A fresh host-packed handle of the module's current weights (same as mlp_handle's)."""
    lins = mlp._linears()
    lib = _lib.load()
    desc = _lib.MlpDesc(mlp.in_size, mlp.init.out_features, len(mlp.layers),
                        mlp.out.out_features, mlp.basis_p.shape[1], mlp.skip, mlp.latent_size,
                        _lib.ACT[mlp.activation_code()])
    basis = _host(mlp.basis_p)
    ws = [_host(lin.weight) for lin in lins]
    bs = [_host(lin.bias) for lin in lins]
    wp = (ctypes.c_void_p * len(ws))(*[w.data_ptr() for w in ws])
    bp = (ctypes.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
    out = ctypes.c_void_p()
    _lib.check(lib.nrt_mlp_create(ctypes.byref(desc), basis.data_ptr(), wp, bp, ctypes.byref(out)),
               "nrt_mlp_create")
    return _Handle(out, "nrt_mlp_destroy")
