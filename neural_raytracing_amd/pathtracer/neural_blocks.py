"""SkipConnMLP with the reference's constructor (neural_blocks.py:12-86); forward runs on the
fused HIP kernel ``nrt_mlp_forward`` (one wavefront = 32 rows, every layer an MFMA GEMM).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib
from ._handles import mlp_handle, train_handle
from .utils import create_fourier_basis2


def _leaky(x):
    return F.leaky_relu(x)


def activation_code(fn):
    """Map a torch activation callable to an NRT_ACT code (raises for anything else)."""
    if fn is None or fn is _leaky or fn is F.leaky_relu:
        return "leaky_relu"
    if isinstance(fn, nn.LeakyReLU) and fn.negative_slope == 0.01:
        return "leaky_relu"
    if fn is F.softplus or (isinstance(fn, nn.Softplus) and fn.beta == 1 and fn.threshold == 20):
        return "softplus"
    if fn in (F.relu, torch.relu) or isinstance(fn, nn.ReLU):
        return "relu"
    if fn in (torch.sigmoid, F.sigmoid) or isinstance(fn, nn.Sigmoid):
        return "sigmoid"
    name = getattr(fn, "__name__", type(fn).__name__)
    raise _lib.NrtError(f"activation {name!r} has no HIP implementation "
                        "(supported: leaky_relu(0.01), softplus, relu, sigmoid)")


class SkipConnMLP(nn.Module):
    """MLP with skip connections and Fourier encoding (neural_blocks.py:12-86).

    Construction consumes the RNG exactly like the reference: Fourier basis, the hidden
    ``nn.Linear`` list, ``init``, ``out``, then optional zero / xavier re-initialisation.
    """

    def __init__(self, num_layers=8, hidden_size=64, in_size=3, out=3, skip=3, freqs=16,
                 sigma=2 << 4, device="cuda", activation=_leaky, latent_size=0,
                 zero_init=False, xavier_init=False):
        super().__init__()
        self.in_size = in_size
        assert type(freqs) == int
        self.basis_p, map_size = create_fourier_basis2(freqs, features=in_size, freq=sigma,
                                                       device=device)
        self.dim_p = map_size + latent_size
        self.skip = skip
        self.latent_size = latent_size
        skip_size = hidden_size + self.dim_p
        self.layers = nn.ModuleList([
            nn.Linear(skip_size if (i % skip) == 0 and i != num_layers - 1 else hidden_size,
                      hidden_size)
            for i in range(num_layers)
        ])
        self.init = nn.Linear(self.dim_p, hidden_size)
        self.out = nn.Linear(hidden_size, out)
        ordered = [self.init, self.out, *self.layers]
        if zero_init:
            for lin in ordered:
                nn.init.zeros_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)
        if xavier_init:
            for lin in ordered:
                nn.init.xavier_uniform_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)
        self.activation = activation

    def _apply(self, fn, *args, **kwargs):
        # basis_p is a plain tensor attribute in the reference too; move it with the module
        out = super()._apply(fn, *args, **kwargs)
        self.basis_p = fn(self.basis_p)
        return out

    def _linears(self):
        return [self.init, *self.layers, self.out]

    def activation_code(self):
        return activation_code(self.activation)

    def nrt(self):
        return mlp_handle(self).value

    def forward(self, p, latent=None):
        if not p.is_cuda:
            raise _lib.NrtError("SkipConnMLP evaluates on the HIP path only: move it and its "
                                "inputs to the GPU")
        batches = p.shape[:-1]
        x = p.reshape(-1, self.in_size).float().contiguous()
        lat = None
        if latent is not None:
            lat = latent.reshape(-1, self.latent_size).float().contiguous()
        params = [t for lin in self._linears() for t in (lin.weight, lin.bias)]
        needs_grad = torch.is_grad_enabled() and (
            x.requires_grad or (lat is not None and lat.requires_grad) or
            any(q.requires_grad for q in params))
        if needs_grad:
            if any(t.device != p.device for t in params):
                # as nn.Linear would: the HIP backward writes gradients next to the parameters
                raise _lib.NrtError("SkipConnMLP parameters and inputs are on different devices: "
                                    "move the module to the GPU (.to(device)) to train it")
            # autograd through the HIP MLP: nrt_mlp_forward, then nrt_mlp_backward (FP32)
            y = _MlpFn.apply(self, x, lat, *params)
        else:
            y = _mlp_forward(self, x, lat)
        return y.reshape(batches + (self.out.out_features,))


def _mlp_forward(mlp, x, lat, handle=None):
    y = torch.empty(x.shape[0], mlp.out.out_features, device=x.device)
    h = mlp.nrt() if handle is None else handle.value
    _lib.call("nrt_mlp_forward", h, _lib.ptr(x), _lib.ptr(lat), x.shape[0],
              _lib.ptr(y), _lib.precision_code(), _lib.stream())
    return y


def _forward_saving(handles, x, outs, keep=True):
    """ys[k] = mlp_k(x) for same-shape MLPs (no latent) in one nrt_mlp_forward_multi call.  Under
    FP32 (and the mixed march's FP32 MLPs) with a ring-backward shape (nrt_mlp_save_bytes > 0) the
    forward also saves the activations its backward reads -> (ys, save buffers) -- else
    (ys, None) and the backward evaluates the forward again.  The save costs (L + 1) M H + 2 M dp
    floats per MLP (about 11 KB a row for LightField 10x256): keep=False (a module in eval mode,
    where a backward is not expected) skips it, and a backward that does come recomputes."""
    import ctypes
    lib = _lib.load(require_device=True)
    n, M = len(handles), x.shape[0]
    ys = [torch.empty(M, o, device=x.device) for o in outs]
    P = ctypes.c_void_p
    hs = (P * n)(*[h.value for h in handles])
    save = None
    if keep and M > 0 and _lib.precision_code() != _lib.NRT_FP16:
        nbytes = [lib.nrt_mlp_save_bytes(h.value, M) for h in handles]
        if all(nbytes):
            save = [torch.empty(b, dtype=torch.uint8, device=x.device) for b in nbytes]
    _lib.call("nrt_mlp_forward_multi", hs, n, _lib.ptr(x), M, (P * n)(*[y.data_ptr() for y in ys]),
              None if save is None else (P * n)(*[b.data_ptr() for b in save]),
              _lib.precision_code(), _lib.stream())
    return ys, save


def _save_versions(ctx, params):
    """The backward kernels read the packed copy of the weights (the training handle, re-packed in
    place by nrt_mlp_refresh after an optimiser step), not saved tensors, so autograd's own
    saved-tensor version check cannot see an in-place update: keep the versions and compare."""
    ctx.param_refs = params
    ctx.param_versions = tuple(q._version for q in params)


def _check_versions(ctx):
    if tuple(q._version for q in ctx.param_refs) != ctx.param_versions:
        raise RuntimeError("one of the variables needed for gradient computation has been "
                           "modified by an inplace operation: a SkipConnMLP weight changed "
                           "(e.g. optimizer.step()) between this graph's forward and backward")


# A backward compacts its rows to those whose incoming gradient is not all zero when that drops
# at least this fraction of them: a zero row adds exactly nothing to any weight or bias gradient
# and its dL/dx is 0.  Under the reference's masks (Direct.sample zeroes missed rays' shading,
# integrators.py:167-189; ComposeSpatialVarying weights every ray, bsdfs.py:515-536) the shading
# MLPs of a training step see dY = 0 on every ray that missed.
COMPACT_MIN_DEAD = 0.1


def _live_rows(dys, M):
    """Indices of the rows with a nonzero (or NaN) incoming gradient in any output, or None when
    compaction would not pay (one host synchronisation per backward call)."""
    live = (dys[0] != 0).any(-1)
    for d in dys[1:]:
        live |= (d != 0).any(-1)
    idx = torch.nonzero(live).reshape(-1)
    return None if idx.numel() > (1.0 - COMPACT_MIN_DEAD) * M else idx


class _MlpFn(torch.autograd.Function):
    """y = SkipConnMLP(x, latent) with gradients for x, latent and every nn.Linear weight and
    bias from nrt_mlp_backward.  basis_p is a plain tensor attribute in the
    reference (no gradient), as here."""

    @staticmethod
    def forward(ctx, mlp, x, lat, *params):
        handle = train_handle(mlp)  # device re-pack after an optimiser step
        ctx.save = None
        with torch.no_grad():
            if lat is None:
                ys, ctx.save = _forward_saving([handle], x.detach(), [mlp.out.out_features],
                                               keep=mlp.training)
                y = ys[0]
            else:
                y = _mlp_forward(mlp, x.detach(), lat.detach(), handle)
        ctx.mlp = mlp
        ctx.handle = handle  # the packed weights this forward used
        _save_versions(ctx, params)
        ctx.has_lat = lat is not None
        ctx.save_for_backward(x, lat if lat is not None else x.new_empty(0))
        return y

    @staticmethod
    def backward(ctx, dy):
        _check_versions(ctx)
        if torch.is_grad_enabled():
            return _MlpFn._backward_create_graph(ctx, dy)
        dx, dlat, grads = _MlpFn._first_order(ctx, dy)
        return (None, dx, dlat, *grads)

    @staticmethod
    def _first_order(ctx, dy):
        """dL/dx, dL/dlatent and the nn.Linear gradients from nrt_mlp_backward (no graph)."""
        import ctypes
        x, lat = ctx.saved_tensors
        x = x.detach()
        lat = lat.detach() if ctx.has_lat else None
        mlp = ctx.mlp
        lib = _lib.load(require_device=True)
        M = x.shape[0]
        dy = dy.detach().float().contiguous()
        lins = mlp._linears()
        idx = _live_rows([dy], M)
        if idx is not None:  # the rows with a gradient only (COMPACT_MIN_DEAD)
            full_x, full_lat = x, lat
            x, dy = x[idx].contiguous(), dy[idx].contiguous()
            lat = None if lat is None else lat[idx].contiguous()
            M = x.shape[0]
        dx = torch.empty_like(x) if ctx.needs_input_grad[1] else None
        dlat = torch.empty_like(lat) if (lat is not None and ctx.needs_input_grad[2]) else None
        zeros = M == 0
        mk = torch.zeros_like if zeros else torch.empty_like
        dws = [mk(lin.weight) if lin.weight.requires_grad else None for lin in lins]
        dbs = [mk(lin.bias) if lin.bias.requires_grad else None for lin in lins]
        wp = (ctypes.c_void_p * len(lins))(*[0 if t is None else t.data_ptr() for t in dws])
        bp = (ctypes.c_void_p * len(lins))(*[0 if t is None else t.data_ptr() for t in dbs])
        if not zeros and ctx.save is not None:  # the forward saved the activations
            P = ctypes.c_void_p
            ws = torch.empty(lib.nrt_mlp_backward_multi_workspace_bytes((P * 1)(ctx.handle.value), 1, M),
                             dtype=torch.uint8, device=x.device)
            rows = None if idx is None else idx.to(torch.int32)
            _lib.call("nrt_mlp_backward_saved", (P * 1)(ctx.handle.value), 1, _lib.ptr(x), M,
                      _lib.ptr(rows), (P * 1)(ctx.save[0].data_ptr()), full_x.shape[0] if idx is not None else M,
                      (P * 1)(dy.data_ptr()), None if dx is None else (P * 1)(dx.data_ptr()),
                      wp, bp, _lib.ptr(ws), _lib.stream())
        elif not zeros:
            ws = torch.empty(lib.nrt_mlp_backward_workspace_bytes(ctx.handle.value, M),
                             dtype=torch.uint8, device=x.device)
            _lib.call("nrt_mlp_backward", ctx.handle.value, _lib.ptr(x), _lib.ptr(lat), M,
                      _lib.ptr(dy), _lib.ptr(dx), _lib.ptr(dlat), wp, bp, _lib.ptr(ws),
                      _lib.stream())
        if idx is not None:  # scatter back: dL/dx = 0 on the rows without a gradient
            if dx is not None:
                dx = torch.zeros_like(full_x).index_copy_(0, idx, dx)
            if dlat is not None:
                dlat = torch.zeros_like(full_lat).index_copy_(0, idx, dlat)
        return dx, dlat, [g for pair in zip(dws, dbs) for g in pair]

    @staticmethod
    def _backward_create_graph(ctx, dy):
        """backward under create_graph=True -- SDF.autograd_diff (sdfs.py:184-197) through an SDF
        callable that wraps a trainable SkipConnMLP (edit_dtu.py:86-100: bend / disp): the input
        gradient as a differentiable function of the weights.  For a one-output MLP,
        dL/dx = dy * g(x) with g = d y / d x (input_gradient: nrt_mlp_backward forward,
        nrt_mlp_grad_backward for its weight gradients) and dy a differentiable tensor too.  The
        second derivative with respect to x itself is not formed: the points come from the no-grad
        march, and a graph from x back to a trainable parameter raises.  The nn.Linear gradients
        returned beside it carry no graph (autograd_diff asks for the points' gradient only)."""
        x, lat = ctx.saved_tensors
        mlp = ctx.mlp
        if ctx.has_lat:
            raise _lib.NrtError("second derivatives through a latent SkipConnMLP are not on the "
                                "HIP path")
        if mlp.out.out_features != 1:
            raise _lib.NrtError("second derivatives through SkipConnMLP.forward are on the HIP "
                                "path for one-output MLPs (an SDF) only")
        if _parameters_upstream(x):
            raise _lib.NrtError("second derivatives with respect to the MLP's inputs are not on "
                                "the HIP path: the SDF callable's points depend on a tensor that "
                                "takes gradients")
        with torch.no_grad():
            _, dlat, grads = _MlpFn._first_order(ctx, dy)
        dx = None
        if ctx.needs_input_grad[1]:
            g = input_gradient(mlp, x.detach())
            dx = dy.reshape(-1, 1).to(g.dtype) * g
        return (None, dx, dlat, *grads)


def diff_points(p):
    """A leaf copy of the points p that autograd differentiates an SDF at (SDF.autograd_diff,
    sdfs.py:184-197): tagged so the create_graph backward knows the leaf is the point set the
    normal is taken at, not a trainable input (_parameters_upstream)."""
    q = p.detach().requires_grad_(True)
    q._nrt_diff_points = True
    return q


def _trainable_leaf(v, x):
    """A leaf of x's graph that takes gradients and is not the point set being differentiated:
    an nn.Parameter, or a requires_grad tensor of another size than x (a learned pose or offset
    held as a bare tensor).  A bare leaf with x's element count is the points themselves --
    SDF.autograd_diff's p.requires_grad_() (sdfs.py:186), possibly warped into x -- as is a
    diff_points leaf."""
    if v is None or not v.requires_grad or getattr(v, "_nrt_diff_points", False):
        return False
    return isinstance(v, nn.Parameter) or v.numel() != x.numel()


def _parameters_upstream(t, limit=20000):
    """True when the autograd graph of `t` (the MLP's input) reaches a leaf that takes gradients
    other than the point set itself (_trainable_leaf).  A graph larger than `limit` nodes counts as
    reaching one (the caller then refuses rather than dropping a term silently)."""
    fn = t.grad_fn
    if fn is None:
        return isinstance(t, nn.Parameter)
    seen, stack = set(), [fn]
    while stack:
        if len(seen) >= limit:
            return True
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        if _trainable_leaf(getattr(f, "variable", None), t):  # AccumulateGrad of a leaf
            return True
        stack.extend(n for n, _ in getattr(f, "next_functions", ()))
    return False


def _shape_key(m):
    return (m.in_size, m.init.out_features, len(m.layers), m.out.out_features, m.skip,
            m.latent_size, m.activation_code(), tuple(m.basis_p.shape))


def same_shape(mlps):
    """True when the SkipConnMLPs share one architecture (nrt_mlp_backward_multi's condition)."""
    k = _shape_key(mlps[0])
    return all(_shape_key(m) == k for m in mlps[1:])


def mlp_multi(mlps, x):
    """[mlp(x) for mlp in mlps] for same-shape SkipConnMLPs (no latent) on one input -- the
    NeuralBSDFs of a spatially varying mixture on the shared Rusinkiewicz features
    (bsdfs.py:634-637).  Under autograd the backward of all of them is one
    nrt_mlp_backward_multi call (one backward launch, one weight-gradient launch)."""
    flat = x.reshape(-1, mlps[0].in_size).float().contiguous()
    params = [t for m in mlps for lin in m._linears() for t in (lin.weight, lin.bias)]
    if not (torch.is_grad_enabled() and (flat.requires_grad or any(q.requires_grad for q in params))):
        return [m(x) for m in mlps]
    if any(t.device != x.device for t in params):
        raise _lib.NrtError("SkipConnMLP parameters and inputs are on different devices: "
                            "move the module to the GPU (.to(device)) to train it")
    ys = _MultiMlpFn.apply(tuple(mlps), flat, *params)
    return [y.reshape(x.shape[:-1] + (m.out.out_features,)) for y, m in zip(ys, mlps)]


class _MultiMlpFn(torch.autograd.Function):
    """ys[i] = mlps[i](x): the forwards on the HIP MLP kernels; the backward (dL/dx summed over
    the MLPs, every nn.Linear weight and bias) in one nrt_mlp_backward_multi call."""

    @staticmethod
    def forward(ctx, mlps, x, *params):
        import ctypes
        handles = [train_handle(m) for m in mlps]
        with torch.no_grad():
            ys, ctx.save = _forward_saving(handles, x.detach(), [m.out.out_features for m in mlps],
                                           keep=all(m.training for m in mlps))
        ctx.mlps = mlps
        ctx.handles = handles
        _save_versions(ctx, params)
        ctx.save_for_backward(x)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys):
        import ctypes
        _check_versions(ctx)
        if torch.is_grad_enabled():
            raise _lib.NrtError("second derivatives through SkipConnMLP.forward are not on the HIP "
                                "path")
        (x,) = ctx.saved_tensors
        mlps, n, M = ctx.mlps, len(ctx.mlps), x.shape[0]
        lib = _lib.load(require_device=True)
        dys = [dy.float().contiguous() for dy in dys]
        idx = _live_rows(dys, M)
        if idx is not None:  # the rows where any of the MLPs has a gradient (COMPACT_MIN_DEAD)
            full_x = x
            x = x[idx].contiguous()
            dys = [dy[idx].contiguous() for dy in dys]
            M = x.shape[0]
        zeros = M == 0
        mk = torch.zeros_like if zeros else torch.empty_like
        dx = torch.empty(n, M, x.shape[1], device=x.device) if ctx.needs_input_grad[1] else None
        grads, wptr, bptr = [], [], []
        for m in mlps:
            for lin in m._linears():
                dw = mk(lin.weight) if lin.weight.requires_grad else None
                db = mk(lin.bias) if lin.bias.requires_grad else None
                grads += [dw, db]
                wptr.append(0 if dw is None else dw.data_ptr())
                bptr.append(0 if db is None else db.data_ptr())
        P = ctypes.c_void_p
        hs = (P * n)(*[h.value for h in ctx.handles])
        dyp = (P * n)(*[d.data_ptr() for d in dys])
        dxp = None if dx is None else (P * n)(*[dx[i].data_ptr() for i in range(n)])
        wp, bp = (P * len(wptr))(*wptr), (P * len(bptr))(*bptr)
        if not zeros:
            ws = torch.empty(lib.nrt_mlp_backward_multi_workspace_bytes(hs, n, M),
                             dtype=torch.uint8, device=x.device)
            if ctx.save is not None:  # the forward saved the activations
                rows = None if idx is None else idx.to(torch.int32)
                Ms = full_x.shape[0] if idx is not None else M
                _lib.call("nrt_mlp_backward_saved", hs, n, _lib.ptr(x), M, _lib.ptr(rows),
                          (P * n)(*[b.data_ptr() for b in ctx.save]), Ms, dyp, dxp, wp, bp,
                          _lib.ptr(ws), _lib.stream())
            else:
                _lib.call("nrt_mlp_backward_multi", hs, n, _lib.ptr(x), M, dyp, dxp, wp, bp,
                          _lib.ptr(ws), _lib.stream())
        dxs = None if dx is None else (dx.sum(0) if not zeros else torch.zeros_like(x))
        if idx is not None and dxs is not None:
            dxs = torch.zeros_like(full_x).index_copy_(0, idx, dxs)
        return (None, dxs, *grads)


def input_gradient(mlp, x):
    """d(sum_o mlp(x)_o)/dx -- torch.autograd.grad(mlp(x), x, ones, create_graph=True), the SDF
    normal of SDF.autograd_diff (sdfs.py:184-197) -- on the HIP path: nrt_mlp_backward for the
    value, nrt_mlp_grad_backward for its gradients with respect to every nn.Linear.  ``x`` is
    not differentiated (second derivatives in x are not on the HIP path)."""
    if not x.is_cuda:
        raise _lib.NrtError("SkipConnMLP evaluates on the HIP path only: move it and its "
                            "inputs to the GPU")
    if mlp.latent_size:
        raise _lib.NrtError("input_gradient: latent MLPs are not supported")
    if torch.is_grad_enabled() and x.requires_grad:
        raise _lib.NrtError("input_gradient: second derivatives with respect to the inputs are "
                            "not on the HIP path (detach the points)")
    lead = x.shape[:-1]
    flat = x.reshape(-1, mlp.in_size).float().contiguous()
    params = [t for lin in mlp._linears() for t in (lin.weight, lin.bias)]
    if torch.is_grad_enabled() and any(q.requires_grad for q in params):
        if any(t.device != x.device for t in params):
            raise _lib.NrtError("SkipConnMLP parameters and inputs are on different devices: "
                                "move the module to the GPU (.to(device)) to train it")
        g = _InputGradFn.apply(mlp, flat, *params)
    else:
        g = _input_grad(mlp, flat)
    return g.reshape(lead + (mlp.in_size,))


def _input_grad(mlp, x, handle=None):
    lib = _lib.load(require_device=True)
    M = x.shape[0]
    g = torch.empty_like(x)
    if M == 0:
        return g
    h = mlp.nrt() if handle is None else handle.value
    dy = torch.ones(M, mlp.out.out_features, device=x.device)
    ws = torch.empty(lib.nrt_mlp_backward_workspace_bytes(h, M), dtype=torch.uint8,
                     device=x.device)
    _lib.call("nrt_mlp_backward", h, _lib.ptr(x), None, M, _lib.ptr(dy), _lib.ptr(g),
              None, None, None, _lib.ptr(ws), _lib.stream())
    return g


class _InputGradFn(torch.autograd.Function):
    """g = d(sum_o y_o)/dx with parameter gradients of <dL/dg, g> from nrt_mlp_grad_backward."""

    @staticmethod
    def forward(ctx, mlp, x, *params):
        handle = train_handle(mlp)
        with torch.no_grad():
            g = _input_grad(mlp, x.detach(), handle)
        ctx.mlp = mlp
        ctx.handle = handle
        _save_versions(ctx, params)
        ctx.save_for_backward(x)
        return g

    @staticmethod
    def backward(ctx, dg):
        import ctypes
        _check_versions(ctx)
        (x,) = ctx.saved_tensors
        mlp = ctx.mlp
        lib = _lib.load(require_device=True)
        M = x.shape[0]
        dg = dg.float().contiguous()
        lins = mlp._linears()
        dws = [torch.empty_like(lin.weight) if lin.weight.requires_grad else None for lin in lins]
        dbs = [torch.empty_like(lin.bias) if lin.bias.requires_grad else None for lin in lins]
        wp = (ctypes.c_void_p * len(lins))(*[0 if t is None else t.data_ptr() for t in dws])
        bp = (ctypes.c_void_p * len(lins))(*[0 if t is None else t.data_ptr() for t in dbs])
        ws = torch.empty(max(lib.nrt_mlp_grad_backward_workspace_bytes(ctx.handle.value, M), 1),
                         dtype=torch.uint8, device=x.device)
        _lib.call("nrt_mlp_grad_backward", ctx.handle.value, _lib.ptr(x), None, M, _lib.ptr(dg),
                  wp, bp, _lib.ptr(ws), _lib.stream())
        grads = [g for pair in zip(dws, dbs) for g in pair]
        return (None, None, *grads)
