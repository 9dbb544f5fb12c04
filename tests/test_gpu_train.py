"""Autograd through the HIP SkipConnMLP (first slice): nrt_mlp_backward vs
torch autograd of the oracle's SkipMLP (neural_blocks.py:12-86 restated) in float64 on the CPU.
Tolerance per tensor: max|got - want64| <= max(1e-4 * max(1, max|want64|), 4 * e32), where e32 is
the error of the same oracle run in float32 (the reference's own precision): gradients through
sigma-32 Fourier features of 70 inputs are ill-conditioned in FP32 for any implementation."""
import pytest
import torch
import torch.nn.functional as F

from oracle import pathtracer_ref as R
from tests.helpers import copy_mlp, seeded

SHAPES = {
    "8x64_leaky": dict(num_layers=8, hidden_size=64, in_size=3, out=3, freqs=16),
    "sdf_shift_8x128_softplus": dict(num_layers=8, hidden_size=128, in_size=3, out=1, freqs=32,
                                     activation="softplus"),
    "nerfle_second_70in": dict(num_layers=8, hidden_size=64, in_size=70, out=3, freqs=16),
    "latent_4x32": dict(num_layers=4, hidden_size=32, in_size=3, out=4, freqs=8, latent_size=8),
    # the shading MLPs of the bench scene (bsdfs.py:487-496, 613-624; lights.py:160-163)
    "neural_bsdf_6x96_F64": dict(num_layers=6, hidden_size=96, in_size=3, out=3, freqs=64),
    "sp_var_16x256_F128": dict(num_layers=16, hidden_size=256, in_size=3, out=8, freqs=128,
                               sigma=128, xavier_init=True),
    "light_field_10x256": dict(num_layers=10, hidden_size=256, in_size=3, out=3, freqs=16),
}


def _pair(kw, seed):
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    seeded(seed)
    act = kw.get("activation", "leaky_relu")
    ref = R.SkipMLP(**kw)
    pkw = {k: v for k, v in kw.items() if k != "activation"}
    if act == "softplus":
        pkw["activation"] = F.softplus
    mine = SkipConnMLP(device="cpu", **pkw)
    copy_mlp(mine, ref)
    return ref, mine.cuda()


def _close(got, want, ref32, what):
    scale = max(1.0, want.abs().max().item())
    err = (got.detach().cpu().double() - want).abs().max().item()
    e32 = (ref32.detach().double() - want).abs().max().item()
    tol = max(1e-4 * scale, 4 * e32)
    assert err <= tol, f"{what}: max|diff| {err:.3g} > {tol:.3g} (scale {scale:.3g}, fp32 ref {e32:.3g})"


def _grads(ref, x, lat, dy, dtype):
    import copy
    m = copy.deepcopy(ref).to(dtype)
    m.basis_p = ref.basis_p.to(dtype)
    xr = x.detach().clone().to(dtype).requires_grad_(True)
    lr = lat.detach().clone().to(dtype).requires_grad_(True) if lat is not None else None
    (m(xr, lr) * dy.to(dtype)).sum().backward()
    out = {"dx": xr.grad}
    if lr is not None:
        out["dlatent"] = lr.grad
    for i, lin in enumerate([m.init, *m.layers, m.out]):
        out[f"dW[{i}]"] = lin.weight.grad
        out[f"db[{i}]"] = lin.bias.grad
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 33, 1000])
@pytest.mark.parametrize("name", list(SHAPES))
def test_mlp_backward_matches_autograd(name, M):
    from neural_raytracing_amd import set_precision
    kw = SHAPES[name]
    ref, mine = _pair(kw, 40 + M)
    set_precision("fp32")
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5)
    lat = torch.randn(M, kw["latent_size"], generator=g) if kw.get("latent_size") else None
    dy = torch.randn(M, kw["out"], generator=g)
    want = _grads(ref, x, lat, dy, torch.float64)
    ref32 = _grads(ref, x, lat, dy, torch.float32)
    # HIP
    xm = x.cuda().requires_grad_(True)
    lm = lat.cuda().requires_grad_(True) if lat is not None else None
    y = mine(xm, lm)
    (y * dy.cuda()).sum().backward()
    got = {"dx": xm.grad}
    if lat is not None:
        got["dlatent"] = lm.grad
    for i, a in enumerate(mine._linears()):
        got[f"dW[{i}]"] = a.weight.grad
        got[f"db[{i}]"] = a.bias.grad
    assert set(got) == set(want)
    for k in want:
        _close(got[k], want[k], ref32[k], k)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SHAPES))
def test_weight_gradients_batch_kernel_matches_autograd(name):
    """The weight gradients on k_wgrad_batch (option wgrad_tile 0: 64 x 64 tiles fed by direct
    loads, separate bias column sums) as well as on the default k_wgrad_tile (128 x 128 tiles
    staged through LDS, biases summed on the first weight tiles): both at the float64 bar, and
    within FP32 summation-order noise of each other."""
    from neural_raytracing_amd import _lib, set_precision
    kw = SHAPES[name]
    M = 2000
    ref, mine = _pair(kw, 140)
    set_precision("fp32")
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5)
    lat = torch.randn(M, kw["latent_size"], generator=g) if kw.get("latent_size") else None
    dy = torch.randn(M, kw["out"], generator=g)
    want = _grads(ref, x, lat, dy, torch.float64)
    ref32 = _grads(ref, x, lat, dy, torch.float32)

    def run(tile):
        with _lib.options(wgrad_tile=tile):
            mine.zero_grad(set_to_none=True)
            xm = x.cuda().requires_grad_(True)
            lm = lat.cuda() if lat is not None else None
            (mine(xm, lm) * dy.cuda()).sum().backward()
            return {**{f"dW[{i}]": a.weight.grad.clone() for i, a in enumerate(mine._linears())},
                    **{f"db[{i}]": a.bias.grad.clone() for i, a in enumerate(mine._linears())}}
    a, b = run(0), run(1)
    for k in a:
        _close(a[k], want[k], ref32[k], "batch " + k)
        _close(b[k], want[k], ref32[k], "tile " + k)
        scale = a[k].abs().max().clamp_min(1e-6)
        assert float((a[k] - b[k]).abs().max() / scale) < 1e-4, k


@pytest.mark.gpu
@pytest.mark.parametrize("dead", [0.6, 1.0])
@pytest.mark.parametrize("name", ["sp_var_16x256_F128", "latent_4x32", "neural_bsdf_6x96_F64"])
def test_mlp_backward_compacts_zero_gradient_rows(name, dead):
    """A backward whose dY is zero on most rows (the missed rays of a masked training step) runs
    on the rows with a gradient only (neural_blocks.COMPACT_MIN_DEAD); the gradients still match
    float64 autograd over all rows, dL/dx (and dL/dlatent) is 0 on the dropped rows, and an
    all-zero dY gives all-zero gradients.  The mixture's multi-MLP backward the same way."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer import neural_blocks as nb
    kw = SHAPES[name]
    M = 1500
    ref, mine = _pair(kw, 77)
    set_precision("fp32")
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5)
    lat = torch.randn(M, kw["latent_size"], generator=g) if kw.get("latent_size") else None
    dy = torch.randn(M, kw["out"], generator=g)
    dy[torch.rand(M, generator=g) < dead] = 0.0
    want = _grads(ref, x, lat, dy, torch.float64)
    ref32 = _grads(ref, x, lat, dy, torch.float32)
    xm = x.cuda().requires_grad_(True)
    lm = lat.cuda().requires_grad_(True) if lat is not None else None
    (mine(xm, lm) * dy.cuda()).sum().backward()
    got = {"dx": xm.grad}
    if lat is not None:
        got["dlatent"] = lm.grad
    for i, a in enumerate(mine._linears()):
        got[f"dW[{i}]"] = a.weight.grad
        got[f"db[{i}]"] = a.bias.grad
    for k in want:
        _close(got[k], want[k], ref32[k], k)
    dead_rows = (dy == 0).all(-1)
    assert torch.equal(xm.grad.cpu()[dead_rows], torch.zeros_like(x[dead_rows]))
    if dead == 1.0:
        assert all(float(v.abs().max()) == 0.0 for v in got.values())
    if lat is None:  # the multi-MLP backward (two copies of the MLP on one input)
        from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
        mine2 = _pair(kw, 78)[1]
        xm2 = x.cuda().requires_grad_(True)
        ys = mlp_multi([mine, mine2], xm2)
        for q in list(mine.parameters()) + list(mine2.parameters()):
            q.grad = None
        (ys[0] * dy.cuda()).sum().backward()  # mine2's output unused: its dY is all zero
        for i, a in enumerate(mine._linears()):
            _close(a.weight.grad, want[f"dW[{i}]"], ref32[f"dW[{i}]"], f"multi dW[{i}]")
        _close(xm2.grad, want["dx"], ref32["dx"], "multi dx")
        for a in mine2._linears():
            assert a.weight.grad is None or float(a.weight.grad.abs().max()) == 0.0
    assert nb.COMPACT_MIN_DEAD < 0.6


@pytest.mark.gpu
def test_mlp_training_steps_reduce_loss():
    """A few Adam steps of an 8x64 SkipConnMLP fitting a smooth target on the HIP path."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    set_precision("fp32")
    seeded(3)
    mlp = SkipConnMLP(num_layers=4, hidden_size=64, in_size=3, out=1, freqs=8, sigma=2,
                      device="cuda").to("cuda")
    x = torch.rand(4096, 3, device="cuda") * 2 - 1
    t = (x.norm(dim=-1, keepdim=True) - 0.5)
    opt = torch.optim.Adam(mlp.parameters(), lr=1e-3)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = (mlp(x) - t).square().mean()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses


@pytest.mark.gpu
def test_mlp_parameters_on_another_device_are_refused():
    """Parameters left on the CPU with GPU inputs fail loudly (as nn.Linear does), before any
    HIP launch could be handed host pointers."""
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    mlp = SkipConnMLP(num_layers=2, hidden_size=32, in_size=3, out=1, freqs=4, device="cuda")
    with pytest.raises(NrtError):
        mlp(torch.rand(8, 3, device="cuda"))


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["fp32", "fp16"])
def test_refreshed_handle_matches_a_fresh_pack(prec):
    """nrt_mlp_refresh (device re-pack after an optimiser step) gives the same forward outputs
    and gradients as a handle packed from scratch on the host: after in-place weight updates the
    autograd path (refreshed training handle) and the no-grad path (fresh host pack) agree
    bit for bit; the refreshed handle refuses the FP16 program engine."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    seeded(12)
    mlp = SkipConnMLP(num_layers=8, hidden_size=64, in_size=3, out=3, freqs=16,
                      device="cpu").cuda()
    x = torch.rand(777, 3, device="cuda") - 0.5
    set_precision(prec)
    try:
        opt = torch.optim.SGD(mlp.parameters(), lr=0.05)
        for _ in range(3):
            opt.zero_grad()
            y = mlp(x)  # training handle: created, then refreshed on the device
            y.square().mean().backward()
            opt.step()
        y_train = mlp(x).detach()  # refreshed after the last step
        with torch.no_grad():
            y_fresh = mlp(x)  # mlp_handle: re-packed on the host from the same weights
        assert torch.equal(y_train, y_fresh)
        h = mlp._nrt_train[2]
        assert h.value != mlp.nrt()
    finally:
        set_precision("fp32")
    # gradients through the refreshed handle vs float64 autograd of the same weights
    ref = R.SkipMLP(num_layers=8, hidden_size=64, in_size=3, out=3, freqs=16)
    with torch.no_grad():
        ref.basis_p = mlp.basis_p.detach().cpu().clone()
        for a, b in zip([ref.init, *ref.layers, ref.out], mlp._linears()):
            a.weight.copy_(b.weight.cpu())
            a.bias.copy_(b.bias.cpu())
    dy = torch.randn(777, 3, generator=torch.Generator().manual_seed(1))
    want = _grads(ref, x.cpu(), None, dy, torch.float64)
    ref32 = _grads(ref, x.cpu(), None, dy, torch.float32)
    mlp.zero_grad()
    (mlp(x) * dy.cuda()).sum().backward()
    for i, a in enumerate(mlp._linears()):
        _close(a.weight.grad, want[f"dW[{i}]"], ref32[f"dW[{i}]"], f"dW[{i}]")


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 77, 5000])
@pytest.mark.parametrize("name", ["neural_bsdf_6x96_F64", "sp_var_16x256_F128"])
def test_mlp_backward_multi_matches_single(name, M):
    """nrt_mlp_backward_multi (n same-shape MLPs on one input: the mixture's NeuralBSDFs, one
    batched launch) against each MLP's own nrt_mlp_backward through autograd: dL/dx summed over
    the MLPs and every weight / bias gradient, relative 1e-5 (only the split-K slice count of the
    weight gradients differs)."""
    from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
    kw = SHAPES[name]
    mlps = [_pair(kw, seed)[1] for seed in (1, 2, 3)]
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, kw["in_size"], generator=g) * 2 - 1).cuda()
    dys = [torch.randn(M, kw["out"], generator=g).cuda() for _ in mlps]
    params = [q for m in mlps for q in m.parameters()]

    def grads(batched):
        xx = x.clone().requires_grad_(True)
        ys = mlp_multi(mlps, xx) if batched else [m(xx) for m in mlps]
        loss = sum((y * dy).sum() for y, dy in zip(ys, dys))
        return torch.autograd.grad(loss, [xx] + params)
    got, want = grads(True), grads(False)
    for a, b in zip(got, want):
        scale = b.abs().max().clamp_min(1e-6)
        assert ((a - b).abs().max() / scale) < 1e-5, (name, M, (a - b).abs().max(), scale)


@pytest.mark.gpu
@pytest.mark.parametrize("frozen", ["biases", "weights_of_odd_layers"])
def test_mlp_backward_with_frozen_parameters(frozen):
    """Some parameters frozen (requires_grad=False: a null gradient pointer at the boundary) at a
    batch large enough that the weight-gradient batch has fewer tiles than the full plan the
    workspace was sized for: the batch keeps the full plan's slice count (a re-plan
    chose more slices and wrote past the workspace).  The requested gradients match float64
    autograd; the frozen ones stay None."""
    from neural_raytracing_amd import set_precision
    kw = SHAPES["8x64_leaky"]
    ref, mine = _pair(kw, 91)
    set_precision("fp32")
    lins = mine._linears()
    for i, a in enumerate(lins):
        if frozen == "biases":
            a.bias.requires_grad_(False)
        elif i % 2 == 1:
            a.weight.requires_grad_(False)
    M = 20000
    g = torch.Generator().manual_seed(5)
    x = torch.rand(M, 3, generator=g) - 0.5
    dy = torch.randn(M, 3, generator=g)
    want = _grads(ref, x, None, dy, torch.float64)
    ref32 = _grads(ref, x, None, dy, torch.float32)
    xm = x.cuda().requires_grad_(True)
    (mine(xm) * dy.cuda()).sum().backward()
    _close(xm.grad, want["dx"], ref32["dx"], "dx")
    for i, a in enumerate(lins):
        for nm, t in (("dW", a.weight), ("db", a.bias)):
            if t.requires_grad:
                _close(t.grad, want[f"{nm}[{i}]"], ref32[f"{nm}[{i}]"], f"{nm}[{i}]")
            else:
                assert t.grad is None


@pytest.mark.gpu
def test_mlp_backward_multi_with_frozen_biases():
    """The batched mixture backward with frozen biases at a large batch matches the per-MLP
    backward (same slice-count rule as the single-MLP batch)."""
    from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
    kw = SHAPES["neural_bsdf_6x96_F64"]
    mlps = [_pair(kw, seed)[1] for seed in (4, 5)]
    for m in mlps:
        for a in m._linears():
            a.bias.requires_grad_(False)
    M = 30000
    g = torch.Generator().manual_seed(9)
    x = (torch.rand(M, 3, generator=g) * 2 - 1).cuda()
    dys = [torch.randn(M, 3, generator=g).cuda() for _ in mlps]
    params = [q for m in mlps for q in m.parameters() if q.requires_grad]

    def grads(batched):
        xx = x.clone().requires_grad_(True)
        ys = mlp_multi(mlps, xx) if batched else [m(xx) for m in mlps]
        loss = sum((y * dy).sum() for y, dy in zip(ys, dys))
        return torch.autograd.grad(loss, [xx] + params)
    got, want = grads(True), grads(False)
    for a, b in zip(got, want):
        scale = b.abs().max().clamp_min(1e-6)
        assert ((a - b).abs().max() / scale) < 1e-5, ((a - b).abs().max(), scale)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", list(SHAPES))
def test_mlp_backward_column_split_bit_equal_to_per_wave(name, mode):
    """The column-split backward kernels (option bwd_colsplit 1: encoding tiles where they double
    the blocks per CU, 2: the slab) do the per-wave kernels' operations in the same order: every
    gradient bit-equal to bwd_colsplit 0, on a ragged row count, single and multi-MLP launches."""
    from neural_raytracing_amd import _lib, set_precision
    kw = SHAPES[name]
    _, mine = _pair(kw, 7)
    set_precision("fp32")
    M = 3001
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5).cuda()
    lat = torch.randn(M, kw["latent_size"], generator=g).cuda() if kw.get("latent_size") else None
    dy = torch.randn(M, kw["out"], generator=g).cuda()

    def run(opt):
        with _lib.options(bwd_colsplit=opt, bwd_ring=0):  # the slab kernels, not the ring
            mine.zero_grad(set_to_none=True)
            xm = x.clone().requires_grad_(True)
            lm = lat.clone().requires_grad_(True) if lat is not None else None
            (mine(xm, lm) * dy).sum().backward()
            out = [xm.grad.clone()] + ([lm.grad.clone()] if lm is not None else [])
            out += [p.grad.clone() for p in mine.parameters() if p.grad is not None]
        return out

    base = run(0)
    got = run(mode)
    assert len(base) == len(got) > 2
    for i, (a, b) in enumerate(zip(base, got)):
        assert torch.equal(a, b), (name, mode, i, (a - b).abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_mlp_backward_multi_column_split_bit_equal(mode):
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
    kw = SHAPES["neural_bsdf_6x96_F64"]
    mlps = [_pair(kw, seed)[1] for seed in (1, 2, 3)]
    g = torch.Generator().manual_seed(11)
    x = (torch.rand(2999, kw["in_size"], generator=g) * 2 - 1).cuda()
    dys = [torch.randn(2999, kw["out"], generator=g).cuda() for _ in mlps]
    params = [q for m in mlps for q in m.parameters()]

    def grads(opt):
        with _lib.options(bwd_colsplit=opt, bwd_ring=0):
            xx = x.clone().requires_grad_(True)
            loss = sum((y * dy).sum() for y, dy in zip(mlp_multi(mlps, xx), dys))
            return torch.autograd.grad(loss, [xx] + params)
    for a, b in zip(grads(0), grads(mode)):
        assert torch.equal(a, b), (a - b).abs().max().item()


RING_SHAPES = ["neural_bsdf_6x96_F64", "sp_var_16x256_F128", "light_field_10x256"]


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 17, 129, 5000])
@pytest.mark.parametrize("name", RING_SHAPES)
def test_ring_backward_matches_autograd_and_slab(name, M):
    """The ring backward (option bwd_ring, nrt_train_ring.h: 16-row tiles, the transposed weights
    streamed through the block's LDS ring, dZ in registers) on the shading MLPs' shapes: every
    gradient against float64 autograd at the FP32 bar of this file, and against the column-split
    slab kernels (bwd_ring 0) within FP32 summation-order noise; ragged row counts (one row, a
    partial tile, a partial block, many blocks)."""
    from neural_raytracing_amd import _lib, set_precision
    kw = SHAPES[name]
    ref, mine = _pair(kw, 90 + M)
    set_precision("fp32")
    g = torch.Generator().manual_seed(M + 3)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5)
    dy = torch.randn(M, kw["out"], generator=g)
    want = _grads(ref, x, None, dy, torch.float64)
    ref32 = _grads(ref, x, None, dy, torch.float32)

    def run(ring):
        with _lib.options(bwd_ring=ring):
            mine.zero_grad(set_to_none=True)
            xm = x.cuda().requires_grad_(True)
            (mine(xm) * dy.cuda()).sum().backward()
            got = {"dx": xm.grad.clone()}
            for i, a in enumerate(mine._linears()):
                got[f"dW[{i}]"] = a.weight.grad.clone()
                got[f"db[{i}]"] = a.bias.grad.clone()
        return got
    _lib.profile_enable(True)
    _lib.profile_reset()
    ring = run(1)
    _lib.profile_enable(False)
    slab = run(0)
    assert _lib.profile_read("k_mlp_backward32")[1] == 1
    for k in want:
        # both implementations at the float64 bar; against each other only a sanity bound (the
        # sigma-128 Fourier features make dL/dx ill-conditioned in FP32: measured 7e-4 relative
        # between the two summation orders at M = 5000, each within the bar)
        _close(ring[k], want[k], ref32[k], k)
        _close(slab[k], want[k], ref32[k], "slab " + k)
        scale = slab[k].abs().max().clamp_min(1e-6)
        assert float((ring[k] - slab[k]).abs().max() / scale) < 1e-2, k


@pytest.mark.gpu
@pytest.mark.parametrize("M", [40, 4100])
def test_ring_backward_multi_matches_single(M):
    """nrt_mlp_backward_multi on the ring (blockIdx.y = MLP) for the mixture's NeuralBSDFs equals
    the per-MLP ring backward, and dL/dx is the sum over the MLPs."""
    from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
    kw = SHAPES["neural_bsdf_6x96_F64"]
    mlps = [_pair(kw, seed)[1] for seed in (4, 5, 6, 7)]
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, 3, generator=g) * 2 - 1).cuda()
    dys = [torch.randn(M, 3, generator=g).cuda() for _ in mlps]
    params = [q for m in mlps for q in m.parameters()]

    def grads(batched):
        xx = x.clone().requires_grad_(True)
        ys = mlp_multi(mlps, xx) if batched else [m(xx) for m in mlps]
        loss = sum((y * dy).sum() for y, dy in zip(ys, dys))
        return torch.autograd.grad(loss, [xx] + params)
    for a, b in zip(grads(True), grads(False)):
        scale = b.abs().max().clamp_min(1e-6)
        assert float((a - b).abs().max() / scale) < 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("name,n,M", [("neural_bsdf_6x96_F64", 3, 1), ("neural_bsdf_6x96_F64", 8, 4100),
                                      ("neural_bsdf_6x96_F64", 17, 300), ("light_field_10x256", 2, 129),
                                      ("8x64_leaky", 3, 500)])
def test_mlp_forward_multi_equals_single(name, n, M):
    """nrt_mlp_forward_multi (one launch for same-shape MLPs on the ring engine, blockIdx.y = MLP;
    more than 16 MLPs in launches of 16; other shapes as per-MLP calls) equals nrt_mlp_forward of
    each MLP bit for bit, and the per-MLP forwards match the float64 oracle at the FP32 bar."""
    import ctypes
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer._handles import mlp_handle
    set_precision("fp32")
    kw = SHAPES[name]
    pairs = [_pair(kw, 200 + s) for s in range(n)]
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, kw["in_size"], generator=g) - 0.5)
    xc = x.cuda().contiguous()
    hs = [mlp_handle(m) for _, m in pairs]
    single = []
    for h, (_, m) in zip(hs, pairs):
        y = torch.empty(M, kw["out"], device="cuda")
        _lib.call("nrt_mlp_forward", h.value, _lib.ptr(xc), None, M, _lib.ptr(y),
                  _lib.precision_code(), _lib.stream())
        single.append(y)
    multi = [torch.full((M, kw["out"]), float("nan"), device="cuda") for _ in range(n)]
    P = ctypes.c_void_p
    _lib.profile_enable(True)
    _lib.profile_reset()
    _lib.call("nrt_mlp_forward_multi", (P * n)(*[h.value for h in hs]), n, _lib.ptr(xc), M,
              (P * n)(*[y.data_ptr() for y in multi]), None, _lib.precision_code(), _lib.stream())
    torch.cuda.synchronize()
    launches = _lib.profile_read("k_mlp_ring32")[1]
    _lib.profile_enable(False)
    if name != "8x64_leaky":
        assert launches == (n + 15) // 16
    for a, b in zip(multi, single):
        assert torch.equal(a, b)
    import copy
    for (ref, _), y in zip(pairs[:2], single[:2]):
        m64 = copy.deepcopy(ref).double()
        m64.basis_p = ref.basis_p.double()
        with torch.no_grad():
            want = m64(x.double(), None)
        assert (y.cpu().double() - want).abs().max().item() <= 1e-4 * max(1.0, want.abs().max().item())


@pytest.mark.gpu
@pytest.mark.parametrize("dead", [0.0, 0.5])
@pytest.mark.parametrize("name", RING_SHAPES)
def test_saved_activation_backward_equals_recompute(name, dead):
    """The training forward saves the activations (nrt_mlp_forward_multi with save buffers,
    nrt_mlp_save_bytes > 0) and nrt_mlp_backward_saved runs the backward chain on them: y and every
    gradient bit-equal to the ring backward that evaluates the forward again (option train_save
    0), with and without row compaction (dead: the fraction of rows whose dL/dy is 0, so the
    saved backward reads saved rows through the live-row index)."""
    from neural_raytracing_amd import _lib, set_precision
    set_precision("fp32")
    kw = SHAPES[name]
    _, mine = _pair(kw, 31)
    M = 3001
    g = torch.Generator().manual_seed(5)
    x = (torch.rand(M, 3, generator=g) - 0.5).cuda()
    dy = torch.randn(M, kw["out"], generator=g)
    dy[torch.rand(M, generator=g) < dead] = 0.0
    dy = dy.cuda()

    def run(save):
        with _lib.options(train_save=save):
            mine.zero_grad(set_to_none=True)
            xm = x.clone().requires_grad_(True)
            y = mine(xm)
            (y * dy).sum().backward()
            return [y.detach().clone(), xm.grad.clone()] + [q.grad.clone() for q in mine.parameters()
                                                            if q.grad is not None]
    _lib.profile_enable(True)
    _lib.profile_reset()
    a = run(1)
    saved_launches = _lib.profile_read("k_mlp_backward32")[1]
    _lib.profile_enable(False)
    b = run(0)
    assert saved_launches == 1
    assert len(a) == len(b) > 3
    for u, v in zip(a, b):
        assert torch.equal(u, v), (u - v).abs().max().item()


@pytest.mark.gpu
def test_saved_activation_multi_backward_equals_recompute():
    """The mixture's NeuralBSDFs through mlp_multi: one saving forward launch for all of them,
    one saved backward; every gradient bit-equal to the recomputing ring backward."""
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import mlp_multi
    set_precision("fp32")
    kw = SHAPES["neural_bsdf_6x96_F64"]
    mlps = [_pair(kw, seed)[1] for seed in (4, 5, 6)]
    M = 2500
    g = torch.Generator().manual_seed(9)
    x = (torch.rand(M, 3, generator=g) * 2 - 1).cuda()
    dys = [torch.randn(M, 3, generator=g) for _ in mlps]
    dead = torch.rand(M, generator=g) < 0.4
    dys = [d.masked_fill(dead[:, None], 0.0).cuda() for d in dys]
    params = [q for m in mlps for q in m.parameters()]

    def grads(save):
        with _lib.options(train_save=save):
            xx = x.clone().requires_grad_(True)
            ys = mlp_multi(mlps, xx)
            loss = sum((y * dy).sum() for y, dy in zip(ys, dys))
            return [y.detach() for y in ys] + list(torch.autograd.grad(loss, [xx] + params))
    for u, v in zip(grads(1), grads(0)):
        assert torch.equal(u, v), (u - v).abs().max().item()
