"""The FP32 ring march (k_march32 / k_scan_best32, nrt_device.h ring32): reference-precision sphere
tracing + coarse scan with the SDF MLP on v_mfma_f32_16x16x4_f32 and the weights streamed through
the block's LDS ring.

* against the oracle (sdfs.py:111-160, 232-249) on the configurations it serves: SphereSDF(n=128)
  + 8x128 F=32 shift (the training SDF), the bare 8x256 F=16 MLP SDF, leaky_relu shifts;
* against the FP32 slab kernel k_intersect (option ring32=0) on the same inputs;
* independent of the persistent grid's size (option march_blocks);
* after nrt_mlp_refresh (the training handle re-gathers stream32 on the device) the march equals a
  freshly packed handle's.
FP32 bar: 1e-4 abs on rays whose hit flag and step count agree; flips reported and bounded.
"""
import os
import random

import pytest
import torch
import torch.nn.functional as F

import bench
from oracle import pathtracer_ref as R
from tests.helpers import copy_mlp, product_mlp_like, seeded
from tests.report import report
from tests.helpers import lib_opt as _lib_opt

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


def _rays(n, seed, eye=(0.0, 0.1, 1.0), spread=0.9):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor(eye).expand(1, n, n, 1, 3)
    d = F.normalize(torch.cat([torch.rand(1, n, n, 1, 2, generator=g) * spread - spread / 2,
                               -torch.ones(1, n, n, 1, 1)], -1), dim=-1)
    return torch.cat([o, d], -1)


def _blob(n, hidden, freqs, act, seed=5):
    """oracle SphereBlobSDF + the product SphereSDF with the same tensors; the shift gets a
    visible residual (out weights x0.05) so the MLP part shapes the surface."""
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    seeded(seed)
    ref = R.SphereBlobSDF(n=n, shift_hidden=hidden, shift_freqs=freqs, shift_zero_init=False)
    if act != "softplus":
        ref.shift = R.SkipMLP(num_layers=8, hidden_size=hidden, out=1, freqs=freqs, activation=act)
    with torch.no_grad():
        ref.radii.add_(0.12)
        ref.tfs.copy_(0.05 * torch.randn_like(ref.tfs))
        ref.shift.out.weight.mul_(0.05)
        ref.shift.out.bias.mul_(0.05)
    mine = SphereSDF(n=n, device="cpu")
    kw = {"activation": F.softplus} if act == "softplus" else {}
    mine.shift = SkipConnMLP(num_layers=8, hidden_size=hidden, in_size=3, out=1, freqs=freqs,
                             device="cpu", **kw)
    with torch.no_grad():
        mine.centers.copy_(ref.centers)
        mine.radii.copy_(ref.radii)
        mine.tfs.copy_(ref.tfs)
    copy_mlp(mine.shift, ref.shift)
    return ref, mine.cuda()


def _march(sdf, rays, primary=True, steps=64, seed=12):
    """(it, hit, kernel launches of k_march32) of SDF.intersect on the HIP path."""
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.shapes import SDF
    _lib.profile_enable(True)
    _lib.profile_reset()
    random.seed(seed)
    with torch.no_grad():
        it, hit = SDF(sdf=sdf, max_steps=steps).intersect(rays.cuda(), primary=primary)
    n32 = _lib.profile_read("k_march32")[1]
    _lib.profile_enable(False)
    return it, hit, n32


def _intersect_raw(sh, rays, max_steps, precision=None):
    """nrt_sdf_intersect (FP32 unless `precision`, primary) on a raw handle: (t, hit, p, n,
    throughput)."""
    import ctypes
    from neural_raytracing_amd import _lib
    P, dev = rays.shape[0], rays.device
    t = torch.empty(P, device=dev)
    hit = torch.empty(P, dtype=torch.uint8, device=dev)
    p, n, raw, wi = (torch.empty(P, 3, device=dev) for _ in range(4))
    thr = torch.empty(P, device=dev)
    idx = torch.empty(P, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.load(require_device=True)
    ws = torch.empty(max(lib.nrt_intersect_workspace_bytes(sh, P), 1), dtype=torch.uint8, device=dev)
    mp = _lib.MarchParams(max_steps, 5e-3, 10.0, 1, 2.2,
                          _lib.NRT_FP32 if precision is None else precision)
    _lib.call("nrt_sdf_intersect", sh, _lib.ptr(rays), P, ctypes.byref(mp), _lib.ptr(t),
              _lib.ptr(hit), _lib.ptr(p), _lib.ptr(n), _lib.ptr(raw), _lib.ptr(wi), _lib.ptr(thr),
              _lib.ptr(idx), _lib.ptr(cnt), _lib.ptr(ws), _lib.stream())
    torch.cuda.synchronize()
    return t, hit, p, n, thr


def _compare(name, it, hit, rit, rhit, tol=1e-4, flip_frac=0.005):
    hit, rhit = hit.cpu().reshape(-1), rhit.cpu().reshape(-1)
    t, rt = it.t.cpu().reshape(-1), rit.t.cpu().reshape(-1)
    step = (hit & rhit) & ((t - rt).abs() > tol)
    m = (hit & rhit) & ~step
    flips = int((hit != rhit).sum())
    errs = {
        "t_maxabs": (t[m] - rt[m]).abs().max().item() if m.any() else 0.0,
        "n_maxabs": (it.n.cpu().reshape(-1, 3)[m] - rit.n.cpu().reshape(-1, 3)[m]).abs().max().item() if m.any() else 0.0,
    }
    thr = None
    if getattr(it, "throughput", None) is not None and getattr(rit, "throughput", None) is not None:
        thr = (it.throughput.cpu().reshape(-1) - rit.throughput.cpu().reshape(-1)).abs()
        errs["thr_maxabs"] = thr.max().item()
    report(name, rays=hit.numel(), hits=int(rhit.sum()), flips=flips, step_flips=int(step.sum()),
           **errs)
    assert flips + int(step.sum()) <= flip_frac * hit.numel(), (flips, int(step.sum()))
    assert errs["t_maxabs"] <= tol and errs["n_maxabs"] <= tol
    if thr is not None:  # -1000 sdf(best): 1e-4 on the sdf is 0.1
        assert (thr <= 0.1).float().mean() >= 0.995
    return m


@pytest.mark.parametrize("hidden,freqs,act", [(128, 32, "softplus"), (256, 16, "softplus"),
                                              (128, 16, "leaky_relu"), (256, 32, "leaky_relu")])
def test_ring32_sphere_sdf_matches_oracle(hidden, freqs, act):
    ref, mine = _blob(128, hidden, freqs, act)
    rays = _rays(36, 7, eye=(0.0, 0.2, 1.1))
    it, hit, n32 = _march(mine, rays)
    assert n32 >= 1, "the FP32 ring kernel did not run"
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=64).intersect(rays, primary=True, jitter=jit)
    assert 0.1 < rhit.float().mean() < 0.9
    _compare(f"ring32_sphere_sdf_vs_oracle[{hidden},{freqs},{act}]", it, hit, rit, rhit)


def test_ring32_bare_mlp_matches_slab_kernel():
    """k_march32 vs the FP32 slab k_intersect on the bare 8x256 MLP SDF (cfg2 / cfg4 kind)."""
    seeded(41)
    ref = R.SkipMLP(num_layers=8, hidden_size=256, out=1, freqs=16, activation="softplus")
    bench.shape_mlp_sdf(ref, radius=0.3)
    mine = product_mlp_like(ref, "softplus")
    rays = _rays(40, 3)
    it, hit, n32 = _march(mine, rays)
    assert n32 >= 1
    _lib_opt("ring32", 0)
    sit, shit, n32b = _march(mine, rays)
    assert n32b == 0
    _compare("ring32_vs_slab[bare 8x256]", it, hit, sit, shit)
    # the coarse-scan argmin (throughput's sample) agrees on all but rounding ties
    assert (it.throughput - sit.throughput).abs().le(0.1).float().mean().item() >= 0.995


def test_ring32_independent_of_grid_size():
    """The job lists are per wave and the scan merge is an order-independent min: any persistent
    grid gives bit-identical results (1 block: 72 rays per wave, 8 of them scanned as whole jobs;
    the default grid: every scan segmented)."""
    _, mine = _blob(128, 128, 32, "softplus", seed=9)
    rays = _rays(24, 11, eye=(0.0, 0.2, 1.1))
    base, bh, _ = _march(mine, rays)
    # (blocks, xcd_lines, march_queue): the launch-wide queue too (every scan segmented, jobs
    # taken 16 at a time in launch order, so lanes, waves and blocks differ from the lists')
    for blocks, xcd, q in ((1, 1, 0), (5, 1, 0), (13, 1, 0), (0, 0, 0), (5, 0, 0), (0, 0, 1),
                           (1, 0, 1), (13, 0, 1)):
        _lib_opt("march_blocks", blocks)
        _lib_opt("xcd_lines", xcd)
        _lib_opt("march_queue", q)
        it, h, _ = _march(mine, rays)
        assert torch.equal(h, bh)
        assert torch.equal(it.t, base.t) and torch.equal(it.throughput, base.throughput)
        assert torch.equal(it.p, base.p) and torch.equal(it.n, base.n)


@pytest.mark.parametrize("prec", ["fp16", "fp32-split", "mixed"])
def test_march_queue_matches_job_lists(prec):
    """Option march_queue (one launch-wide job queue) on the FP16, split and NRT_MIXED marches
    (k_march16, k_march3, the mixed flagging march + k_refine3 + k_best3): bit-identical t, hit,
    p, n and throughput to the per-wave job lists, at the default grid and at 3 blocks."""
    from neural_raytracing_amd import set_precision
    _, mine = _blob(128, 128, 32, "softplus", seed=9)
    rays = _rays(24, 11, eye=(0.0, 0.2, 1.1))
    set_precision(prec)
    base, bh, _ = _march(mine, rays)
    assert bh.any() and not bh.all()
    for blocks in (0, 3):
        _lib_opt("march_blocks", blocks)
        _lib_opt("march_queue", 1)
        it, h, _ = _march(mine, rays)
        assert torch.equal(h, bh)
        assert torch.equal(it.t, base.t) and torch.equal(it.throughput, base.throughput)
        assert torch.equal(it.p, base.p) and torch.equal(it.n, base.n)


@pytest.mark.parametrize("hidden", [128, 256])
@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp32-split", "mixed"])
def test_march_line_staging_matches_per_ray_stores(prec, hidden):
    """Option march_stage (the launch queue's march writes each wave's finished packed t and
    whole-scan keys through per-wave LDS line stages, nrt_kernels.h LineStage): bit-identical t,
    hit, p, n and throughput to one store per ray -- 37^2 = 1,369 rays (a ragged last line), 3
    blocks (24 waves: 384 segmented scans, the rest whole, a line split between the two), and the
    default grid; the 128- and 256-wide shifts (the headline's width)."""
    from neural_raytracing_amd import set_precision
    _, mine = _blob(32, hidden, 16, "softplus", seed=21)
    rays = _rays(37, 23, eye=(0.0, 0.2, 1.1))
    set_precision(prec)
    _lib_opt("march_queue", 1)
    try:
        for blocks in (3, 0):
            _lib_opt("march_blocks", blocks)
            _lib_opt("march_stage", 0)
            base, bh, _ = _march(mine, rays)
            assert bh.any() and not bh.all()
            _lib_opt("march_stage", 1)
            it, h, _ = _march(mine, rays)
            assert torch.equal(h, bh)
            assert torch.equal(it.t, base.t) and torch.equal(it.throughput, base.throughput)
            assert torch.equal(it.p, base.p) and torch.equal(it.n, base.n)
    finally:
        _lib_opt("march_stage", 1)


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp32-split", "mixed"])
def test_ring32_after_device_refresh_matches_fresh_pack(prec):
    """nrt_mlp_refresh re-gathers stream32 / bias32, the split stream and the FP16 ring stream
    (folded, rounded to f16) on the device: a handle refreshed to new weights marches exactly like
    a handle packed from them on the host, at every precision (fp16 / mixed: the FP16 ring march
    of a training loop, which refused refreshed handles before round 4)."""
    import ctypes
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer._handles import train_handle, mlp_handle
    _, mine = _blob(64, 128, 32, "softplus", seed=13)
    mlp = mine.shift
    th = train_handle(mlp)  # packed from the current weights
    with torch.no_grad():
        for lin in mlp._linears():
            lin.weight.add_(0.01 * torch.randn_like(lin.weight))
            lin.bias.add_(0.01 * torch.randn_like(lin.bias))
    th2 = train_handle(mlp)  # same handle, refreshed on the device
    assert th2 is th
    fresh = mlp_handle(mlp)  # host-packed from the new weights
    assert fresh is not th
    rays = _rays(24, 17, eye=(0.0, 0.2, 1.1)).cuda().reshape(-1, 6).contiguous()
    P = rays.shape[0]
    c, r, t = (x.detach().cpu().contiguous() for x in (mine.centers, mine.radii, mine.tfs))
    outs = []
    for h in (th, fresh):
        sh = ctypes.c_void_p()
        _lib.check(_lib.load().nrt_sdf_create_sphere_blob(
            c.shape[0], c.data_ptr(), r.data_ptr(), t.data_ptr(), 32.0, h.value, ctypes.byref(sh)),
            "nrt_sdf_create_sphere_blob")
        try:
            _lib.profile_reset()
            _lib.profile_enable(True)
            outs.append(_intersect_raw(sh, rays, max_steps=64,
                                       precision=_lib._PRECISIONS[prec]))
            _lib.profile_enable(False)
            if prec in ("fp16", "mixed"):  # both handles on the FP16 ring march
                assert _lib.profile_read("k_march16")[1] >= 1
        finally:
            _lib.load().nrt_sdf_destroy(sh)
    if prec in ("fp32", "fp16"):
        for a, b in zip(outs[0], outs[1]):
            assert torch.equal(a, b)
    else:
        # the split stream keeps its pack-time per-layer scales across refreshes (they only keep
        # the lo halves normal), so the hi / lo halves -- not the products -- differ from a fresh
        # pack's in the last bits
        (t, h, p, n, thr), (t2, h2, p2, n2, thr2) = outs
        assert torch.equal(h, h2)
        assert (t - t2).abs().max().item() <= 1e-5 and (p - p2).abs().max().item() <= 1e-5
        assert (n - n2).abs().max().item() <= 1e-4 and (thr - thr2).abs().max().item() <= 1e-2


@pytest.mark.parametrize("n", [1, 15, 16, 17, 511, 3001])
def test_ring32_ragged_ray_counts_match_slab_kernel(n):
    """Ray counts that are not a multiple of the 16-ray tile, fewer rays than one wave / block,
    and more rays than waves: every ray's t / hit / p / throughput equal the FP32 slab kernel's
    up to the summation-order tolerance, and no ray is dropped or written twice."""
    _, mine = _blob(64, 128, 32, "softplus", seed=23)
    g = torch.Generator().manual_seed(n)
    o = torch.tensor([0.0, 0.2, 1.1]) + 0.05 * torch.randn(1, n, 1, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, n, 1, 1, 2, generator=g) * 0.8 - 0.4,
                               -torch.ones(1, n, 1, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    it, hit, n32 = _march(mine, rays)
    assert n32 >= 1
    _lib_opt("ring32", 0)
    sit, shit, _ = _march(mine, rays)
    assert torch.isfinite(it.t).all() and torch.isfinite(it.throughput).all()
    _compare(f"ring32_ragged[{n}]", it, hit, sit, shit, flip_frac=max(0.005, 1.0 / n))
