"""The fp32-split precision (include/nrt.h NRT_FP32_SPLIT, nrt_ring3.h): the SDF march + coarse
scan with every MLP layer on v_mfma_f32_16x16x32_f16, each f32 operand split into two f16 halves
and three products per block, f32 accumulation.

* accuracy of one SDF evaluation against float64 (the oracle's MLP in double), side by side with
  the FP32 fma-chain path (exact-f32 MFMA): the split path must be FP32-class -- within 2x of the
  FP32 path's max error and well inside the 1e-4 parity bar;
* the march against the oracle with the FP32 bar (1e-4 abs on t / p / n on agreeing rays, flips +
  step flips <= 0.5 %, throughput within 0.1 on 99.5 % of rays): the bare 8x256 MLP SDF (cfg2 /
  cfg4 kind, KH = 8, KQ = 2), SphereSDF(128) + 8x128 F=32 shift (KH = 4, KQ = 3) and the bench's
  metric scene on a crop across the silhouette;
* schedule invariance (persistent grid size) and ragged ray counts.
"""
import copy
import math
import random

import pytest
import torch

import bench
from oracle import pathtracer_ref as R
from tests.helpers import lib_opt as _lib_opt
from tests.report import report
from tests.test_gpu_configs import _agreement, _camera_rays, _mlp_sdf_pair
from tests.test_gpu_ring32 import _blob, _compare, _intersect_raw, _rays

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


def _double(mod):
    """float64 copy of an oracle module, plain tensor attributes (basis_p) included."""
    m = copy.deepcopy(mod).double()
    for sub in m.modules():
        for k, v in list(vars(sub).items()):
            if isinstance(v, torch.Tensor) and not isinstance(v, torch.nn.Parameter):
                setattr(sub, k, v.double())
    return m


def _eval(mine, pts, prec, kernel):
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_eval
    set_precision(prec)
    _lib.profile_enable(True)
    _lib.profile_reset()
    with torch.no_grad():
        v = sdf_eval(mine, pts.cuda()).cpu().double()
    n = _lib.profile_read(kernel)[1] if kernel else None
    _lib.profile_enable(False)
    set_precision("fp32")
    return v, n


def _points(n, seed, scale=1.2):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(n, 3, generator=g) * 2 - 1) * scale


@pytest.mark.parametrize("kind", ["bare_8x256_f16", "blob128_8x128_f32", "blob1_8x256_f16"])
def test_split_sdf_eval_accuracy_vs_float64(kind):
    if kind == "bare_8x256_f16":
        ref, mine = _mlp_sdf_pair()
        f64 = _double(ref)

        def want(p):
            return f64(p.double())[..., 0]
    elif kind == "blob128_8x128_f32":
        ref, mine = _blob(128, 128, 32, "softplus")
        f64 = _double(ref)

        def want(p):
            return f64(p.double())
    else:  # the bench scene's SDF (one-sphere prior + default-init 8x256 shift)
        scene = bench.build_scene("cuda", 64, seed=0)
        osc = bench.oracle_scene(scene)
        mine = scene["shape"].sdf
        f64 = _double(osc["shape"].sdf)

        def want(p):
            return f64(p.double())
    pts = _points(8000, 3)
    w = want(pts).reshape(-1)
    s32, _ = _eval(mine, pts, "fp32", None)
    s3, n3 = _eval(mine, pts, "fp32-split", "k_sdf_eval3")
    assert n3 == 1, "the split engine did not run"
    e32, e3 = (s32 - w).abs(), (s3 - w).abs()
    report(f"split_eval_vs_f64[{kind}]", points=pts.shape[0], fp32_max=e32.max().item(),
           fp32_mean=e32.mean().item(), split_max=e3.max().item(), split_mean=e3.mean().item(),
           value_absmax=w.abs().max().item())
    assert e3.max().item() <= 2 * e32.max().item() + 1e-7
    assert e3.mean().item() <= 2 * e32.mean().item() + 1e-8
    assert e3.max().item() <= 1e-5


def _march_split(sdf, rays, primary=True, steps=64, seed=12):
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    set_precision("fp32-split")
    _lib.profile_enable(True)
    _lib.profile_reset()
    random.seed(seed)
    with torch.no_grad():
        it, hit = SDF(sdf=sdf, max_steps=steps).intersect(rays.cuda(), primary=primary)
    n3 = _lib.profile_read("k_march3")[1]
    _lib.profile_enable(False)
    set_precision("fp32")
    return it, hit, n3


def test_split_bare_mlp_march_matches_oracle():
    ref, mine = _mlp_sdf_pair()
    rays = _camera_rays(40, 3)
    it, hit, n3 = _march_split(mine, rays)
    assert n3 == 1
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=lambda p: ref(p)[..., 0], max_steps=64).intersect(
            rays, primary=True, jitter=jit)
    assert 0.15 < rhit.float().mean() < 0.85
    _compare("split_bare_mlp_vs_oracle[8x256,F16]", it, hit, rit, rhit)


@pytest.mark.parametrize("hidden,freqs,act", [(128, 32, "softplus"), (256, 16, "leaky_relu")])
def test_split_sphere_sdf_march_matches_oracle(hidden, freqs, act):
    ref, mine = _blob(128, hidden, freqs, act)
    rays = _rays(36, 7, eye=(0.0, 0.2, 1.1))
    it, hit, n3 = _march_split(mine, rays)
    assert n3 == 1
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=64).intersect(rays, primary=True, jitter=jit)
    assert 0.1 < rhit.float().mean() < 0.9
    _compare(f"split_sphere_sdf_vs_oracle[{hidden},{freqs},{act}]", it, hit, rit, rhit)


def test_split_metric_config_crop_matches_oracle():
    """bench.py's headline scene on the 64x64 silhouette crop (as test_metric_config_crop_matches_
    oracle[fp32]) in fp32-split: the FP32 bar."""
    import neural_raytracing_amd as nra
    scene = bench.build_scene("cuda", samples=64, seed=0)
    pt = scene["pt"]
    size, crop = 800, 64
    c0, c1 = (size - crop) // 2, 72
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    osc = bench.oracle_scene(scene)
    ocam = R.NeRFCameraRef(c2w, focal)
    random.seed(5)
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], ocam, osc["integrator"], osc["bsdf"],
                        size=size, chunk_size=size, background=0.0, with_noise=0.0,
                        crop=(c0, c1, crop))
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    nra.set_precision("fp32-split")
    random.seed(5)
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(scene["shape"], scene["lights"], cam, scene["integrator"],
                                     bsdf=scene["bsdf"], size=size, chunk_size=size,
                                     bundle_size=1, crop_size=crop, uv=(c0, c1), background=0,
                                     with_noise=0.0)
        agree, rh, flips, steps = _agreement(
            scene["shape"], osc["shape"], cam.rays_tile(c0, c1, crop, crop, size),
            ocam.sample_positions(R._tile_positions(c0, c1, crop), size))
    nra.set_precision("fp32")
    got = got.cpu()
    agree = agree.reshape(crop, crop)
    err = (got - want).abs().amax(-1)
    report("split_metric_config_crop", pixels=crop * crop, hits=int(rh.sum()), flips=flips,
           step_flips=steps, maxabs_agreeing=err[agree].max().item(),
           pixels_over_1e4=int((err > 1e-4).sum()))
    assert 0.1 < rh.float().mean() < 0.95
    assert int((~agree).sum()) <= 0.005 * crop * crop
    assert err[agree].max().item() <= 1e-4


def test_split_march_schedule_invariant():
    _, mine = _blob(64, 256, 16, "softplus", seed=9)
    rays = _rays(24, 11, eye=(0.0, 0.2, 1.1))
    base, bh, _ = _march_split(mine, rays)
    for blocks, xcd in ((1, 1), (5, 1), (13, 1), (0, 0), (5, 0)):
        _lib_opt("march_blocks", blocks)
        _lib_opt("xcd_lines", xcd)
        it, h, _ = _march_split(mine, rays)
        assert torch.equal(h, bh)
        assert torch.equal(it.t, base.t) and torch.equal(it.throughput, base.throughput)
        assert torch.equal(it.p, base.p) and torch.equal(it.n, base.n)


@pytest.mark.parametrize("n", [1, 33, 3001])
def test_split_ragged_ray_counts(n):
    import torch.nn.functional as F
    ref, mine = _blob(64, 128, 32, "softplus", seed=23)
    g = torch.Generator().manual_seed(n)
    o = torch.tensor([0.0, 0.2, 1.1]) + 0.05 * torch.randn(1, n, 1, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, n, 1, 1, 2, generator=g) * 0.8 - 0.4,
                               -torch.ones(1, n, 1, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    it, hit, n3 = _march_split(mine, rays)
    assert n3 == 1
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=64).intersect(rays, primary=True, jitter=jit)
    assert torch.isfinite(it.t).all() and torch.isfinite(it.throughput).all()
    _compare(f"split_ragged[{n}]", it, hit, rit, rhit, flip_frac=max(0.005, 1.0 / n))


def test_split_after_device_refresh_matches_fresh_pack():
    """nrt_mlp_refresh re-splits stream3 / bias3 on the device (fold, hi / lo halves: the
    packer's arithmetic) at the handle's pack-time power-of-two scales, where a fresh host pack
    picks the scales of the new weights: the two representations of the same weights march to
    the same hits and depths to FP32 rounding."""
    import ctypes
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer._handles import train_handle, mlp_handle
    _, mine = _blob(64, 128, 32, "softplus", seed=13)
    mlp = mine.shift
    th = train_handle(mlp)
    with torch.no_grad():
        for lin in mlp._linears():
            lin.weight.add_(0.01 * torch.randn_like(lin.weight))
            lin.bias.add_(0.01 * torch.randn_like(lin.bias))
    th2 = train_handle(mlp)  # same handle, refreshed on the device
    assert th2 is th
    fresh = mlp_handle(mlp)
    assert fresh is not th
    rays = _rays(24, 17, eye=(0.0, 0.2, 1.1)).cuda().reshape(-1, 6).contiguous()
    c, r, t = (x.detach().cpu().contiguous() for x in (mine.centers, mine.radii, mine.tfs))
    outs = []
    for h in (th, fresh):
        sh = ctypes.c_void_p()
        _lib.check(_lib.load().nrt_sdf_create_sphere_blob(
            c.shape[0], c.data_ptr(), r.data_ptr(), t.data_ptr(), 32.0, h.value, ctypes.byref(sh)),
            "nrt_sdf_create_sphere_blob")
        try:
            _lib.profile_enable(True)
            _lib.profile_reset()
            outs.append(_intersect_raw(sh, rays, max_steps=64, precision=_lib.NRT_FP32_SPLIT))
            assert _lib.profile_read("k_march3")[1] == 1, "the split march did not run"
            _lib.profile_enable(False)
        finally:
            _lib.load().nrt_sdf_destroy(sh)
    (t, hit, p, n, thr), (t2, hit2, p2, n2, thr2) = outs
    assert torch.equal(hit, hit2)
    m = hit.bool()
    assert m.any()
    assert (t - t2).abs().max().item() <= 1e-5
    assert (p[m] - p2[m]).abs().max().item() <= 1e-5 and (n[m] - n2[m]).abs().max().item() <= 1e-5
    assert (thr - thr2).abs().max().item() <= 0.05  # -1000 sdf(best): 5e-5 on the sdf
