"""HIP path vs the CPU oracle (FP32 parity bar 1e-4 abs; FP16 judged by relative error/PSNR)."""
import math
import random

import pytest
import torch
import torch.nn.functional as F

from oracle import pathtracer_ref as R
from oracle import recipes
from tests.helpers import copy_mlp, product_mlp_like, seeded
from tests.helpers import lib_opt as _lib_opt
from tests.report import report

pytestmark = pytest.mark.gpu

# FP16 render bars (PSNR against the oracle, dB): the measured level minus about 5 dB
# (round 5: render 106.2 dB, program shading 98.5 dB)
PSNR_FP16_RENDER = 101.0
PSNR_FP16_PROGRAM = 93.0

MLP_CASES = [
    # name, ctor kwargs, activation, init
    ("sdf_8x256_softplus", dict(num_layers=8, hidden_size=256, out=1, freqs=16), "softplus", None),
    ("neural_bsdf_6x96", dict(num_layers=6, hidden_size=96, out=3, freqs=64), "leaky_relu", None),
    ("light_field_10x256", dict(num_layers=10, hidden_size=256, out=3, freqs=16), "leaky_relu", None),
    ("sp_var_16x256", dict(num_layers=16, hidden_size=256, out=8, freqs=128, sigma=128,
                           xavier_init=True), "leaky_relu", None),
    ("shift_8x128", dict(num_layers=8, hidden_size=128, out=1, freqs=32), "softplus", None),
    ("nerfle_first_5x128", dict(num_layers=5, hidden_size=128, out=65, freqs=16), "leaky_relu", None),
    ("default_8x64", dict(num_layers=8, hidden_size=64, out=3, freqs=16), "leaky_relu", None),
    ("plain_nerf_latent", dict(num_layers=5, hidden_size=32, out=33, latent_size=32), "leaky_relu", None),
]


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


@pytest.mark.parametrize("name,kw,act,_", MLP_CASES, ids=[c[0] for c in MLP_CASES])
@pytest.mark.parametrize("M", [1, 31, 1000])
def test_mlp_forward_fp32(name, kw, act, _, M):
    seeded(1)
    ref = R.SkipMLP(activation=act, **kw)
    mine = product_mlp_like(ref, act)
    x = torch.rand(M, 3) * 2 - 1
    lat = torch.randn(M, kw["latent_size"]) if kw.get("latent_size") else None
    with torch.no_grad():
        want = ref(x, lat)
        got = mine(x.cuda(), None if lat is None else lat.cuda()).cpu()
    scale = max(1.0, want.abs().max().item())
    assert (got - want).abs().max().item() <= 1e-4 * scale, (got - want).abs().max()


@pytest.mark.parametrize("name,kw,act,_", MLP_CASES[:5], ids=[c[0] for c in MLP_CASES[:5]])
def test_mlp_forward_fp16_close(name, kw, act, _):
    from neural_raytracing_amd import set_precision
    seeded(2)
    ref = R.SkipMLP(activation=act, **kw)
    mine = product_mlp_like(ref, act)
    x = (torch.rand(4096, 3) * 2 - 1)
    with torch.no_grad():
        want = ref(x)
        set_precision("fp16")
        got = mine(x.cuda()).cpu()
    err = (got - want).abs().max().item()
    assert err <= 2e-2 * max(1.0, want.abs().max().item()), err


def _blob_pair(n=32, shift_hidden=128, nonzero_shift=True):
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    seeded(3)
    ref = R.SphereBlobSDF(n=n, shift_hidden=shift_hidden, shift_zero_init=not nonzero_shift)
    if nonzero_shift:
        with torch.no_grad():
            ref.shift.out.weight.mul_(0.05)
    mine = SphereSDF(n=n, device="cpu")
    if shift_hidden != 128:
        raise ValueError
    with torch.no_grad():
        mine.centers.copy_(ref.centers)
        mine.radii.copy_(ref.radii)
        mine.tfs.copy_(ref.tfs + 0.05 * torch.randn_like(ref.tfs))
        ref.tfs.copy_(mine.tfs)
    copy_mlp(mine.shift, ref.shift)
    return ref, mine.cuda()


def test_sphere_sdf_eval_and_grad_fp32():
    ref, mine = _blob_pair()
    p = torch.rand(777, 3) - 0.5
    with torch.no_grad():
        want = ref(p)
        got = mine(p.cuda()).cpu()
    assert (got - want).abs().max().item() < 1e-5
    from neural_raytracing_amd.pathtracer.shapes import SDF
    g_ref = R.MarchedSDF(sdf=ref).gradient(p)
    with torch.no_grad():
        g = SDF(sdf=mine).autograd_diff(p.cuda()).cpu()
    assert (g - g_ref).abs().max().item() < 1e-4


def test_mlp_sdf_grad_fp32():
    from neural_raytracing_amd.pathtracer.shapes import SDF
    seeded(4)
    ref = R.SkipMLP(num_layers=8, hidden_size=256, out=1, freqs=16, activation="softplus")
    mine = product_mlp_like(ref, "softplus")
    p = torch.rand(300, 3) - 0.5
    g_ref = R.MarchedSDF(sdf=ref).gradient(p)
    with torch.no_grad():
        g = SDF(sdf=mine).autograd_diff(p.cuda()).cpu()
    assert (g - g_ref).abs().max().item() < 1e-4 * max(1.0, g_ref.abs().max().item())


def test_unit_sphere_intersect_kat():
    from neural_raytracing_amd.pathtracer.shapes import SDF, SPHERE_SDF
    rays = torch.tensor([[0.0, 0.0, 1.5, 0.0, 0.0, -1.0],
                         [0.3, 0.0, 1.5, 0.0, 0.0, -1.0],
                         [0.0, 3.0, 1.5, 0.0, 0.0, -1.0]])
    shape = SDF(sdf=SPHERE_SDF, max_steps=16)
    with torch.no_grad():
        it, hit = shape.intersect(rays.cuda(), primary=False)
    ref_it, ref_hit = R.MarchedSDF(max_steps=16).intersect(rays, primary=False)
    assert hit.cpu().tolist() == ref_hit.tolist() == [True, True, False]
    assert torch.allclose(it.t.cpu(), ref_it.t, atol=1e-6)
    assert torch.allclose(it.n.cpu(), ref_it.n, atol=1e-6)
    assert torch.allclose(it.p.cpu(), ref_it.p, atol=1e-6)
    assert torch.allclose(it.wi.cpu(), ref_it.wi, atol=1e-6)
    assert torch.allclose(it.frame.cpu(), ref_it.frame, atol=1e-6)


def test_blob_intersect_matches_oracle():
    from neural_raytracing_amd.pathtracer.shapes import SDF
    ref, mine = _blob_pair()
    seeded(5)
    o = torch.tensor([0.0, 0.0, 1.0]).expand(1, 48, 48, 1, 3)
    d = F.normalize(torch.cat([torch.rand(1, 48, 48, 1, 2) * 0.6 - 0.3,
                               -torch.ones(1, 48, 48, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    with torch.no_grad():
        it, hit = SDF(sdf=mine, max_steps=32).intersect(rays.cuda(), primary=True)
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=32).intersect(rays, primary=True,
                                                                    jitter=_last_jitter())
    agree = (hit.cpu() == rhit).reshape(-1)
    assert agree.float().mean() > 0.99
    m = agree & rhit.reshape(-1)
    assert m.sum() > 100
    assert (it.t.cpu().reshape(-1)[m] - rit.t.reshape(-1)[m]).abs().max() < 1e-4
    assert (it.n.cpu().reshape(-1, 3)[m] - rit.n.reshape(-1, 3)[m]).abs().max() < 1e-3
    thr_diff = (it.throughput.cpu().reshape(-1) - rit.throughput.reshape(-1)).abs()
    # the scan argmin can pick a different sample when two samples tie to ~1 ulp
    assert (thr_diff < 1e-2).float().mean() > 0.99


_JIT = {}


def _last_jitter():
    # the product drew random.random() once; replay the same draw for the oracle
    random.seed(5)
    return random.random()


def _scene_pair(scene_fn=recipes.baseline_checksum_scene):
    """Oracle scene and the product scene with identical weights (same seed, same order)."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, NeuralBSDF
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from neural_raytracing_amd.pathtracer.lights import LightField
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    ref = scene_fn()
    torch.manual_seed(0)
    random.seed(0)
    sphere = SphereSDF(n=128, device="cpu")
    shape = SDF(sdf=sphere, device="cpu", max_steps=32)
    bsdf = ComposeSpatialVarying([NeuralBSDF(activation=torch.nn.Softplus(), device="cpu")
                                  for _ in range(8)], device="cpu")
    lights = LightField(device="cpu")
    integ = NeRFIntegrator(Direct())
    # identical RNG order => identical weights; verify instead of assuming
    assert torch.equal(sphere.centers, ref["shape"].sdf.centers)
    assert torch.equal(bsdf.sp_var_fn.out.weight, ref["bsdf"].sp_var_fn.out.weight)
    assert torch.equal(lights.light_field_approx.init.weight,
                       ref["lights"].light_field_approx.init.weight)
    sphere.cuda()
    for b in bsdf.bsdfs:
        b.mlp.cuda()
    bsdf.sp_var_fn.cuda()
    lights.cuda()
    cam = pt.cameras.NeRFCamera(cam_to_world=ref["camera"].cam_to_world.cuda(),
                                focal=ref["camera"].focal, device="cuda")
    return ref, dict(shape=shape, bsdf=bsdf, lights=lights, integrator=integ, camera=cam)


def test_render_matches_oracle_fp32():
    """The BASELINE.md §2 scene (no camera jitter) rendered by both paths."""
    import neural_raytracing_amd.pathtracer as pt
    ref, mine = _scene_pair()
    random.seed(11)
    with torch.no_grad():
        want = R.render(ref["shape"], ref["lights"], ref["camera"], ref["integrator"], ref["bsdf"],
                        size=256, chunk_size=256, background=0.0, with_noise=0.0,
                        crop=(96, 96, 64))
    random.seed(11)
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"],
                                     mine["integrator"], bsdf=mine["bsdf"], size=256,
                                     chunk_size=256, bundle_size=1, crop_size=64, uv=(96, 96),
                                     background=0, with_noise=0.0, device="cuda")
    got = got.cpu()
    assert got.shape == want.shape == (64, 64, 4)
    diff = (got - want).abs()
    assert diff.max().item() <= 1e-4, diff.max()


def test_render_fp16_psnr():
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    ref, mine = _scene_pair()
    random.seed(11)
    with torch.no_grad():
        want = R.render(ref["shape"], ref["lights"], ref["camera"], ref["integrator"], ref["bsdf"],
                        size=256, chunk_size=256, background=0.0, with_noise=0.0,
                        crop=(96, 96, 64))
    random.seed(11)
    set_precision("fp16")
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"],
                                     mine["integrator"], bsdf=mine["bsdf"], size=256,
                                     chunk_size=256, bundle_size=1, crop_size=64, uv=(96, 96),
                                     background=0, with_noise=0.0, device="cuda")
    mse = ((got.cpu().clamp(0, 1) - want.clamp(0, 1)) ** 2).mean()
    psnr = -10 * math.log10(max(mse.item(), 1e-12))
    report("render_fp16_psnr", pixels=64 * 64, psnr=psnr,
           maxabs=float((got.cpu() - want).abs().max()))
    assert psnr > PSNR_FP16_RENDER, psnr


def test_nerf_raygen_matches_oracle():
    import neural_raytracing_amd.pathtracer as pt
    c2w = recipes.look_at_c2w((0.3, 0.4, 0.866)).unsqueeze(0)
    focal = recipes.nerf_focal(64)
    ref = R.NeRFCameraRef(c2w, focal)
    pos = R._tile_positions(8, 16, 32)
    want = ref.sample_positions(pos, 64, 0.0)
    got = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal).rays_tile(8, 16, 32, 32, 64)
    assert torch.allclose(got.cpu(), want, atol=1e-6)


def test_dtu_raygen_matches_oracle():
    import neural_raytracing_amd.pathtracer as pt
    K = torch.eye(4)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2], K[0, 1] = 2890.0, 2890.0, 800.0, 600.0, 0.3
    pose = torch.eye(4)
    pose[:3, :4] = recipes.look_at_c2w((0.0, 0.5, 0.866))
    pose[:3, 1:3] *= -1  # DTU looks down +z
    ref = R.DTUCameraRef(pose[None], K[None])
    pos = R._tile_positions(0, 0, 16)
    want = ref.sample_positions(pos, 64)
    got = pt.cameras.DTUCamera(pose=pose[None].cuda(), intrinsic=K[None].cuda()).rays_tile(0, 0, 16, 16, 64)
    assert torch.allclose(got.cpu(), want, atol=2e-6)


def test_all_miss_tile_and_empty_batch():
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.shapes import SDF, SPHERE_SDF
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    m = SkipConnMLP(device="cuda")
    with torch.no_grad():
        assert m(torch.empty(0, 3, device="cuda")).shape == (0, 3)
        rays = torch.tensor([[0.0, 5.0, 1.5, 0.0, 0.0, -1.0]] * 70).cuda()
        it, hit = SDF(sdf=SPHERE_SDF).intersect(rays, primary=False)
    assert not hit.any()
    assert (it.n == 0).all()


def test_pathtrace_fused_tiles_match_oracle():
    """Full-frame pathtrace (fused tile path, 4 tiles) vs the oracle's tile loop."""
    import neural_raytracing_amd.pathtracer as pt
    ref, mine = _scene_pair()
    for integ_ref, integ in [(ref["integrator"], mine["integrator"]),
                             (R.DirectRef(), mine["integrator"].sub_integrator)]:
        random.seed(21)
        with torch.no_grad():
            want = R.render(ref["shape"], ref["lights"], ref["camera"], integ_ref, ref["bsdf"],
                            size=64, chunk_size=32, background=0.25, with_noise=0.0)
        random.seed(21)
        with torch.no_grad():
            got, _ = pt.pathtrace(mine["shape"], mine["lights"], mine["camera"], integ,
                                  bsdf=mine["bsdf"], size=64, chunk_size=32, bundle_size=1,
                                  background=0.25, with_noise=0.0)
        assert got.shape == want.shape
        assert (got.cpu() - want).abs().max().item() <= 1e-4


@pytest.mark.parametrize("hidden,freqs", [(256, 16), (128, 32)])
def test_ring_fp16_intersect_matches_oracle(hidden, freqs):
    """The block-cooperative FP16 kernel (LDS weight ring, log2-folded softplus) vs the oracle."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    seeded(7)
    ref = R.SphereBlobSDF(n=1, shift_hidden=hidden, shift_freqs=freqs, shift_zero_init=False)
    with torch.no_grad():
        ref.centers.zero_()
        ref.radii.fill_(0.25)
        ref.shift.out.weight.mul_(0.1)
        ref.shift.out.bias.mul_(0.1)
    mine = SphereSDF(n=1, device="cpu")
    mine.shift = SkipConnMLP(num_layers=8, hidden_size=hidden, in_size=3, out=1, freqs=freqs,
                             activation=F.softplus, device="cpu")
    with torch.no_grad():
        mine.centers.copy_(ref.centers)
        mine.radii.copy_(ref.radii)
    copy_mlp(mine.shift, ref.shift)
    mine = mine.cuda()
    o = torch.tensor([0.0, 0.2, 1.0]).expand(1, 40, 40, 1, 3)
    d = F.normalize(torch.cat([torch.rand(1, 40, 40, 1, 2) * 0.7 - 0.35,
                               -torch.ones(1, 40, 40, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    set_precision("fp16")
    random.seed(9)
    with torch.no_grad():
        it, hit = SDF(sdf=mine, max_steps=48).intersect(rays.cuda(), primary=True)
    random.seed(9)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=48).intersect(rays, primary=True, jitter=jit)
    agree = (hit.cpu() == rhit).reshape(-1)
    assert agree.float().mean() > 0.98, agree.float().mean()
    m = agree & rhit.reshape(-1)
    assert m.sum() > 200
    assert (it.t.cpu().reshape(-1)[m] - rit.t.reshape(-1)[m]).abs().max() < 2e-2
    thr = (it.throughput.cpu().reshape(-1) - rit.throughput.reshape(-1)).abs()
    assert (thr < 5.0).float().mean() > 0.95
    # FP16 forward-mode normals (k_normal16) vs the oracle's autograd normals: unit length,
    # within 1 degree on 99 % of the agreeing hits
    n16 = it.n.cpu().reshape(-1, 3)[m]
    nref = rit.n.reshape(-1, 3)[m]
    assert (n16.norm(dim=-1) - 1).abs().max() < 1e-4
    cos = (n16 * nref).sum(-1).clamp(-1, 1)
    assert (cos > math.cos(math.radians(1.0))).float().mean() > 0.99, cos.min()
    assert cos.min() > math.cos(math.radians(5.0)), cos.min()


@pytest.mark.gpu
def test_fp16_normals_match_f32_backward(monkeypatch):
    """k_normal16 (FP16 forward mode) vs k_sdf_grad (FP32 reverse mode) on the same hit points:
    raw gradients agree to FP16 accuracy."""
    from neural_raytracing_amd import set_precision, _lib
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    seeded(3)
    mine = SphereSDF(n=1, device="cpu")
    mine.shift = SkipConnMLP(num_layers=8, hidden_size=256, in_size=3, out=1, freqs=16,
                             activation=F.softplus, device="cpu")
    with torch.no_grad():
        mine.centers.zero_()
        mine.radii.fill_(0.25)
        mine.shift.out.weight.mul_(0.1)
    mine = mine.cuda()
    o = torch.tensor([0.0, 0.0, 1.0]).expand(1, 64, 64, 1, 3)
    d = F.normalize(torch.cat([torch.rand(1, 64, 64, 1, 2) * 0.6 - 0.3,
                               -torch.ones(1, 64, 64, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1).cuda()
    set_precision("fp16")
    out = {}
    for mode in ("f16", "f32"):
        if mode == "f32":
            _lib_opt("normals16", 0)
        random.seed(5)
        with torch.no_grad():
            it, hit = SDF(sdf=mine, max_steps=48).intersect(rays, primary=True)
            out[mode] = (hit.clone(), it.raw_normals.clone(), it.n.clone(), it.p.clone())
    _lib_opt("normals16", 1)
    set_precision("fp32")
    h16, g16, n16, p16 = out["f16"]
    h32, g32, n32, p32 = out["f32"]
    assert torch.equal(h16, h32)
    m = h16.reshape(-1)
    assert m.sum() > 500
    rel = (g16 - g32).norm(dim=-1) / g32.norm(dim=-1)
    assert rel.max() < 2e-2, rel.max()
    assert (n16.reshape(-1, 3)[m] - n32.reshape(-1, 3)[m]).abs().max() < 2e-2
    assert (p16.reshape(-1, 3)[m] - p32.reshape(-1, 3)[m]).abs().max() < 1e-5
    # misses keep zero normals
    assert n16.reshape(-1, 3)[~m].abs().max() == 0


@pytest.mark.gpu
def test_program_shading_nerf_synthetic_scene(monkeypatch):
    """k_light16 + k_bsdf16 (program engine: LightField 10x256, spatial 16x256 F=128, 8 x
    NeuralBSDF 6x96 F=64) against the per-wave FP16 register path (same MFMA order: equal to
    rounding) and against the oracle (PSNR)."""
    import bench
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    scene = bench.build_scene("cuda", samples=32, seed=2)
    pt = scene["pt"]
    size, crop = 200, 40
    c0 = (size - crop) // 2
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)

    def render():
        random.seed(7)
        with torch.no_grad():
            img, _ = pt.pathtrace_sample(scene["shape"], scene["lights"], cam, scene["integrator"],
                                         bsdf=scene["bsdf"], size=size, chunk_size=size,
                                         bundle_size=1, crop_size=crop, uv=(c0, c0), background=0,
                                         with_noise=0.0)
        return img.cpu()

    nra.set_precision("fp16")
    _lib.profile_enable(True)
    _lib.profile_reset()
    prog = render()
    _, n_bsdf = _lib.profile_read("k_bsdf16")
    _, n_light = _lib.profile_read("k_light16")
    _lib.profile_enable(False)
    assert n_bsdf >= 1 and n_light >= 1, "program shading path did not run"
    _lib_opt("shade_program", 0)
    regs = render()
    _lib_opt("shade_program", 1)
    nra.set_precision("fp32")
    assert (prog - regs).abs().max() < 2e-3, (prog - regs).abs().max()
    # oracle (fp32 restatement) on the same crop
    from oracle import pathtracer_ref as R
    osc = bench.oracle_scene(scene)
    random.seed(7)
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], R.NeRFCameraRef(c2w, focal), osc["integrator"],
                        osc["bsdf"], size=size, chunk_size=size, background=0.0, with_noise=0.0,
                        crop=(c0, c0, crop))
    hit = prog[..., 3] if prog.shape[-1] == 4 else None
    assert hit is None or (prog[..., :3].abs().sum() > 0)
    mse = ((prog.clamp(0, 1) - want.clamp(0, 1)) ** 2).mean().item()
    psnr = -10 * math.log10(max(mse, 1e-12))
    report("program_shading_fp16_psnr", pixels=crop * crop, psnr=psnr,
           program_vs_per_component=float((prog - regs).abs().max()))
    assert psnr > PSNR_FP16_PROGRAM, psnr


def _ring_blob(hidden, freqs, seed, zero_out=False):
    """Oracle SphereBlobSDF (one sphere r = 0.25) + the product copy with an 8-layer shift MLP."""
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    seeded(seed)
    ref = R.SphereBlobSDF(n=1, shift_hidden=hidden, shift_freqs=freqs, shift_zero_init=False)
    with torch.no_grad():
        ref.centers.zero_()
        ref.radii.fill_(0.25)
        ref.shift.out.weight.mul_(0.0 if zero_out else 0.1)
        ref.shift.out.bias.mul_(0.0 if zero_out else 0.1)
    mine = SphereSDF(n=1, device="cpu")
    mine.shift = SkipConnMLP(num_layers=8, hidden_size=hidden, in_size=3, out=1, freqs=freqs,
                             activation=F.softplus, device="cpu")
    with torch.no_grad():
        mine.centers.copy_(ref.centers)
        mine.radii.copy_(ref.radii)
    copy_mlp(mine.shift, ref.shift)
    return ref, mine.cuda()


def _scene_rays(P, seed):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.0, 0.1, 1.0]) + 0.05 * torch.randn(P, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(P, 2, generator=g) * 0.9 - 0.45, -torch.ones(P, 1)], -1), dim=-1)
    return torch.cat([o, d], -1).reshape(1, P, 1, 1, 6)


@pytest.mark.parametrize("P", [1, 33, 2500])
def test_ring_march_zero_shift_matches_oracle(P):
    """FP16 ring march with a zero output layer: the MLP contributes exactly 0, so the SDF is the
    f32 sphere blob and march, coarse-scan argmin, sdf(best) and normals must match the oracle
    tightly -- this pins the load-balanced job lists (march jobs, 8 scan segments per ray merged
    by 64-bit atomic min, sdf(best) pass) to the reference loop semantics (sdfs.py:119-131,
    232-249)."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    ref, mine = _ring_blob(256, 16, 5, zero_out=True)
    rays = _scene_rays(P, 11)
    set_precision("fp16")
    random.seed(4)
    with torch.no_grad():
        it, hit = SDF(sdf=mine, max_steps=40).intersect(rays.cuda(), primary=True)
    random.seed(4)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=40).intersect(rays, primary=True, jitter=jit)
    hit, rhit = hit.cpu().reshape(-1), rhit.reshape(-1)
    assert (hit == rhit).float().mean() >= (0.99 if P > 100 else 1.0)
    m = hit & rhit
    assert (it.t.cpu().reshape(-1)[m] - rit.t.reshape(-1)[m]).abs().max().item() < 1e-4 if m.any() else True
    thr = (it.throughput.cpu().reshape(-1) - rit.throughput.reshape(-1)).abs()
    assert (thr < 1e-2).float().mean() >= (0.99 if P > 100 else 1.0), thr.max()
    if m.any():
        cos = (it.n.cpu().reshape(-1, 3)[m] * rit.n.reshape(-1, 3)[m]).sum(-1)
        assert cos.min() > 0.9999


def test_ring_march_schedule_invariant(monkeypatch):
    """Results of the persistent load-balanced march do not depend on the grid: 1, 5 and the
    default number of blocks give bit-identical t, hit, p, n and throughput (each ray's
    arithmetic is its own; only which lane runs it changes).  At 1 and 5 blocks a wave owns 375 /
    75 rays, so most scans run as whole 129-point jobs with a plain key store; at the default grid
    every ray is in the segmented tail (atomicMin merge): the two scan paths agree bit for bit."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    _, mine = _ring_blob(256, 16, 8)
    rays = _scene_rays(3001, 12).cuda()
    set_precision("fp16")
    outs = []
    # (blocks, xcd_lines): the default grid with both ray deals, and grids of 1, 5, 13 blocks
    # (fewer XCD groups than XCDs, a group with one block more than another)
    # and the launch-wide job queue (option march_queue) at the default grid and at 5 blocks
    for blocks, xcd, q in ((0, 1, 0), (0, 0, 0), (1, 1, 0), (5, 1, 0), (13, 1, 0), (5, 0, 0),
                           (0, 0, 1), (5, 0, 1)):
        _lib_opt("march_blocks", blocks)
        _lib_opt("xcd_lines", xcd)
        _lib_opt("march_queue", q)
        random.seed(2)
        with torch.no_grad():
            it, hit = SDF(sdf=mine, max_steps=64).intersect(rays, primary=True)
        outs.append([hit.cpu(), it.t.cpu(), it.p.cpu(), it.n.cpu(), it.throughput.cpu()])
    assert outs[0][0].any() and not outs[0][0].all()
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert torch.equal(a, b)


def _shadow_scene():
    """A large sphere with a small one floating between it and a point light (it casts a shadow
    on the large one); Diffuse BSDF; NeRF camera.  Oracle and product objects, same numbers."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import Diffuse
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    seeded(3)
    ref = R.SphereBlobSDF(n=2, shift_zero_init=True)
    with torch.no_grad():
        ref.centers.copy_(torch.tensor([[0.0, 0.0, 0.0], [0.05, 0.45, 0.12]]))
        ref.radii.copy_(torch.tensor([0.3, 0.1]))
    mine = SphereSDF(n=2, device="cpu")
    with torch.no_grad():
        mine.centers.copy_(ref.centers)
        mine.radii.copy_(ref.radii)
    copy_mlp(mine.shift, ref.shift)
    loc = (0.15, 1.4, 0.4)
    c2w = recipes.look_at_c2w((0.0, 0.7, 0.9)).unsqueeze(0)
    focal = recipes.nerf_focal(64)
    oracle = dict(shape=R.MarchedSDF(sdf=ref, max_steps=48), bsdf=R.DiffuseRef(),
                  lights=R.PointLightRef(location=loc, scale=5.0),
                  camera=R.NeRFCameraRef(c2w, focal))
    prod = dict(shape=SDF(sdf=mine.cuda(), max_steps=48), bsdf=Diffuse(device="cuda"),
                lights=PointLights(location=list(loc), scale=5.0, device="cuda"),
                camera=pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal, device="cuda"))
    return oracle, prod


@pytest.mark.parametrize("prec", ["fp32", "fp32-split", "fp16", "mixed"])
def test_direct_shadow_rays_match_oracle(prec):
    """Direct with w_isect=True (sample_emitter_dir_w_isect, scene.py:290-298 + intersect_test,
    sdfs.py:162-181): HIP shadow march + masked shading vs the oracle.  FP32 within 1e-4 except
    at most 0.5 % of pixels (shadow-boundary flips from ulp-level march differences); FP16 by
    PSNR."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Direct
    ref, mine = _shadow_scene()
    imgs = {}
    for w_isect in (False, True):
        random.seed(8)
        with torch.no_grad():
            imgs[w_isect] = R.render(ref["shape"], ref["lights"], ref["camera"], R.DirectRef(),
                                     ref["bsdf"], size=64, chunk_size=64, background=0.0,
                                     with_noise=0.0, w_isect=w_isect)
    shadowed = (imgs[False] - imgs[True]).abs().amax(-1) > 1e-3
    assert shadowed.sum() > 40, "the scene must cast a shadow for this test to mean anything"
    set_precision(prec)
    random.seed(8)
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"], Direct(),
                                     bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                     crop_size=64, uv=(0, 0), background=0, with_noise=0.0,
                                     w_isect=True)
    got = got.cpu()
    want = imgs[True]
    assert got.shape == want.shape
    err = (got - want).abs().amax(-1)
    report(f"direct_shadow_rays[{prec}]", pixels=err.numel(), shadowed=int(shadowed.sum()),
           over_1e4=int((err > 1e-4).sum()), maxabs=err.max().item())
    # fp32 and fp32-split: the FP32 bar (flips at a shadow boundary aside); fp16 measured
    # 4e-7 here (the Diffuse shading is FP32 math on FP16-march hits): the same bar
    close = err <= 1e-4
    assert close.float().mean() >= 0.995, (got - want).abs().max()


def _occ_pair(out=1, seed=21):
    """An occlusion MLP (SkipConnMLP 5 -> out, as w_isect takes it, scene.py:301-319): oracle
    and product copies with the same weights."""
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    seeded(seed)
    ref = R.SkipMLP(num_layers=4, hidden_size=64, in_size=5, out=out)
    mine = SkipConnMLP(num_layers=4, hidden_size=64, in_size=5, out=out, device="cpu")
    copy_mlp(mine, ref)
    return ref, mine.cuda()


@pytest.mark.parametrize("prec,out", [("fp32", 1), ("fp32", 3), ("fp16", 1)])
def test_direct_learned_occlusion_matches_oracle(prec, out):
    """Direct with w_isect=<SkipConnMLP> (sample_emitter_dir_w_learned_occ, scene.py:301-319):
    shadow march, occ([p, dir_to_elev_azim(d)]) on the HIP MLP, sigmoid-scaled Le where occluded.
    FP32 within 1e-4 except shadow-boundary flips (<= 0.5 % of pixels); FP16 by PSNR."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Direct
    ref, mine = _shadow_scene()
    occ_ref, occ_mine = _occ_pair(out)
    random.seed(8)
    with torch.no_grad():
        want = R.render(ref["shape"], ref["lights"], ref["camera"], R.DirectRef(), ref["bsdf"],
                        size=64, chunk_size=64, background=0.0, with_noise=0.0, w_isect=occ_ref)
        hard = R.render(ref["shape"], ref["lights"], ref["camera"], R.DirectRef(), ref["bsdf"],
                        size=64, chunk_size=64, background=0.0, with_noise=0.0, w_isect=True)
    # the learned term must light up pixels the hard shadow leaves black
    lit = (want - hard).abs().amax(-1) > 1e-3
    assert lit.sum() > 40
    set_precision(prec)
    random.seed(8)
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"], Direct(),
                                     bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                     crop_size=64, uv=(0, 0), background=0, with_noise=0.0,
                                     w_isect=occ_mine)
    got = got.cpu()
    assert got.shape == want.shape
    if prec == "fp32":
        close = (got - want).abs().amax(-1) <= 1e-4
        assert close.float().mean() >= 0.995, (got - want).abs().max()
    else:
        mse = ((got.clamp(0, 1) - want.clamp(0, 1)) ** 2).mean().item()
        assert -10 * math.log10(max(mse, 1e-12)) > 40


def test_learned_occlusion_needs_5_inputs():
    """nrt_shade_direct_learned_occ refuses an occlusion MLP that is not 5 -> 1|3."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    _, mine = _shadow_scene()
    bad = SkipConnMLP(num_layers=2, hidden_size=32, in_size=5, out=2, device="cuda")
    with pytest.raises(NrtError):
        with torch.no_grad():
            pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"], Direct(),
                                bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                crop_size=32, uv=(0, 0), background=0, with_noise=0.0,
                                w_isect=bad)


def test_direct_shadow_rays_need_point_light():
    """The reference's LightField samples carry no distance (lights.py:175-195), so
    w_isect=True cannot run with it there; the HIP path refuses it loudly."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.lights import LightField
    _, mine = _shadow_scene()
    with pytest.raises(NrtError):
        with torch.no_grad():
            pt.pathtrace_sample(mine["shape"], LightField(device="cuda"), mine["camera"], Direct(),
                                bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                crop_size=32, uv=(0, 0), background=0, with_noise=0.0,
                                w_isect=True)


def test_fov_raygen_matches_oracle():
    """nrt_raygen(NRT_CAM_FOV) vs FoVPerspectiveCameras.sample_positions (renderer/cameras.py:
    539-575), without and with the sampler's jitter (the same uniforms injected into both)."""
    from neural_raytracing_amd.pathtracer.cameras import OpenGLPerspectiveCameras
    Rm, Tm = R.look_at_view_transform_ref(dist=1.0, elev=30.0, azim=45.0)
    ref = R.FoVCameraRef(Rm, Tm, znear=1.0, zfar=100.0)
    cam = OpenGLPerspectiveCameras(R=Rm, T=Tm, device="cuda")
    pos = R._tile_positions(8, 16, 32)
    want = ref.sample_positions(pos, 64)
    got = cam.rays_tile(8, 16, 32, 32, 64)
    assert torch.allclose(got.cpu(), want, atol=2e-6)
    noise = torch.rand(32, 32, 2)
    want = ref.sample_positions(pos, 64, with_noise=0.5, noise=noise.unsqueeze(-2))
    got = cam.rays_tile(8, 16, 32, 32, 64, with_noise=0.5, noise=noise.cuda())
    assert torch.allclose(got.cpu(), want, atol=2e-6)


def _colocate_pair():
    """cfg3-like scene (colocate.py:63-80, 109): SphereSDF(n=64), OpenGLPerspectiveCameras from
    look_at_view_transform(dist=1, elev=30, azim=45), PointLights(scale=5) at 1.05 x the camera
    centre, ComposeSpatialVarying([NeuralBSDF x 2, Diffuse(Softplus).random(),
    Conductor(Softplus).random()]), Direct().  Oracle built first, product copies its numbers."""
    from neural_raytracing_amd.pathtracer.bsdf import (ComposeSpatialVarying, Conductor, Diffuse,
                                                        NeuralBSDF)
    from neural_raytracing_amd.pathtracer.cameras import OpenGLPerspectiveCameras
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    seeded(13)
    ref_sdf = R.SphereBlobSDF(n=64)
    parts = [R.NeuralBSDFRef(), R.NeuralBSDFRef(),
             R.DiffuseRef(reflectance=torch.rand(3).tolist(), preprocess="softplus"),
             R.ConductorRef(specular=torch.rand(3).tolist(), activation="softplus")]
    ref_bsdf = R.SpatialMixBSDF(parts)
    Rm, Tm = R.look_at_view_transform_ref(dist=1.0, elev=30.0, azim=45.0)
    ref_cam = R.FoVCameraRef(Rm, Tm, znear=1.0, zfar=100.0)
    loc = (ref_cam.center()[0] * 1.05).tolist()
    ref = dict(shape=R.MarchedSDF(sdf=ref_sdf, max_steps=64), bsdf=ref_bsdf,
               lights=R.PointLightRef(location=loc, scale=5.0), camera=ref_cam)
    sphere = SphereSDF(n=64, device="cpu")
    with torch.no_grad():
        sphere.centers.copy_(ref_sdf.centers)
        sphere.radii.copy_(ref_sdf.radii)
        sphere.tfs.copy_(ref_sdf.tfs)
    copy_mlp(sphere.shift, ref_sdf.shift)
    comps = [NeuralBSDF(device="cpu"), NeuralBSDF(device="cpu"),
             Diffuse(reflectance=parts[2].reflectance.tolist(), preprocess=torch.nn.Softplus(),
                     device="cuda"),
             Conductor(specular=parts[3].specular.tolist(), activation=torch.nn.Softplus(),
                       device="cuda")]
    for c, r in zip(comps[:2], parts[:2]):
        copy_mlp(c.mlp, r.mlp)
        c.mlp.cuda()
    bsdf = ComposeSpatialVarying(comps, device="cpu")
    copy_mlp(bsdf.sp_var_fn, ref_bsdf.sp_var_fn)
    bsdf.sp_var_fn.cuda()
    mine = dict(shape=SDF(sdf=sphere.cuda(), max_steps=64), bsdf=bsdf,
                lights=PointLights(location=loc, scale=5.0, device="cuda"),
                camera=OpenGLPerspectiveCameras(R=Rm, T=Tm, device="cuda"))
    return ref, mine


@pytest.mark.parametrize("prec", ["fp32", "fp32-split", "fp16", "mixed"])
def test_colocate_fov_render_matches_oracle(prec):
    """Full-frame pathtrace of the colocate-like scene (FoV camera, point light, 4-component
    spatially varying BSDF incl. Diffuse and Conductor) on the fused tile path vs the oracle."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Direct
    ref, mine = _colocate_pair()
    random.seed(17)
    with torch.no_grad():
        want = R.render(ref["shape"], ref["lights"], ref["camera"], R.DirectRef(), ref["bsdf"],
                        size=64, chunk_size=32, background=0.5, with_noise=0.0)
    assert (want != 0.5).any(-1).float().mean() > 0.1  # the object covers part of the frame
    set_precision(prec)
    random.seed(17)
    with torch.no_grad():
        got, _ = pt.pathtrace(mine["shape"], mine["lights"], mine["camera"], Direct(),
                              bsdf=mine["bsdf"], size=64, chunk_size=32, bundle_size=1,
                              background=0.5, with_noise=0.0)
    got = got.cpu()
    assert got.shape == want.shape == (64, 64, 3)
    err = (got - want).abs().amax(-1)
    # where the pixels past 1e-4 come from: primary-ray hit / step flips at the silhouette
    # (ulp-level march differences) and the Conductor's (refl . wo) > 0.94 switch (bsdfs.py:371)
    from tests.test_gpu_configs import _agreement
    with torch.no_grad():
        agree, rh, flips, steps = _agreement(
            mine["shape"], ref["shape"], mine["camera"].rays_tile(0, 0, 64, 64, 64),
            ref["camera"].sample_positions(R._tile_positions(0, 0, 64), 64))
    agree = agree.reshape(64, 64)
    report(f"colocate_fov_render[{prec}]", pixels=err.numel(), hits=int(rh.sum()), flips=flips,
           step_flips=steps, over_1e4=int((err > 1e-4).sum()),
           over_1e4_on_agreeing=int((err[agree] > 1e-4).sum()), maxabs=err.max().item())
    # measured (round 4, 64^2): 0 hit / 0 step flips at every precision; 2 allowed
    assert int((~agree).sum()) <= 2
    if prec != "fp16":  # fp32, fp32-split, mixed: the FP32 bar on every ray whose march agrees
        assert int((err[agree] > 1e-4).sum()) == 0, err[agree].max()
    else:  # measured 4.9e-4 max (FP16 SDF / shading MLP error), 298 of 4096 pixels (7.3 %) > 1e-4
        assert err[agree].max().item() <= 2e-3, err[agree].max()
        assert int((err > 1e-4).sum()) <= 0.09 * err.numel()


def _nerfle_pair(seed=19, envmap=False):
    from neural_raytracing_amd.pathtracer.shapes import NeRFLE
    seeded(seed)
    ref = R.NeRFLERef(envmap=envmap)
    mine = NeRFLE(envmap=envmap, device="cpu")
    copy_mlp(mine.first, ref.first)
    copy_mlp(mine.second, ref.second)
    return ref, mine.cuda()


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16-unfused"])
def test_nerfle_matches_oracle(prec, monkeypatch):
    """NeRFLE (nerf.py:153-214): 64 samples per ray through both MLPs and the reference's
    rolled-cumprod compositing, on nrt_nerfle_forward, vs the oracle; ragged ray count.
    "fp16" runs the fused k_nerfle16 program kernel, "fp16-unfused" the per-MLP kernels."""
    from neural_raytracing_amd import set_precision
    if prec == "fp16-unfused":
        _lib_opt("nerf_fused", 0)
        prec = "fp16"
    else:
        _lib_opt("nerf_fused", 1)
    from neural_raytracing_amd.pathtracer.lights import PointLights
    ref, mine = _nerfle_pair()
    g = torch.Generator().manual_seed(4)
    o = torch.tensor([0.0, 0.2, 1.2]) + 0.1 * torch.randn(1, 13, 11, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 13, 11, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 13, 11, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    loc = torch.tensor([[0.3, 1.0, 0.2]])
    lights = PointLights(location=loc.cuda(), device="cuda")
    set_precision(prec)
    random.seed(6)
    with torch.no_grad():
        got = mine(rays.cuda(), lights).cpu()
    random.seed(6)
    with torch.no_grad():
        want = ref(rays, loc, jitter=random.random())
    assert got.shape == want.shape == (1, 13, 11, 1, 3)
    tol = 1e-4 if prec == "fp32" else 2e-2
    assert (got - want).abs().max().item() <= tol, (got - want).abs().max()


@pytest.mark.parametrize("prec,steps", [("fp32", 37), ("fp16", 1), ("fp16", 37), ("fp16", 200)])
def test_nerfle_depth_counts(prec, steps, monkeypatch):
    """NeRFLE with depth counts other than 64 (BASELINE cfg5 asks 256): the fused kernel's
    ray-major sample order and the wave-scan compositing across partial 64-depth steps, and the
    S == 1 roll edge case, vs the oracle."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.shapes import NeRFLE
    from neural_raytracing_amd.pathtracer.lights import PointLights
    _lib_opt("nerf_fused", 1)
    seeded(31)
    ref = R.NeRFLERef(steps=steps)
    mine = NeRFLE(device="cpu", steps=steps)
    copy_mlp(mine.first, ref.first)
    copy_mlp(mine.second, ref.second)
    mine = mine.cuda()
    g = torch.Generator().manual_seed(8)
    o = torch.tensor([0.0, 0.1, 1.1]) + 0.1 * torch.randn(1, 7, 5, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 7, 5, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 7, 5, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    loc = torch.tensor([[0.2, 1.0, 0.4]])
    lights = PointLights(location=loc.cuda(), device="cuda")
    set_precision(prec)
    random.seed(3)
    with torch.no_grad():
        got = mine(rays.cuda(), lights).cpu()
    random.seed(3)
    with torch.no_grad():
        want = ref(rays, loc, jitter=random.random())
    tol = 1e-4 if prec == "fp32" else 2e-2
    assert (got - want).abs().max().item() <= tol, (got - want).abs().max()


@pytest.mark.parametrize("prec", ["fp32", "fp16", "fp16-unfused"])
def test_nerfle_envmap_matches_oracle(prec):
    """NeRFLE(envmap=True) (NeRF+LE, nerf.py:183-191): the colour MLP's light input is the point
    light's envmap at 16 directions (nrt_light_envmap) -> second MLP 115 -> 3.  "fp16" runs the
    fused k_nerfle16 with the envmap folded into one constant input column (build_nerf_program),
    "fp16-unfused" the per-MLP kernels on the 115 inputs."""
    from neural_raytracing_amd import set_precision
    if prec == "fp16-unfused":
        _lib_opt("nerf_fused", 0)
        prec = "fp16"
    else:
        _lib_opt("nerf_fused", 1)
    from neural_raytracing_amd.pathtracer.lights import PointLights
    ref, mine = _nerfle_pair(29, envmap=True)
    g = torch.Generator().manual_seed(5)
    o = torch.tensor([0.0, 0.2, 1.2]) + 0.1 * torch.randn(1, 9, 7, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 9, 7, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 9, 7, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    kw = dict(intensity=(0.9, 0.5, 0.3), location=(0.3, 1.0, 0.2), scale=3.0)
    lref = R.PointLightRef(**kw)
    lights = PointLights(intensity=list(kw["intensity"]), location=list(kw["location"]),
                         scale=kw["scale"], device="cuda")
    set_precision(prec)
    random.seed(6)
    with torch.no_grad():
        got = mine(rays.cuda(), lights).cpu()
    random.seed(6)
    with torch.no_grad():
        want = ref(rays, None, jitter=random.random(), light=lref)
    _lib_opt("nerf_fused", 1)
    assert got.shape == want.shape == (1, 9, 7, 1, 3)
    tol = 1e-4 if prec == "fp32" else 2e-2
    assert (got - want).abs().max().item() <= tol, (got - want).abs().max()


def test_nerfle_envmap_fused_psnr_and_refold():
    """NeRF+LE on the fused FP16 kernel over 2,048 rays x 64 depths: PSNR against the oracle
    (FP32 arithmetic) at least the unfused FP16 path's less 3 dB and above 60 dB; a changed light
    (another envmap) rebuilds the folded program, a repeated one reuses it (same bits)."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.lights import PointLights
    ref, mine = _nerfle_pair(31, envmap=True)
    g = torch.Generator().manual_seed(9)
    o = torch.tensor([0.0, 0.2, 1.2]) + 0.1 * torch.randn(1, 32, 64, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 32, 64, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 32, 64, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)

    def psnr(a, b):
        mse = float(((a - b) ** 2).mean())
        return 10 * math.log10(float(b.abs().max()) ** 2 / mse) if mse > 0 else float("inf")
    res = {}
    for kw in (dict(intensity=(0.9, 0.5, 0.3), location=(0.3, 1.0, 0.2), scale=3.0),
               dict(intensity=(0.2, 0.8, 0.6), location=(-0.5, 0.7, 0.4), scale=2.0)):
        lref = R.PointLightRef(**kw)
        lights = PointLights(intensity=list(kw["intensity"]), location=list(kw["location"]),
                             scale=kw["scale"], device="cuda")
        random.seed(2)
        with torch.no_grad():
            want = ref(rays, None, jitter=random.random(), light=lref)
        set_precision("fp16")
        outs = {}
        for fused in (1, 0, 1):
            _lib_opt("nerf_fused", fused)
            random.seed(2)
            with torch.no_grad():
                outs.setdefault(fused, []).append(mine(rays.cuda(), lights).cpu())
        _lib_opt("nerf_fused", 1)
        set_precision("fp32")
        fused_a, fused_b = outs[1]
        assert torch.equal(fused_a, fused_b)
        res[kw["scale"]] = (psnr(fused_a, want), psnr(outs[0][0], want), fused_a)
        report("nerfle_envmap_fused_psnr", scale=kw["scale"], fused_db=res[kw["scale"]][0],
               unfused_db=res[kw["scale"]][1])
    for fused_db, unfused_db, _ in res.values():
        assert fused_db >= min(unfused_db - 3.0, 80.0) and fused_db > 60.0, res
    assert not torch.equal(res[3.0][2], res[2.0][2])  # the second light was not served stale


def test_nerfle_pathtrace_nerf_reproduce():
    """pathtrace with NeRFReproduce (integrators.py:260-267) renders the NeRFLE tile by tile;
    each tile equals the direct NeRFLE call on the camera's rays with the same jitter draw."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import NeRFReproduce
    from neural_raytracing_amd.pathtracer.lights import PointLights
    ref, mine = _nerfle_pair(23)
    c2w = recipes.look_at_c2w((0.0, 0.3, 1.3)).unsqueeze(0)
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=recipes.nerf_focal(32), device="cuda")
    lights = PointLights(location=[0.0, 1.0, 0.0], device="cuda")
    random.seed(2)
    with torch.no_grad():
        img, _ = pt.pathtrace(mine, lights, cam, NeRFReproduce(), size=32, chunk_size=16,
                              bundle_size=1, background=0.0, with_noise=0.0)
    assert img.shape == (32, 32, 3)
    random.seed(2)
    ocam = R.NeRFCameraRef(c2w, recipes.nerf_focal(32))
    for (x0, y0) in [(0, 0), (16, 0), (0, 16), (16, 16)]:  # main.py:63-71 tile order
        rays = ocam.sample_positions(R._tile_positions(x0, y0, 16), 32)
        with torch.no_grad():
            want = ref(rays, torch.tensor([[0.0, 1.0, 0.0]]), jitter=random.random())
        got = img[x0:x0 + 16, y0:y0 + 16].cpu()
        assert (got - want[0, :, :, 0]).abs().max().item() <= 1e-4


def _path_pair(seed=31):
    """path_nerv-like scene (path_nerv.py:42-100): SphereSDF blob with a small learned shift,
    ComposeSpatialVarying([NeuralBSDF(sigmoid) x 2, Diffuse]), a point light."""
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, Diffuse, NeuralBSDF
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    seeded(seed)
    ref_sdf = R.SphereBlobSDF(n=16)
    with torch.no_grad():
        ref_sdf.radii.add_(0.15)
    parts = [R.NeuralBSDFRef(), R.NeuralBSDFRef(), R.DiffuseRef()]
    ref_bsdf = R.SpatialMixBSDF(parts)
    loc = (0.4, 0.9, 0.8)
    ref = dict(shape=R.MarchedSDF(sdf=ref_sdf, max_steps=48), bsdf=ref_bsdf,
               lights=R.PointLightRef(location=loc, scale=5.0))
    sphere = SphereSDF(n=16, device="cpu")
    with torch.no_grad():
        sphere.centers.copy_(ref_sdf.centers)
        sphere.radii.copy_(ref_sdf.radii)
    copy_mlp(sphere.shift, ref_sdf.shift)
    comps = [NeuralBSDF(device="cpu"), NeuralBSDF(device="cpu"), Diffuse(device="cuda")]
    for c, r in zip(comps[:2], parts[:2]):
        copy_mlp(c.mlp, r.mlp)
        c.mlp.cuda()
    bsdf = ComposeSpatialVarying(comps, device="cpu")
    copy_mlp(bsdf.sp_var_fn, ref_bsdf.sp_var_fn)
    bsdf.sp_var_fn.cuda()
    mine = dict(shape=SDF(sdf=sphere.cuda(), max_steps=48), bsdf=bsdf,
                lights=PointLights(location=list(loc), scale=5.0, device="cuda"))
    return ref, mine


@pytest.mark.parametrize("prec,w_isect", [("fp32", False), ("fp32", True), ("fp16", True),
                                          ("fp32", "occ"), ("fp32-split", False),
                                          ("fp32-split", True), ("mixed", True)])
def test_path_integrator_matches_oracle(prec, w_isect):
    """Path (integrators.py:275-354), two bounces, with injected BSDF-sampling uniforms: the
    emitter term per bounce (optionally shadowed), ComposeSpatialVarying.sample, throughput
    update and the secondary intersection, vs the oracle's PathRef."""
    if w_isect == "occ":
        occ_ref, occ_mine = _occ_pair(1, seed=23)
        w_ref, w_mine = occ_ref, occ_mine
    else:
        w_ref = w_mine = w_isect
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Path
    ref, mine = _path_pair()
    c2w = recipes.look_at_c2w((0.1, 0.5, 0.9)).unsqueeze(0)
    ocam = R.NeRFCameraRef(c2w, recipes.nerf_focal(48))
    rays = ocam.sample_positions(R._tile_positions(0, 0, 48), 48)
    g = torch.Generator().manual_seed(9)
    lead = rays.shape[:-1]
    uniforms = [(torch.rand(*lead, 3, 2, generator=g), torch.rand(*lead, generator=g))
                for _ in range(2)]
    with torch.no_grad():
        want, wmask, _ = R.PathRef().sample(ref["shape"], rays, ref["bsdf"], ref["lights"],
                                            w_isect=w_ref, uniforms=uniforms)
    assert wmask.float().mean() > 0.2
    set_precision(prec)
    with torch.no_grad():
        got, mask, _ = Path().sample(mine["shape"], rays.cuda(), mine["bsdf"],
                                     lights=mine["lights"], w_isect=w_mine, uniforms=uniforms)
    got = got.cpu()
    assert torch.equal(mask.cpu(), wmask)
    assert got.shape == want.shape
    err = (got - want).abs().amax(-1)
    # Path's pixels past 1e-4: a secondary (bounce) ray's hit / step flip or a shadow-ray flip
    # changes that pixel's whole bounce contribution; reported with the count
    report(f"path_integrator[{prec},{w_isect}]", pixels=err.numel(), hits=int(wmask.sum()),
           over_1e4=int((err > 1e-4).sum()), over_1e2=int((err > 1e-2).sum()),
           maxabs=err.max().item())
    if prec != "fp16":  # fp32 and fp32-split: no bounce flips on this scene (reported 0)
        assert int((err > 1e-4).sum()) == 0, err.max()
    else:  # measured 1.7e-4 max, 46 of 2304 pixels > 1e-4
        assert err.max().item() <= 1e-3, err.max()
        assert int((err > 1e-4).sum()) <= 0.05 * err.numel()


@pytest.mark.parametrize("prec,w_isect", [("fp32", True), ("fp32", False), ("mixed", True)])
def test_path_batched_tiles_and_compaction_bit_equal(prec, w_isect):
    """Path on pathtrace's batched tiles (main._path_tiles): four 24^2 tiles concatenated into
    one Path.sample -- one primary march, one bounce kernel and one compacted secondary march per
    bounce -- equal the four tiles sampled one at a time, and the compacted secondary march
    (Path.compact, the live spawned rays only) equals marching every spawned ray, bit for bit,
    with the same injected uniforms (integrators.py:309-350)."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Path
    _, mine = _path_pair()
    c2w = recipes.look_at_c2w((0.1, 0.5, 0.9)).unsqueeze(0)
    ocam = R.NeRFCameraRef(c2w, recipes.nerf_focal(48))
    tiles = [ocam.sample_positions(R._tile_positions(x0, y0, 24), 48)
             for x0 in (0, 24) for y0 in (0, 24)]
    g = torch.Generator().manual_seed(17)
    lead = tiles[0].shape[:-1]
    unif = [[(torch.rand(*lead, 3, 2, generator=g), torch.rand(*lead, generator=g))
             for _ in range(2)] for _ in tiles]
    set_precision(prec)
    try:
        with torch.no_grad():
            per_tile = [Path().sample(mine["shape"], t.cuda(), mine["bsdf"], lights=mine["lights"],
                                      w_isect=w_isect, uniforms=u) for t, u in zip(tiles, unif)]
            cat_u = [tuple(torch.cat([u[d][i] for u in unif], 0) for i in range(2))
                     for d in range(2)]
            batched, bmask, _ = Path().sample(mine["shape"], torch.cat(tiles, 0).cuda(),
                                              mine["bsdf"], lights=mine["lights"],
                                              w_isect=w_isect, uniforms=cat_u)
            full = Path()
            full.compact = False
            uncompacted, umask, _ = full.sample(mine["shape"], torch.cat(tiles, 0).cuda(),
                                                mine["bsdf"], lights=mine["lights"],
                                                w_isect=w_isect, uniforms=cat_u)
    finally:
        set_precision("fp32")
    assert torch.equal(torch.cat([v for v, _, _ in per_tile], 0), batched)
    assert torch.equal(torch.cat([m for _, m, _ in per_tile], 0), bmask)
    assert torch.equal(batched, uncompacted) and torch.equal(bmask, umask)
    assert float(bmask.float().mean()) > 0.2 and float(batched.abs().max()) > 0


def test_pathtrace_path_batches_its_tiles(monkeypatch):
    """pathtrace(integrator=Path(), w_isect=True) (path_nerv.py:86-99) calls Path.sample once for
    all its tiles and composites each tile from its slice; with BATCH_PATH off it calls it per
    tile.  Both frames have the same hit mask (the primary march) and background."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer import main
    from neural_raytracing_amd.pathtracer.integrators import Path
    import neural_raytracing_amd.pathtracer as pt
    _, mine = _path_pair()
    set_precision("fp32")
    calls = []
    orig = Path.sample

    def spy(self, shapes, rays, bsdf, **kw):
        calls.append(tuple(rays.shape))
        return orig(self, shapes, rays, bsdf, **kw)
    monkeypatch.setattr(Path, "sample", spy)
    cam = pt.cameras.NeRFCamera(cam_to_world=recipes.look_at_c2w((0.1, 0.5, 0.9)).unsqueeze(0).cuda(),
                                focal=recipes.nerf_focal(48), device="cuda")
    frames = []
    for batch in (True, False):
        monkeypatch.setattr(main, "BATCH_PATH", batch)
        calls.clear()
        torch.manual_seed(0)
        random.seed(0)
        with torch.no_grad():
            img, _ = pt.pathtrace(mine["shape"], mine["lights"], cam, Path(), bsdf=mine["bsdf"],
                                  size=48, chunk_size=24, bundle_size=1, background=0,
                                  device="cuda", w_isect=True)
        frames.append((img.cpu(), list(calls)))
    (fb, cb), (ft, ct) = frames
    assert cb == [(4, 24, 24, 1, 6)] and ct == [(1, 24, 24, 1, 6)] * 4
    assert torch.equal(fb.abs().sum(-1) > 0, ft.abs().sum(-1) > 0)  # the same lit pixels
    assert float((fb.abs().sum(-1) > 0).float().mean()) > 0.2
