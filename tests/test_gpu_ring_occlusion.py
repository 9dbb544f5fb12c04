"""Shadow rays (SDF.intersect_test, sdfs.py:162-181) on the ring engines: k_occl16 / k_occl32 /
k_occl3 (march_body mode 3) against the per-wave k_occlusion (option ring_occlusion = 0) and the
oracle's MarchedSDF.intersect_test, on the headline scene's SDF (SphereSDF prior + 8x256 shift)
and the colocate SDF (64 spheres + 8x128 shift).  Rays leave points on the surface towards
random light positions, so visibility changes across the set; each ray's own distance to the
light is its max_t; ragged counts; the ring march's stop at t >= max_t (the visibility is decided
there) must not change any answer."""
import math

import pytest
import torch
import torch.nn.functional as F

import bench
from tests.helpers import lib_opt
from tests.report import report

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


def _scene(name):
    if name == "nerf_synthetic":
        sc = bench.build_scene("cuda", 64, seed=0)
        return sc["shape"], bench.oracle_scene(sc)["shape"]
    sc = bench.build_other_scene("colocate", torch.device("cuda"), 64)
    return sc["shape"], None


def _shadow_rays(shape, n, seed):
    """Points on the surface (FP32 march of camera-like rays), directions to random lights."""
    from neural_raytracing_amd import set_precision
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.0, 0.3, 1.2]).expand(n, 3) + 0.05 * torch.randn(n, 3, generator=g)
    tgt = 0.4 * (torch.rand(n, 3, generator=g) * 2 - 1)
    d = F.normalize(tgt - o, dim=-1)
    rays = torch.cat([o, d], -1).cuda()
    set_precision("fp32")
    with torch.no_grad():
        it, hit = shape.intersect(rays, primary=False)
    p = it.p[hit]
    m = p.shape[0]
    lights = 2.0 * F.normalize(torch.randn(m, 3, generator=g), dim=-1).cuda()
    dirv = lights - p
    dist = dirv.norm(dim=-1, keepdim=True)
    return torch.cat([p, dirv / dist], -1).contiguous(), dist.squeeze(-1).contiguous()


def _visible(shape, rays, dist, prec, ring):
    from neural_raytracing_amd import set_precision, _lib
    set_precision(prec)
    lib_opt("ring_occlusion", 1 if ring else 0)
    _lib.profile_reset()
    _lib.profile_enable(True)
    with torch.no_grad():
        v = shape.intersect_test(rays, max_t=dist[:, None])  # [..., 1], as scene.py passes it
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    set_precision("fp32")
    return v.cpu()


@pytest.mark.parametrize("name", ["nerf_synthetic", "colocate"])
@pytest.mark.parametrize("prec", ["fp32", "fp32-split", "mixed", "fp16"])
def test_ring_shadow_march_matches_per_wave_kernel(name, prec):
    shape, _ = _scene(name)
    rays, dist = _shadow_rays(shape, 3001, 7)
    assert rays.shape[0] > 200
    ring = _visible(shape, rays, dist, prec, True)
    from neural_raytracing_amd import _lib
    kern = {"fp32": "k_occl32", "fp16": "k_occl16"}.get(prec, "k_occl3")
    # (the profile counts the k_occlusion scope around every occlusion launch)
    assert _lib.profile_read("k_occlusion")[1] >= 1
    slab = _visible(shape, rays, dist, "fp16" if prec == "fp16" else "fp32", False)
    diff = int((ring != slab).sum())
    report(f"ring_shadow_vs_slab[{name},{prec}]", rays=ring.numel(), visible=int(ring.sum()),
           differ=diff, kernel=kern)
    assert 0.05 < ring.float().mean() < 0.95
    # FP32-accurate engines: the summation order only (a ray grazing eps); FP16 against FP16
    assert diff <= max(2, (0.02 if prec == "fp16" else 0.005) * ring.numel())


@pytest.mark.parametrize("n", [1, 77, 1000])
def test_ring_shadow_march_matches_oracle(n):
    shape, oshape = _scene("nerf_synthetic")
    rays, dist = _shadow_rays(shape, max(n, 400) * 2, 11)
    rays, dist = rays[:n], dist[:n]
    ring = _visible(shape, rays, dist, "fp32", True)
    with torch.no_grad():
        want = oshape.intersect_test(rays.cpu(), max_t=dist.cpu()[:, None])
    diff = int((ring != want).sum())
    report(f"ring_shadow_vs_oracle[{n}]", rays=n, visible=int(want.sum()), differ=diff)
    assert diff <= max(1, 0.005 * n)


def test_ring_shadow_march_empty_and_far_light():
    """No rays; and a light far past max_steps of marching: visible only if no hit."""
    shape, _ = _scene("nerf_synthetic")
    empty = torch.zeros(0, 6, device="cuda")
    assert shape.intersect_test(empty, max_t=torch.zeros(0, 1, device="cuda")).numel() == 0
    rays, dist = _shadow_rays(shape, 800, 13)
    far = torch.full_like(dist, 1e6)
    ring = _visible(shape, rays, far, "fp32", True)
    slab = _visible(shape, rays, far, "fp32", False)
    assert int((ring != slab).sum()) <= max(1, 0.005 * ring.numel())
    assert math.isfinite(float(dist.max()))


@pytest.mark.parametrize("prec", ["fp32", "mixed"])
@pytest.mark.parametrize("mode", ["direct", "nerf", "occ"])
def test_fused_shadowed_tiles_match_integrator_path(prec, mode):
    """pathtrace(..., w_isect=True | <occlusion MLP>) now renders on the fused tile path (every
    tile of a batch in one intersect + shadowed-shading chain, render.direct_kernels); it must
    equal the per-tile integrator path (forced by an `addition` hook, main.py _fused) pixel for
    pixel: same rays, same scan draws, same kernels per ray."""
    import random
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from tests.test_gpu_parity import _occ_pair, _shadow_scene
    _, mine = _shadow_scene()
    w = _occ_pair(1)[1] if mode == "occ" else True
    integ = NeRFIntegrator(Direct()) if mode == "nerf" else Direct()
    set_precision(prec)
    outs = []
    for hook in (None, lambda it: None):
        random.seed(21)
        kw = {} if hook is None else {"addition": hook}
        with torch.no_grad():
            img, _ = pt.pathtrace(mine["shape"], mine["lights"], mine["camera"], integ,
                                  bsdf=mine["bsdf"], size=64, chunk_size=32, bundle_size=1,
                                  background=0.5, with_noise=0.0, w_isect=w, **kw)
        outs.append(img.cpu())
    set_precision("fp32")
    fused, plain = outs
    err = (fused - plain).abs().max().item()
    report(f"fused_shadowed_tiles[{prec},{mode}]", pixels=fused[..., 0].numel(), maxabs=err)
    assert fused.shape == plain.shape
    assert err <= 1e-6, err


@pytest.mark.gpu
def test_pathtrace_trainable_occlusion_mlp_keeps_its_gradients():
    """pathtrace under autograd with a trainable learned-occlusion MLP (w_isect = SkipConnMLP,
    scene.py:313-318) must not take the gradient-free fused tile path: the occlusion weights get
    the gradients of the per-tile integrator path (forced by an `addition` hook)."""
    import random
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from tests.test_gpu_parity import _occ_pair, _shadow_scene
    _, mine = _shadow_scene()
    for key in ("shape", "bsdf", "lights"):  # only the occlusion MLP trains
        for q in getattr(mine[key], "parameters", lambda: [])():
            q.requires_grad_(False)
    occ = _occ_pair(1)[1]
    for q in occ.parameters():
        q.requires_grad_(True)
    grads = []
    for hook in (None, lambda it: None):
        random.seed(21)
        kw = {} if hook is None else {"addition": hook}
        occ.zero_grad()
        img, _ = pt.pathtrace(mine["shape"], mine["lights"], mine["camera"], Direct(),
                              bsdf=mine["bsdf"], size=32, chunk_size=32, bundle_size=1,
                              background=0.5, with_noise=0.0, w_isect=occ, **kw)
        img.sum().backward()
        grads.append([q.grad.detach().clone() for q in occ.parameters()])
    for a, b in zip(*grads):
        assert a is not None and torch.isfinite(a).all()
        assert torch.equal(a, b)
    assert any(float(g.abs().max()) > 0 for g in grads[0])
