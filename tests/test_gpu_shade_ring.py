"""FP32 / fp32-split shading on the row-program ring kernels (nrt_shade_ring.h: k_light32 /
k_bsdf32, k_light3 / k_bsdf3) -- Direct.sample's emitter + spatially varying BSDF evaluation
(integrators.py:173-189) with the reference's shading MLPs (LightField 10x256 F=16, spatial
weights 16x256 F=128, NeuralBSDF 6x96 F=64).

* the C-ABI entry nrt_shade_direct on synthetic hit lists (ragged counts, the hit list in any
  order, shadow-scaled and component-weight outputs) against the per-wave FP32 kernel
  k_shade_direct (option shade_ring = 0): both are exact-f32 MFMA products with f32 accumulation
  in different orders, so they agree to f32 rounding (1e-5 abs on RGB values up to ~1); the split
  path is held to the same bar;
* the bench scene's pathtrace_sample crop against the oracle at the FP32 bar (1e-4 abs per
  channel on agreeing pixels) with the ring kernels verified to run;
* other component mixes (Diffuse / Conductor beside NeuralBSDFs, no spatial MLP, a point light)
  against the per-wave kernel.
"""
import math
import random

import pytest
import torch

import bench
from tests.helpers import lib_opt as _lib_opt
from tests.report import report

pytestmark = pytest.mark.gpu

KERNELS = {"fp32": ("k_light32", "k_bsdf32"), "fp32-split": ("k_light3", "k_bsdf3")}


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


def _hits(P, n_hit, seed):
    """P ray slots, n_hit of them hit (random order in the list); points in the unit ball,
    normals / wi unit vectors."""
    g = torch.Generator().manual_seed(seed)
    p = (torch.rand(P, 3, generator=g) * 2 - 1) * 0.5
    n = torch.nn.functional.normalize(torch.randn(P, 3, generator=g), dim=-1)
    wi = torch.nn.functional.normalize(torch.randn(P, 3, generator=g), dim=-1)
    idx = torch.randperm(P, generator=g)[:n_hit].to(torch.int32)
    full = torch.zeros(P, dtype=torch.int32)
    full[:n_hit] = idx
    return p.cuda(), n.cuda(), wi.cuda(), full.cuda(), torch.tensor([n_hit], dtype=torch.int32).cuda()


def _shade(bsdf, lights, p, n, wi, idx, cnt, prec, ring, nc):
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.integrators.integrators import _bsdf_handle, _light_handle
    set_precision(prec)
    _lib_opt("shade_ring", 1 if ring else 0)
    P = p.shape[0]
    rgb = torch.zeros(P, 3, device="cuda")
    wout = torch.zeros(P, nc, device="cuda")
    _lib.profile_enable(True)
    _lib.profile_reset()
    _lib.call("nrt_shade_direct", _bsdf_handle(bsdf), _light_handle(lights), _lib.ptr(p),
              _lib.ptr(n), _lib.ptr(wi), _lib.ptr(idx), _lib.ptr(cnt), P, _lib.ptr(rgb),
              _lib.ptr(wout), _lib.precision_code(), _lib.stream())
    torch.cuda.synchronize()
    counts = {k: _lib.profile_read(k)[1] for ks in KERNELS.values() for k in ks}
    _lib.profile_enable(False)
    _lib_opt("shade_ring", 1)
    set_precision("fp32")
    return rgb.cpu(), wout.cpu(), counts


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
@pytest.mark.parametrize("P,n_hit", [(1, 1), (300, 17), (5000, 3001), (70000, 65000)])
def test_ring_shading_matches_per_wave_kernel(prec, P, n_hit):
    scene = bench.build_scene("cuda", samples=16, seed=3, light_gain=10.0)
    p, n, wi, idx, cnt = _hits(P, n_hit, seed=P)
    nc = len(scene["bsdf"].bsdfs)
    want, wwant, _ = _shade(scene["bsdf"], scene["lights"], p, n, wi, idx, cnt, "fp32", False, nc)
    got, wgot, counts = _shade(scene["bsdf"], scene["lights"], p, n, wi, idx, cnt, prec, True, nc)
    kl, kb = KERNELS[prec]
    assert counts[kl] >= 1 and counts[kb] >= 1, counts
    hit = idx[:n_hit].long().cpu()
    d = (got[hit] - want[hit]).abs()
    dw = (wgot[hit] - wwant[hit]).abs()
    report(f"ring_shading_vs_per_wave[{prec}-{P}-{n_hit}]", rays=n_hit,
           rgb_maxabs=float(d.max()), weights_maxabs=float(dw.max()),
           rgb_peak=float(want[hit].abs().max()))
    assert d.max() < 1e-5, d.max()
    assert dw.max() < 1e-5, dw.max()
    # rays off the hit list are left alone
    miss = torch.ones(P, dtype=torch.bool)
    miss[hit] = False
    assert got[miss].abs().max() == 0 if miss.any() else True


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
def test_ring_shading_render_matches_oracle(prec):
    """The bench scene (light gain 10, RGB spanning most of [0, 1]) through pathtrace_sample on a
    64^2 crop across the silhouette, against the oracle: 1e-4 abs on pixels whose hit agrees."""
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    from oracle import pathtracer_ref as R
    scene = bench.build_scene("cuda", samples=32, seed=0, light_gain=10.0)
    pt = scene["pt"]
    size, crop = 200, 64
    c0 = 40
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    nra.set_precision(prec)
    _lib.profile_enable(True)
    _lib.profile_reset()
    random.seed(7)
    with torch.no_grad():
        img, _ = pt.pathtrace_sample(scene["shape"], scene["lights"], cam, scene["integrator"],
                                     bsdf=scene["bsdf"], size=size, chunk_size=size, bundle_size=1,
                                     crop_size=crop, uv=(c0, c0), background=0, with_noise=0.0)
    img = img.cpu()
    kl, kb = KERNELS[prec]
    assert _lib.profile_read(kb)[1] >= 1 and _lib.profile_read(kl)[1] >= 1
    _lib.profile_enable(False)
    nra.set_precision("fp32")
    osc = bench.oracle_scene(scene)
    random.seed(7)
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], R.NeRFCameraRef(c2w, focal), osc["integrator"],
                        osc["bsdf"], size=size, chunk_size=size, background=0.0, with_noise=0.0,
                        crop=(c0, c0, crop))
    a_got, a_want = img[..., 3], want[..., 3]
    hit_got, hit_want = a_got > 0.5, a_want > 0.5
    agree = hit_got == hit_want
    d = (img - want).abs().amax(-1)
    report(f"ring_shading_render_vs_oracle[{prec}]", pixels=int(d.numel()),
           hits=int(hit_want.sum()), flips=int((~agree).sum()),
           maxabs_agreeing=float(d[agree].max()), rgb_peak=float(want[..., :3].max()),
           pixels_over_1e4=int((d[agree] > 1e-4).sum()))
    assert want[..., :3].max() > 0.3  # a bright frame, not a dark crop
    assert (~agree).float().mean() <= 0.005
    assert (d[agree] > 1e-4).float().mean() <= 0.005, int((d[agree] > 1e-4).sum())


def _mixed_bsdf(kind, seed):
    """Component mixes the ring kernels must reproduce: NeuralBSDFs beside Diffuse / Conductor
    (colocate.py's family), with or without the spatial-weight MLP."""
    from neural_raytracing_amd.pathtracer.bsdf import (ComposeSpatialVarying, Conductor, Diffuse,
                                                        NeuralBSDF)
    torch.manual_seed(seed)
    comps = [NeuralBSDF(activation=torch.nn.Softplus(), device="cpu"), Diffuse(device="cpu"),
             NeuralBSDF(device="cpu"), Conductor(device="cpu")]
    if kind == "single":
        b = comps[0]
        b.mlp.to("cuda")
        return b, 1
    bsdf = ComposeSpatialVarying(comps, device="cpu")
    for c in bsdf.bsdfs:
        if getattr(c, "mlp", None) is not None:
            c.mlp.to("cuda")
    bsdf.sp_var_fn.to("cuda")
    return bsdf, len(comps)


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
@pytest.mark.parametrize("kind", ["mixed", "single"])
@pytest.mark.parametrize("light", ["field", "point"])
def test_ring_shading_component_mixes(prec, kind, light):
    from neural_raytracing_amd.pathtracer.lights import LightField, PointLights
    bsdf, nc = _mixed_bsdf(kind, seed=5)
    torch.manual_seed(6)
    if light == "field":
        lights = LightField(device="cpu").to("cuda")
    else:
        lights = PointLights(location=[[0.3, 1.5, 1.0]], device="cuda")
    p, n, wi, idx, cnt = _hits(4000, 2500, seed=11)
    want, wwant, _ = _shade(bsdf, lights, p, n, wi, idx, cnt, "fp32", False, nc)
    got, wgot, counts = _shade(bsdf, lights, p, n, wi, idx, cnt, prec, True, nc)
    kl, kb = KERNELS[prec]
    assert counts[kb] >= 1, counts
    if light == "field":
        assert counts[kl] >= 1, counts
    hit = idx[:2500].long().cpu()
    # relative to the ray's magnitude: a point light (scale 1e2 over a quadratic falloff) puts
    # RGB far above 1
    mag = want[hit].abs().amax(-1).clamp_min(1.0)
    d = (got[hit] - want[hit]).abs().amax(-1) / mag
    # Conductor's specular test (r . wo > 0.94, bsdfs.py:384-386) is a step: a ray whose light
    # direction sits within rounding of the threshold flips between 0 and the full value
    over = d > 1e-5
    report(f"ring_shading_mix[{prec}-{kind}-{light}]", rays=2500, rgb_relmax=float(d.max()),
           rgb_relmax_agreeing=float(d[~over].max()), rays_over_1e5=int(over.sum()),
           rgb_peak=float(want[hit].abs().max()))
    assert int(over.sum()) <= 5, int(over.sum())
