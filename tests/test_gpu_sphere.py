"""The analytic Sphere shape (shapes/shapes.py:31-97, HIP nrt_sphere_intersect) and the renderer's
PointLights as a pathtracer light (renderer/lighting.py:221-304), against the oracle
restatements SphereRef / RendererPointLightRef -- and utils.sphere_examples (utils.py:409-431),
which renders every BSDF basis on them (VERDICT r3 "What's missing" 1)."""
import math
import random

import pytest
import torch
import torch.nn.functional as F

from oracle import pathtracer_ref as R
from tests.helpers import copy_mlp, seeded
from tests.report import report

pytestmark = pytest.mark.gpu


def _rays(n, seed):
    """Rays from outside (hits, misses, grazing), from inside the sphere, and pointing away."""
    g = torch.Generator().manual_seed(seed)
    o = torch.randn(n, 3, generator=g)
    o = o / o.norm(dim=-1, keepdim=True) * (1.0 + 2.5 * torch.rand(n, 1, generator=g))
    o[: n // 8] *= 0.3  # inside
    tgt = 1.3 * (torch.rand(n, 3, generator=g) * 2 - 1)
    d = F.normalize(tgt - o, dim=-1) * (0.5 + torch.rand(n, 1, generator=g))  # not unit length
    d[n // 8: n // 4] = -d[n // 8: n // 4]  # some pointing away
    return torch.cat([o + torch.tensor([0.1, -0.2, 0.05]), d], dim=-1)


@pytest.mark.parametrize("n", [1, 77, 5000])
def test_sphere_intersect_matches_oracle(n):
    from neural_raytracing_amd.pathtracer.shapes import Sphere
    center, radius = (0.1, -0.2, 0.05), 0.9
    ref = R.SphereRef(center, radius)
    mine = Sphere(list(center), radius, device="cuda")
    rays = _rays(n, n).reshape(1, n, 1, 1, 6)
    want, wmask = ref.intersect(rays)
    got, mask = mine.intersect(rays.cuda())
    mask = mask.cpu()
    assert torch.equal(mask, wmask)
    if n > 10:
        assert 0.1 < wmask.float().mean() < 0.9
    h = wmask
    for name, a, b in (("t", got.t.cpu(), want.t), ("p", got.p.cpu(), want.p),
                       ("n", got.n.cpu(), want.n), ("wi", got.wi.cpu(), want.wi)):
        err = (a[h] - b[h]).abs().max().item() if h.any() else 0.0
        report(f"sphere_intersect[{n}].{name}", rays=n, hits=int(h.sum()), maxabs=err)
        assert err <= 1e-6, (name, err)
    # misses keep the reference's t (from the unsquared discriminant) where it is finite
    miss_t, want_t = got.t.cpu()[~h], want.t[~h]
    fin = torch.isfinite(want_t)
    assert torch.equal(torch.isfinite(miss_t), fin)
    assert (miss_t[fin] - want_t[fin]).abs().max().item() <= 1e-5 if fin.any() else True
    assert torch.equal(mine.intersect_test(rays.cuda()).cpu(), ref.intersect_test(rays))
    lo, hi, m2 = mine.intersect_limits(rays.cuda())
    wlo, whi, wm2 = ref.intersect_limits(rays)
    assert torch.equal(m2.cpu(), wm2)
    assert torch.allclose(lo.cpu()[wm2], wlo[wm2], atol=1e-6)
    assert torch.allclose(hi.cpu()[wm2], whi[wm2], atol=1e-6)
    # the compacted hit list is the hit mask
    idx, cnt, _ = got._nrt_hits
    listed = torch.zeros(n, dtype=torch.bool)
    listed[idx[: int(cnt.item())].long().cpu()] = True
    assert torch.equal(listed, wmask.reshape(-1))


def test_sphere_empty_batch():
    from neural_raytracing_amd.pathtracer.shapes import Sphere
    it, mask = Sphere([0, 0, 0], 1).intersect(torch.zeros(0, 6, device="cuda"))
    assert mask.numel() == 0 and it.p.shape == (0, 3)


def _bases(seed=5):
    """A NeuralBSDF, a Diffuse and a Conductor basis, oracle and product with equal numbers."""
    from neural_raytracing_amd.pathtracer.bsdf import (ComposeSpatialVarying, Conductor, Diffuse,
                                                        NeuralBSDF)
    seeded(seed)
    parts = [R.NeuralBSDFRef(activation="sigmoid"),
             R.DiffuseRef(reflectance=torch.rand(3).tolist(), preprocess="sigmoid"),
             R.ConductorRef(specular=torch.rand(3).tolist(), activation="sigmoid")]
    comps = [NeuralBSDF(activation=torch.sigmoid, device="cpu"),
             Diffuse(reflectance=parts[1].reflectance.tolist(), preprocess=torch.sigmoid,
                     device="cuda"),
             Conductor(specular=parts[2].specular.tolist(), activation=torch.sigmoid,
                       device="cuda")]
    copy_mlp(comps[0].mlp, parts[0].mlp)
    comps[0].mlp.cuda()
    bsdf = ComposeSpatialVarying(comps, device="cpu")
    bsdf.sp_var_fn.cuda()
    return parts, bsdf


def test_sphere_scene_renders_match_oracle():
    """utils.sphere_examples' scene -- unit Sphere, look_at_view_transform(dist=2, elev=0,
    azim=0), OpenGLPerspectiveCameras, renderer PointLights at (0, 1, 4) scale 100, Direct() --
    for each basis, pathtrace without camera jitter vs the oracle: the FP32 bar on every pixel."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.utils import _sphere_scene
    parts, bsdf = _bases()
    sphere, cameras, lights = _sphere_scene("cuda", 100)
    Rm, Tm = R.look_at_view_transform_ref(dist=2.0, elev=0.0, azim=0.0)
    ocam = R.FoVCameraRef(Rm, Tm, znear=1.0, zfar=100.0)
    olight = R.RendererPointLightRef(location=[[0.0, 1.0, 4.0]], scale=100)
    size = 64
    for k, (ref_basis, basis) in enumerate(zip(parts, bsdf.bsdfs)):
        with torch.no_grad():
            want = R.render(R.SphereRef(), olight, ocam, R.DirectRef(), ref_basis, size=size,
                            chunk_size=32, background=1.0)
            got, _ = pt.pathtrace(sphere, lights, cameras, Direct(), bsdf=basis, size=size,
                                  chunk_size=32, bundle_size=1, with_noise=0.0, silent=True)
        got = got.cpu()
        assert got.shape == want.shape == (size, size, 3)
        hit = (want != 1.0).any(-1)
        assert 0.2 < hit.float().mean() < 0.95
        lit = (want[hit] > 1e-3).any(-1).float().mean()
        err = (got - want).abs().amax(-1)
        report(f"sphere_scene_render[{type(ref_basis).__name__}]", pixels=err.numel(),
               hits=int(hit.sum()), lit=float(lit), maxabs=err.max().item(),
               over_1e4=int((err > 1e-4).sum()), peak=float(want.max()))
        # the Conductor lights only its highlight ((refl . wo) > 0.94, bsdfs.py:371)
        assert lit > (0.01 if isinstance(ref_basis, R.ConductorRef) else 0.3)
        assert int((err > 1e-4).sum()) == 0, (k, err.max().item())


def test_sphere_examples_runs_every_basis():
    """utils.sphere_examples itself (bundle 4, camera jitter 1e-3 as pathtrace's defaults):
    one image per basis, finite, lit, and within the jitter's effect of the jitter-free render."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.utils import _sphere_scene, sphere_examples
    _, bsdf = _bases(7)
    random.seed(0)
    torch.manual_seed(0)
    with torch.no_grad():
        outs = sphere_examples(bsdf, size=64, chunk_size=32)
    assert len(outs) == 3
    sphere, cameras, lights = _sphere_scene("cuda", 100)
    for img, basis in zip(outs, bsdf.bsdfs):
        assert img.shape == (64, 64, 3) and torch.isfinite(img).all()
        with torch.no_grad():
            ref, _ = pt.pathtrace(sphere, lights, cameras, Direct(), bsdf=basis, size=64,
                                  chunk_size=32, bundle_size=1, with_noise=0.0, silent=True)
        inner = (ref != 1.0).all(-1)
        # interior pixels move by the 1e-3 sub-pixel jitter only
        assert (img[inner] - ref[inner]).abs().mean().item() < 2e-2


def test_renderer_point_light_kat_and_training_path():
    """sample_direction of the renderer light (torch) equals the closed form; the training path
    (autograd through the BSDF) shades with it like the fused kernel."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.lights import RendererPointLights
    from neural_raytracing_amd.pathtracer.utils import _sphere_scene
    light = RendererPointLights(location=[[0.0, 1.0, 4.0]], scale=100, device="cuda")

    class It:
        p = torch.tensor([[0.0, 0.0, 1.0]], device="cuda")
    ds, le = light.sample_direction(It())
    dist = math.sqrt(10.0)
    assert torch.allclose(ds.d.cpu(), torch.tensor([[0.0, 1.0, 3.0]]) / (1e-7 + dist))
    assert torch.allclose(le.cpu(), torch.full((1, 3), 100 * 0.5 / (1e-7 + dist) ** 2))
    _, bsdf = _bases(9)
    basis = bsdf.bsdfs[0]
    sphere, cameras, _ = _sphere_scene("cuda", 100)
    with torch.no_grad():
        fused, _ = pt.pathtrace(sphere, light, cameras, Direct(), bsdf=basis, size=32,
                                chunk_size=32, bundle_size=1, with_noise=0.0, silent=True)
    trained, _ = pt.pathtrace(sphere, light, cameras, Direct(), bsdf=basis, size=32,
                              chunk_size=32, bundle_size=1, with_noise=0.0, silent=True)
    assert any(q.requires_grad for q in basis.parameters())
    assert (trained.detach() - fused).abs().max().item() <= 1e-5
