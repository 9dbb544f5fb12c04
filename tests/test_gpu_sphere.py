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


def _cloud_rays(n, seed, lead=1):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor([0.0, 0.1, 2.5]) + 0.3 * torch.randn(lead, n, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(lead, n, 1, 2, generator=g) * 1.2 - 0.6,
                               -torch.ones(lead, n, 1, 1)], -1), dim=-1)
    return torch.cat([o, d], -1)


@pytest.mark.parametrize("t_max", [math.inf, 2.3])
@pytest.mark.parametrize("n", [1, 300, 4000])
def test_sphere_cloud_one_sphere_matches_oracle(n, t_max):
    """SphereCloud (shapes.py:99-206) where the reference's broadcasting is well-formed: one
    sphere, rays [1, n, 1, 6] for intersect and [3, n, 1, 6] for intersect_test; t, p, n, wi of
    the hits at the Sphere test's bar, the hit masks and the misses' t (t_max) equal."""
    from neural_raytracing_amd.pathtracer.shapes import SphereCloud
    centers, radius = [[0.05, 0.1, 0.2]], 0.6
    ref = R.SphereCloudRef(centers=centers, radii=radius)
    mine = SphereCloud(centers=centers, radii=radius, device="cuda")
    rays = _cloud_rays(n, n)
    want, wmask = ref.intersect(rays, t_max=t_max)
    got, mask = mine.intersect(rays.cuda(), t_max=t_max)
    assert torch.equal(mask.cpu(), wmask)
    if n > 10:
        assert 0.1 < wmask.float().mean() < 0.9
    h = wmask
    for name, a, b in (("t", got.t.cpu(), want.t), ("p", got.p.cpu(), want.p),
                       ("n", got.n.cpu(), want.n), ("wi", got.wi.cpu(), want.wi)):
        err = (a[h] - b[h]).abs().max().item() if h.any() else 0.0
        report(f"sphere_cloud[{n},{t_max}].{name}", rays=n, hits=int(h.sum()), maxabs=err)
        assert err <= 1e-6, (name, err)
    assert torch.equal(got.t.cpu()[~h], want.t[~h])
    assert torch.equal(got.n.cpu()[~h], want.n[~h])
    rays3 = _cloud_rays(n, n + 1, lead=3)
    assert torch.equal(mine.intersect_test(rays3.cuda(), t_max=t_max).cpu(),
                       ref.intersect_test(rays3, t_max=t_max))
    idx, cnt, _ = got._nrt_hits
    listed = torch.zeros(n, dtype=torch.bool)
    listed[idx[: int(cnt.item())].long().cpu()] = True
    assert torch.equal(listed, wmask.reshape(-1))


def _cloud_restated(centers, radii, rays, t_max, split_n):
    """SphereCloud.intersect's per-ray statements (shapes.py:111-179) for N spheres, sphere by
    sphere on the CPU in float32 (the reference's own broadcasting is well-formed for N = 1 only):
    per chunk the first minimum's index within the chunk names the normal's centre."""
    r_o, r_d = torch.split(rays, 3, dim=-1)
    lead = r_o.shape[:-1]
    out_active = torch.zeros(lead, dtype=torch.bool)
    best = torch.full(lead, t_max, dtype=torch.float)
    face = torch.full(lead, -1, dtype=torch.long)
    for j0 in range(0, centers.shape[0], split_n):
        ts = []
        for j in range(j0, min(j0 + split_n, centers.shape[0])):
            fs = r_o - centers[j]
            a = torch.sum(r_d * r_d, dim=-1)
            b = 2 * torch.sum(r_d * fs, dim=-1)
            c = torch.sum(fs * fs, dim=-1) - radii[j] * radii[j]
            inter, mask = R.quad_solve(a, b, c)
            mask = mask & ((inter >= R.SPHERE_EPS) & (inter < t_max)).any(-1)
            inter[inter < R.SPHERE_EPS] = math.inf
            t, _ = inter.min(dim=-1)
            t[~mask] = math.inf
            ts.append((t, mask))
        t = torch.stack([q[0] for q in ts])
        valid = torch.stack([q[1] for q in ts]).any(0)
        out_active |= valid
        min_t, idx = t.min(dim=0)
        rep = valid & (best > min_t)
        best[rep] = min_t[rep]
        face[rep] = idx[rep]
    p = r_o + best[..., None] * r_d
    n = torch.zeros_like(p)
    n[out_active] = F.normalize(p[out_active] - centers[face[out_active]], dim=-1)
    return best, p + n * 1e-5, n, out_active


@pytest.mark.parametrize("split_n", [256, 7])
def test_sphere_cloud_many_spheres_matches_restatement(split_n):
    """37 spheres (the reference's broadcasting breaks past one sphere, so the per-ray statements
    are restated sphere by sphere): nearest hit, chunks of split_n (7: six chunks, the normal's
    centre named by the index within the chunk, as the reference keeps it), t_max = 3.1."""
    from neural_raytracing_amd.pathtracer.shapes import SphereCloud
    g = torch.Generator().manual_seed(11)
    centers = (torch.rand(37, 3, generator=g) * 2 - 1) * torch.tensor([1.0, 1.0, 0.5])
    mine = SphereCloud(centers=centers.tolist(), radii=0.18, device="cuda")
    rays = _cloud_rays(3000, 4)
    radii = torch.full([37], 0.18)
    t_max = 3.1
    wt, wp, wn, wmask = _cloud_restated(centers, radii, rays, t_max, split_n)
    got, mask = mine.intersect(rays.cuda(), t_max=t_max, split_n=split_n)
    assert torch.equal(mask.cpu(), wmask)
    assert 0.05 < wmask.float().mean() < 0.95
    h = wmask
    # n = normalize(p - c) scales p's last-bit differences by 1 / r = 5.6 (radius 0.18): 4e-6
    for name, a, b, tol in (("t", got.t.cpu(), wt, 1e-6), ("p", got.p.cpu(), wp, 1e-6),
                            ("n", got.n.cpu(), wn, 4e-6)):
        err = (a[h] - b[h]).abs().max().item()
        report(f"sphere_cloud_many[{split_n}].{name}", rays=3000, hits=int(h.sum()), maxabs=err)
        assert err <= tol, (name, err)
    assert torch.equal(got.t.cpu()[~h], wt[~h])
    assert torch.equal(mine.intersect_test(rays.cuda(), t_max=t_max, split_n=split_n).cpu(), wmask)


def test_sphere_cloud_empty_batch():
    from neural_raytracing_amd.pathtracer.shapes import SphereCloud
    it, mask = SphereCloud().intersect(torch.zeros(0, 6, device="cuda"))
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
