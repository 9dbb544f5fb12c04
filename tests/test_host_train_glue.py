"""CPU checks of the element-wise glue the training path differentiates through
(neural_raytracing_amd/pathtracer/differentiable.py) against the oracle's restatement:
values and autograd gradients agree to float32 rounding (atol 1e-6 on unit-scale inputs)."""
import torch

from oracle import pathtracer_ref as R
from tests.helpers import seeded


def test_coordinate_system_matches_oracle_frames():
    from neural_raytracing_amd.pathtracer import differentiable as D
    seeded(1)
    n = torch.randn(500, 3)
    n[0] = torch.tensor([0.0, 0.0, -1.0])  # the s_z clamp branch
    n[1] = torch.tensor([0.0, 0.0, 1.0])
    a = n.clone().requires_grad_(True)
    b = n.clone().requires_grad_(True)
    fa, fb = D.coordinate_system(a), R.shading_frame(b)
    assert torch.allclose(fa, fb, atol=1e-6)
    w = torch.randn_like(fa)
    (fa * w).sum().backward()
    (fb * w).sum().backward()
    assert torch.allclose(a.grad, b.grad, atol=1e-5, rtol=1e-5)


def test_param_rusin2_matches_oracle():
    from neural_raytracing_amd.pathtracer import differentiable as D
    seeded(2)
    wo = torch.nn.functional.normalize(torch.randn(400, 3), dim=-1)
    wi = torch.nn.functional.normalize(torch.randn(400, 3), dim=-1)
    wi[0] = wo[0] = torch.tensor([0.0, 0.0, 1.0])  # SURVEY §8c KAT 6
    a, b = wo.clone().requires_grad_(True), wo.clone().requires_grad_(True)
    ra, rb = D.param_rusin2(a, wi), R.rusinkiewicz(b, wi)
    assert torch.allclose(ra, rb, atol=1e-6)
    ra.sum().backward()
    rb.sum().backward()
    assert torch.allclose(a.grad, b.grad, atol=1e-4, rtol=1e-4)


def test_fresnel_and_reflect_match_oracle():
    from neural_raytracing_amd.pathtracer import differentiable as D
    c = torch.linspace(-1, 1, 101)
    assert torch.allclose(D.fresnel_conductor(c, 1.3, 0.0), R.fresnel_conductor(c, 1.3, 0.0),
                          atol=1e-7)


def test_sphere_part_and_gradient_match_oracle():
    """SphereSDF's smooth-min part: values, d/dp with create_graph, and the parameter gradients
    of an eikonal-style loss on that normal."""
    from neural_raytracing_amd.pathtracer import differentiable as D
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    seeded(3)
    ref = R.SphereBlobSDF(n=16)
    seeded(3)
    mine = SphereSDF(n=16, device="cpu")
    assert torch.equal(mine.centers, ref.centers)
    with torch.no_grad():
        for t in (ref.tfs, mine.tfs):
            t.copy_(0.05 * torch.sin(torch.arange(t.numel(), dtype=torch.float)).reshape(t.shape))
    p = torch.randn(64, 3) * 0.3
    assert torch.allclose(D.sphere_part(mine, p), ref.spheres(p), atol=1e-6)
    for m, fn in ((mine, lambda q: D.sphere_part(mine, q)), (ref, ref.spheres)):
        q = p.clone().requires_grad_(True)
        out = fn(q)
        (g,) = torch.autograd.grad(out, q, torch.ones_like(out), create_graph=True)
        (g.norm(dim=-1) - 1).square().mean().backward()
    for a, b in ((mine.centers, ref.centers), (mine.radii, ref.radii), (mine.tfs, ref.tfs)):
        assert torch.allclose(a.grad, b.grad, atol=1e-5, rtol=1e-4)


def test_needs_grad_follows_autograd_mode():
    from neural_raytracing_amd.pathtracer import differentiable as D
    from neural_raytracing_amd.pathtracer.shapes import SPHERE_SDF, SDF, SphereSDF
    s = SphereSDF(n=4, device="cpu")
    assert D.needs_grad(s)
    assert not D.needs_grad(SDF(sdf=SPHERE_SDF, device="cpu"))  # no parameters
    with torch.no_grad():
        assert not D.needs_grad(s)
    for q in s.parameters():
        q.requires_grad_(False)
    assert not D.needs_grad(s)


def _jit_float_scale(c, e: float):
    return c * e


def test_conductor_eta_gets_no_gradient_like_the_reference():
    """Conductor.eval_and_pdf passes F.softplus(self.eta) into fresnel_conductor, which the
    reference compiles with @torch.jit.script and annotates ``eta_r: float`` (bsdfs.py:327-328,
    :371): TorchScript converts the 0-d tensor to a Python float, so eta receives no gradient and
    AdamW never moves it.  The training path keeps that (differentiable.bsdf_eval detaches eta);
    specular still gets its gradient."""
    import inspect
    import torch
    import torch.nn.functional as F
    from neural_raytracing_amd.pathtracer.bsdf import Conductor
    from neural_raytracing_amd.pathtracer.differentiable import bsdf_eval

    # the TorchScript float conversion itself (what the reference's call does)
    f = torch.jit.script(_jit_float_scale)
    eta = torch.tensor(1.3, requires_grad=True)
    c = torch.rand(4, requires_grad=True)
    f(c, F.softplus(eta)).sum().backward()
    assert eta.grad is None and c.grad is not None

    cond = Conductor(specular=[0.5, 0.6, 0.7], device="cpu")

    class It:
        pass
    it = It()
    it.wi = F.normalize(torch.tensor([[0.1, 0.2, 0.9]]), dim=-1)
    it.p = torch.zeros(1, 3)
    wo = torch.cat([-it.wi[:, :2], it.wi[:, 2:]], -1)  # the mirror direction: above the 0.94 cut
    f_, _ = bsdf_eval(cond, it, wo, torch.ones(1, dtype=torch.bool))
    f_.sum().backward()
    assert cond.eta.grad is None
    assert cond.specular.grad is not None and cond.specular.grad.abs().sum() > 0
    assert inspect.signature(Conductor.__init__).parameters["eta"].default == 1.3


def test_point_light_per_camera_broadcast_matches_oracle():
    """PointLights with one location / intensity per camera (colocate.py:109): the training
    path's light sample broadcasts row n over camera n like lights.py:91, :106 (the oracle's
    PointLightRef.sample_direction); one row broadcasts to every camera."""
    from neural_raytracing_amd.pathtracer import differentiable as D
    from neural_raytracing_amd.pathtracer.lights import PointLights

    class It:
        pass
    torch.manual_seed(5)
    p = torch.randn(3, 4, 5, 1, 3)
    active = torch.rand(3, 4, 5, 1) > 0.3
    it = It()
    it.p = p
    locs = torch.randn(3, 3)
    inten = torch.rand(3, 3) + 0.1
    mine = PointLights(location=locs, intensity=inten, scale=5.0, device="cpu")
    assert mine.per_camera() == 3
    d, le, pdf, dist = D.light_sample(mine, it, active)
    ref = R.PointLightRef(location=locs.reshape(-1).tolist(), scale=5.0)
    ref.intensity = inten.clone()
    rs, rle = ref.sample_direction(it, active)
    assert torch.allclose(d, rs.d, atol=1e-6) and torch.allclose(dist, rs.dist, atol=1e-6)
    assert torch.allclose(le, rle, atol=1e-6)
    v = mine.camera(1)
    assert torch.equal(v.location, locs[1:2]) and torch.equal(v.intensity, inten[1:2])
    assert v.per_camera() is None
    one = PointLights(location=locs[:1].expand(3, 3).clone(), scale=5.0, device="cpu")
    assert one.per_camera() is None
