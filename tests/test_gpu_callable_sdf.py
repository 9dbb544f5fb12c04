"""SDF callables the library cannot pack: SDF(sdf=f) for any function f of the points -- the warp
and displacement lambdas of edit_dtu.py:86-100 around a trained SDF, a plain torch lambda.  The
callable runs between the HIP steps (nrt_march_callable_step / nrt_scan_callable_step /
nrt_occlusion_callable_step, nrt_callable.hip); the normals are autograd through the callable
(sdfs.py:184-197).

Against the oracle (MarchedSDF with the same callable around the oracle SDF, sdfs.py:111-181):
hit masks, t / p / normals on agreeing rays at the FP32 bar (1e-4 abs), throughput = -1000
sdf(best_pos) within 2e-3 (the x1000 logit of an f32 SDF), shadow visibility; flips reported.
Then the bench scene with its SDF bent, rendered through pathtrace_sample (NeRFIntegrator(Direct),
HIP shading on the callable's hit list) against the oracle's render, and Debug normals through
pathtrace as edit_dtu.py calls it."""
import math
import random

import pytest
import torch

import bench
from oracle import pathtracer_ref as R
from tests.report import report
from tests.test_gpu_ring32 import _blob, _rays

pytestmark = pytest.mark.gpu


def bend(shape, k=-3.0):
    """edit_dtu.py:85-95's warp (k = -10 there, on a DTU-scale object)."""
    def f(p):
        x, y, z = p.split(1, dim=-1)
        v = z * k
        c, s = v.cos(), v.sin()
        return shape(torch.cat([c * x - s * z, y, s * x + c * z], dim=-1))
    return f


def disp(shape):
    """edit_dtu.py:96-99's displacement add-on."""
    def f(p):
        x, y, z = p.split(1, dim=-1)
        out = shape(p)
        return out + 0.05 * ((20 * x).cos() * (20 * y).cos() * (20 * z).cos()).reshape_as(out)
    return f


def _pair(kind):
    ref, mine = _blob(128, 128, 32, "softplus")
    if kind == "bend":
        return bend(ref), bend(mine)
    if kind == "disp":
        return disp(ref), disp(mine)
    lam = lambda p: torch.norm(p - torch.tensor([0.05, 0.0, 0.0], device=p.device), dim=-1) - 0.3  # noqa: E731
    return lam, lam


@pytest.mark.parametrize("kind", ["bend", "disp", "lambda"])
def test_callable_intersect_matches_oracle(kind):
    from neural_raytracing_amd.pathtracer.shapes import SDF
    from neural_raytracing_amd import _lib
    f_ref, f_mine = _pair(kind)
    rays = _rays(40, 3, eye=(0.0, 0.2, 1.1))
    steps = 48
    random.seed(21)
    _lib.profile_enable(True)
    _lib.profile_reset()
    with torch.no_grad():
        it, hit = SDF(sdf=f_mine, max_steps=steps).intersect(rays.cuda())
    n_step, n_scan = (_lib.profile_read(k)[1] for k in ("k_march_step", "k_scan_step"))
    _lib.profile_enable(False)
    assert (n_step, n_scan) == (steps + 1, 129)
    random.seed(21)
    want, whit = R.MarchedSDF(sdf=f_ref, max_steps=steps).intersect(rays)
    hit, whit = hit.cpu().reshape(-1), whit.reshape(-1)
    agree = hit == whit
    flips = int((~agree).sum())
    both = (hit & whit)
    p, wp = it.p.cpu().reshape(-1, 3), want.p.reshape(-1, 3)
    n, wn = it.n.cpu().reshape(-1, 3), want.n.reshape(-1, 3)
    t, wt = it.t.cpu().reshape(-1), want.t.reshape(-1)
    thr, wthr = it.throughput.detach().cpu().reshape(-1), want.throughput.detach().reshape(-1)
    dp = (p[agree] - wp[agree]).abs().amax(-1)
    dn = (n[both] - wn[both]).abs().amax(-1)
    dt = (t[agree] - wt[agree]).abs()
    dthr = (thr - wthr).abs()
    report(f"callable_intersect[{kind}]", rays=hit.numel(), hits=int(whit.sum()), hit_flips=flips,
           p_maxabs=float(dp.max()), n_maxabs=float(dn.max()) if both.any() else 0.0,
           t_maxabs=float(dt.max()), rays_p_over_1e4=int((dp > 1e-4).sum()),
           thr_maxabs=float(dthr.max()), rays_thr_over_2e3=int((dthr > 2e-3).sum()),
           march_step_launches=n_step)
    assert int(whit.sum()) > 100 and int((~whit).sum()) > 100
    assert flips <= 0.005 * hit.numel()
    assert (dp > 1e-4).float().mean() <= 0.005 and (dt > 1e-4).float().mean() <= 0.005
    assert (dn > 1e-4).float().mean() <= 0.005
    assert (dthr > 2e-3).float().mean() <= 0.005
    # raw normals of the hit rays (sdfs.py:154: setattr(si, "raw_normals", ...))
    raw = it.raw_normals
    assert raw is not None and raw.shape == (int(hit.sum()), 3)


@pytest.mark.parametrize("kind", ["bend", "disp"])
def test_callable_intersect_test_matches_oracle(kind):
    from neural_raytracing_amd.pathtracer.shapes import SDF
    f_ref, f_mine = _pair(kind)
    rays = _rays(40, 4, eye=(0.0, 0.2, 1.1))
    g = torch.Generator().manual_seed(9)
    max_t = 0.6 + 1.2 * torch.rand(rays.shape[:-1] + (1,), generator=g)
    with torch.no_grad():
        vis = SDF(sdf=f_mine, max_steps=32).intersect_test(rays.cuda(), max_t=max_t.cuda()).cpu()
    want = R.MarchedSDF(sdf=f_ref, max_steps=32).intersect_test(rays, max_t=max_t)
    diff = int((vis != want).sum())
    report(f"callable_occlusion[{kind}]", rays=vis.numel(), visible=int(want.sum()), flips=diff)
    assert 0 < int(want.sum()) < want.numel()
    assert diff <= 0.005 * vis.numel()


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
def test_callable_render_matches_oracle(prec):
    """The bench scene with its SDF bent (edit_dtu.py's warp) through pathtrace_sample:
    NeRFIntegrator(Direct) shading on the HIP kernels over the callable march's hit list
    (fp32-split: the shading row programs k_light3 / k_bsdf3)."""
    import neural_raytracing_amd as nra
    nra.set_precision(prec)
    try:
        _callable_render(prec)
    finally:
        nra.set_precision("fp32")


def _callable_render(prec):
    scene = bench.build_scene("cuda", samples=32, seed=0, light_gain=10.0)
    osc = bench.oracle_scene(scene)
    pt = scene["pt"]
    scene["shape"].sdf = bend(scene["shape"].sdf, k=-4.0)
    osc["shape"].sdf = bend(osc["shape"].sdf, k=-4.0)
    size, crop, c0 = 200, 64, 40
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    random.seed(7)
    with torch.no_grad():
        img, _ = pt.pathtrace_sample(scene["shape"], scene["lights"], cam, scene["integrator"],
                                     bsdf=scene["bsdf"], size=size, chunk_size=size, bundle_size=1,
                                     crop_size=crop, uv=(c0, c0), background=0, with_noise=0.0)
    img = img.cpu()
    random.seed(7)
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], R.NeRFCameraRef(c2w, focal), osc["integrator"],
                        osc["bsdf"], size=size, chunk_size=size, background=0.0, with_noise=0.0,
                        crop=(c0, c0, crop))
    hit_got, hit_want = img[..., 3] > 0.5, want[..., 3] > 0.5
    agree = hit_got == hit_want
    d = (img - want).abs().amax(-1)
    report(f"callable_render_vs_oracle[bend,{prec}]", pixels=int(d.numel()),
           hits=int(hit_want.sum()), flips=int((~agree).sum()),
           maxabs_agreeing=float(d[agree].max()), rgb_peak=float(want[..., :3].max()),
           pixels_over_1e4=int((d[agree] > 1e-4).sum()))
    assert int(hit_want.sum()) > 200
    assert (~agree).float().mean() <= 0.005
    assert int((d[agree] > 1e-4).sum()) == 0, float(d[agree].max())


def test_callable_debug_pathtrace():
    """pathtrace with Debug (edit_dtu.py's integrator): (n + 1) / 2 on hits, through the callable
    march tile by tile (the fused kernels decline an SDF callable)."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Debug
    from neural_raytracing_amd.pathtracer.shapes import SDF
    f_ref, f_mine = _pair("bend")
    size = 32
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    shape = SDF(sdf=f_mine, max_steps=48)
    with torch.no_grad():
        img, _ = pt.pathtrace(shape, None, cam, Debug(), size=size, chunk_size=16, bundle_size=1,
                              background=0, with_noise=0.0)
    img = img.cpu()
    # the same normals from SDF.intersect over the whole frame's rays
    rays = cam.rays_tile(0, 0, size, size, size, 0.0)
    with torch.no_grad():
        it, hit = shape.intersect(rays)
    want = torch.where(hit.unsqueeze(-1), (it.n + 1) / 2, torch.tensor(0.0, device=hit.device))
    want = want.mean(dim=-2).cpu().reshape(img.shape)
    assert int(hit.sum()) > 20
    assert (img - want).abs().max() < 1e-5


def test_callable_shadow_rays_match_oracle():
    """Direct with w_isect=True over a bent shape (sample_emitter_dir_w_isect, scene.py:290-298):
    the shading kernel cannot march a callable, so Direct shades on the composed path (HIP MLPs,
    the shadow march by nrt_occlusion_callable_step) -- against the oracle's render, the FP32 bar
    on all but 0.5 % of pixels (shadow-boundary flips)."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from tests.test_gpu_parity import _shadow_scene
    ref, mine = _shadow_scene()
    ref["shape"].sdf = bend(ref["shape"].sdf, k=-1.5)
    mine["shape"].sdf = bend(mine["shape"].sdf, k=-1.5)
    imgs = {}
    for w_isect in (False, True):
        random.seed(8)
        with torch.no_grad():
            imgs[w_isect] = R.render(ref["shape"], ref["lights"], ref["camera"], R.DirectRef(),
                                     ref["bsdf"], size=64, chunk_size=64, background=0.0,
                                     with_noise=0.0, w_isect=w_isect)
    shadowed = (imgs[False] - imgs[True]).abs().amax(-1) > 1e-3
    random.seed(8)
    with torch.no_grad():
        got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"], Direct(),
                                     bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                     crop_size=64, uv=(0, 0), background=0, with_noise=0.0,
                                     w_isect=True)
    got = got.cpu()
    d = (got - imgs[True]).abs().amax(-1)
    report("callable_shadow_rays_vs_oracle[bend]", pixels=int(d.numel()),
           shadowed=int(shadowed.sum()), maxabs=float(d.max()), pixels_over_1e4=int((d > 1e-4).sum()))
    assert shadowed.sum() > 40, "the scene must cast a shadow for this test to mean anything"
    assert (d > 1e-4).float().mean() <= 0.005


class _Blob(torch.nn.Module):
    """A trainable torch SDF callable: a wobbly sphere with learnable centre and radius."""

    def __init__(self, device):
        super().__init__()
        self.c = torch.nn.Parameter(torch.tensor([0.03, -0.02, 0.01], device=device))
        self.r = torch.nn.Parameter(torch.tensor(0.28, device=device))

    def forward(self, p):
        q = p - self.c
        return q.norm(dim=-1) - self.r + 0.01 * (7 * q[..., 0]).sin() * (5 * q[..., 1]).cos()


def test_callable_training_gradients_match_oracle():
    """Training through an SDF callable (sdfs.py:133-158 under autograd): throughput =
    -1000 sdf(best_pos) and the create_graph normals carry gradients for the callable's
    parameters; a loss over both (mask BCE-style + eikonal, utils.py:307-359 / :295) against the
    oracle's autograd of the same loss -- relative 1e-4 per parameter."""
    import torch.nn.functional as F
    from neural_raytracing_amd.pathtracer.shapes import SDF
    rays = _rays(24, 5, eye=(0.0, 0.2, 1.1))
    mine, ref = _Blob("cuda"), _Blob("cpu")

    def loss_of(it):
        thr = it.throughput.reshape(-1)
        raw = it.raw_normals
        return F.softplus(-thr / 1000.0).mean() + ((raw.norm(dim=-1) - 1) ** 2).mean()
    random.seed(3)
    it, hit = SDF(sdf=mine, max_steps=48).intersect(rays.cuda())
    g = torch.autograd.grad(loss_of(it), [mine.c, mine.r])
    random.seed(3)
    want, whit = R.MarchedSDF(sdf=ref, max_steps=48, create_graph=True).intersect(rays)
    gw = torch.autograd.grad(loss_of(want), [ref.c, ref.r])
    assert torch.equal(hit.cpu().reshape(-1), whit.reshape(-1))
    rel = [float((a.cpu() - b).norm() / b.norm()) for a, b in zip(g, gw)]
    report("callable_training_grads", hits=int(whit.sum()), rel_c=rel[0], rel_r=rel[1])
    assert int(whit.sum()) > 50
    assert max(rel) < 1e-4, rel


def _oracle_callable_grads(ref, kind, p, w, dtype):
    """Oracle autograd of <w, f(p)> + eikonal(autograd normal of f at p) for the callable f
    around a copy of the oracle blob in ``dtype``; every parameter's gradient."""
    import copy
    m = copy.deepcopy(ref).to(dtype)
    for sub in m.modules():
        if hasattr(sub, "basis_p"):
            sub.basis_p = sub.basis_p.to(dtype)
    f = bend(m) if kind == "bend" else disp(m)
    q = p.detach().clone().to(dtype).requires_grad_(True)
    out = f(q).reshape(-1)
    (n,) = torch.autograd.grad(out, q, torch.ones_like(out), create_graph=True)
    loss = (out * w.to(dtype)).sum() + ((n.norm(dim=-1) - 1) ** 2).mean()
    loss.backward()
    return {k: v.grad.detach().double() for k, v in m.named_parameters()}


@pytest.mark.parametrize("kind", ["bend", "disp"])
def test_callable_training_through_a_hip_mlp(kind):
    """Training through an SDF callable that wraps a trainable HIP SkipConnMLP (edit_dtu.py:86-100
    around a SphereSDF with its 8x128 shift): SDF.autograd_diff's create_graph normal (sdfs.py:
    184-197) differentiates the MLP's input gradient through _MlpFn's create_graph backward
    (input_gradient: nrt_mlp_backward + nrt_mlp_grad_backward).  A loss of the callable's
    values and the eikonal term of its normals at fixed points near the surface; every
    parameter's gradient against float64 oracle autograd: max|HIP - f64| <= max(2e-3 max|f64|,
    4 max|oracle f32 - f64|)."""
    ref, mine = _blob(128, 128, 32, "softplus")
    g = torch.Generator().manual_seed(4)
    d = torch.nn.functional.normalize(torch.randn(600, 3, generator=g), dim=-1)
    p = d * (0.3 + 0.1 * torch.rand(600, 1, generator=g))
    w = torch.randn(600, generator=g) * 0.1
    f = bend(mine) if kind == "bend" else disp(mine)
    q = p.cuda().requires_grad_(True)
    out = f(q).reshape(-1)
    (n,) = torch.autograd.grad(out, q, torch.ones_like(out), create_graph=True)
    loss = (out * w.cuda()).sum() + ((n.norm(dim=-1) - 1) ** 2).mean()
    names = dict(mine.named_parameters())
    grads = torch.autograd.grad(loss, list(names.values()), allow_unused=True)
    got = {k: (torch.zeros_like(v) if gr is None else gr).detach().cpu().double()
           for (k, v), gr in zip(names.items(), grads)}
    want = _oracle_callable_grads(ref, kind, p, w, torch.float64)
    w32 = _oracle_callable_grads(ref, kind, p, w, torch.float32)
    # product names (init / layers / out of shift, centers / radii / tfs) equal the oracle's
    worst = 0.0
    for k, g64 in want.items():
        err = (got[k] - g64).abs().max().item()
        e32 = (w32[k] - g64).abs().max().item()
        tol = max(2e-3 * g64.abs().max().item(), 4 * e32, 1e-9)
        worst = max(worst, err / tol)
        assert err <= tol, f"{k}: {err:.3g} > {tol:.3g}"
    report(f"callable_hip_mlp_training[{kind}]", params=len(want), worst_err_over_tol=worst)
    # the eikonal term reaches the shift MLP's weights through the double backward
    assert want["shift.layers.3.weight"].abs().max() > 0


def test_callable_training_step_through_a_hip_mlp():
    """One optimiser step of SDF.intersect's training outputs (throughput = -1000 sdf(best_pos)
    and the create_graph normals) through disp(HIP SphereSDF): finite, nonzero gradients for the
    shift MLP and the spheres, and the loss moves."""
    from neural_raytracing_amd.pathtracer.shapes import SDF
    _, mine = _blob(128, 128, 32, "softplus")
    f = disp(mine)
    rays = _rays(24, 5, eye=(0.0, 0.2, 1.1)).cuda()
    opt = torch.optim.Adam(mine.parameters(), lr=1e-3)
    losses = []
    for _ in range(2):
        random.seed(3)
        opt.zero_grad()
        it, hit = SDF(sdf=f, max_steps=48).intersect(rays)
        loss = torch.nn.functional.softplus(-it.throughput.reshape(-1) / 1000.0).mean() + \
            ((it.raw_normals.norm(dim=-1) - 1) ** 2).mean()
        loss.backward()
        losses.append(float(loss))
        gs = [q.grad for q in mine.shift.parameters()]
        assert all(g is not None and torch.isfinite(g).all() for g in gs)
        assert any(float(g.abs().max()) > 0 for g in gs)
        opt.step()
    assert losses[0] != losses[1] and all(math.isfinite(x) for x in losses)


def test_callable_over_frozen_mlp_with_grad_mode_on():
    """grad mode on but nothing the callable closes over takes gradients (a bend
    around a loaded, frozen SDF): the normals need no graph, so the intersect runs and equals the
    no_grad one (sdfs.py:184-197 differentiates any callable)."""
    from neural_raytracing_amd.pathtracer.shapes import SDF
    ref, mine = _blob(128, 128, 32, "softplus")
    for q in mine.parameters():
        q.requires_grad_(False)
    f = bend(mine)
    rays = _rays(20, 6, eye=(0.0, 0.2, 1.1)).cuda()
    random.seed(3)
    it, hit = SDF(sdf=f, max_steps=32).intersect(rays)
    random.seed(3)
    with torch.no_grad():
        it0, hit0 = SDF(sdf=f, max_steps=32).intersect(rays)
    assert torch.equal(hit, hit0) and bool(hit.any())
    assert torch.equal(it.n, it0.n) and torch.equal(it.p, it0.p)
    assert not it.n.requires_grad
