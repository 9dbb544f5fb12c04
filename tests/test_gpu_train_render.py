"""Training through the fused render path: gradients of a loss on
``pathtrace_sample`` -- throughput = -1000 sdf(best_pos), the create_graph SDF normals
(``nrt_mlp_grad_backward``), the shading MLPs -- against torch autograd of the oracle.

Tolerances are written per test: the double backward is compared with float64 autograd of the
oracle's SkipMLP (as tests/test_gpu_train.py does for the first backward); whole-render
gradients are FP32 on both sides with different batch-reduction orders, so they are compared at
2e-3 of each tensor's largest entry (plus 1e-6 absolute)."""
import copy
import math
import random

import pytest
import torch
import torch.nn.functional as F

from oracle import pathtracer_ref as R
from oracle import recipes
from tests.helpers import copy_mlp, seeded
from tests.report import report

SHAPES = {
    "sdf_8x256_softplus_F16": dict(num_layers=8, hidden_size=256, in_size=3, out=1, freqs=16,
                                   activation="softplus"),
    "shift_8x128_softplus_F32": dict(num_layers=8, hidden_size=128, in_size=3, out=1, freqs=32,
                                     activation="softplus"),
    "8x64_leaky_out3": dict(num_layers=8, hidden_size=64, in_size=3, out=3, freqs=16),
    "sigmoid_4x32": dict(num_layers=4, hidden_size=32, in_size=3, out=1, freqs=8,
                         activation="sigmoid"),
}


def _pair(kw, seed):
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    seeded(seed)
    act = kw.get("activation", "leaky_relu")
    ref = R.SkipMLP(**kw)
    pkw = {k: v for k, v in kw.items() if k != "activation"}
    if act != "leaky_relu":
        pkw["activation"] = {"softplus": F.softplus, "sigmoid": torch.sigmoid}[act]
    mine = SkipConnMLP(device="cpu", **pkw)
    copy_mlp(mine, ref)
    return ref, mine.cuda()


def _double_backward(ref, x, v, dtype):
    m = copy.deepcopy(ref).to(dtype)
    m.basis_p = ref.basis_p.to(dtype)
    xr = x.detach().clone().to(dtype).requires_grad_(True)
    y = m(xr)
    (g,) = torch.autograd.grad(y, xr, torch.ones_like(y), create_graph=True)
    (g * v.to(dtype)).sum().backward()
    out = {"g": g.detach()}
    for i, lin in enumerate([m.init, *m.layers, m.out]):
        out[f"dW[{i}]"] = lin.weight.grad if lin.weight.grad is not None else torch.zeros_like(lin.weight)
        out[f"db[{i}]"] = lin.bias.grad if lin.bias.grad is not None else torch.zeros_like(lin.bias)
    return out


def _close(got, want, ref32, what, rel=1e-4):
    scale = max(1.0, want.abs().max().item())
    err = (got.detach().cpu().double() - want.double()).abs().max().item()
    e32 = (ref32.detach().double() - want.double()).abs().max().item()
    tol = max(rel * scale, 4 * e32)
    assert err <= tol, f"{what}: max|diff| {err:.3g} > {tol:.3g} (scale {scale:.3g}, fp32 ref {e32:.3g})"


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 45, 700])
@pytest.mark.parametrize("name", list(SHAPES))
def test_mlp_grad_backward_matches_autograd(name, M):
    """d/dtheta of sum(v . d(sum y)/dx): nrt_mlp_grad_backward vs float64 double backward."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import input_gradient
    kw = SHAPES[name]
    ref, mine = _pair(kw, 70 + M)
    # the zero / default init leaves the deep layers' second-order terms tiny: widen the weights
    with torch.no_grad():
        for a in [ref.init, *ref.layers, ref.out]:
            a.weight.mul_(1.5)
    copy_mlp(mine, ref)
    set_precision("fp32")
    g = torch.Generator().manual_seed(M)
    x = (torch.rand(M, 3, generator=g) - 0.5)
    v = torch.randn(M, 3, generator=g)
    want = _double_backward(ref, x, v, torch.float64)
    ref32 = _double_backward(ref, x, v, torch.float32)
    gm = input_gradient(mine, x.cuda())
    (gm * v.cuda()).sum().backward()
    got = {"g": gm}
    for i, a in enumerate(mine._linears()):
        got[f"dW[{i}]"] = a.weight.grad
        got[f"db[{i}]"] = a.bias.grad
    for k in want:
        _close(got[k], want[k], ref32[k], k)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(SHAPES))
def test_mlp_grad_backward_column_split_bit_equal(name):
    """k_mlp_grad_backward32_cs (option bwd_colsplit != 0) against the per-wave kernel
    (bwd_colsplit 0): the same operations per element, every parameter gradient bit-equal, on a
    ragged row count."""
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.neural_blocks import input_gradient
    kw = SHAPES[name]
    _, mine = _pair(kw, 3)
    set_precision("fp32")
    g = torch.Generator().manual_seed(9)
    x = (torch.rand(2011, 3, generator=g) - 0.5).cuda()
    v = torch.randn(2011, 3, generator=g).cuda()

    def run(opt):
        with _lib.options(bwd_colsplit=opt):
            mine.zero_grad(set_to_none=True)
            (input_gradient(mine, x) * v).sum().backward()
            return [p.grad.clone() for p in mine.parameters() if p.grad is not None]
    base, got = run(0), run(1)
    assert len(base) == len(got) > 2
    for i, (a, b) in enumerate(zip(base, got)):
        assert torch.equal(a, b), (name, i, (a - b).abs().max().item())


@pytest.mark.gpu
def test_mlp_grad_backward_empty_and_refusals():
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.neural_blocks import input_gradient
    ref, mine = _pair(SHAPES["8x64_leaky_out3"], 1)
    g = input_gradient(mine, torch.empty(0, 3, device="cuda"))
    assert g.shape == (0, 3)
    g.sum().backward()
    assert all(float(p.grad.abs().max()) == 0 for p in mine.parameters())
    with pytest.raises(NrtError):
        input_gradient(mine, torch.rand(4, 3, device="cuda", requires_grad=True))


def _perturbed_scene(smooth=False):
    """The BASELINE.md §2 scene with a non-zero SphereSDF shift MLP (the recorded scene's shift is
    zero-initialised, which would leave the double-backward terms zero).

    ``smooth=True`` switches the leaky-ReLU shading MLPs (NeuralBSDFs, spatial weights,
    LightField) to softplus on both sides: leaky_relu's kink makes per-element gradients
    discontinuous -- this crop has a NeuralBSDF pre-activation at |z| = 3.4e-7, within FP32
    rounding of 0, whose derivative flips between 1 and 0.01 between any two FP32
    implementations (measured: the oracle's own FP32 run is 1.3 % off its float64 run there)."""
    import tests.test_gpu_parity as P
    ref, mine = P._scene_pair()
    if smooth:
        pairs = [(ref["bsdf"].sp_var_fn, mine["bsdf"].sp_var_fn),
                 (ref["lights"].light_field_approx, mine["lights"].light_field_approx)]
        pairs += [(a.mlp, b.mlp) for a, b in zip(ref["bsdf"].bsdfs, mine["bsdf"].bsdfs)]
        for a, b in pairs:
            a.act_name = "softplus"
            b.activation = F.softplus
    seeded(21)
    with torch.no_grad():
        sh = ref["shape"].sdf.shift
        for a in [sh.init, *sh.layers]:
            a.weight.normal_(0.0, 0.02)
            a.bias.zero_()
        sh.out.weight.normal_(0.0, 0.002)  # |shift| ~ 0.02: every ray of the crop still hits
        sh.out.bias.zero_()
    copy_mlp(mine["shape"].sdf.shift, sh)
    ref["shape"].create_graph = True
    return ref, mine


def _named_params(scene, oracle):
    out = {}
    sdf = scene["shape"].sdf
    out["centers"], out["radii"], out["tfs"] = sdf.centers, sdf.radii, sdf.tfs
    sh = sdf.shift
    lins = [sh.init, *sh.layers, sh.out]
    for i, a in enumerate(lins):
        out[f"shift.W{i}"], out[f"shift.b{i}"] = a.weight, a.bias
    sp = scene["bsdf"].sp_var_fn
    for i, a in enumerate([sp.init, *sp.layers, sp.out]):
        out[f"sp.W{i}"], out[f"sp.b{i}"] = a.weight, a.bias
    for j, b in enumerate(scene["bsdf"].bsdfs):
        for i, a in enumerate([b.mlp.init, *b.mlp.layers, b.mlp.out]):
            out[f"bsdf{j}.W{i}"], out[f"bsdf{j}.b{i}"] = a.weight, a.bias
    lf = scene["lights"].light_field_approx
    for i, a in enumerate([lf.init, *lf.layers, lf.out]):
        out[f"light.W{i}"], out[f"light.b{i}"] = a.weight, a.bias
    out["light.color"] = scene["lights"].color
    return out


def _oracle_render_grads(ref, dtype, w, crop):
    """Oracle render of the crop + loss <img, w> + 0.1 eikonal(raw normals) in ``dtype``;
    returns the image, the hit-point normals and every parameter's gradient."""
    r = {k: copy.deepcopy(v) for k, v in ref.items()}
    for m in (r["shape"].sdf, r["bsdf"], r["lights"]):
        m.to(dtype)
        for sub in m.modules():
            if hasattr(sub, "basis_p"):
                sub.basis_p = sub.basis_p.to(dtype)
    r["camera"].cam_to_world = r["camera"].cam_to_world.to(dtype)
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        random.seed(11)
        img = R.render(r["shape"], r["lights"], r["camera"], r["integrator"], r["bsdf"],
                       size=256, chunk_size=256, background=0.0, with_noise=0.0,
                       crop=(crop[0], crop[1], crop[2]))
        # the interaction record is internal to DirectRef: recompute its normals the same way
        rays = r["camera"].sample_positions(R._tile_positions(*crop), 256, 0.0)
        o, d = rays.split(3, dim=-1)
        t, hit = r["shape"].march(o, d)
        raw = r["shape"].gradient((o + t * d)[hit])
        loss = (img * w.to(dtype)).sum() + 0.1 * (raw.norm(dim=-1) - 1).square().mean()
        loss.backward()
    finally:
        torch.set_default_dtype(old)
    grads = {k: (a.grad if a.grad is not None else torch.zeros_like(a)).detach().double()
             for k, a in _named_params(r, True).items()}
    return img.detach(), raw.detach(), grads


@pytest.mark.gpu
def test_pathtrace_sample_gradients_match_oracle():
    """loss = <img, w> + 0.1 eikonal(raw_normals) on a 32x32 crop: every parameter's gradient
    (SphereSDF spheres and shift MLP through throughput and the create_graph normals, the
    spatial-weights MLP, 8 NeuralBSDFs, the LightField).  Bar per tensor:
    max|HIP - f64| <= max(2e-3 * max|f64|, 4 * max|oracle f32 - f64|) -- the deep shading MLPs'
    FP32 gradients carry ~1 % rounding noise whichever implementation computes them."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    ref, mine = _perturbed_scene(smooth=True)
    crop = (112, 112, 32)
    w = torch.randn(32, 32, 4, generator=torch.Generator().manual_seed(5))
    img64, raw64, want = _oracle_render_grads(ref, torch.float64, w, crop)
    img32, _, ref32 = _oracle_render_grads(ref, torch.float32, w, crop)
    random.seed(11)
    captured = {}
    img, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"],
                                 mine["integrator"], bsdf=mine["bsdf"], size=256, chunk_size=256,
                                 bundle_size=1, crop_size=32, uv=crop[:2], background=0,
                                 with_noise=0.0, device="cuda",
                                 addition=lambda it: captured.setdefault("raw", it.raw_normals))
    assert img.requires_grad
    diff = (img.detach().cpu() - img32).abs().max().item()
    assert diff <= 1e-4, f"forward differs from the FP32 oracle by {diff}"
    raw = captured["raw"]
    assert raw is not None and raw.requires_grad and raw.shape == raw64.shape
    loss = (img * w.cuda()).sum() + 0.1 * (raw.norm(dim=-1) - 1).square().mean()
    loss.backward()
    got = _named_params(mine, False)
    bad = []
    for k, g64 in want.items():
        gb = got[k].grad
        gb = torch.zeros_like(g64) if gb is None else gb.detach().cpu().double()
        scale = g64.abs().max().item()
        err = (gb - g64).abs().max().item()
        e32 = (ref32[k] - g64).abs().max().item()
        if err > max(2e-3 * scale, 4 * e32) + 1e-9:
            bad.append(f"{k}: err {err:.3g} scale {scale:.3g} fp32-oracle err {e32:.3g}")
    assert not bad, "\n".join(bad)
    assert want["shift.W0"].abs().max() > 0  # the double-backward terms are exercised


@pytest.mark.gpu
def test_training_steps_reduce_render_loss():
    """A few Adam steps of the full scene through pathtrace_sample lower an image loss."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    _, mine = _perturbed_scene()
    target = torch.zeros(32, 32, 4, device="cuda")
    target[..., :3] = 0.5
    target[..., 3] = 1.0
    params = [*mine["shape"].sdf.parameters(), *mine["bsdf"].parameters(),
              *mine["lights"].parameters()]
    opt = torch.optim.Adam(params, lr=1e-3)
    losses = []
    for step in range(8):
        random.seed(step)
        opt.zero_grad()
        img, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"],
                                     mine["integrator"], bsdf=mine["bsdf"], size=256,
                                     chunk_size=256, bundle_size=1, crop_size=32, uv=(112, 112),
                                     background=0, with_noise=0.0, device="cuda")
        loss = F.mse_loss(img, target)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses


def _nerfle_grads(ref, rays, loc, w, dtype, jitter):
    r = copy.deepcopy(ref).to(dtype)
    for sub in r.modules():
        if hasattr(sub, "basis_p"):
            sub.basis_p = sub.basis_p.to(dtype)
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        out = r(rays.to(dtype), loc.to(dtype), jitter=jitter)
        (out * w.to(dtype)).sum().backward()
    finally:
        torch.set_default_dtype(old)
    lins = {"first": r.first, "second": r.second}
    return out.detach(), {f"{n}.{k}{i}": getattr(a, "weight" if k == "W" else "bias").grad.double()
                          for n, m in lins.items()
                          for i, a in enumerate([m.init, *m.layers, m.out]) for k in ("W", "b")}


@pytest.mark.gpu
def test_nerfle_training_gradients_match_oracle():
    """NeRFLE (nerf.py:175-214) with autograd: both MLPs' gradients of <rgb, w> against float64
    autograd of the oracle (softplus MLPs, so the gradients are smooth in the weights; same
    bar as the render test)."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from tests.test_gpu_parity import _nerfle_pair
    ref, mine = _nerfle_pair()
    for m in (ref.first, ref.second):
        m.act_name = "softplus"
    for m in (mine.first, mine.second):
        m.activation = F.softplus
    g = torch.Generator().manual_seed(8)
    o = torch.tensor([0.0, 0.2, 1.2]) + 0.1 * torch.randn(1, 9, 7, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 9, 7, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 9, 7, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    loc = torch.tensor([[0.3, 1.0, 0.2]])
    w = torch.randn(1, 9, 7, 1, 3, generator=g)
    random.seed(6)
    jitter = random.random()
    want_img, want = _nerfle_grads(ref, rays, loc, w, torch.float64, jitter)
    _, ref32 = _nerfle_grads(ref, rays, loc, w, torch.float32, jitter)
    set_precision("fp32")
    lights = PointLights(location=loc.cuda(), device="cuda")
    random.seed(6)
    got_img = mine(rays.cuda(), lights)
    assert got_img.requires_grad
    assert (got_img.detach().cpu().double() - want_img).abs().max().item() <= 1e-4
    (got_img * w.cuda()).sum().backward()
    got = {f"{n}.{k}{i}": getattr(a, "weight" if k == "W" else "bias").grad
           for n, m in {"first": mine.first, "second": mine.second}.items()
           for i, a in enumerate(m._linears()) for k in ("W", "b")}
    bad = []
    for k, g64 in want.items():
        err = (got[k].detach().cpu().double() - g64).abs().max().item()
        e32 = (ref32[k] - g64).abs().max().item()
        if err > max(2e-3 * g64.abs().max().item(), 4 * e32) + 1e-9:
            bad.append(f"{k}: err {err:.3g} scale {g64.abs().max().item():.3g} fp32 {e32:.3g}")
    assert not bad, "\n".join(bad)


@pytest.mark.gpu
def test_envmap_refuses_a_light_field():
    """NeRFLE's envmap needs a PointLights: a LightField fails loudly instead of dropping the
    light encoding."""
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.shapes import NeRFLE
    _, mine = _perturbed_scene()
    rays = mine["camera"].rays_tile(120, 120, 4, 4, 256)
    nerf = NeRFLE(envmap=True, device="cuda")
    with pytest.raises(NrtError):
        nerf(rays, mine["lights"])


def _path_grad_pair():
    """tests/test_gpu_parity.py's path_nerv-like scene with smooth (softplus) shading MLPs (the
    leaky_relu kink: see _perturbed_scene) and a non-zero SDF shift."""
    import tests.test_gpu_parity as P
    ref, mine = P._path_pair()
    pairs = [(ref["bsdf"].sp_var_fn, mine["bsdf"].sp_var_fn)]
    pairs += [(a.mlp, b.mlp) for a, b in zip(ref["bsdf"].bsdfs[:2], mine["bsdf"].bsdfs[:2])]
    for a, b in pairs:
        a.act_name = "softplus"
        b.activation = F.softplus
    seeded(33)
    with torch.no_grad():
        sh = ref["shape"].sdf.shift
        for a in [sh.init, *sh.layers]:
            a.weight.normal_(0.0, 0.02)
            a.bias.zero_()
        sh.out.weight.normal_(0.0, 0.002)
        sh.out.bias.zero_()
    copy_mlp(mine["shape"].sdf.shift, sh)
    ref["shape"].create_graph = True
    return ref, mine


def _path_params(scene):
    out = {}
    sdf = scene["shape"].sdf
    out["centers"], out["radii"], out["tfs"] = sdf.centers, sdf.radii, sdf.tfs
    for name, m in [("shift", sdf.shift), ("sp", scene["bsdf"].sp_var_fn),
                    ("bsdf0", scene["bsdf"].bsdfs[0].mlp), ("bsdf1", scene["bsdf"].bsdfs[1].mlp)]:
        for i, a in enumerate([m.init, *m.layers, m.out]):
            out[f"{name}.W{i}"], out[f"{name}.b{i}"] = a.weight, a.bias
    return out


def _oracle_path_grads(ref, dtype, rays, uniforms, w):
    r = {k: copy.deepcopy(v) for k, v in ref.items()}
    for m in (r["shape"].sdf, r["bsdf"]):
        m.to(dtype)
        for sub in m.modules():
            if hasattr(sub, "basis_p"):
                sub.basis_p = sub.basis_p.to(dtype)
            for k, v in list(vars(sub).items()):
                if isinstance(v, torch.Tensor) and not isinstance(v, torch.nn.Parameter):
                    setattr(sub, k, v.to(dtype))
    for k, v in list(vars(r["lights"]).items()):
        if isinstance(v, torch.Tensor):
            setattr(r["lights"], k, v.to(dtype))
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        uni = [(a.to(dtype), b.to(dtype)) for a, b in uniforms]
        img, mask, _ = R.PathRef().sample(r["shape"], rays.to(dtype), r["bsdf"], r["lights"],
                                          uniforms=uni)
        (img * w.to(dtype)).sum().backward()
    finally:
        torch.set_default_dtype(old)
    grads = {k: (a.grad if a.grad is not None else torch.zeros_like(a)).detach().double()
             for k, a in _path_params(r).items()}
    return img.detach(), grads


@pytest.mark.gpu
def test_path_gradients_match_oracle():
    """Path (integrators.py:275-354) under autograd, two bounces with injected BSDF-sampling
    uniforms: loss = <img, w>; the gradient of every parameter -- SphereSDF spheres and shift
    (both bounces' normals, the secondary hit points through the differentiable spawned rays),
    the spatial-weights MLP, the NeuralBSDFs -- against float64 oracle autograd, with the
    reference's detached throughput (:336-337).  Bar per tensor as for pathtrace_sample."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Path
    set_precision("fp32")
    ref, mine = _path_grad_pair()
    c2w = recipes.look_at_c2w((0.1, 0.5, 0.9)).unsqueeze(0)
    ocam = R.NeRFCameraRef(c2w, recipes.nerf_focal(32))
    rays = ocam.sample_positions(R._tile_positions(0, 0, 32), 32)
    g = torch.Generator().manual_seed(9)
    lead = rays.shape[:-1]
    uniforms = [(torch.rand(*lead, 3, 2, generator=g), torch.rand(*lead, generator=g))
                for _ in range(2)]
    w = torch.randn(*lead, 3, generator=g)
    img64, want = _oracle_path_grads(ref, torch.float64, rays, uniforms, w)
    img32, ref32 = _oracle_path_grads(ref, torch.float32, rays, uniforms, w)
    img, mask, _ = Path().sample(mine["shape"], rays.cuda(), mine["bsdf"], lights=mine["lights"],
                                 uniforms=uniforms)
    assert img.requires_grad
    diff = (img.detach().cpu() - img32).abs().amax(-1)
    # a bounce ray's hit / step flip moves that pixel's whole second-bounce term
    assert (diff <= 1e-4).float().mean() >= 0.99, diff.max()
    (img * w.cuda()).sum().backward()
    got = _path_params(mine)
    bad, worst = [], 0.0
    for k, g64 in want.items():
        gb = got[k].grad
        gb = torch.zeros_like(g64) if gb is None else gb.detach().cpu().double()
        scale = g64.abs().max().item()
        err = (gb - g64).abs().max().item()
        e32 = (ref32[k] - g64).abs().max().item()
        worst = max(worst, err / max(scale, 1e-12))
        if err > max(2e-3 * scale, 4 * e32) + 1e-9:
            bad.append(f"{k}: err {err:.3g} scale {scale:.3g} fp32-oracle err {e32:.3g}")
    report("path_gradients_vs_f64", params=len(want), worst_rel=worst,
           pixels_over_1e4=int((diff > 1e-4).sum()))
    assert not bad, "\n".join(bad)
    assert want["shift.W0"].abs().max() > 0 and want["sp.W0"].abs().max() > 0


@pytest.mark.gpu
def test_nerfle_envmap_training_gradients_match_oracle():
    """NeRF+LE (envmap=True) with autograd: the colour MLP sees the point light's envmap at
    bins^2 directions (nerf.py:183-191); both MLPs' gradients vs float64 oracle autograd."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from tests.test_gpu_parity import _nerfle_pair
    ref, mine = _nerfle_pair(envmap=True)
    for m in (ref.first, ref.second):
        m.act_name = "softplus"
    for m in (mine.first, mine.second):
        m.activation = F.softplus
    g = torch.Generator().manual_seed(9)
    o = torch.tensor([0.0, 0.2, 1.2]) + 0.1 * torch.randn(1, 6, 5, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, 6, 5, 1, 2, generator=g) - 0.5,
                               -torch.ones(1, 6, 5, 1, 1)], -1), dim=-1)
    rays = torch.cat([o, d], -1)
    w = torch.randn(1, 6, 5, 1, 3, generator=g)
    loc = (0.3, 1.0, 0.2)
    random.seed(4)
    jitter = random.random()

    def oracle(dtype):
        r = copy.deepcopy(ref).to(dtype)
        for sub in r.modules():
            if hasattr(sub, "basis_p"):
                sub.basis_p = sub.basis_p.to(dtype)
        light = R.PointLightRef(location=loc)
        for a in ("scale", "intensity", "location", "const", "linear", "square"):
            setattr(light, a, getattr(light, a).to(dtype))
        old = torch.get_default_dtype()
        torch.set_default_dtype(dtype)
        try:
            out = r(rays.to(dtype), None, jitter=jitter, light=light)
            (out * w.to(dtype)).sum().backward()
        finally:
            torch.set_default_dtype(old)
        return out.detach(), {f"{n}.{k}{i}": getattr(a, "weight" if k == "W" else "bias").grad.double()
                              for n, m in {"first": r.first, "second": r.second}.items()
                              for i, a in enumerate([m.init, *m.layers, m.out]) for k in ("W", "b")}
    want_img, want = oracle(torch.float64)
    _, ref32 = oracle(torch.float32)
    set_precision("fp32")
    random.seed(4)
    got_img = mine(rays.cuda(), PointLights(location=list(loc), device="cuda"))
    assert got_img.requires_grad
    assert (got_img.detach().cpu().double() - want_img).abs().max().item() <= 1e-4
    (got_img * w.cuda()).sum().backward()
    bad = []
    for n, m in {"first": mine.first, "second": mine.second}.items():
        for i, a in enumerate(m._linears()):
            for k in ("W", "b"):
                g64 = want[f"{n}.{k}{i}"]
                gb = getattr(a, "weight" if k == "W" else "bias").grad.detach().cpu().double()
                err = (gb - g64).abs().max().item()
                e32 = (ref32[f"{n}.{k}{i}"] - g64).abs().max().item()
                if err > max(2e-3 * g64.abs().max().item(), 4 * e32) + 1e-9:
                    bad.append(f"{n}.{k}{i}: err {err:.3g} fp32 {e32:.3g}")
    assert not bad, "\n".join(bad)


@pytest.mark.gpu
def test_mixed_precision_training_steps():
    """set_precision("fp16") with autograd: FP16 march / scan (ring kernels, scan argmin from the
    64-bit keys) and MLP forwards, FP32 backward; the loop still lowers the loss and the
    gradients stay finite."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    _, mine = _perturbed_scene()
    set_precision("fp16")
    try:
        target = torch.full((32, 32, 4), 0.5, device="cuda")
        params = [*mine["shape"].sdf.parameters(), *mine["bsdf"].parameters(),
                  *mine["lights"].parameters()]
        opt = torch.optim.Adam(params, lr=1e-3)
        losses = []
        for step in range(6):
            random.seed(step)
            opt.zero_grad()
            img, mi = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"],
                                          mine["integrator"], bsdf=mine["bsdf"], size=256,
                                          chunk_size=256, bundle_size=1, crop_size=32,
                                          uv=(112, 112), background=0, with_noise=0.0,
                                          device="cuda", addition=lambda m: m)
            loss = F.mse_loss(img, target) + 0.1 * (mi.raw_normals.norm(dim=-1) - 1).square().mean()
            loss.backward()
            assert all(p.grad is None or bool(torch.isfinite(p.grad).all()) for p in params)
            opt.step()
            losses.append(loss.item())
        assert losses[-1] < losses[0], losses
    finally:
        set_precision("fp32")


def _shadow_oracle(ref, occ_ref, dtype, w, kind):
    """Oracle Direct render of the shadow scene with w_isect = True | occ MLP, in ``dtype``;
    returns the image and the gradients of <img, w> for the SDF, Diffuse and occlusion MLP."""
    r = {k: copy.deepcopy(v) for k, v in ref.items()}
    r["shape"].create_graph = True  # differentiable normals, as the reference's autograd_diff
    occ = copy.deepcopy(occ_ref)
    mods = [r["shape"].sdf, occ]
    for m in mods:
        m.to(dtype)
        for sub in m.modules():
            if hasattr(sub, "basis_p"):
                sub.basis_p = sub.basis_p.to(dtype)
    r["bsdf"].reflectance = r["bsdf"].reflectance.to(dtype).requires_grad_(True)
    li = r["lights"]
    for a in ("scale", "intensity", "location", "const", "linear", "square"):
        setattr(li, a, getattr(li, a).to(dtype))
    r["camera"].cam_to_world = r["camera"].cam_to_world.to(dtype)
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        random.seed(8)
        img = R.render(r["shape"], r["lights"], r["camera"], R.DirectRef(), r["bsdf"], size=64,
                       chunk_size=64, background=0.0, with_noise=0.0,
                       w_isect=True if kind == "hard" else occ)
        if w is not None:
            (img * w.to(dtype)).sum().backward()
    finally:
        torch.set_default_dtype(old)
    grads = {}
    if w is not None:
        sdf = r["shape"].sdf
        grads = {"centers": sdf.centers.grad, "radii": sdf.radii.grad,
                 "reflectance": r["bsdf"].reflectance.grad}
        for i, a in enumerate([occ.init, *occ.layers, occ.out]):
            grads[f"occ.W{i}"], grads[f"occ.b{i}"] = a.weight.grad, a.bias.grad
        grads = {k: (torch.zeros(1) if g is None else g.detach().double()) for k, g in grads.items()}
    return img.detach(), grads


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["hard", "learned_occ"])
def test_shadowed_direct_gradients_match_oracle(kind):
    """Direct with w_isect=True / an occlusion MLP under autograd (colocate.py trains with the
    latter, :137): gradients of <img, w> for the SDF spheres, the Diffuse reflectance and the
    occlusion MLP vs float64 oracle autograd.  Pixels whose shadow test flips between
    implementations (ulp-level march differences at the shadow boundary) get w = 0 on both
    sides, so every compared gradient comes from rays all three runs agree on."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.integrators import Direct
    import tests.test_gpu_parity as P
    ref, mine = P._shadow_scene()
    occ_ref, occ_mine = P._occ_pair(1)
    occ_ref.act_name = "softplus"
    occ_mine.activation = F.softplus
    img64, _ = _shadow_oracle(ref, occ_ref, torch.float64, None, kind)
    img32, _ = _shadow_oracle(ref, occ_ref, torch.float32, None, kind)
    set_precision("fp32")
    random.seed(8)
    got, _ = pt.pathtrace_sample(mine["shape"], mine["lights"], mine["camera"], Direct(),
                                 bsdf=mine["bsdf"], size=64, chunk_size=64, bundle_size=1,
                                 crop_size=64, uv=(0, 0), background=0, with_noise=0.0,
                                 w_isect=True if kind == "hard" else occ_mine)
    assert got.requires_grad
    agree = ((got.detach().cpu().double() - img64).abs().amax(-1) <= 1e-4) & \
        ((img32.double() - img64).abs().amax(-1) <= 1e-4)
    assert agree.float().mean() >= 0.99
    w = torch.randn(64, 64, 3, generator=torch.Generator().manual_seed(2)) * agree[..., None]
    _, want = _shadow_oracle(ref, occ_ref, torch.float64, w, kind)
    _, ref32 = _shadow_oracle(ref, occ_ref, torch.float32, w, kind)
    (got * w.cuda()).sum().backward()
    sdf = mine["shape"].sdf
    have = {"centers": sdf.centers.grad, "radii": sdf.radii.grad,
            "reflectance": mine["bsdf"].reflectance.grad}
    for i, a in enumerate(occ_mine._linears()):
        have[f"occ.W{i}"], have[f"occ.b{i}"] = a.weight.grad, a.bias.grad
    bad = []
    for k, g64 in want.items():
        gb = have[k]
        gb = torch.zeros_like(g64) if gb is None else gb.detach().cpu().double().reshape(g64.shape)
        err = (gb - g64).abs().max().item()
        e32 = (ref32[k].reshape(g64.shape) - g64).abs().max().item()
        if err > max(2e-3 * g64.abs().max().item(), 4 * e32) + 1e-9:
            bad.append(f"{k}: err {err:.3g} scale {g64.abs().max().item():.3g} fp32 {e32:.3g}")
    assert not bad, "\n".join(bad)
    assert want["reflectance"].abs().max() > 0
    if kind == "learned_occ":
        assert want["occ.W0"].abs().max() > 0  # the occlusion MLP is on the gradient path


@pytest.mark.gpu
@pytest.mark.parametrize("loop", ["nerf", "dtu"])
def test_training_loops_run_on_the_hip_path(loop, tmp_path):
    """training_utils.train_nerf / train_dtu (training_utils.py:211-300, 347-434): a few
    iterations over synthetic views with the scripts' extra eikonal loss; finite losses, images
    written, parameters moved."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer import training_utils as TU
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.utils import eikonal_loss
    set_precision("fp32")
    _, mine = _perturbed_scene()
    size, n_views = 64, 4
    g = torch.Generator().manual_seed(3)
    imgs = [torch.rand(size, size, 3, generator=g).cuda() for _ in range(n_views)]
    masks = [torch.ones(size, size, device="cuda") for _ in range(n_views)]
    before = mine["shape"].sdf.centers.detach().clone()
    opt = torch.optim.AdamW([*mine["shape"].parameters(), *mine["bsdf"].parameters(),
                             *mine["lights"].parameters()], lr=1e-3, weight_decay=0)
    extra = lambda mi, got, exp, mask: eikonal_loss(mi.raw_normals) if mi.raw_normals is not None else 0
    common = dict(opt=opt, size=size, crop_size=16, N=2, iters=3, num_ckpts=1, save_freq=2,
                  valid_freq=0, extra_loss=extra, silent=False,
                  name_fn=lambda i: str(tmp_path / f"train_{i}.png"),
                  uv_select=lambda mask, crop: (20, 24))
    random.seed(0)
    if loop == "nerf":
        c2w = mine["camera"].cam_to_world.reshape(-1, 3, 4)[0]
        losses = TU.train_nerf(mine["shape"], mine["bsdf"], Direct(), mine["lights"],
                               [c2w] * n_views, mine["camera"].focal, imgs, masks, **common)
    else:
        pose = torch.eye(4)
        pose[:3, :4] = mine["camera"].cam_to_world.reshape(-1, 3, 4)[0].cpu()
        pose[:3, 1:3] *= -1  # DTU looks down +z
        K = torch.eye(4)
        K[0, 0] = K[1, 1] = 2890.0
        K[0, 2], K[1, 2] = 800.0, 600.0
        losses = TU.train_dtu(mine["shape"], mine["bsdf"], Direct(), mine["lights"],
                              [pose.cuda()] * n_views, [K.cuda()] * n_views, imgs, masks,
                              **common)
    assert len(losses) == 3 and all(math.isfinite(x) for x in losses), losses
    assert (tmp_path / "train_0.png").exists()
    assert not torch.equal(before, mine["shape"].sdf.centers.detach())
