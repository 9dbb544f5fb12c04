"""The drivers' render entry points and model formats on the GPU, against the oracle:

* ``test_nerf`` (training_utils.py:302-345, the call at nerf_synthetic.py:129) through the
  ``pytorch3d`` import surface with a ``torch.jit.load``-ed SphereSDF as the SDF (nerf_synthetic.py:
  63-64): every rendered view vs the oracle's render of the same view (camera jitter and scan
  jitter replayed);
* ``test_dtu`` (training_utils.py:436-485, dtu.py:179) with a DTUCamera;
* training through a TorchScript SDF: gradients land on the ScriptModule's own tensors and equal
  those of the same weights in a SphereSDF module;
* model files: a ``torch.save`` pickle of ComposeSpatialVarying / LightField
  under the reference's module paths and a ``torch.jit.save`` SphereSDF, read by
  ``model_io.load`` (nothing executed from the files), rendered on HIP vs the oracle.
"""
import math
import random

import pytest
import torch
import torch.nn as nn

from oracle import pathtracer_ref as R
from oracle import recipes
from tests.report import report
from tests.test_model_io import (RefComposeSpatialVarying, RefDiffuse, RefLightField,  # noqa: F401
                                 RefNeuralBSDF, SphereSDF as ScriptableSphereSDF, ref_paths)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


def _copy_linear(dst, src):
    with torch.no_grad():
        dst.weight.copy_(src.weight)
        dst.bias.copy_(src.bias)


def _scripted_sphere_sdf(src, device="cuda"):
    """A TorchScript module with the reference SphereSDF's attribute layout (sdfs.py:16-44) holding
    the tensors of ``src`` (an oracle SphereBlobSDF or a product SphereSDF), saved with
    torch.jit.save and loaded back with torch.jit.load, as the drivers do."""
    import io
    torch.manual_seed(123)
    n = src.centers.shape[0]
    m = ScriptableSphereSDF(n)
    with torch.no_grad():
        m.centers.copy_(src.centers)
        m.radii.copy_(src.radii)
        m.tfs.copy_(src.tfs)
        m.shift.basis_p = src.shift.basis_p.detach().cpu().clone()
        lins = [src.shift.init, *src.shift.layers, src.shift.out]
        for a, b in zip([m.shift.init, *m.shift.layers, m.shift.out], lins):
            _copy_linear(a, b)
    buf = io.BytesIO()
    torch.jit.save(torch.jit.script(m), buf)
    buf.seek(0)
    return torch.jit.load(buf, map_location=device)


def _capture_plots(monkeypatch):
    import pytorch3d.pathtracer.training_utils as tu
    got = []
    monkeypatch.setattr(tu, "save_plot", lambda exp, img, name: got.append(img.detach().cpu()))
    return got


def test_test_nerf_with_a_torchscript_sdf_matches_oracle(monkeypatch):
    """nerf_synthetic.py:63-67, 123-140 in miniature: SDF(sdf=torch.jit.load(...)), Direct(),
    ComposeSpatialVarying([NeuralBSDF(Softplus)] x 8), LightField, test_nerf over two views."""
    import pytorch3d.pathtracer as pt
    from pytorch3d.pathtracer.integrators import Direct
    from pytorch3d.pathtracer.shapes.sdfs import SDF
    from pytorch3d.pathtracer.training_utils import test_nerf
    from tests.test_gpu_parity import _scene_pair
    ref, mine = _scene_pair()
    sm = _scripted_sphere_sdf(ref["shape"].sdf)
    assert isinstance(sm, torch.jit.ScriptModule)
    density_field = SDF(sdf=sm)
    density_field.max_steps = 32
    size = 64
    focal = recipes.nerf_focal(size)
    c2ws = [recipes.look_at_c2w(e) for e in [(0.0, 0.2, 1.0), (0.6, 0.3, 0.75)]]
    # the RNG the product draws per view: camera jitter (cuda, rays_tile) and scan jitter (python)
    torch.manual_seed(5)
    random.seed(5)
    noises = [torch.rand(2, size, size, device="cuda").cpu() for _ in c2ws]
    jits = [random.random() for _ in c2ws]
    got = _capture_plots(monkeypatch)
    torch.manual_seed(5)
    random.seed(5)
    test_nerf(density_field, integrator=Direct(), bsdf=mine["bsdf"], lights=mine["lights"],
              cam_to_worlds=[c.cuda() for c in c2ws], focal=focal,
              exp_imgs=[torch.zeros(size, size, 3, device="cuda") for _ in c2ws], size=size,
              name_fn=lambda i: f"/tmp/unused_{i}.png")
    assert len(got) == len(c2ws)
    for v, (c2w, noise, jit) in enumerate(zip(c2ws, noises, jits)):
        cam = R.NeRFCameraRef(c2w.unsqueeze(0), focal)
        with torch.no_grad():
            want = R.render(ref["shape"], ref["lights"], cam, R.DirectRef(), ref["bsdf"],
                            size=size, chunk_size=size, background=0.0, with_noise=1e-3,
                            jitter=jit,
                            camera_noise=lambda pos, n=noise: (n[0].unsqueeze(-1),
                                                               n[1].unsqueeze(-1)))
        want = want.clamp(0, 1)
        err = (got[v] - want).abs().amax(-1)
        report(f"test_nerf_view{v}", pixels=err.numel(), maxabs=err.max().item(),
               pixels_over_1e4=int((err > 1e-4).sum()),
               lit=int((want.amax(-1) > 0).sum()))
        assert (want.amax(-1) > 0).float().mean() > 0.1
        assert (err <= 1e-4).float().mean() >= 0.995, err.max()
    assert pt.pathtrace is not None


def test_test_dtu_matches_oracle(monkeypatch):
    """dtu.py:179-185: test_dtu over a DTU pose (DTUCamera ignores with_noise), masked metrics."""
    import bench
    from pytorch3d.pathtracer.integrators import Direct
    from pytorch3d.pathtracer.training_utils import test_dtu
    from tests.test_gpu_configs import _dtu_oracle
    sc = bench.build_other_scene("dtu", torch.device("cuda"), 64)
    osc = _dtu_oracle(sc)
    size = 64
    got = _capture_plots(monkeypatch)
    random.seed(9)
    jit = random.random()
    random.seed(9)
    test_dtu(sc["shape"], integrator=Direct(), bsdf=sc["bsdf"], lights=sc["lights"],
             poses=[sc["cameras"].pose[0]], intrinsics=[sc["cameras"].intrinsic[0]],
             exp_imgs=[torch.zeros(size, size, 3, device="cuda")],
             exp_masks=[torch.ones(size, size, device="cuda")], size=size,
             name_fn=lambda i: f"/tmp/unused_{i}.png")
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], osc["camera"], R.DirectRef(), osc["bsdf"],
                        size=size, chunk_size=size, background=0.0, jitter=jit).clamp(0, 1)
    err = (got[0] - want).abs().amax(-1)
    report("test_dtu_view0", pixels=err.numel(), maxabs=err.max().item(),
           pixels_over_1e4=int((err > 1e-4).sum()))
    assert (want.amax(-1) > 0).float().mean() > 0.1
    assert (err <= 1e-4).float().mean() >= 0.995, err.max()


def test_training_through_a_torchscript_sdf():
    """The optimiser of nerf_synthetic.py:81-85 holds density_field.parameters() -- the
    ScriptModule's tensors: a pathtrace_sample loss backward fills their .grad, equal to the
    gradients of the same weights held by a SphereSDF module."""
    import pytorch3d.pathtracer as pt
    from pytorch3d.pathtracer.shapes.sdfs import SDF
    from tests.test_gpu_parity import _scene_pair
    ref, mine = _scene_pair()
    with torch.no_grad():  # a non-zero shift so its gradients are non-trivial
        for lin in [mine["shape"].sdf.shift.init, *mine["shape"].sdf.shift.layers]:
            lin.weight.normal_(0, 0.02)
        mine["shape"].sdf.shift.out.weight.normal_(0, 0.002)
    sm = _scripted_sphere_sdf(mine["shape"].sdf)
    grads = []
    for sdf in (sm, mine["shape"].sdf):
        shape = SDF(sdf=sdf, max_steps=32)
        for p in shape.parameters():
            p.grad = None
        random.seed(3)
        img, mi = pt.pathtrace_sample(shape, mine["lights"], mine["camera"], mine["integrator"],
                                      bsdf=mine["bsdf"], size=256, chunk_size=256, bundle_size=1,
                                      crop_size=16, uv=(120, 110), background=0, with_noise=0.0,
                                      addition=lambda m: m)
        loss = img.square().mean() + (mi.raw_normals.norm(dim=-1) - 1).square().mean()
        loss.backward()
        grads.append({"centers": sdf.centers.grad.clone(), "radii": sdf.radii.grad.clone(),
                      "shift_init": sdf.shift.init.weight.grad.clone(),
                      "shift_out": sdf.shift.out.weight.grad.clone()})
    for k in grads[0]:
        a, b = grads[0][k], grads[1][k]
        assert a.abs().sum() > 0, k
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-7), (k, (a - b).abs().max())


def test_model_files_render_like_the_oracle(tmp_path, ref_paths):
    """dtu.py:93-108's formats -- torch.jit.save(SphereSDF), torch.save(
    ComposeSpatialVarying), torch.save(LightField) -- written under the reference's module paths,
    read by model_io.load (restricted unpickler, nothing executed), rendered on HIP and compared
    with the oracle built from the same tensors."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer import model_io
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    torch.manual_seed(0)
    random.seed(0)
    o_sdf = R.SphereBlobSDF(n=32)
    with torch.no_grad():
        o_sdf.shift.out.weight.normal_(0, 0.01)  # a non-zero residual
    bsdf_rec = RefComposeSpatialVarying([RefNeuralBSDF(nn.Softplus()), RefNeuralBSDF(nn.Softplus()),
                                         RefDiffuse()])
    lf_rec = RefLightField()
    sm = _scripted_sphere_sdf(o_sdf, device="cpu")
    torch.jit.save(sm, str(tmp_path / "sdf.pt"))
    torch.save(bsdf_rec, tmp_path / "bsdf.pt")
    torch.save(lf_rec, tmp_path / "lights.pt")
    shape = pt.shapes.SDF(sdf=model_io.load(str(tmp_path / "sdf.pt")), max_steps=32)
    bsdf = model_io.load(str(tmp_path / "bsdf.pt"))
    lights = model_io.load(str(tmp_path / "lights.pt"))

    # the oracle from the same tensors
    def o_mlp(rec, act):
        m = R.SkipMLP(num_layers=len(rec.layers), hidden_size=rec.init.out_features,
                      in_size=rec.in_size, out=rec.out.out_features, skip=rec.skip,
                      freqs=rec.basis_p.shape[1], activation=act)
        m.basis_p = rec.basis_p.clone()
        for a, b in zip([m.init, *m.layers, m.out], [rec.init, *rec.layers, rec.out]):
            _copy_linear(a, b)
        return m
    parts = []
    for b in bsdf_rec.bsdfs[:2]:
        o = R.NeuralBSDFRef(activation="softplus")
        o.mlp = o_mlp(b.mlp, "leaky_relu")
        parts.append(o)
    parts.append(R.DiffuseRef(reflectance=bsdf_rec.bsdfs[2].reflectance.tolist()))
    o_bsdf = R.SpatialMixBSDF(parts)
    o_bsdf.sp_var_fn = o_mlp(bsdf_rec.sp_var_fn, "leaky_relu")
    o_lights = R.LightFieldRef()
    o_lights.light_field_approx = o_mlp(lf_rec.light_field_approx, "leaky_relu")
    with torch.no_grad():
        o_lights.color.copy_(lf_rec.color)
    c2w = recipes.look_at_c2w((0.2, 0.3, 0.9)).unsqueeze(0)
    focal = recipes.nerf_focal(64)
    random.seed(4)
    with torch.no_grad():
        want = R.render(R.MarchedSDF(sdf=o_sdf, max_steps=32), o_lights, R.NeRFCameraRef(c2w, focal),
                        R.NeRFIntegratorRef(R.DirectRef()), o_bsdf, size=64, chunk_size=64,
                        background=0.0)
    random.seed(4)
    with torch.no_grad():
        got, _ = pt.pathtrace(shape, lights, pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(),
                                                                  focal=focal),
                              NeRFIntegrator(Direct()), bsdf=bsdf, size=64, chunk_size=64,
                              bundle_size=1, background=0.0, with_noise=0.0)
    got = got.cpu()
    err = (got - want).abs().amax(-1)
    report("model_files_render", pixels=err.numel(), maxabs=err.max().item(),
           pixels_over_1e4=int((err > 1e-4).sum()))
    assert (want[..., :3].amax(-1) > 0).float().mean() > 0.05
    assert (err <= 1e-4).float().mean() >= 0.995, err.max()
    assert math.isfinite(err.max().item())


def test_train_sample_colocated_lights_per_camera(tmp_path, monkeypatch):
    """colocate.py's training call (colocate.py:109-137): train_sample with N = 2 cameras per step,
    a point light moved onto each camera (light.location = cameras.get_camera_center() * 1.05,
    one light per camera), Direct() (colocate.py:78) and a learned occlusion MLP (w_isect=occ_mlp)
    -- every step shades each camera with its own light on the training path.  Two steps and a
    validation render run; the losses are finite and the weights move."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, Diffuse, NeuralBSDF
    from neural_raytracing_amd.pathtracer.cameras import look_at_view_transform
    from neural_raytracing_amd.pathtracer.integrators import Direct
    from neural_raytracing_amd.pathtracer.lights import PointLights
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.shapes import SDF, SphereSDF
    from neural_raytracing_amd.pathtracer.training_utils import train_sample
    monkeypatch.chdir(tmp_path)
    (tmp_path / "outputs").mkdir()
    torch.manual_seed(21)
    random.seed(21)
    dev = "cuda"
    shape = SDF(sdf=SphereSDF(n=32, device=dev), device=dev, max_steps=32)
    bsdf = ComposeSpatialVarying([NeuralBSDF(device=dev), Diffuse(device=dev)], device=dev)
    lights = PointLights(device=dev, scale=5)
    occ = SkipConnMLP(in_size=5, out=1, device=dev).to(dev)
    views = [look_at_view_transform(dist=1.0, elev=e, azim=a) for e, a in ((30, 45), (10, -60),
                                                                         (45, 150))]
    Rs = [r.to(dev) for r, _ in views]
    Ts = [t.to(dev) for _, t in views]
    size = 32
    exp_imgs = [torch.rand(size, size, 3, device=dev) for _ in views]
    exp_masks = [torch.ones(size, size, device=dev) for _ in views]
    params = list(shape.parameters()) + list(bsdf.parameters()) + list(occ.parameters())
    opt = torch.optim.Adam(params, lr=1e-4)
    before = [p.detach().clone() for p in params]
    seen = []

    def light_update(cam, light):
        light.location = cam.get_camera_center().to(dev) * 1.05
        seen.append(light.per_camera())

    losses = train_sample(shape, bsdf=bsdf, integrator=Direct(), lights=lights,
                          Rs=Rs, Ts=Ts, exp_imgs=exp_imgs, exp_masks=exp_masks, opt=opt,
                          size=size, crop_size=16, N=2, iters=2, save_freq=10_000, valid_freq=1,
                          max_valid_size=16, uv_select=lambda _, cs: (8, 8),
                          light_update=light_update, silent=True, w_isect=occ)
    assert len(losses) == 2 and all(math.isfinite(x) for x in losses)
    assert 2 in seen  # a step with one light per camera
    assert any(not torch.equal(b, p.detach()) for b, p in zip(before, params))
