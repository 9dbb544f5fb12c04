"""Round-3 API items on the GPU, against the oracle or against the API's own untrimmed /
un-optioned result:

* ``pathtrace(trim > 0)`` (main.py:52, 67-68): every tile rendered with a trim-pixel border and
  cropped back gives the untrimmed image (rays are per pixel, so the interior is unchanged);
* option ``scan_best32`` (include/nrt.h "Runtime options"): on the FP16 march, the throughput
  -1000 sdf(best) (sdfs.py:137, 249) evaluated by the FP32 engine -- the FP16 SDF error the x1000
  logit amplifies into alpha drops, and the flip / depth statistics do not change.
"""
import math
import random

import pytest
import torch

import bench
from oracle import pathtracer_ref as R
from tests.helpers import lib_opt as _lib_opt
from tests.report import report
from tests.test_gpu_configs import _camera_rays, _mlp_sdf_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fp32():
    from neural_raytracing_amd import set_precision
    set_precision("fp32")
    yield
    set_precision("fp32")


@pytest.mark.parametrize("trim", [1, 3])
def test_pathtrace_trim_matches_untrimmed(trim):
    scene = bench.build_scene("cuda", samples=32, seed=3)
    pt = scene["pt"]
    size = 64
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    cam = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1).unsqueeze(0).cuda(), focal=focal)
    imgs = []
    for tr in (0, trim):
        random.seed(11)
        with torch.no_grad():
            img, _ = pt.pathtrace(scene["shape"], scene["lights"], cam, scene["integrator"],
                                  bsdf=scene["bsdf"], size=size, chunk_size=32, bundle_size=1,
                                  background=0, with_noise=0.0, trim=tr, silent=True)
        imgs.append(img.cpu())
    assert imgs[0].shape == imgs[1].shape == (size, size, 4)
    assert (imgs[0][..., 3] > 0.5).any() and (imgs[0][..., 3] < 0.5).any()
    assert (imgs[0] - imgs[1]).abs().max().item() <= 1e-6


def test_pathtrace_trim_negative_raises():
    scene = bench.build_scene("cuda", samples=8, seed=3)
    pt = scene["pt"]
    cam = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1).unsqueeze(0).cuda(), focal=50.0)
    with pytest.raises(ValueError):
        pt.pathtrace(scene["shape"], scene["lights"], cam, scene["integrator"], bsdf=scene["bsdf"],
                     size=32, chunk_size=32, trim=-1)


def test_fp16_scan_best32_cuts_throughput_error():
    """The bare 8x256 MLP SDF (cfg2 / cfg4 kind) marched in FP16 with and without the FP32
    sdf(best) pass, against the oracle's throughput."""
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    ref, mine = _mlp_sdf_pair()
    rays = _camera_rays(40, 3)
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=lambda p: ref(p)[..., 0], max_steps=64).intersect(
            rays, primary=True, jitter=jit)
    want = rit.throughput.reshape(-1)
    set_precision("fp16")
    res = {}
    for best32 in (0, 1):
        _lib_opt("scan_best32", best32)
        _lib.profile_enable(True)
        _lib.profile_reset()
        random.seed(12)
        with torch.no_grad():
            it, hit = SDF(sdf=mine, max_steps=64).intersect(rays.cuda(), primary=True)
        n32 = _lib.profile_read("k_scan_best32")[1]
        n16 = _lib.profile_read("k_scan_best16")[1]
        _lib.profile_enable(False)
        assert (n32, n16) == ((1, 0) if best32 else (0, 1))
        err = (it.throughput.cpu().reshape(-1) - want).abs()
        alpha_err = (torch.sigmoid(it.throughput.cpu().reshape(-1)) - torch.sigmoid(want)).abs()
        res[best32] = (hit.cpu().reshape(-1), it.t.cpu().reshape(-1), err, alpha_err)
        report(f"fp16_scan_best32[{best32}]", rays=err.numel(), thr_maxabs=err.max().item(),
               thr_over_0p1=int((err > 0.1).sum()), alpha_maxabs=alpha_err.max().item(),
               alpha_over_1e4=int((alpha_err > 1e-4).sum()))
    # the march itself is the same FP16 march either way
    # (bitwise: the FP16 log2-domain softplus overflows to NaN on the shaped SDF's far points,
    # pre-activations above 88, so some missed rays carry t = NaN -- DESIGN.md §3 k_march16)
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1].view(torch.int32), res[1][1].view(torch.int32))
    e16, e32 = res[0][2], res[1][2]
    assert int((e32 > 0.1).sum()) < int((e16 > 0.1).sum())
    assert e32.median().item() < 0.25 * e16.median().item()


def test_fp16_ring_march_repeatable():
    """Two identical FP16 ring marches of the bare 8x256 MLP SDF give identical bits."""
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    _, mine = _mlp_sdf_pair()
    rays = _camera_rays(40, 3).cuda()
    set_precision("fp16")
    outs = []
    for _ in range(3):
        random.seed(12)
        with torch.no_grad():
            it, hit = SDF(sdf=mine, max_steps=64).intersect(rays, primary=True)
        outs.append((hit.cpu(), it.t.cpu(), it.throughput.cpu(), it.n.cpu()))
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            if a.dtype == torch.float32:
                a, b = a.view(torch.int32), b.view(torch.int32)
            assert torch.equal(a, b)


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
def test_pathtrace_batched_tiles_with_jitter_match_oracle(prec):
    """pathtrace's fused tiles are marched / shaded in one batch (render.render_tiles): 16 tiles,
    each with its own scan jitter (random.random(), sdfs.py:236) and camera jitter (two rand_like
    draws per tile, cameras.py:35-36) in tile order, vs the oracle's tile loop fed the same
    draws."""
    import neural_raytracing_amd.pathtracer as pt
    from neural_raytracing_amd import _lib, set_precision
    from tests.test_gpu_parity import _scene_pair
    ref, mine = _scene_pair()
    size, chunk, amp = 64, 16, 0.5
    n_tiles = (size // chunk) ** 2
    torch.manual_seed(77)
    draws = [torch.rand(2, chunk, chunk, device="cuda").cpu() for _ in range(n_tiles)]
    it = iter(draws)

    def camera_noise(pos):
        nz = next(it)
        return nz[0][..., None], nz[1][..., None]

    random.seed(21)
    with torch.no_grad():
        want = R.render(ref["shape"], ref["lights"], ref["camera"], ref["integrator"], ref["bsdf"],
                        size=size, chunk_size=chunk, background=0.25, with_noise=amp,
                        camera_noise=camera_noise)
    set_precision(prec)
    torch.manual_seed(77)
    random.seed(21)
    _lib.profile_enable(True)
    _lib.profile_reset()
    with torch.no_grad():
        got, _ = pt.pathtrace(mine["shape"], mine["lights"], mine["camera"], mine["integrator"],
                              bsdf=mine["bsdf"], size=size, chunk_size=chunk, bundle_size=1,
                              background=0.25, with_noise=amp, silent=True)
    n_isect = _lib.profile_read("k_intersect")[1]
    _lib.profile_enable(False)
    assert n_isect == 1, "the 16 tiles were not batched into one intersect launch"
    err = (got.cpu() - want).abs()
    report(f"batched_tiles_vs_oracle[{prec}]", tiles=n_tiles, maxabs=err.max().item(),
           pixels_over_1e4=int((err.amax(-1) > 1e-4).sum()))
    assert err.max().item() <= 1e-4


@pytest.mark.parametrize("alpha", [True, False])
@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
def test_render_tile_entry_matches_python_chain(alpha, prec):
    """nrt_render_tile (one C-ABI call per pathtrace tile: raygen, march + scan + normals,
    Direct shading, composite) equals the Python launch chain render.render_tile bit for bit:
    same camera jitter uniforms, same scan jitter draw (NeRFIntegrator(Direct): alpha channel;
    Direct: background fill)."""
    import ctypes
    import random
    import bench
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.integrators import Direct, NeRFIntegrator
    from neural_raytracing_amd.pathtracer.integrators.integrators import _bsdf_handle, _light_handle
    from neural_raytracing_amd.pathtracer.render import fused_integrator, render_tile
    from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_handle
    nra.set_precision(prec)
    try:
        sc = bench.build_scene("cuda", 32, seed=2, light_gain=bench.LIGHT_GAIN)
        pt = sc["pt"]
        size, chunk, x0, y0 = 96, 32, 32, 16
        focal = float(0.5 * size / math.tan(0.5 * 0.6911))
        cam = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].cuda(), focal=focal)
        integ = NeRFIntegrator(Direct()) if alpha else Direct()
        C = 4 if alpha else 3
        bg = 0.25
        want = torch.full((1, size, size, C), bg, device="cuda")
        got = want.clone()
        torch.manual_seed(3)
        random.seed(4)
        with torch.no_grad():
            render_tile(fused_integrator(integ), sc["shape"], sc["lights"], cam, sc["bsdf"], want,
                        x0, y0, chunk, size, 1e-3, bg)
        torch.manual_seed(3)
        noise = torch.rand(2, chunk, chunk, device="cuda")
        random.seed(4)
        shapes = sc["shape"]
        mp = _lib.MarchParams(int(shapes.max_steps), float(shapes.epsilon), 10.0, 1,
                              float(shapes.dist + random.random() * (2 / 128)),
                              _lib.precision_code())
        sh = sdf_handle(shapes.sdf)
        lib = _lib.load(require_device=True)
        ws = torch.empty(lib.nrt_render_tile_workspace_bytes(sh, 1, chunk, chunk), dtype=torch.uint8,
                         device="cuda")
        arr = (_lib.Camera * 1)(*cam._structs(size))
        with torch.no_grad():
            _lib.call("nrt_render_tile", ctypes.cast(arr, ctypes.c_void_p), 1, x0, y0, chunk, chunk,
                      1e-3, _lib.ptr(noise), sh, ctypes.byref(mp), _bsdf_handle(sc["bsdf"]),
                      _light_handle(sc["lights"]), int(alpha), bg, _lib.ptr(got), size, size, C, x0,
                      y0, _lib.ptr(ws), _lib.stream())
        torch.cuda.synchronize()
        tile = (slice(None), slice(x0, x0 + chunk), slice(y0, y0 + chunk))
        assert torch.equal(got, want)
        assert (want[tile] != bg).any() and (want[..., :3][tile] > 0).any()
    finally:
        nra.set_precision("fp32")
