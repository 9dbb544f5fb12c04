"""The fp32-split range guard (nrt_ring3.h header; VERDICT r3 "What's weak" 2): activations past
f16's range (|a| >= 65520) must not reach an f16 half unscaled.

The networks here are the usual test networks "inflated": for pairs of consecutive plain layers
(i, i + 1) -- neither a skip layer, i + 1 possibly the out layer -- layer i's weights and bias are
multiplied by k and layer i + 1's weights divided by k.  leaky_relu is positively homogeneous, so
the function is unchanged while the inputs of layer i + 1 are k times larger: 1e4 .. 1e9 here,
checked on the oracle, so the guard has to raise an exponent once or twice.  (Whole matrices are
scaled, so no layer's weights get a wide dynamic range: the split's weight halves are scaled per
layer.)  An unguarded split evaluation turns these into inf / NaN; the guarded one must stay at
the FP32 bar against the float64 oracle and the oracle's march / render, like the FP32 path on the
same weights.  Tolerances are the FP32 tests' (1e-4 absolute on agreeing rays / pixels, flips
<= 0.5 %)."""
import copy
import math
import random

import pytest
import torch

import bench
from oracle import pathtracer_ref as R
from tests.report import report
from tests.test_gpu_ring32 import _blob, _compare, _rays
from tests.test_gpu_split import _double, _eval, _points

pytestmark = pytest.mark.gpu
KS = (2.0e5, 1.0e9, 3.0e6)  # one factor per inflated layer pair, in turn


def inflate(mlp, ks=KS):
    """In place: the same function with the inputs of some plain layers x k (leaky_relu MLPs;
    product SkipConnMLP and oracle SkipMLP alike: init / layers / out)."""
    L = len(mlp.layers)
    plain = [i for i in range(L) if not (i != L - 1 and i % mlp.skip == 0)]
    pairs = [i for i in plain if i + 1 == L or (i + 1) in plain]
    picked, last = [], -2
    for i in pairs:  # disjoint pairs
        if i > last + 1:
            picked.append(i)
            last = i + 1
    with torch.no_grad():
        for n, i in enumerate(picked):
            k = ks[n % len(ks)]
            lin = mlp.layers[i]
            nxt = mlp.layers[i + 1] if i + 1 < L else mlp.out
            lin.weight.mul_(k)
            lin.bias.mul_(k)
            nxt.weight.div_(k)
    return mlp


def _hidden_absmax(ref_mlp, pts):
    """Largest |activation| inside the oracle MLP at pts (forward hooks on the hidden linears)."""
    seen = []
    hooks = [lin.register_forward_hook(lambda m, i, o: seen.append(o.abs().max().item()))
             for lin in [ref_mlp.init, *ref_mlp.layers]]
    with torch.no_grad():
        ref_mlp(pts)
    for h in hooks:
        h.remove()
    return max(seen)


def _inflated_blob(hidden, freqs, seed=5):
    ref, mine = _blob(64, hidden, freqs, "leaky_relu", seed=seed)
    inflate(ref.shift)
    inflate(mine.shift)
    return ref, mine


@pytest.mark.parametrize("hidden,freqs", [(256, 16), (128, 32)])
def test_split_guard_sdf_eval_large_activations(hidden, freqs):
    ref, mine = _inflated_blob(hidden, freqs)
    pts = _points(6000, 4)
    amax = _hidden_absmax(ref.shift, pts)
    assert amax > 1e4, amax  # past f16's range
    f64 = _double(ref)
    w = f64(pts.double()).reshape(-1)
    s32, _ = _eval(mine, pts, "fp32", None)
    s3, n3 = _eval(mine, pts, "fp32-split", "k_sdf_eval3")
    assert n3 == 1
    assert torch.isfinite(s3).all(), "split evaluation overflowed"
    e32, e3 = (s32 - w).abs(), (s3 - w).abs()
    report(f"split_guard_eval[{hidden},{freqs}]", points=pts.shape[0], act_absmax=amax,
           fp32_max=e32.max().item(), split_max=e3.max().item(), split_mean=e3.mean().item())
    assert e3.max().item() <= 2 * e32.max().item() + 1e-6
    assert e3.max().item() <= 1e-4


@pytest.mark.parametrize("hidden,freqs", [(256, 16), (128, 32)])
def test_split_guard_march_matches_oracle(hidden, freqs):
    """March + scan (k_march3 / k_scan_best3) and normals (k_normal3) of the inflated SDF."""
    from neural_raytracing_amd import _lib, set_precision
    from neural_raytracing_amd.pathtracer.shapes import SDF
    ref, mine = _inflated_blob(hidden, freqs, seed=8)
    rays = _rays(36, 7, eye=(0.0, 0.2, 1.1))
    out = {}
    for prec in ("fp32", "fp32-split"):
        set_precision(prec)
        _lib.profile_enable(True)
        _lib.profile_reset()
        random.seed(12)
        with torch.no_grad():
            out[prec] = SDF(sdf=mine, max_steps=64).intersect(rays.cuda(), primary=True)
        if prec == "fp32-split":
            assert _lib.profile_read("k_march3")[1] == 1
            assert _lib.profile_read("k_normal3")[1] == 1
        _lib.profile_enable(False)
    set_precision("fp32")
    random.seed(12)
    jit = random.random()
    with torch.no_grad():
        rit, rhit = R.MarchedSDF(sdf=ref, max_steps=64).intersect(rays, primary=True, jitter=jit)
    assert 0.1 < rhit.float().mean() < 0.9
    it, hit = out["fp32-split"]
    assert torch.isfinite(it.t).all() and torch.isfinite(it.throughput).all()
    assert torch.isfinite(it.n).all()
    _compare(f"split_guard_march_vs_oracle[{hidden},{freqs}]", it, hit, rit, rhit)
    it32, hit32 = out["fp32"]
    _compare(f"fp32_inflated_march_vs_oracle[{hidden},{freqs}]", it32, hit32, rit, rhit)


def _inflate_scene(scene, osc):
    for a, b in [(scene["lights"].light_field_approx, osc["lights"].light_field_approx),
                 (scene["bsdf"].sp_var_fn, osc["bsdf"].sp_var_fn),
                 *[(p.mlp, o.mlp) for p, o in zip(scene["bsdf"].bsdfs, osc["bsdf"].bsdfs)]]:
        inflate(a)
        inflate(b)


def test_split_guard_shading_render_matches_oracle():
    """Direct shading on the row programs (k_light3 / k_bsdf3) with every shading MLP inflated
    (LightField 10x256, the spatial-weight MLP 16x256 F=128, the eight NeuralBSDF 6x96): a crop of
    the bench frame across the silhouette, split vs the oracle render and vs the FP32 path."""
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    scene = bench.build_scene("cuda", samples=32, seed=0, light_gain=bench.LIGHT_GAIN)
    osc = bench.oracle_scene(scene)
    _inflate_scene(scene, osc)
    pts = torch.rand(512, 3) - 0.5
    amax = min(_hidden_absmax(osc["lights"].light_field_approx, pts),
               _hidden_absmax(osc["bsdf"].sp_var_fn, pts))
    assert amax > 1e4, amax
    pt = scene["pt"]
    size, crop = 320, 40
    c0, c1 = (size - crop) // 2, 30
    focal = float(0.5 * size / math.tan(0.5 * 0.6911))
    c2w = bench.view_c2w(0, 1).unsqueeze(0)
    ocam = R.NeRFCameraRef(c2w, focal)
    random.seed(5)
    with torch.no_grad():
        want = R.render(osc["shape"], osc["lights"], ocam, osc["integrator"], osc["bsdf"],
                        size=size, chunk_size=size, background=0.0, with_noise=0.0,
                        crop=(c0, c1, crop))
    cam = pt.cameras.NeRFCamera(cam_to_world=c2w.cuda(), focal=focal)
    got = {}
    for prec in ("fp32", "fp32-split"):
        nra.set_precision(prec)
        _lib.profile_enable(True)
        _lib.profile_reset()
        random.seed(5)
        with torch.no_grad():
            got[prec], _ = pt.pathtrace_sample(scene["shape"], scene["lights"], cam,
                                               scene["integrator"], bsdf=scene["bsdf"], size=size,
                                               chunk_size=size, bundle_size=1, crop_size=crop,
                                               uv=(c0, c1), background=0, with_noise=0.0)
        if prec == "fp32-split":
            assert _lib.profile_read("k_bsdf3")[1] >= 1 and _lib.profile_read("k_light3")[1] >= 1
        _lib.profile_enable(False)
    nra.set_precision("fp32")
    want_hit = want[..., 3] > 0.5
    assert 0.1 < want_hit.float().mean() < 0.95
    for prec, g in got.items():
        g = g.cpu()
        assert torch.isfinite(g).all(), prec
        err = (g - want).abs().amax(-1)
        report(f"guard_shading_vs_oracle[{prec}]", pixels=crop * crop, act_absmax=amax,
               maxabs=err.max().item(), pixels_over_1e4=int((err > 1e-4).sum()))
        # a march flip moves a pixel by O(1): at most 0.5 % of them
        assert int((err > 1e-4).sum()) <= 0.005 * crop * crop, (prec, int((err > 1e-4).sum()))
    d = (got["fp32-split"].cpu() - got["fp32"].cpu()).abs().amax(-1)
    assert int((d > 1e-4).sum()) <= 0.005 * crop * crop


def test_split_guard_is_free_when_not_needed():
    """On ordinary weights the guard never switches on: the split evaluation of the un-inflated
    network is bit-identical before and after an inflated one ran (exponents are per launch)."""
    _, mine = _blob(64, 256, 16, "leaky_relu", seed=5)
    _, big = _inflated_blob(256, 16)
    pts = _points(4000, 6)
    a, _ = _eval(mine, pts, "fp32-split", "k_sdf_eval3")
    b, _ = _eval(big, pts, "fp32-split", "k_sdf_eval3")
    c, _ = _eval(mine, pts, "fp32-split", "k_sdf_eval3")
    assert torch.isfinite(b).all()
    assert torch.equal(a, c)
