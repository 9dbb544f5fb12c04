"""The training loop's SDF handle (shapes/sdfs.py train_sdf_handle): the march of a training step
runs over the MLP's device-refreshed training handle (nrt_mlp_refresh) and a sphere table
rewritten on the device (nrt_sdf_refresh_spheres) -- no host re-pack per optimiser step.  It
must march exactly like a freshly host-packed handle of the same weights, before and after the
parameters change in place (what AdamW does), in FP32 and fp32-split."""
import ctypes

import pytest
import torch

from tests.test_gpu_ring32 import _rays

pytestmark = pytest.mark.gpu


def _march(h, rays, code):
    from neural_raytracing_amd import _lib
    P, dev = rays.shape[0], rays.device
    t = torch.empty(P, device=dev)
    hit = torch.zeros(P, dtype=torch.uint8, device=dev)
    p, n, raw, wi = (torch.zeros(P, 3, device=dev) for _ in range(4))
    thr = torch.empty(P, device=dev)
    idx = torch.empty(P, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.load(require_device=True)
    ws = torch.empty(max(lib.nrt_intersect_workspace_bytes(h, P), 1), dtype=torch.uint8, device=dev)
    mp = _lib.MarchParams(48, 5e-3, 10.0, 1, 2.2, code)
    _lib.call("nrt_sdf_intersect", h, _lib.ptr(rays), P, ctypes.byref(mp), _lib.ptr(t),
              _lib.ptr(hit), _lib.ptr(p), _lib.ptr(n), _lib.ptr(raw), _lib.ptr(wi), _lib.ptr(thr),
              _lib.ptr(idx), _lib.ptr(cnt), _lib.ptr(ws), _lib.stream())
    torch.cuda.synchronize()
    return [x.cpu() for x in (t, hit, p, n, raw, thr)]


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
def test_train_sdf_handle_marches_like_a_fresh_pack(prec):
    import neural_raytracing_amd as nra
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    from neural_raytracing_amd.pathtracer.shapes.sdfs import march_handle, sdf_handle
    torch.manual_seed(3)
    sdf = SphereSDF(n=128, device="cpu")
    with torch.no_grad():
        sdf.radii.add_(0.1)
        for a in [sdf.shift.init, *sdf.shift.layers]:
            a.weight.normal_(0.0, 0.02)
        sdf.shift.out.weight.normal_(0.0, 0.002)
    sdf = sdf.cuda()
    nra.set_precision(prec)
    code = _lib.precision_code()
    rays = _rays(40, 5, eye=(0.0, 0.2, 1.1)).reshape(-1, 6).contiguous().cuda()
    try:
        for rnd in range(3):
            with torch.enable_grad():
                ht = march_handle(sdf)           # parameters take gradients: the training handle
            got = _march(ht, rays, code)
            with torch.no_grad():
                hr = march_handle(sdf)           # no gradients: the host-packed render handle
            want = _march(hr, rays, code)
            assert hr.value == sdf_handle(sdf).value
            assert int(want[1].sum()) > 100
            for a, b, name in zip(got, want, ("t", "hit", "p", "n", "raw", "thr")):
                assert torch.equal(a, b), (rnd, name, (a.float() - b.float()).abs().max())
            # an optimiser-like in-place update of every parameter (versions bump)
            with torch.no_grad():
                sdf.centers.add_(0.01 * torch.randn_like(sdf.centers))
                sdf.radii.add_(0.005)
                sdf.tfs.add_(0.01 * torch.randn_like(sdf.tfs))
                for q in sdf.shift.parameters():
                    q.mul_(1.01)
    finally:
        nra.set_precision("fp32")


SHAPES = {  # the shading MLPs nrt_mlp_forward runs on the ring engine (nrt_shade_ring.hip)
    "light_10x256_f16": dict(num_layers=10, hidden_size=256, out=3, freqs=16),
    "spatial_16x256_f128": dict(num_layers=16, hidden_size=256, out=8, freqs=128, sigma=2 << 6),
    "bsdf_6x96_f64": dict(num_layers=6, hidden_size=96, out=3, freqs=64),
}


def _forward(handle, x, ring=True):
    from neural_raytracing_amd import _lib
    from tests.helpers import lib_opt
    y = torch.empty(x.shape[0], handle_out(handle), device="cuda")
    lib_opt("shade_ring", 1 if ring else 0)
    _lib.profile_enable(True)
    _lib.profile_reset()
    _lib.call("nrt_mlp_forward", handle.value, _lib.ptr(x), None, x.shape[0], _lib.ptr(y),
              _lib.NRT_FP32, _lib.stream())
    torch.cuda.synchronize()
    n = _lib.profile_read("k_mlp_ring32")[1]
    _lib.profile_enable(False)
    lib_opt("shade_ring", 1)
    return y.cpu(), n


_OUT = {}


def handle_out(h):
    return _OUT[id(h)]


@pytest.mark.parametrize("shape", list(SHAPES))
def test_mlp_forward_on_the_ring_engine(shape):
    """nrt_mlp_forward (FP32) of the shading MLP shapes on the ring engine against the per-wave slab
    kernel (option shade_ring = 0): exact-f32 MFMA both, different summation orders (1e-5 of the
    output scale); then the training handle after an in-place weight change (nrt_mlp_refresh
    gathers the ring program too) against a freshly packed handle of the same weights: equal."""
    from neural_raytracing_amd.pathtracer._handles import mlp_handle, train_handle
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    torch.manual_seed(11)
    mlp = SkipConnMLP(in_size=3, device="cpu", **SHAPES[shape]).cuda()
    x = (torch.rand(5003, 3) * 2 - 1).cuda()
    h = mlp_handle(mlp)
    _OUT[id(h)] = mlp.out.out_features
    ring, n = _forward(h, x, True)
    slab, n0 = _forward(h, x, False)
    assert n >= 1 and n0 == 0
    scale = slab.abs().max().clamp_min(1e-3)
    assert ((ring - slab).abs().max() / scale) < 1e-5, (ring - slab).abs().max()
    th = train_handle(mlp)
    _OUT[id(th)] = mlp.out.out_features
    for rnd in range(2):
        with torch.no_grad():
            for q in mlp.parameters():
                q.mul_(1.02)
        th = train_handle(mlp)            # refreshed on the device
        _OUT[id(th)] = mlp.out.out_features
        got, n1 = _forward(th, x, True)
        fresh = mlp_handle(mlp)           # re-packed on the host (the version changed)
        _OUT[id(fresh)] = mlp.out.out_features
        want, _ = _forward(fresh, x, True)
        assert n1 >= 1
        assert torch.equal(got, want), (rnd, (got - want).abs().max())
