"""Forward-mode SDF normals on the FP32 / fp32-split ring engines (k_normal32 / k_normal3 =
k_normal_r, nrt_kernels.h): the normal pass of nrt_sdf_intersect (sdfs.py:152-158, autograd normal
sdfs.py:184-197) after a ring32 / ring3 march.

* against the per-wave FP32 reverse-mode kernel k_sdf_grad (option normals_ring = 0) on the same
  march: unit normals and offset points within 1e-5, raw gradients within 1e-5 relative to their
  norm (both are FP32-class: forward and reverse mode differ only in rounding order);
* against the oracle's autograd gradient in float64 near the march's hit points: the ring path
  is within 2x of k_sdf_grad's error (or 1e-5 relative);
* the configurations the ring engines serve: SphereSDF(128) + 8x128 / 8x256 shifts (F = 16 / 32,
  softplus / leaky_relu); ragged hit counts.  (The bare 8x256 MLP SDF runs through the same
  kernels in tests/test_gpu_configs.py and tests/test_gpu_split.py against the oracle.)
"""
import copy

import pytest
import torch

from tests.helpers import lib_opt as _lib_opt
from tests.report import report
from tests.test_gpu_ring32 import _blob, _rays

pytestmark = pytest.mark.gpu

CONFIGS = [(128, 32, "softplus"), (256, 16, "softplus"), (128, 16, "leaky_relu"),
           (256, 32, "leaky_relu")]


def _intersect(sh, rays, code, max_steps=48):
    """nrt_sdf_intersect (primary) on a raw handle: (hit, p, n, raw gradient) on the host."""
    import ctypes
    from neural_raytracing_amd import _lib
    P, dev = rays.shape[0], rays.device
    t = torch.empty(P, device=dev)
    hit = torch.zeros(P, dtype=torch.uint8, device=dev)
    p, n, raw, wi = (torch.zeros(P, 3, device=dev) for _ in range(4))
    thr = torch.empty(P, device=dev)
    idx = torch.empty(P, dtype=torch.int32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = _lib.load(require_device=True)
    ws = torch.empty(max(lib.nrt_intersect_workspace_bytes(sh, P), 1), dtype=torch.uint8, device=dev)
    mp = _lib.MarchParams(max_steps, 5e-3, 10.0, 1, 2.2, code)
    _lib.call("nrt_sdf_intersect", sh, _lib.ptr(rays), P, ctypes.byref(mp), _lib.ptr(t),
              _lib.ptr(hit), _lib.ptr(p), _lib.ptr(n), _lib.ptr(raw), _lib.ptr(wi), _lib.ptr(thr),
              _lib.ptr(idx), _lib.ptr(cnt), _lib.ptr(ws), _lib.stream())
    torch.cuda.synchronize()
    return hit.cpu().bool(), p.cpu(), n.cpu(), raw.cpu()


def _run(sh, rays, code, ring):
    from neural_raytracing_amd import _lib
    _lib_opt("normals_ring", 1 if ring else 0)
    _lib.profile_enable(True)
    _lib.profile_reset()
    out = _intersect(sh, rays, code)
    counts = {k: _lib.profile_read(k)[1] for k in ("k_normal32", "k_normal3", "k_sdf_grad")}
    _lib.profile_enable(False)
    _lib_opt("normals_ring", 1)
    return (*out, counts)


def _double(mod):
    m = copy.deepcopy(mod).double()
    for sub in m.modules():
        for k, v in list(vars(sub).items()):
            if isinstance(v, torch.Tensor) and not isinstance(v, torch.nn.Parameter):
                setattr(sub, k, v.double())
    return m


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
@pytest.mark.parametrize("hidden,freqs,act", CONFIGS)
def test_ring_normals_match_reverse_mode(prec, hidden, freqs, act):
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_handle
    ref, mine = _blob(128, hidden, freqs, act)
    sh = sdf_handle(mine)
    code = _lib.NRT_FP32 if prec == "fp32" else _lib.NRT_FP32_SPLIT
    rays = _rays(48, 3, eye=(0.0, 0.2, 1.1)).reshape(-1, 6).contiguous().cuda()
    hit, p, n, raw, counts = _run(sh, rays, code, True)
    hit0, p0, n0, raw0, counts0 = _run(sh, rays, code, False)
    want = "k_normal32" if prec == "fp32" else "k_normal3"
    assert counts[want] >= 1 and counts["k_sdf_grad"] == 0, counts
    assert counts0["k_sdf_grad"] >= 1 and counts0[want] == 0, counts0
    assert torch.equal(hit, hit0)  # the march is the same; only the normal pass differs
    assert hit.sum() > 100
    dn = (n[hit] - n0[hit]).abs().max().item()
    dp = (p[hit] - p0[hit]).abs().max().item()
    dg = ((raw[hit] - raw0[hit]).norm(dim=-1) / raw0[hit].norm(dim=-1)).max().item()
    # float64 autograd of the oracle SDF near the hit points (p - 5 eps n, recomputed in f64)
    q = (p0[hit].double() - 5 * 5e-3 * n0[hit].double()).requires_grad_(True)
    g64 = torch.autograd.grad(_double(ref)(q).sum(), q)[0].detach()
    e_ring = ((raw[hit].double() - g64).norm(dim=-1) / g64.norm(dim=-1)).max().item()
    e_rev = ((raw0[hit].double() - g64).norm(dim=-1) / g64.norm(dim=-1)).max().item()
    report(f"ring_normals[{prec}-{hidden}-{freqs}-{act}]", hits=int(hit.sum()), n_maxabs=dn,
           p_maxabs=dp, grad_relerr_vs_reverse=dg, grad_relerr_ring_vs_f64=e_ring,
           grad_relerr_reverse_vs_f64=e_rev)
    assert dn < 1e-5 and dp < 1e-6 and dg < 1e-5, (dn, dp, dg)
    assert e_ring <= max(2 * e_rev, 1e-5), (e_ring, e_rev)


@pytest.mark.parametrize("prec", ["fp32", "fp32-split"])
@pytest.mark.parametrize("n", [1, 5, 67])
def test_ring_normals_ragged_hit_counts(prec, n):
    """Ray counts (n x n) whose hit lists are not multiples of the 4-ray tile or a block's rays."""
    from neural_raytracing_amd import _lib
    from neural_raytracing_amd.pathtracer.shapes.sdfs import sdf_handle
    _, mine = _blob(128, 128, 32, "softplus")
    sh = sdf_handle(mine)
    code = _lib.NRT_FP32 if prec == "fp32" else _lib.NRT_FP32_SPLIT
    rays = _rays(n, 9, eye=(0.0, 0.2, 1.1), spread=0.3).reshape(-1, 6).contiguous().cuda()
    hit, _, n1, raw, _ = _run(sh, rays, code, True)
    hit0, _, n0, raw0, _ = _run(sh, rays, code, False)
    assert torch.equal(hit, hit0)
    if hit.any():
        d = ((raw[hit] - raw0[hit]).norm(dim=-1) / raw0[hit].norm(dim=-1)).max().item()
        report(f"ring_normals_ragged[{prec}-{n}]", rays=n * n, hits=int(hit.sum()),
               grad_relerr_vs_reverse=d)
        assert d < 1e-5, d
    assert (n1[~hit] == n0[~hit]).all()
