"""CPU tests of the boundary: the C ABI library loads and exports every declared symbol, the
host mirror constructs the same weights as the oracle, and the multi-GPU row shard / gather."""
import os
import re
import subprocess

import pytest
import torch

from oracle import pathtracer_ref as R
from oracle import recipes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nrt.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nrt_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from neural_raytracing_amd import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (nrt_[a-z0-9_]+)", out))
    assert set(names) <= exported, set(names) - exported
    assert set(_lib.exported_symbols()) == set(names)


def test_library_is_gfx950_code_object():
    """The fat binary embeds a gfx950 code object (and no other GPU target)."""
    from neural_raytracing_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_no_cpu_fallback():
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    m = SkipConnMLP(device="cpu")
    with torch.no_grad(), pytest.raises(NrtError):
        m(torch.zeros(4, 3))


@pytest.mark.parametrize("kw", [
    dict(num_layers=8, hidden_size=256, out=1, freqs=16),
    dict(num_layers=6, hidden_size=96, out=3, freqs=64),
    dict(num_layers=16, hidden_size=256, out=8, freqs=128, sigma=128, xavier_init=True),
    dict(num_layers=8, hidden_size=128, out=1, freqs=32, zero_init=True),
])
def test_mlp_construction_matches_oracle_rng(kw):
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    torch.manual_seed(5)
    ref = R.SkipMLP(**kw)
    torch.manual_seed(5)
    mine = SkipConnMLP(device="cpu", **kw)
    assert torch.equal(ref.basis_p, mine.basis_p)
    for a, b in zip([ref.init, *ref.layers, ref.out], mine._linears()):
        assert torch.equal(a.weight, b.weight) and torch.equal(a.bias, b.bias)


def test_checksum_scene_construction_matches_oracle():
    """Building the BASELINE §2 scene with the product classes draws the same weights."""
    import random
    from neural_raytracing_amd.pathtracer.bsdf import ComposeSpatialVarying, NeuralBSDF
    from neural_raytracing_amd.pathtracer.lights import LightField
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    ref = recipes.baseline_checksum_scene()
    torch.manual_seed(0)
    random.seed(0)
    sphere = SphereSDF(n=128, device="cpu")
    bsdf = ComposeSpatialVarying([NeuralBSDF(activation=torch.nn.Softplus(), device="cpu")
                                  for _ in range(8)], device="cpu")
    lights = LightField(device="cpu")
    assert torch.equal(sphere.centers, ref["shape"].sdf.centers)
    assert torch.equal(sphere.radii, ref["shape"].sdf.radii)
    for a, b in zip(bsdf.bsdfs, ref["bsdf"].bsdfs):
        assert torch.equal(a.mlp.init.weight, b.mlp.init.weight)
    assert torch.equal(bsdf.sp_var_fn.layers[7].weight, ref["bsdf"].sp_var_fn.layers[7].weight)
    assert torch.equal(lights.light_field_approx.out.weight, ref["lights"].light_field_approx.out.weight)


def test_activation_codes():
    import torch.nn.functional as F
    from neural_raytracing_amd import NrtError
    from neural_raytracing_amd.pathtracer.neural_blocks import activation_code
    assert activation_code(torch.nn.Softplus()) == "softplus"
    assert activation_code(F.softplus) == "softplus"
    assert activation_code(torch.sigmoid) == "sigmoid"
    assert activation_code(torch.nn.LeakyReLU()) == "leaky_relu"
    with pytest.raises(NrtError):
        activation_code(torch.tanh)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("size,tile", [(800, 10), (256, 16), (64, 5)])
def test_row_shard_partitions_rows(world, size, tile):
    from neural_raytracing_amd.pathtracer.render import row_shard
    shards = [row_shard(size, r, world, tile) for r in range(world)]
    flat = sorted(x for s in shards for x in s)
    assert flat == list(range(size))
    if size % (tile * world) == 0:
        assert len({len(s) for s in shards}) == 1


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    from neural_raytracing_amd.pathtracer.render import gather_rows, row_shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    size, tile, N, W = 50, 5, 2, 7
    full = torch.arange(N * size * W * 4, dtype=torch.float32).reshape(N, size, W, 4)
    rows = row_shard(size, rank, world, tile)
    got = gather_rows(full[:, rows].contiguous(), size, rank, world, tile)
    q.put((rank, bool(torch.equal(got, full))))
    dist.destroy_process_group()


def test_gather_rows_gloo_world2():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _spawn(target, world, timeout=180):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=timeout) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return res


def _bench_step_worker(rank, world, port, q):
    """bench.make_step / max_over_ranks with a stub row renderer: every rank renders only its
    shard's rows (a function of view, row, column), several steps, uneven shards."""
    import torch.distributed as dist
    import bench
    from neural_raytracing_amd.pathtracer.render import row_shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    size, tile = 37, 4  # 37 rows over tiles of 4: ranks get different row counts
    rows = row_shard(size, rank, world, tile)
    calls = {"n": 0}
    v = torch.arange(world).view(world, 1, 1, 1).float()
    r = torch.tensor(rows).view(1, -1, 1, 1).float()
    c = torch.arange(size).view(1, 1, size, 1).float()
    ch = torch.arange(4).view(1, 1, 1, 4).float()

    def render():  # [views, my rows, size, 4]
        calls["n"] += 1
        return 1000 * v + 10 * r + 0.01 * c + 0.001 * ch + calls["n"]

    step = bench.make_step(render, rows, size, rank, world, tile, torch.device("cpu"))
    ok = True
    rr = torch.arange(size).view(1, -1, 1, 1).float()
    for k in range(1, 4):
        full = step()
        want = 1000 * v + 10 * rr + 0.01 * c + 0.001 * ch + k
        ok = ok and bool(torch.equal(full, want))
    el = bench.max_over_ranks(float(rank + 1), world, torch.device("cpu"))
    q.put((rank, (ok, el)))
    dist.destroy_process_group()


def test_bench_step_assembly_gloo_world2():
    """The multi-rank bookkeeping of bench.py (frame assembly across uneven row shards, repeated
    steps through the cached buffers, MAX of the elapsed times) run on gloo, world size 2."""
    res = _spawn(_bench_step_worker, 2)
    assert res == {0: (True, 2.0), 1: (True, 2.0)}


def _broadcast_worker(rank, world, port, q):
    import torch.distributed as dist
    from neural_raytracing_amd.pathtracer.neural_blocks import SkipConnMLP
    from neural_raytracing_amd.pathtracer.render import broadcast_module
    from neural_raytracing_amd.pathtracer.shapes import SphereSDF
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    torch.manual_seed(100 + rank)  # every rank a different model
    m = torch.nn.ModuleList([SphereSDF(n=8, device="cpu"),
                             SkipConnMLP(num_layers=3, hidden_size=32, freqs=4, device="cpu")])
    versions = [p._version for p in m.parameters()]
    broadcast_module(m)
    flat = torch.cat([t.reshape(-1) for t in list(m.parameters()) + [m[1].basis_p, m[0].shift.basis_p]])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    bumped = all(p._version > v for p, v in zip(m.parameters(), versions))
    q.put((rank, (all(torch.equal(g, gathered[0]) for g in gathered), bumped)))
    dist.destroy_process_group()


def test_broadcast_module_gloo_world2():
    """broadcast_module replicates rank 0's parameters and tensor attributes (basis_p) on every
    rank, in place (version counters move, so packed handles are rebuilt)."""
    res = _spawn(_broadcast_worker, 2)
    assert res == {0: (True, True), 1: (True, True)}


def _bench_scene_broadcast_worker(rank, world, port, q):
    """bench.py's multi-GPU branch broadcasts its real scene objects -- the SDF shape
    (a plain class with parameters() only), the BSDF and the lights, including a PointLights
    whose falloff tensors stay on the host."""
    import torch.distributed as dist
    import bench
    from neural_raytracing_amd.pathtracer.render import _module_tensors, broadcast_module
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    dev = torch.device("cpu")
    scene = bench.build_scene(dev, 64, seed=10 + rank)  # every rank a different scene
    other = bench.build_other_scene("colocate", dev, 64)
    with torch.no_grad():
        for t in _module_tensors(other["lights"]):
            t.add_(rank)
    objs = [scene["shape"], scene["bsdf"], scene["lights"], other["lights"], other["shape"]]
    for o in objs:
        broadcast_module(o)
    flat = torch.cat([t.reshape(-1).float() for o in objs for t in _module_tensors(o)])
    gathered = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    q.put((rank, (flat.numel() > 1_000_000, all(torch.equal(g, gathered[0]) for g in gathered))))
    dist.destroy_process_group()


def test_broadcast_bench_scene_gloo_world2():
    res = _spawn(_bench_scene_broadcast_worker, 2)
    assert res == {0: (True, True), 1: (True, True)}


def test_runtime_options_roundtrip():
    """nrt_set_option / nrt_get_option / nrt_reset_options (include/nrt.h "Runtime options"):
    named, validated, restored -- the library reads no environment variables."""
    import os
    from neural_raytracing_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libnrt_hip.so not built")
    lib = _lib.load()
    names = ["ring16", "ring32", "normals16", "scan_best32", "march_blocks", "shade_program",
             "nerf_fused", "max_waves", "shade_ring", "normals_ring", "xcd_lines",
             "mixed_refine_d", "mixed_refine_s", "mixed_restart", "mixed_drift",
             "ring_occlusion", "mixed_zone", "bwd_colsplit", "bwd_ring", "march_queue", "train_save", "wgrad_tile",
             "march_stage"]
    defaults = {n: _lib.get_option(n) for n in names}
    assert defaults == {"ring16": 1, "ring32": 1, "normals16": 1, "scan_best32": 1,
                        "march_blocks": 0, "shade_program": 1, "nerf_fused": 1, "max_waves": 0,
                        "shade_ring": 1, "normals_ring": 1, "xcd_lines": 0,
                        "mixed_refine_d": 20000, "mixed_refine_s": 2000, "mixed_restart": 1,
                        "mixed_drift": 0, "ring_occlusion": 1, "mixed_zone": 500000,
                        "bwd_colsplit": 1, "bwd_ring": 1, "march_queue": 2,
                        "train_save": 1, "wgrad_tile": 0, "march_stage": 1}
    with _lib.options(march_blocks=5, ring32=0):
        assert _lib.get_option("march_blocks") == 5 and _lib.get_option("ring32") == 0
    assert _lib.get_option("march_blocks") == 0 and _lib.get_option("ring32") == 1
    with pytest.raises(_lib.NrtError):
        _lib.set_option("no_such_option", 1)
    with pytest.raises(_lib.NrtError):
        _lib.set_option("ring16", -1)
    _lib.set_option("normals16", 0)
    assert lib.nrt_reset_options() == 0
    assert _lib.get_option("normals16") == 1
    src = open(os.path.join(os.path.dirname(_lib.HERE), "include", "nrt.h")).read()
    for n in names:
        assert f'"{n}"' in src


class _StubCameras:
    """A camera batch for the sharding tests: rays_tile gives [N, W, H, 1, 6] rays whose
    components encode (view, row, column) plus the torch.rand jitter the NeRF camera draws
    (cameras.py:45-48), so a frame shows whether each tile saw its single-process draws."""

    def __init__(self, n=2):
        self.n = n

    def __len__(self):
        return self.n

    def rays_tile(self, x0, y0, W, H, size, with_noise=False, positions=None):
        v = torch.arange(self.n).view(-1, 1, 1).float().expand(self.n, W, H)
        r = (x0 + torch.arange(W)).view(1, -1, 1).float().expand(self.n, W, H)
        c = (y0 + torch.arange(H)).view(1, 1, -1).float().expand(self.n, W, H)
        jit = torch.rand(2, W, H) if with_noise else torch.zeros(2, W, H)
        rays = torch.stack([v, r, c, jit[0].expand(self.n, W, H), jit[1].expand(self.n, W, H),
                            torch.zeros(self.n, W, H)], dim=-1)
        return rays.reshape(self.n, W, H, 1, 6)


def _stub_fused_path(monkeypatch, rendered):
    """Replace the HIP launches of pathtrace's fused tile path (render.direct_kernels and the
    tile composite) by torch stand-ins: a ray's colour is (view + 1000 scan jitter, row + u,
    column + v) -- what the real kernels would make of these rays is beside the point; the
    test checks which tiles each rank renders and that every tile sees its own draws."""
    import types
    from neural_raytracing_amd.pathtracer import main, render
    from neural_raytracing_amd.pathtracer.integrators import Direct

    def direct_kernels(direct, shapes, rays_flat, bsdf, lights, scan_groups=None, w_isect=False,
                       scan_draws=None):
        G = scan_groups or 1
        per = rays_flat.shape[0] // G
        scan = torch.tensor(scan_draws).repeat_interleave(per).view(-1, 1)
        rgb = rays_flat[:, :3] + rays_flat[:, 3:6] * torch.tensor([0.0, 1.0, 1.0]) + \
            1000 * scan * torch.tensor([1.0, 0.0, 0.0])
        rendered.extend(sorted(set(rays_flat[:, 1].long().tolist())))
        return types.SimpleNamespace(rgb=rgb)

    def composite_slice(b, sl, N, W, H, with_alpha, background, out, X0, Y0):
        out[:, X0:X0 + W, Y0:Y0 + H, :3] = b.rgb[sl].view(N, W, H, 3)

    monkeypatch.setattr(render, "direct_kernels", direct_kernels)
    monkeypatch.setattr(render, "composite_slice", composite_slice)
    monkeypatch.setattr(main, "is_hip_sdf", lambda sdf: True)
    shapes = types.SimpleNamespace(sdf=object(), dist=2.2)
    direct = Direct()
    direct.training = True  # primary rays: every tile draws its scan jitter
    return main, shapes, direct


def _pathtrace_frame(main, shapes, direct, seed, views=2, size=48, chunk=8, **kw):
    import random
    torch.manual_seed(seed)
    random.seed(seed)
    out, _ = main.pathtrace(shapes, None, _StubCameras(views), direct, bsdf=None, size=size,
                            chunk_size=chunk, bundle_size=1, background=0.25, silent=True,
                            device="cpu", with_noise=1e-3, **kw)
    return out, random.random(), torch.rand(1)  # the RNG states after the frame


def _pathtrace_shard_worker(rank, world, port, q):
    import torch.distributed as dist
    from _pytest.monkeypatch import MonkeyPatch
    from neural_raytracing_amd.pathtracer.render import tile_shard_rows
    mpatch = MonkeyPatch()
    rendered = []
    main, shapes, direct = _stub_fused_path(mpatch, rendered)
    cases = [(48, 8), (64, 64)]  # tiles of 8 rows; one 64-row tile (test_nerf: chunk == size)
    want = [_pathtrace_frame(main, shapes, direct, 5, size=s, chunk=c, shard=False)
            for s, c in cases]  # before any process group
    n_single = len(set(rendered))
    rendered.clear()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    res = []
    for (s, c), w in zip(cases, want):
        rendered.clear()
        got = _pathtrace_frame(main, shapes, direct, 5, size=s, chunk=c)  # automatic: sharded
        mine = sorted(set(rendered))
        res.append((bool(torch.equal(got[0], w[0])), got[1] == w[1], bool(torch.equal(got[2], w[2])),
                    mine == sorted(tile_shard_rows(s, c, rank, world)), len(mine)))
    # ranks asking for different frames (here: different camera counts) each render their own
    rendered.clear()
    own = _pathtrace_frame(main, shapes, direct, 6, views=2 + rank)
    n_own = len(set(rendered))
    q.put((rank, (res, n_single, n_own, tuple(own[0].shape))))
    dist.destroy_process_group()
    mpatch.undo()


def test_pathtrace_row_tile_shard_gloo_world2():
    """pathtrace under a 2-rank process group (gloo): each rank renders its row slices of every
    tile only (render.tile_slice_rows), the all-gather assembles the frame, and the frame and
    both RNG states afterwards equal the single-process render's (main.py:54-90, the parallelism
    TODO at :60) -- for 8-row tiles and for the one-tile frame test_nerf asks for
    (chunk_size == size, training_utils.py:325), where each rank renders half the rows."""
    res = _spawn(_pathtrace_shard_worker, 2)
    for rank in (0, 1):
        cases, n_single, n_own, shape = res[rank]
        for frame_eq, py_rng_eq, torch_rng_eq, rows_ok, n_rows in cases:
            assert frame_eq and py_rng_eq and torch_rng_eq and rows_ok, res
        assert cases[0][4] == 24 and cases[1][4] == 32  # half the rows of each frame
        assert n_single == 64  # unsharded: every row
        assert n_own == 48 and shape == (2 + rank, 48, 48, 3)  # different frames: not sharded


def test_pathtrace_shard_off_without_process_group(monkeypatch):
    """No process group: the whole frame, and shard=True is an error."""
    from neural_raytracing_amd import NrtError
    rendered = []
    main, shapes, direct = _stub_fused_path(monkeypatch, rendered)
    out, _, _ = _pathtrace_frame(main, shapes, direct, 3)
    assert sorted(set(rendered)) == list(range(48)) and out.shape == (2, 48, 48, 3)
    with pytest.raises(NrtError):
        _pathtrace_frame(main, shapes, direct, 3, shard=True)


def _stub_nerfle():
    """A NeRFLE whose forward is a torch stand-in with the reference's draw (one random.random()
    per call for the depths, nerf.py:178): what pathtrace's NeRFReproduce shard must preserve."""
    from neural_raytracing_amd.pathtracer.shapes import NeRFLE

    class StubNeRF(NeRFLE):
        def forward(self, rays, lights):
            u = random.random()
            return rays[..., :3] + u * rays[..., 3:6]

    import random
    return StubNeRF(device="cpu")


def _nerf_frame(nerf, seed, **kw):
    import random
    from neural_raytracing_amd.pathtracer import main
    from neural_raytracing_amd.pathtracer.integrators import NeRFReproduce
    torch.manual_seed(seed)
    random.seed(seed)
    with torch.no_grad():  # as the scripts render (training_utils.py:319)
        out, _ = main.pathtrace(nerf, None, _StubCameras(2), NeRFReproduce(), size=32,
                                chunk_size=32, bundle_size=1, background=0, device="cpu",
                                with_noise=1e-3, **kw)
    return out, random.random(), torch.rand(1)


def _nerf_shard_worker(rank, world, port, q):
    import torch.distributed as dist
    torch.manual_seed(0)
    nerf = _stub_nerfle()
    seen = []
    fwd = nerf.forward

    def spy(rays, lights):
        seen.append(rays.shape)
        return fwd(rays, lights)
    nerf.forward = spy
    want = _nerf_frame(nerf, 7, shard=False)
    seen.clear()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    got = _nerf_frame(nerf, 7)
    q.put((rank, (bool(torch.equal(got[0], want[0])), got[1] == want[1],
                  bool(torch.equal(got[2], want[2])), [tuple(s) for s in seen])))
    dist.destroy_process_group()


def test_pathtrace_nerf_reproduce_shard_gloo_world2():
    """NeRFReproduce over a NeRFLE (cfg5's path, nerf.py:175-214) shards like the fused tiles:
    each of 2 ranks runs the NeRF on half the rows of the one 32-row tile, with the same depth
    draw, and the gathered frame and RNG states equal the single-process render's."""
    res = _spawn(_nerf_shard_worker, 2)
    for rank in (0, 1):
        frame_eq, py_eq, torch_eq, seen = res[rank]
        assert frame_eq and py_eq and torch_eq, res
        assert seen == [(2, 16, 32, 1, 6)], seen
