"""The multi-GPU path on the RCCL (``nccl``) backend, in-process at world size 1 (SURVEY §8e;
the reference's per-GPU loop is main.py:54-90).  The 8-GPU node is the driver's; this runs the
same collectives bench.py's N > 1 branch issues -- the scene broadcast (with a PointLights whose
falloff tensors live on the host, staged through the device), the row-slab all-gather of a
10-row-tile shard and the MAX all-reduce of the step time -- on the real scene objects, and
requires the gathered frame to equal the single-process RowRenderer frame bit for bit.  The
rendezvous is a TCP store on 127.0.0.1; nothing is exec'd."""
import random
import socket

import pytest
import torch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture
def nccl_group():
    import torch.distributed as dist
    from neural_raytracing_amd.pathtracer.render import clear_gathers
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=dev)
    try:
        yield dev
    finally:
        clear_gathers()
        dist.destroy_process_group()


def _frame(render, seed):
    torch.manual_seed(seed)
    random.seed(seed)
    return render().clone()


@pytest.mark.gpu
def test_rccl_scene_broadcast_row_gather_and_max(nccl_group):
    import torch.distributed as dist
    import bench
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer.render import (RowRenderer, _module_tensors,
                                                         broadcast_module, row_shard)
    dev = nccl_group
    assert dist.get_backend() == "nccl"
    set_precision("fp32")
    size, samples, tile = 96, 16, 10
    scene = bench.build_scene(dev, samples, light_gain=bench.LIGHT_GAIN)
    other = bench.build_other_scene("colocate", dev, samples)
    objs = [scene["shape"], scene["bsdf"], scene["lights"], other["lights"], other["shape"]]
    before = [t.detach().clone() for o in objs for t in _module_tensors(o)]
    assert any(t.device.type == "cpu" for t in before)  # the point light's falloff: staged
    for o in objs:
        broadcast_module(o)
    after = [t for o in objs for t in _module_tensors(o)]
    assert all(torch.equal(a.detach(), b) and a.device == b.device for a, b in zip(after, before))

    pt = scene["pt"]
    focal = float(0.5 * size / torch.tan(torch.tensor(0.5 * 0.6911)).item())
    cameras = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev), focal=focal,
                                    device=dev)
    rows = row_shard(size, 0, 1, tile)
    assert rows == list(range(size))
    with torch.no_grad():
        rr = RowRenderer(scene["shape"], scene["lights"], cameras, scene["integrator"],
                         scene["bsdf"], size, rows, background=0.0, with_noise=1e-3, device=dev)
        want = _frame(rr.render, 7)
        step = bench.make_step(rr.render, rows, size, 0, 1, tile, dev, gather=True)
        got = None
        for _ in range(2):  # the RowGather's cached staging buffers, twice
            got = _frame(step, 7)
        torch.cuda.synchronize()
    assert got.shape == (1, size, size, 4)
    assert torch.equal(got, want)
    assert float((want[..., 3] > 0.5).float().mean()) > 0.05  # a frame with hits in it
    assert bench.max_over_ranks(1.25, 1, dev, force=True) == 1.25


@pytest.mark.gpu
def test_rccl_row_gather_of_uneven_shards(nccl_group):
    """RowGather over the nccl group with 10-row tiles of a side that is not a multiple of the
    tile: the padded slab, the all-gather and the index copy on the device."""
    from neural_raytracing_amd.pathtracer.render import gather_rows, row_shard
    dev = nccl_group
    size, tile, N, W = 57, 10, 2, 9
    full = torch.arange(N * size * W * 4, dtype=torch.float32, device=dev).reshape(N, size, W, 4)
    rows = row_shard(size, 0, 1, tile)
    got = gather_rows(full[:, rows].contiguous(), size, 0, 1, tile)
    assert torch.equal(got, full)


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [32, 64])
def test_rccl_pathtrace_sharded_equals_unsharded(nccl_group, chunk):
    """pathtrace through its row-tile shard path (shard=True: the frame fingerprint all-gather,
    the tile-band deal, every tile's jitter drawn in order, the RowGather all-gather of the
    bands) on the nccl group is bit-equal to the unsharded call (shard=False) with the same seeds
    -- test_nerf's call (training_utils.py:323-329, size 128 here)."""
    import bench
    from neural_raytracing_amd import set_precision
    dev = nccl_group
    set_precision("fp32")
    size = 128
    scene = bench.build_scene(dev, 24, light_gain=bench.LIGHT_GAIN)
    pt = scene["pt"]
    focal = float(0.5 * size / torch.tan(torch.tensor(0.5 * 0.6911)).item())
    cameras = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev), focal=focal,
                                    device=dev)
    outs = []
    for shard in (False, True):
        torch.manual_seed(3)
        random.seed(3)
        with torch.no_grad():
            img, _ = pt.pathtrace(scene["shape"], scene["lights"], cameras, scene["integrator"],
                                  bsdf=scene["bsdf"], size=size, chunk_size=chunk, bundle_size=1,
                                  background=0, silent=True, device=dev, shard=shard)
        outs.append((img.clone(), random.random(), torch.rand(1, device=dev).item()))
    torch.cuda.synchronize()
    (a, ra, ta), (b, rb, tb) = outs
    assert torch.equal(a, b) and ra == rb and ta == tb
    assert float((a[..., 3] > 0.5).float().mean()) > 0.05


def _simulated_shards(monkeypatch, world, render):
    """Run `render()` once per simulated rank of a `world`-rank group on this one GPU: shard_of
    answers (rank, world) and the all-gather is replaced by a scatter of the rank's own rows, so
    each pass renders only that rank's row slices of every tile (render.tile_slice_rows) with
    every draw of the frame taken.  Returns the frame assembled from the ranks' rows, the rows
    each rank rendered, and the RNG states after every pass."""
    from neural_raytracing_amd.pathtracer import render as R
    frame, rows_of, states = None, [], []
    for r in range(world):
        monkeypatch.setattr(R, "shard_of", lambda *a, _r=r, **k: (_r, world))

        def gather(slab, out, chunk, rank, w, group=None):
            rows = R.tile_shard_rows(out.shape[1], chunk, rank, w)
            rows_of.append(rows)
            out[:, torch.tensor(rows, device=out.device)] = slab
        monkeypatch.setattr(R, "gather_tile_shard", gather)
        torch.manual_seed(3)
        random.seed(3)
        with torch.no_grad():
            img = render()
        states.append((random.random(), torch.rand(1).item()))
        idx = torch.tensor(rows_of[-1], device=img.device)
        if frame is None:
            frame = torch.full_like(img, float("nan"))
        frame.index_copy_(img.dim() - 3, idx, img.index_select(img.dim() - 3, idx))
    monkeypatch.undo()
    return frame, rows_of, states


def _unsharded(render):
    torch.manual_seed(3)
    random.seed(3)
    with torch.no_grad():
        img = render()
    return img, (random.random(), torch.rand(1).item())


@pytest.mark.gpu
@pytest.mark.parametrize("scene_name,size,chunk,world", [
    ("nerf_synthetic", 128, 128, 8),   # test_nerf's one tile (chunk_size == size) over 8 ranks
    ("nerf_synthetic", 96, 32, 3),     # 3 ranks, 32-row tiles (11 / 11 / 10 rows a tile)
    ("dtu", 128, 64, 8),               # test_dtu's chunk = size / 2 (training_utils.py:460)
    ("nerfle", 64, 64, 4),             # NeRFReproduce over NeRFLE (cfg5's path)
])
def test_row_slice_shards_assemble_the_unsharded_frame(monkeypatch, scene_name, size, chunk,
                                                       world):
    """pathtrace's within-tile row shard on the real kernels: every simulated rank renders only
    its rows of each tile (half / an eighth of the rays of test_nerf's single 128-row tile), and
    the rows assembled from all ranks equal the unsharded frame bit for bit, with the same RNG
    states after each rank's pass (the draws of the whole frame are taken on every rank)."""
    import bench
    from neural_raytracing_amd import set_precision
    from neural_raytracing_amd.pathtracer import render as R
    dev = torch.device("cuda", 0)
    set_precision("fp32")
    pt = __import__("neural_raytracing_amd.pathtracer", fromlist=["pathtrace"])
    focal = float(0.5 * size / torch.tan(torch.tensor(0.5 * 0.6911)).item())
    nerf_cam = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev),
                                     focal=focal, device=dev)
    if scene_name == "nerf_synthetic":
        sc = bench.build_scene(dev, 24, light_gain=bench.LIGHT_GAIN)
        args = (sc["shape"], sc["lights"], nerf_cam, sc["integrator"])
        kw = dict(bsdf=sc["bsdf"])
    elif scene_name == "dtu":
        sc = bench.build_other_scene("dtu", dev, 24)
        args = (sc["shape"], sc["lights"], sc["cameras"], sc["integrator"])
        kw = dict(bsdf=sc["bsdf"])
    else:
        sc = bench.build_other_scene("nerfle", dev, 32)
        args = (sc["nerf"], sc["lights"], nerf_cam, sc["integrator"])
        kw = {}

    def render():
        img, _ = pt.pathtrace(*args, size=size, chunk_size=chunk, bundle_size=1, background=0,
                              silent=True, device=dev, **kw)
        return img.clone()
    want, want_state = _unsharded(render)
    got, rows_of, states = _simulated_shards(monkeypatch, world, render)
    assert sorted(r for rows in rows_of for r in rows) == list(range(size))
    assert max(len(r) for r in rows_of) - min(len(r) for r in rows_of) <= size // chunk
    assert all(s == want_state for s in states)
    assert torch.equal(got, want)
    if scene_name != "nerfle":
        assert float((want[..., 3] > 0.5).float().mean()) > 0.05  # a frame with hits in it
    else:
        assert float(want.abs().max()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("scene_name", ["nerf_synthetic_one_tile", "dtu", "nerfle"])
def test_rccl_pathtrace_sharded_one_rank_cases(nccl_group, scene_name):
    """shard=True on the nccl group at one rank (the fingerprint all-gather, the slab, the
    RowGather over tile_shard_rows) is bit-equal to shard=False for test_nerf's chunk_size ==
    size call, the DTU scene and NeRFReproduce over NeRFLE."""
    import bench
    from neural_raytracing_amd import set_precision
    dev = nccl_group
    set_precision("fp32")
    pt = __import__("neural_raytracing_amd.pathtracer", fromlist=["pathtrace"])
    size = 64
    focal = float(0.5 * size / torch.tan(torch.tensor(0.5 * 0.6911)).item())
    nerf_cam = pt.cameras.NeRFCamera(cam_to_world=bench.view_c2w(0, 1)[None].to(dev),
                                     focal=focal, device=dev)
    if scene_name == "nerf_synthetic_one_tile":
        sc = bench.build_scene(dev, 24, light_gain=bench.LIGHT_GAIN)
        args, kw = (sc["shape"], sc["lights"], nerf_cam, sc["integrator"]), dict(bsdf=sc["bsdf"])
    elif scene_name == "dtu":
        sc = bench.build_other_scene("dtu", dev, 24)
        args = (sc["shape"], sc["lights"], sc["cameras"], sc["integrator"])
        kw = dict(bsdf=sc["bsdf"])
    else:
        sc = bench.build_other_scene("nerfle", dev, 32)
        args, kw = (sc["nerf"], sc["lights"], nerf_cam, sc["integrator"]), {}
    outs = []
    for shard in (False, True):
        outs.append(_unsharded(lambda: pt.pathtrace(*args, size=size, chunk_size=size,
                                                    bundle_size=1, background=0, silent=True,
                                                    device=dev, shard=shard, **kw)[0].clone()))
    (a, sa), (b, sb) = outs
    assert torch.equal(a, b) and sa == sb
