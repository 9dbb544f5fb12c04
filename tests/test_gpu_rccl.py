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
