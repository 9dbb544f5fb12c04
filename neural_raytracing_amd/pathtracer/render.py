"""Fused render path: one tile = nrt_raygen -> nrt_sdf_intersect -> nrt_shade_direct ->
nrt_composite, all stream-ordered on torch's current stream, with buffers reused across calls.

``pathtrace`` / ``pathtrace_sample`` (main.py) route ``Direct`` and ``NeRFIntegrator(Direct)``
tiles here; ``render_rows`` renders an arbitrary set of image rows (the multi-GPU row shard,
SURVEY §8e).  Semantics are the reference's Direct.sample (integrators.py:156-206) +
NeRFIntegrator (integrators.py:249-257) + the tile composite (main.py:85-90) for bundle_size 1.
"""
import ctypes
import random

import torch

from .. import _lib
from .integrators import Direct, NeRFIntegrator
from .integrators.integrators import _bsdf_handle, _emitter_mode, _light_handle
from .shapes.sdfs import sdf_handle


def fused_integrator(integrator):
    """(direct, with_alpha) if the integrator is Direct or NeRFIntegrator(Direct), else None."""
    if isinstance(integrator, NeRFIntegrator) and type(integrator.sub_integrator) is Direct:
        return integrator.sub_integrator, True
    if type(integrator) is Direct:
        return integrator, False
    return None


class _Buffers:
    def __init__(self, P, nb, device):
        f = dict(device=device)
        self.P = P
        self.t = torch.empty(P, **f)
        self.hit = torch.empty(P, dtype=torch.uint8, **f)
        self.p = torch.empty(P, 3, **f)
        self.n = torch.empty(P, 3, **f)
        self.raw = torch.empty(P, 3, **f)
        self.wi = torch.empty(P, 3, **f)
        self.thr = torch.empty(P, **f)
        self.rgb = torch.empty(P, 3, **f)
        self.weights = torch.empty(P, max(nb, 1), **f)
        self.hit_idx = torch.empty(max(P, 1), dtype=torch.int32, **f)
        self.hit_count = torch.zeros(1, dtype=torch.int32, **f)
        self.ws = None


_BUFS = {}


def _buffers(P, nb, device):
    key = (P, nb, str(device))
    b = _BUFS.get(key)
    if b is None:
        _BUFS.clear()  # keep one set alive
        b = _BUFS[key] = _Buffers(P, nb, device)
    return b


def direct_kernels(direct, shapes, rays_flat, bsdf, lights, scan_groups=None, w_isect=False,
                   scan_draws=None):
    """Run intersect + shade on flat rays [P,6]; returns the buffer set (rgb zero on misses).
    scan_groups: for batched tiles, the number of tiles G; ray r belongs to tile r // (P // G)
    and each tile draws its own scan jitter (random.random(), sdfs.py:236), in tile order.
    scan_draws: those G uniforms already drawn by the caller (render_tiles draws every tile's,
    the ones a rank does not render included, so the frame does not depend on the world size).
    w_isect: Direct's emitter sample with a shadow ray (True) or a learned occlusion MLP, as
    Direct.sample picks it (integrators.py:161-166)."""
    P = rays_flat.shape[0]
    dev = rays_flat.device
    nb = len(getattr(bsdf, "bsdfs", [bsdf]))
    b = _buffers(P, nb, dev)
    lib = _lib.load(require_device=True)
    sh = sdf_handle(shapes.sdf)
    ws_bytes = lib.nrt_intersect_workspace_bytes(sh, P)
    if b.ws is None or b.ws.numel() < ws_bytes:
        b.ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    primary = bool(direct.training)
    scan_max_t = 0.0
    groups = None
    if primary:
        dist = getattr(shapes, "dist", 2.2)
        if scan_draws is None:
            scan_draws = [random.random() for _ in range(scan_groups or 1)]
        if scan_groups is None:
            scan_max_t = dist + scan_draws[0] * (2 / 128)
        else:
            groups = torch.tensor([dist + u * (2 / 128) for u in scan_draws],
                                  dtype=torch.float64).to(dev, non_blocking=True)
    mp = _lib.MarchParams(int(shapes.max_steps), float(shapes.epsilon), 10.0, int(primary),
                          float(scan_max_t), _lib.precision_code())
    if groups is not None:
        mp.scan_max_t_groups = groups.data_ptr()
        mp.group_rays = P // scan_groups
    s = _lib.stream()
    _lib.call("nrt_sdf_intersect", sh, _lib.ptr(rays_flat), P, ctypes.byref(mp), _lib.ptr(b.t),
              _lib.ptr(b.hit), _lib.ptr(b.p), _lib.ptr(b.n), _lib.ptr(b.raw), _lib.ptr(b.wi),
              _lib.ptr(b.thr) if primary else None, _lib.ptr(b.hit_idx), _lib.ptr(b.hit_count),
              _lib.ptr(b.ws), s)
    if not primary:
        b.thr.zero_()
    b.rgb.zero_()
    shadow, occ = _emitter_mode(w_isect)
    if shadow:
        # nrt_shade_direct_shadowed / _learned_occ over the batch's hit list: the shadow march
        # runs on the ring engines once for every tile of the batch
        args = (_lib.ptr(b.p), _lib.ptr(b.n), _lib.ptr(b.wi), _lib.ptr(b.hit_idx),
                _lib.ptr(b.hit_count), P, _lib.ptr(b.rgb), None)
        Direct._shade(shapes, bsdf, lights, shadow, occ, args, P, dev)
        return b
    _lib.call("nrt_shade_direct", _bsdf_handle(bsdf), _light_handle(lights), _lib.ptr(b.p),
              _lib.ptr(b.n), _lib.ptr(b.wi), _lib.ptr(b.hit_idx), _lib.ptr(b.hit_count), P,
              _lib.ptr(b.rgb), None, _lib.precision_code(), s)
    return b


def composite(b, N, W, H, with_alpha, background, out, X0, Y0):
    """Write the tile into out[N, IW, IH, C] (main.py:85-90): Direct fills misses with the
    background, NeRFIntegrator appends sigmoid(throughput) and never fills."""
    _lib.call("nrt_composite", _lib.ptr(b.rgb), _lib.ptr(b.thr), _lib.ptr(b.hit), N, W, H,
              int(with_alpha), int(not with_alpha), float(background), _lib.ptr(out),
              out.shape[1], out.shape[2], out.shape[3], int(X0), int(Y0), _lib.stream())


def render_tile(fused, shapes, lights, cameras, bsdf, out, x0, y0, chunk, size, with_noise,
                background, ox=0, oy=0):
    direct, with_alpha = fused
    rays = cameras.rays_tile(x0, y0, chunk, chunk, size, with_noise)
    N = rays.shape[0]
    b = direct_kernels(direct, shapes, rays.reshape(-1, 6), bsdf, lights)
    composite(b, N, chunk, chunk, with_alpha, background, out, x0 - ox, y0 - oy)
    return b


# rays per batched launch of pathtrace's fused tiles: 4M rays keep every buffer (rays, hits,
# points, normals, frames, rgb: ~100 B a ray) under half a GB while filling the persistent marches
# (65,536 ray slots per round on 256 CUs) many times over
MAX_BATCH_RAYS = 1 << 22


def render_tiles(fused, shapes, lights, cameras, bsdf, out, tiles, chunk, size, with_noise,
                 background, ox=0, oy=0, rows=None):
    """pathtrace's fused tile loop (main.py:63-90) as few launch chains as possible: the rays of
    consecutive tiles are generated tile by tile (same camera-jitter draws, same order), marched,
    scanned and shaded in one nrt_sdf_intersect + nrt_shade_direct over all of them -- each tile
    keeps its own scan jitter (nrt_march_params.scan_max_t_groups) -- and composited tile by
    tile.  Equal to rendering the tiles one at a time; the GPU sees up to MAX_BATCH_RAYS rays per
    launch instead of chunk_size^2.
    rows: tile-local rows (a rank's row slices under torch.distributed, tile_slice_rows) -- every
    tile's rays are generated whole (its camera jitter drawn as in a single-process render), then
    only those rows of it are marched and shaded, and tile (x0, y0) lands in `out` -- the rank's
    slab [N, bands x len(rows), height, C] -- at rows (x0 // chunk) * len(rows) ... ; every tile's
    scan jitter is drawn in tile order, so each rendered ray sees the numbers it would see in a
    single-process render."""
    direct, with_alpha = fused[:2]
    w_isect = fused[2] if len(fused) > 2 else False  # pathtrace's w_isect (main.py _fused)
    N = len(cameras)
    R = chunk if rows is None else len(rows)
    per_tile = N * R * chunk
    dev = out.device
    sel = None if rows is None else torch.tensor(list(rows), dtype=torch.long, device=dev)
    step = max(1, MAX_BATCH_RAYS // max(per_tile, 1))
    primary = bool(direct.training)
    # the scan jitter of every tile (sdfs.py:236) in tile order: python's RNG, independent of the
    # camera's torch draws, so drawing them up front leaves both sequences as the per-tile loop
    scan = [random.random() for _ in tiles] if primary else None
    for t0 in range(0, len(tiles), step):
        batch = range(t0, min(t0 + step, len(tiles)))
        rays = torch.empty(len(batch), per_tile, 6, device=dev)
        for k, ti in enumerate(batch):
            x0, y0 = tiles[ti]
            r = cameras.rays_tile(x0, y0, chunk, chunk, size, with_noise)
            if sel is not None:
                r = r.index_select(1, sel)  # [N, chunk rows, chunk cols, ...] -> this rank's rows
            rays[k] = r.reshape(-1, 6)
        if per_tile == 0:
            continue  # (no rows of these tiles here: their draws are taken, nothing to render)
        b = direct_kernels(direct, shapes, rays.reshape(-1, 6), bsdf, lights,
                           scan_groups=len(batch) if len(batch) > 1 else None, w_isect=w_isect,
                           scan_draws=[scan[ti] for ti in batch] if primary else None)
        for k, ti in enumerate(batch):
            x0, y0 = tiles[ti]
            X0 = x0 - ox if rows is None else ((x0 - ox) // chunk) * R
            composite_slice(b, slice(k * per_tile, (k + 1) * per_tile), N, R, chunk, with_alpha,
                            background, out, X0, y0 - oy)


def composite_slice(b, sl, N, W, H, with_alpha, background, out, X0, Y0):
    """composite() of the rays sl of a batched buffer set (one W x H tile, [N, W, H] order)."""
    _lib.call("nrt_composite", _lib.ptr(b.rgb[sl]), _lib.ptr(b.thr[sl]), _lib.ptr(b.hit[sl]),
              N, W, H, int(with_alpha), int(not with_alpha), float(background),
              _lib.ptr(out), out.shape[1], out.shape[2], out.shape[3], int(X0), int(Y0),
              _lib.stream())


def tile_slice_rows(chunk, rank, world):
    """Tile-local rows of `rank` under pathtrace's row sharding: the rows of every chunk-row tile
    are dealt round-robin, one row at a time, so a single chunk_size == size tile (test_nerf's
    call, training_utils.py:325) spreads over every rank and the ranks' row counts differ by at
    most one per tile (a centred object's cost spreads evenly too)."""
    return list(range(rank, chunk, world))


def tile_shard_rows(width, chunk, rank, world):
    """Image rows of `rank` (tile_slice_rows of every band of chunk rows), in slab order."""
    local = tile_slice_rows(chunk, rank, world)
    return [x0 + r for x0 in range(0, width, chunk) for r in local]


def shard_of(cameras, size, width, chunk, background, group=None, shard=None):
    """(rank, world) when pathtrace should render a row shard (images shard by pixel
    rows, one all-gather at frame end), else None.  shard: None = automatic (a process group of
    more than one rank, and every rank asks for the same frame -- checked with one small
    all-gather of the cameras' corner rays and the frame parameters, so ranks that render
    different views each keep rendering their own full frame), False = never, True = always (an
    error if the ranks' frames differ or the frame cannot be sharded).  Once a group of several
    ranks exists, every rank takes part in the fingerprint all-gather whatever its own
    parameters, so ranks that disagree about the frame fall back together instead of hanging."""
    if shard is False:
        return None
    try:
        import torch.distributed as dist
    except ImportError:
        return None
    if not (dist.is_available() and dist.is_initialized()):
        if shard:
            raise _lib.NrtError("pathtrace(shard=True) needs an initialised torch.distributed "
                                "process group")
        return None
    world = dist.get_world_size(group)
    if world <= 1 and not shard:
        return None  # (shard=True at one rank runs the sharded path: the RCCL test's case)
    rank = dist.get_rank(group)
    shardable = width % chunk == 0 and chunk >= world
    if shard and not shardable:
        raise _lib.NrtError(f"pathtrace(shard=True): width {width} must be a multiple of "
                            f"chunk_size {chunk} and chunk_size >= the {world} ranks")
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend(group) == "nccl" else torch.device("cpu")
    # a fixed-length fingerprint (the collective needs equal shapes on every rank): the frame
    # parameters, whether this rank can shard it, and three moments of the cameras' corner rays
    corners = torch.cat([cameras.rays_tile(x, y, 1, 1, size, False).reshape(-1).double().cpu()
                         for x, y in ((0, 0), (width - 1, size - 1))])
    w = torch.arange(1, corners.numel() + 1, dtype=torch.float64)
    key = torch.tensor([float(len(cameras)), float(size), float(width), float(chunk),
                        float(background), float(shardable), float(corners.sum()),
                        float((corners * w).sum()), float((corners * corners).sum())],
                       dtype=torch.float64).to(dev)
    keys = [torch.empty_like(key) for _ in range(world)]
    dist.all_gather(keys, key, group=group)
    same = all(torch.equal(k, keys[0]) for k in keys)
    if not same:
        if shard:
            raise _lib.NrtError("pathtrace(shard=True): the ranks asked for different frames")
        return None
    if not shardable:
        return None
    return rank, world


def gather_tile_shard(slab, out, chunk, rank, world, group=None):
    """After each rank rendered its row slices (tile_shard_rows) into its slab
    [N, bands x rows, height, C], every rank's rows into every rank's `out` [N, width, height, C]
    by one all-gather (RowGather over the ranks' tile_shard_rows)."""
    width = out.shape[1]
    shards = tuple(tuple(tile_shard_rows(width, chunk, r, world)) for r in range(world))
    return gather_rows(slab, width, rank, world, chunk, out=out, group=group, shards=shards)


def row_shard(size, rank, world, tile_rows=16):
    """Image rows of `rank` when tiles of `tile_rows` rows are dealt round-robin."""
    rows = []
    for t0 in range(rank * tile_rows, size, world * tile_rows):
        rows.extend(range(t0, min(t0 + tile_rows, size)))
    return rows


class RowRenderer:
    """Renders a fixed set of rows of every camera of a NeRF/DTU camera batch.

    ``positions`` ([R, size, 2], u = column, v = row) are built once; each ``render`` call is
    raygen + intersect + shade + composite into ``self.image`` [N, R, size, C].
    """

    def __init__(self, shapes, lights, cameras, integrator, bsdf, size, rows, background=0.0,
                 with_noise=1e-3, device="cuda"):
        fused = fused_integrator(integrator)
        if fused is None:
            raise _lib.NrtError("RowRenderer supports Direct and NeRFIntegrator(Direct)")
        self.fused = fused
        self.shapes, self.lights, self.cameras, self.bsdf = shapes, lights, cameras, bsdf
        self.size = size
        self.rows = list(rows)
        self.background = background
        self.with_noise = with_noise
        R = len(self.rows)
        v = torch.tensor(self.rows, dtype=torch.float32, device=device)[:, None].expand(R, size)
        u = torch.arange(size, dtype=torch.float32, device=device)[None, :].expand(R, size)
        self.positions = torch.stack([u, v], dim=-1).contiguous()
        dims = 4 if fused[1] else 3
        self.image = torch.empty(len(cameras), R, size, dims, device=device)

    def render(self):
        direct, with_alpha = self.fused
        R = len(self.rows)
        rays = self.cameras.rays_tile(0, 0, R, self.size, self.size, self.with_noise,
                                      positions=self.positions)
        N = rays.shape[0]
        b = direct_kernels(direct, self.shapes, rays.reshape(-1, 6), self.bsdf, self.lights)
        composite(b, N, R, self.size, with_alpha, self.background, self.image, 0, 0)
        return self.image


class RowGather:
    """The multi-GPU frame assembly: every rank's row slab ([N, R_rank, W, C]) ->
    the full [N, size, W, C] frame on every rank, by one ``all_gather_into_tensor`` of
    equal-sized (padded) slabs -- the only collective of the path (RCCL over xGMI on the box,
    gloo in the CPU tests).  The shard table, padded staging buffers and per-rank row-index
    tensors are built once per frame shape, not per step."""

    def __init__(self, size, rank, world, tile_rows, shape, device, dtype=torch.float32,
                 group=None, shards=None):
        N, W, C = shape
        self.size, self.rank, self.world, self.group = size, rank, world, group
        # shards: every rank's image rows in its slab's order (default: row_shard's tiles)
        self.shards = [list(s) for s in shards] if shards is not None else \
            [row_shard(size, r, world, tile_rows) for r in range(world)]
        self.max_rows = max(len(s) for s in self.shards)
        self.slab = torch.zeros(N, self.max_rows, W, C, device=device, dtype=dtype)
        self.buf = torch.empty(world * N, self.max_rows, W, C, device=device, dtype=dtype)
        self.idx = [torch.tensor(rows, device=device, dtype=torch.long) for rows in self.shards]

    def __call__(self, local, out):
        import torch.distributed as dist
        R = local.shape[1]
        if R != len(self.shards[self.rank]):
            raise ValueError(f"rank {self.rank} renders {R} rows, its shard has "
                             f"{len(self.shards[self.rank])}")
        self.slab[:, :R].copy_(local)
        dist.all_gather_into_tensor(self.buf, self.slab, group=self.group)
        buf = self.buf.view(self.world, *self.slab.shape)
        for r, idx in enumerate(self.idx):
            out.index_copy_(1, idx, buf[r, :, :idx.numel()])
        return out


_GATHERS = {}
_GATHERS_MAX = 4  # RowGathers (each holds world x slab staging buffers) kept, least recent out


def clear_gathers():
    """Drop the cached RowGathers (call after destroy_process_group)."""
    _GATHERS.clear()


def gather_rows(local, size, rank, world, tile_rows, out=None, group=None, shards=None):
    """All-gather every rank's row slab ([N, R_rank, W, C]) and assemble [N, size, W, C]
    (a RowGather per frame shape / device / group from a small LRU; a caller that renders many
    shapes should own its RowGather, as bench.make_step does).  shards: the ranks' row lists
    (tuple of tuples), default row_shard's tiles of tile_rows."""
    N, _, W, C = local.shape
    key = (size, rank, world, tile_rows, N, W, C, local.device, local.dtype, group, shards)
    g = _GATHERS.pop(key, None)
    if g is None:
        g = RowGather(size, rank, world, tile_rows, (N, W, C), local.device, local.dtype, group,
                      shards=shards)
    _GATHERS[key] = g  # most recent last
    while len(_GATHERS) > _GATHERS_MAX:
        _GATHERS.pop(next(iter(_GATHERS)))
    if out is None:
        out = local.new_empty(N, size, W, C)
    return g(local, out)


def broadcast_module(module, src=0, group=None):
    """Make every rank's copy of `module` (its parameters and buffers) equal to rank `src`'s,
    in place: a model loaded from file on one rank (or initialised from different seeds) is
    replicated before the row-sharded render, so every shard is rendered by the same weights.
    Tensors are coalesced by dtype into one flat broadcast each (no per-parameter collective)."""
    import torch.distributed as dist
    uniq = _module_tensors(module)
    # an NCCL (RCCL) group moves device tensors only: CPU tensors (e.g. PointLights' falloff
    # coefficients) are staged through the current device and copied back
    stage = dist.get_backend(group) == "nccl"
    by_dtype = {}
    for t in uniq:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    with torch.no_grad():
        for (dtype, device), ts in by_dtype.items():
            flat = torch.cat([t.reshape(-1) for t in ts])
            if stage and flat.device.type != "cuda":
                flat = flat.to(torch.device("cuda", torch.cuda.current_device()))
            dist.broadcast(flat, src=src, group=group)
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n
    return module


def _module_tensors(obj):
    """Every tensor that defines `obj`'s render: parameters, buffers and plain tensor attributes
    (basis_p of the MLPs) of an nn.Module tree; for an SDF shape (shapes.SDF, a plain class
    with parameters() only, sdfs.py:89-109) those of its ``sdf`` module (SPHERE_SDF has none);
    for any other object its parameters()."""
    if not isinstance(obj, torch.nn.Module):
        inner = getattr(obj, "sdf", None)
        if isinstance(inner, torch.nn.Module):
            return _module_tensors(inner)
        params = getattr(obj, "parameters", None)
        return _uniq(list(params()) if params is not None else [])
    tensors = list(obj.parameters()) + list(obj.buffers())
    for m in obj.modules():
        for v in vars(m).values():
            if isinstance(v, torch.Tensor) and not isinstance(v, torch.nn.Parameter):
                tensors.append(v)
    return _uniq(tensors)


def _uniq(tensors):
    seen, uniq = set(), []
    for t in tensors:
        if id(t) not in seen:
            seen.add(id(t))
            uniq.append(t)
    return uniq
