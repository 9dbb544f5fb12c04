"""Renderer entry points (main.py:13-179) on the HIP path.

The tile loop, crop logic, background fill and the ``addition`` hook follow the reference;
each tile's rays come from ``nrt_raygen`` (cameras with ``rays_tile``) and the integrator runs
its HIP kernels.  Positions follow main.py:66-71: pixel (row x, col y) has u = y, v = x.
"""
import random

import torch

from .. import _lib
from .differentiable import needs_grad
from . import render as _render
from .render import fused_integrator
from .shapes.sdfs import is_hip_sdf
from .samplers import Sampler


def nothing(_):
    return None


def rand_uv(w, h, size):
    return random.randint(0, w - size), random.randint(0, h - size)


def _tile_rays(cameras, x0, y0, chunk, size, sampler, bundle_size, batch_dims, with_noise, device,
               positions=False):
    if hasattr(cameras, "rays_tile") and not positions:
        return cameras.rays_tile(x0, y0, chunk, chunk, size, with_noise)
    gx, gy = torch.meshgrid(torch.arange(x0, x0 + chunk, device=device, dtype=torch.float),
                            torch.arange(y0, y0 + chunk, device=device, dtype=torch.float),
                            indexing="ij")
    positions = torch.stack([gy, gx], dim=-1)
    return cameras.sample_positions(positions, sampler, bundle_size, size=size, N=batch_dims,
                                    with_noise=with_noise)


def _composite(out, values, mask, background, xs, ys, chunk, trim=0, H=None):
    """values [N, W, H, B, C] of a W x H tile (W = chunk rows, H = chunk columns unless given)
    into out[:, xs:xs + W, ys:ys + H] (main.py:85-90)."""
    H = chunk if H is None else H
    valid = mask.any(dim=-1)
    v = torch.mean(values, dim=-2)
    # v[~valid] = background, without the boolean scatter's host sync (and the scalar as a
    # wrapped number: a new_tensor would be a pageable host-to-device copy, a sync of its own)
    v = torch.where(valid.unsqueeze(-1), v, float(background))
    if trim:
        # the tile was rendered with a `trim`-pixel border; keep its interior.  The reference
        # writes this as v[trim:-trim, trim:-trim] (main.py:52), which slices v's camera and row
        # axes ([N, W, H, C]) -- a shape error at the assignment for every trim > 0 -- so the
        # intended crop of the two pixel axes is what runs here.
        v = v[:, trim:-trim, trim:-trim]
    out[:, xs:xs + chunk, ys:ys + H, :] = v


def _fused(integrator, cameras, w_isect, addition):
    """Direct / NeRFIntegrator(Direct) tiles go through the fused kernels when nothing needs the
    interaction record (addition is the default `nothing`); with w_isect (a shadow ray or a
    learned occlusion MLP, integrators.py:161-166) the tuple carries it to render_tiles."""
    if addition is not nothing or not hasattr(cameras, "rays_tile"):
        return None
    fused = fused_integrator(integrator)
    if fused is None or w_isect in (None, False):
        return fused
    return tuple(fused) + (w_isect,)


def _row_separable(integrator, shapes, addition, trim, bsdf, lights, w_isect):
    """Tiles whose rows can be rendered on different ranks with the single-process result: the
    integrator's draws per call must not depend on the number of rays -- NeRFReproduce over a
    NeRFLE (one random.random() per call for its depths, nerf.py:178) -- with no addition hook
    (it would see one rank's interaction), no trim border and no gradients (the all-gather is not
    differentiable).  The fused Direct tiles are the other sharded case (render_tiles)."""
    from .integrators import NeRFReproduce
    from .shapes.nerf import NeRFLE
    if addition is not nothing or trim or needs_grad(shapes, bsdf, lights, w_isect):
        return False
    return type(integrator) is NeRFReproduce and isinstance(shapes, NeRFLE)


# pathtrace(Path) marches all tiles of a frame in one batch (_path_tiles); False: tile by tile
BATCH_PATH = True


def _path_batchable(integrator, shapes, lights, cameras, addition, trim, bsdf, w_isect):
    """Path (integrators.py:275-354) without the coarse scan over a packed SDF, one light for
    every camera, no addition hook / trim / gradients: its tiles can run as one batch."""
    from .integrators import Path
    if not BATCH_PATH or type(integrator) is not Path or integrator.training:
        return False
    if addition is not nothing or trim or not hasattr(cameras, "rays_tile"):
        return False
    if not hasattr(shapes, "sdf") or not is_hip_sdf(shapes.sdf):
        return False
    if getattr(lights, "per_camera", lambda: None)() is not None:
        return False
    return not needs_grad(shapes, bsdf, lights, w_isect)


def _path_tiles(integrator, shapes, lights, cameras, bsdf, out, tiles, chunk, size, bundle_size,
                sampler, with_noise, background, w_isect, device):
    """pathtrace's tile loop for Path as few Path.sample calls as possible (SURVEY §8f rank 3,
    path_nerv.py:86-104: 200^2 in 100^2 tiles, 32 passes a frame): the rays of consecutive tiles
    (each tile's camera jitter drawn in tile order) are concatenated along the camera axis, so one
    primary march, one nrt_path_bounce and one compacted secondary march per bounce serve them
    all, and each tile is composited from its slice.  Per ray the same arithmetic as the tile
    loop; the sampler's draws are taken per batch instead of per tile (every draw is still one
    independent uniform per ray and component: the same distribution, a different stream --
    like the reference's torch.multinomial, which this path already replaces by an inverse CDF)."""
    N = len(cameras)
    per_tile = N * chunk * chunk
    step = max(1, _render.MAX_BATCH_RAYS // per_tile)
    it = None
    for t0 in range(0, len(tiles), step):
        batch = tiles[t0:t0 + step]
        rays = torch.cat([_tile_rays(cameras, x0, y0, chunk, size, sampler, bundle_size, N,
                                     with_noise, device) for x0, y0 in batch], dim=0)
        values, mask, it = integrator.sample(shapes, rays, bsdf=bsdf, lights=lights,
                                             sampler=sampler, w_isect=w_isect)
        for k, (x0, y0) in enumerate(batch):
            _composite(out, values[k * N:(k + 1) * N], mask[k * N:(k + 1) * N], background, x0,
                       y0, chunk)
    return it


def pathtrace(shapes, lights, cameras, integrator, bsdf=None, size=512, width=None, height=None,
              chunk_size=32, bundle_size=4, background=1, addition=nothing, sampler=Sampler(),
              silent=False, trim=0, device="cuda", squeeze_first=True, w_isect=False,
              with_noise=1e-3, shard=None, group=None):
    """main.py:13-93.  trim > 0 renders each tile with a trim-pixel border of extra rays
    (main.py:67-68) and keeps the tile's interior (see _composite).

    Multi-GPU (the parallelism TODO of main.py:60): under an initialised torch.distributed
    process group of several ranks that all ask for the same frame, every rank generates every
    tile's rays (the camera jitter and scan jitter drawn in the reference's order), marches and
    shades only its row slices of each tile -- the tile's rows dealt round-robin, one row at a
    time (render.tile_slice_rows), so one chunk_size == size tile (test_nerf's call) spreads over
    all ranks -- and one all-gather assembles the frame on every rank; the frame and the RNG
    states afterwards are the single-process render's.  Sharded: Direct / NeRFIntegrator(Direct)
    on the fused tile path, and NeRFReproduce over a NeRFLE (_row_separable).  shard: None =
    automatic, False = render the whole frame on every rank, True = require sharding (render.
    shard_of); group: the process group.  The scene's weights must be equal on the ranks
    (render.broadcast_module replicates them)."""
    if trim < 0:
        raise ValueError("trim must be >= 0")
    batch_dims = len(cameras)
    if width is None:
        width = size
    if height is None:
        height = size
    out = torch.full([batch_dims, width, height, integrator.dims()], background, device=device,
                     dtype=torch.float)
    assert (size % chunk_size) == 0, \
        f"Can only specify chunk sizes which evenly divide size, {size} % {chunk_size}"
    xs = list(range(0, width, chunk_size))
    ys = list(range(0, height, chunk_size))
    it = None
    fused = _fused(integrator, cameras, w_isect, addition) if trim == 0 else None
    grads = needs_grad(shapes, bsdf, lights, w_isect)
    if grads:
        # training (a learned occlusion MLP included, as Direct.sample checks it):
        # integrator.sample carries the gradients
        fused = None
    if not hasattr(shapes, "sdf") or not is_hip_sdf(shapes.sdf):
        # an SDF callable (SDF.intersect evaluates it between the HIP march steps) or another
        # shape (the analytic Sphere): integrator.sample on its own intersect, tile by tile
        fused = None
    if getattr(lights, "per_camera", lambda: None)() is not None:
        fused = None  # one light per camera: Direct.sample shades camera by camera
    tiles = []
    for ij in range(len(xs) * len(ys)):  # the reference's tile order (main.py:63-65)
        i, j = divmod(ij, len(ys))
        tiles.append((xs[j], ys[i]))
    sh = None
    if fused is not None or _row_separable(integrator, shapes, addition, trim, bsdf, lights,
                                           w_isect):
        sh = _render.shard_of(cameras, size, width, chunk_size, background, group, shard)
    elif shard:
        raise _lib.NrtError("pathtrace(shard=True) shards Direct / NeRFIntegrator(Direct) tiles "
                            "and NeRFReproduce over NeRFLE (no addition hook, trim 0, no "
                            "gradients)")
    dst, rows = out, None
    if sh is not None:
        # this rank's row slices of every tile (render.tile_slice_rows) into a slab, then one
        # all-gather assembles the frame on every rank
        rows = _render.tile_slice_rows(chunk_size, *sh)
        dst = torch.full([batch_dims, (width // chunk_size) * len(rows), height,
                          integrator.dims()], background, device=device, dtype=torch.float)
    if fused is not None:
        # every tile in the reference's order, batched into few launch chains (render.py)
        _render.render_tiles(fused, shapes, lights, cameras, bsdf, dst, tiles, chunk_size, size,
                             with_noise, background, rows=rows)
    elif sh is None and _path_batchable(integrator, shapes, lights, cameras, addition, trim, bsdf,
                                        w_isect):
        it = _path_tiles(integrator, shapes, lights, cameras, bsdf, out, tiles, chunk_size, size,
                         bundle_size, sampler, with_noise, background, w_isect, device)
    else:
        sel = None if rows is None else torch.tensor(rows, dtype=torch.long, device=device)
        R = chunk_size if rows is None else len(rows)
        for x0, y0 in tiles:
            rays = _tile_rays(cameras, x0 - trim, y0 - trim, chunk_size + 2 * trim, size, sampler,
                              bundle_size, batch_dims, with_noise, device, positions=bool(trim))
            if sel is not None:
                rays = rays.index_select(1, sel)  # this rank's rows of the tile (all its draws made)
            values, mask, it = integrator.sample(shapes, rays, bsdf=bsdf, lights=lights,
                                                 sampler=sampler, w_isect=w_isect)
            X0 = x0 if rows is None else (x0 // chunk_size) * R
            _composite(dst, values, mask, background, X0, y0, R, trim, H=chunk_size)
    if sh is not None:
        _render.gather_tile_shard(dst, out, chunk_size, sh[0], sh[1], group)
    if squeeze_first and batch_dims == 1:
        out = out.squeeze(0)
    return out, addition(it)


def pathtrace_sample(shapes, lights, cameras, integrator, bsdf=None, size=512, chunk_size=32,
                     bundle_size=4, crop_size=128, uv=None, background=1, sampler=Sampler(),
                     addition=nothing, silent=False, mode="crop", device="cuda",
                     squeeze_first=True, w_isect=False, with_noise=1e-2):
    """main.py:97-179."""
    if uv is None:
        uv = rand_uv(size, size, crop_size)
    batch_dims = len(cameras)
    img = [batch_dims, size, size, integrator.dims()]
    if mode == "crop":
        img = [batch_dims, crop_size, crop_size, integrator.dims()]
    out = torch.full(img, background, device=device, dtype=torch.float)
    assert (size % chunk_size) == 0, \
        f"Can only specify chunk sizes which evenly divide size, {size} % {chunk_size}"
    chunk_size = min(chunk_size, crop_size)
    u = max(min(uv[0], size - crop_size), 0)
    v = max(min(uv[1], size - crop_size), 0)
    xs = list(range(u, u + crop_size, chunk_size))
    ys = list(range(v, v + crop_size, chunk_size))
    it = None
    for ij in range(len(xs) * len(ys)):
        i, j = divmod(ij, len(ys))
        x0, y0 = xs[j], ys[i]
        rays = _tile_rays(cameras, x0, y0, chunk_size, size, sampler, bundle_size, batch_dims,
                          with_noise, device)
        values, mask, it = integrator.sample(shapes, rays, bsdf=bsdf, lights=lights,
                                             sampler=sampler, w_isect=w_isect)
        if mode == "crop":
            _composite(out, values, mask, background, x0 - u, y0 - v, chunk_size)
        else:
            _composite(out, values, mask, background, x0, y0, chunk_size)
    if squeeze_first and batch_dims == 1:
        out = out.squeeze(0)
    setattr(it, "crop_uv", uv)
    return out, addition(it)
