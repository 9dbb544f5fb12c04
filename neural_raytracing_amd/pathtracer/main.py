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


def _composite(out, values, mask, background, xs, ys, chunk, trim=0):
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
    out[:, xs:xs + chunk, ys:ys + chunk, :] = v


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


def pathtrace(shapes, lights, cameras, integrator, bsdf=None, size=512, width=None, height=None,
              chunk_size=32, bundle_size=4, background=1, addition=nothing, sampler=Sampler(),
              silent=False, trim=0, device="cuda", squeeze_first=True, w_isect=False,
              with_noise=1e-3, shard=None, group=None):
    """main.py:13-93.  trim > 0 renders each tile with a trim-pixel border of extra rays
    (main.py:67-68) and keeps the tile's interior (see _composite).

    Multi-GPU (the parallelism TODO of main.py:60): under an initialised torch.distributed
    process group of several ranks that all ask for the same frame, the fused tile path renders
    only this rank's bands of tile rows (band j of chunk_size rows when j % world == rank) and
    one all-gather assembles the frame on every rank; the frame is the single-process frame (every
    tile's camera and scan jitter is drawn in the reference's order on every rank).  shard: None =
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
    if needs_grad(shapes, bsdf, lights, w_isect):
        # training (a learned occlusion MLP included, as Direct.sample checks it):
        # integrator.sample carries the gradients
        fused = None
    if not hasattr(shapes, "sdf") or not is_hip_sdf(shapes.sdf):
        # an SDF callable (SDF.intersect evaluates it between the HIP march steps) or another
        # shape (the analytic Sphere): integrator.sample on its own intersect, tile by tile
        fused = None
    if getattr(lights, "per_camera", lambda: None)() is not None:
        fused = None  # one light per camera: Direct.sample shades camera by camera
    if fused is not None:
        # every tile in the reference's order, batched into few launch chains (render.py)
        tiles = []
        for ij in range(len(xs) * len(ys)):
            i, j = divmod(ij, len(ys))
            tiles.append((xs[j], ys[i]))
        sh = _render.shard_of(cameras, size, width, chunk_size, background, group, shard)
        keep = None
        if sh is not None:
            rank, world = sh
            keep = lambda k: (k % len(ys)) % world == rank  # noqa: E731  (band j = k % len(ys))
        _render.render_tiles(fused, shapes, lights, cameras, bsdf, out, tiles, chunk_size, size,
                             with_noise, background, keep=keep)
        if sh is not None:
            _render.gather_tile_rows(out, chunk_size, sh[0], sh[1], group)
    elif shard:
        raise _lib.NrtError("pathtrace(shard=True) renders on the fused tile path only "
                            "(Direct / NeRFIntegrator(Direct), no addition hook, a packed SDF)")
    for ij in range(len(xs) * len(ys) if fused is None else 0):
        i, j = divmod(ij, len(ys))
        x0, y0 = xs[j], ys[i]
        rays = _tile_rays(cameras, x0 - trim, y0 - trim, chunk_size + 2 * trim, size, sampler,
                          bundle_size, batch_dims, with_noise, device, positions=bool(trim))
        values, mask, it = integrator.sample(shapes, rays, bsdf=bsdf, lights=lights,
                                             sampler=sampler, w_isect=w_isect)
        _composite(out, values, mask, background, x0, y0, chunk_size, trim)
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
