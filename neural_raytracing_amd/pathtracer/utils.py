"""Host utilities with the names ``pytorch3d.pathtracer.utils`` exports to the drivers.

Only the Fourier basis constructor feeds the hot path (it fixes the RNG order of SkipConnMLP);
the rest are small host helpers the scripts import (losses, image IO, crops, PSNR).
"""
import math
import random

import numpy as np
import torch
import torch.nn.functional as F


def create_fourier_basis2(batch_size, features=3, freq=40, device="cuda"):
    """utils.py:33-36: ``B = freq * randn(batch_size, features).T``; enc width 2F+in."""
    basis = freq * torch.randn(batch_size, features, device=device).T
    return basis, batch_size * 2 + features


def rand_uv(w: int, h: int, size: int):
    """utils.py:375-376."""
    return random.randint(0, w - size), random.randint(0, h - size)


def mse2psnr(x):
    """utils.py:361."""
    return -10 * torch.log10(x)


def eikonal_loss(grad):
    """utils.py:295."""
    return (torch.norm(grad, dim=-1) - 1).square().mean()


def load_image(src, resize=None):
    """utils.py:365-369."""
    from PIL import Image
    img = Image.open(src)
    if resize is not None:
        img = img.resize(resize)
    return torch.from_numpy(np.array(img, dtype=float) / 255).float()


def crop(img, u, v, size):
    return img[u:u + size, v:v + size, ...]


def elev_azim_to_dir(elev_azim):
    """utils.py:478-486."""
    limit = math.pi - 1e-7
    elev, azim = elev_azim.clamp(min=-limit, max=limit).split(1, dim=-1)
    return torch.cat([azim.sin() * elev.cos(), azim.cos() * elev.cos(), elev.sin()], dim=-1)


def dir_to_elev_azim(direc):
    """utils.py:490-494."""
    x, y, z = F.normalize(direc, dim=-1).clamp(min=-1 + 1e-7, max=1 - 1e-7).split(1, dim=-1)
    elev = z.asin()
    azim = torch.atan2(x, (1 - x.square() - z.square()).clamp(min=1e-10).sqrt())
    return torch.cat([elev, azim], dim=-1)


class LossSampler:
    """View selection weighted by the squared last loss (utils.py:134-147); views not drawn for a
    while gain likelihood by ``likelihood_inc`` per update."""

    def __init__(self, N, default=1e5, likelihood_inc=1.00001):
        self.losses = np.array([default] * N)
        self.l_inc = likelihood_inc

    def update(self, idx, loss):
        self.losses *= self.l_inc
        self.losses[idx] = loss + 1

    def sample(self, n=1, replace=False):
        sq = self.losses * self.losses
        return np.random.choice(len(self.losses), replace=replace, size=n, p=sq / sq.sum())

    def update_idxs(self, idxs, loss):
        for idx in idxs:
            self.update(idx, loss)


def rand_uv_mask(mask, size: int):
    """A crop corner inside the mask's valid region (utils.py:378-383)."""
    half = int(math.ceil(size / 2))
    valid = mask[half:-half - size, half:-half - size, ...]
    p, q = valid.nonzero(as_tuple=True)
    idx = random.randint(0, len(p) - 1)
    return p[idx], q[idx]


def masked_loss(got, exp, throughput, exp_mask, eps: float = 1e-10, trim: int = 0,
                mask_weight: float = 1, with_logits: bool = True, tone_mapping: bool = False):
    """utils.py:307-359: on rays that hit inside the mask, 10 x (L2 + RMSE + L1 - log SSIM) of the
    masked colours (tone-mapped x/(1+x) if asked); on the others, BCE of the throughput logits
    against the mask, weighted by ``mask_weight``."""
    from .metrics import ssim
    active = ((throughput > 0) & (exp_mask == 1)).squeeze(-1)
    misses = ~active
    color_loss = 0
    if active.any():
        got_active = got * active[..., None]
        exp_active = exp * active[..., None]
        if tone_mapping:
            got_active = got_active / (1 + got_active)
            exp_active = exp_active / (1 + exp_active)
        l1_loss = F.l1_loss(got_active, exp_active)
        l2_loss = F.mse_loss(got_active, exp_active)
        rmse_loss = l2_loss.clamp(min=1e-10).sqrt()
        ssim_loss = -ssim(got_active.permute(0, 3, 1, 2), exp_active.permute(0, 3, 1, 2),
                          data_range=1, size_average=True).log()
        color_loss = l2_loss + rmse_loss + l1_loss + ssim_loss
    mask_loss = 0
    if misses.any():
        loss_fn = F.binary_cross_entropy_with_logits if with_logits else F.binary_cross_entropy
        mask_loss = loss_fn(throughput[misses].reshape(-1, 1), exp_mask[misses].reshape(-1, 1))
    return mask_weight * mask_loss + 10 * color_loss


def save_image(name, img):
    """training_utils.py:21 (PNG through PIL; matplotlib is not needed)."""
    from PIL import Image
    arr = (img.detach().cpu().clamp(0, 1).numpy() * 255 + 0.5).astype(np.uint8)
    Image.fromarray(arr).save(name)


def count_parameters(params):
    """utils.py:363."""
    return sum(p.numel() for p in params)


def smooth_min(v, k: float = 32, dim: int = 0):
    """utils.py:386-387 (host form; the HIP SphereSDF evaluates it in-kernel)."""
    return -torch.exp(-k * v).sum(dim).clamp(min=1e-4).log() / k


def depth_image(img):
    """utils.py:441-445: [depth, mask] -> [d/max d, d/max d, d/max d, mask]."""
    l, m = img.split(1, dim=-1)
    l = l / l.max()
    return torch.cat([l, l, l, m], dim=-1)


def heightmap(warp, size=256, device="cuda"):
    """utils.py:434-439: warp.pdf on a size x size (u, v) grid."""
    u, v = torch.meshgrid(torch.linspace(0, 1, size, device=device),
                          torch.linspace(0, 1, size, device=device), indexing="ij")
    return warp.pdf(torch.stack([u, v], dim=-1))


def _sphere_scene(device, scale):
    """utils.py:390-399 / 417-420: the unit Sphere at the origin, look_at_view_transform(dist=2,
    elev=0, azim=0) through OpenGLPerspectiveCameras, the renderer's PointLights at (0, 1, 4)."""
    from .cameras import OpenGLPerspectiveCameras, look_at_view_transform
    from .lights import RendererPointLights
    from .shapes import Sphere
    sphere = Sphere([0, 0, 0], 1, device=device)
    R, T = look_at_view_transform(dist=2., elev=0, azim=0)
    cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
    lights = RendererPointLights(device=device, location=[[0., 1., 4.]], scale=scale)
    return sphere, cameras, lights


def sphere_render_bsdf(bsdf, integrator=None, device="cuda", size=256, chunk_size=128, scale=100):
    """utils.py:389-407: one BSDF on the analytic unit Sphere (Direct by default), on the HIP
    path (nrt_sphere_intersect + the fused shading kernels)."""
    from . import pathtrace
    from .integrators import Direct
    sphere, cameras, lights = _sphere_scene(device, scale)
    if integrator is None:
        integrator = Direct()
    return pathtrace(sphere, cameras=cameras, lights=lights, chunk_size=chunk_size, size=size,
                     bsdf=bsdf, integrator=integrator, device=device, silent=True)[0]


def sphere_examples(bsdf, device="cuda", size=256, chunk_size=128, scale=100):
    """utils.py:409-431: every component of a ComposeSpatialVarying rendered on the analytic unit
    Sphere (shapes/shapes.py:31-97, HIP intersect) lit by the renderer's PointLights
    (renderer/lighting.py:221-304) with Direct()."""
    from . import pathtrace
    from .integrators import Direct
    sphere, cameras, lights = _sphere_scene(device, scale)
    out = []
    for basis in bsdf.bsdfs:
        out.append(pathtrace(sphere, cameras=cameras, lights=lights, chunk_size=chunk_size,
                             size=size, bsdf=basis, integrator=Direct(), device=device,
                             silent=True)[0])
    return out
