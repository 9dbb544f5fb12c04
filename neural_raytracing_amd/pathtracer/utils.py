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


def dir_to_elev_azim(direc):
    """utils.py:490-494."""
    x, y, z = F.normalize(direc, dim=-1).clamp(min=-1 + 1e-7, max=1 - 1e-7).split(1, dim=-1)
    elev = z.asin()
    azim = torch.atan2(x, (1 - x.square() - z.square()).clamp(min=1e-10).sqrt())
    return torch.cat([elev, azim], dim=-1)
