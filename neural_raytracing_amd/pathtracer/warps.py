"""Sample warps (warps.py:7-52), host tensor functions with the reference's names.

The HIP path applies the cosine-hemisphere warp inside ``nrt_path_bounce`` (Path's BSDF
sampling); these are the Python-level functions the reference package exports
(pytorch3d/pathtracer/__init__.py) for drivers and tests.
"""
import math

import torch


def circ(x):
    """warps.py:7-8."""
    return torch.sqrt((1 - x.square()).clamp(min=1e-10))


def square_to_uniform_disk_concentric(sample):
    """warps.py:10-30, including its (r sin(phi), r cos(phi)) output order."""
    v = 2 * sample - 1
    is_zero = (v == 0).all(dim=-1)
    q13 = (v[..., 0].abs() < v[..., 1].abs()).unsqueeze(-1)
    x, y = torch.split(v, 1, dim=-1)
    r = torch.where(q13, y, x)
    rp = torch.where(q13, x, y)
    r = r.sign() * r.abs().clamp(min=1e-12)
    phi = 0.25 * math.pi * rp / r
    phi = torch.where(q13, 0.5 * math.pi - phi, phi)
    phi = torch.where(is_zero.unsqueeze(-1), torch.zeros_like(phi), phi)
    s, c = phi.sin(), phi.cos()
    return torch.cat([r * s, r * c], dim=-1)


def square_to_uniform_sphere(sample):
    """warps.py:33-40."""
    z = 1 - 2 * sample[..., 1]
    r = circ(z)
    tmp = 2 * math.pi * sample[..., 0] - math.pi
    return torch.stack([r * tmp.cos(), r * tmp.sin(), z], dim=-1)


def square_to_uniform_sphere_pdf(sample):
    """warps.py:42."""
    return 1 / (4 * math.pi)


def square_to_cos_hemisphere(sample):
    """warps.py:44-49."""
    p = square_to_uniform_disk_concentric(sample)
    z = (1 - (p * p).sum(dim=-1, keepdim=True)).clamp(min=1e-7).sqrt()
    return torch.cat([p, z], dim=-1)


def square_to_cos_hemisphere_pdf(d):
    """warps.py:51-52."""
    return d[..., 2] / math.pi
