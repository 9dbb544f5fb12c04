"""Interaction records (interaction.py:53-119).  Frames come from the HIP kernel
``nrt_frames``; to_local / from_local on a record are host-side glue on device tensors."""
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .. import _lib


def coordinate_system(n):
    """interaction.py:9-27 via the HIP kernel: [..., 3] -> [..., 3, 3] columns [s, t, n]."""
    flat = n.reshape(-1, 3).float().contiguous()
    frame = torch.empty(flat.shape[0], 9, device=n.device)
    _lib.call("nrt_frames", None, _lib.ptr(flat), flat.shape[0], _lib.ptr(frame), None,
              _lib.stream())
    return frame.reshape(n.shape[:-1] + (3, 3))


def to_local(frame, wo):
    """interaction.py:37-41."""
    wo = wo.unsqueeze(-1).expand_as(frame)
    return F.normalize((frame * wo).mean(dim=-2), eps=1e-7, dim=-1)


def from_local(frame, v):
    """interaction.py:44-51."""
    s, t, n = frame.split(1, dim=-1)
    x, y, z = v.split(1, dim=-1)
    wo = s.squeeze(-1) * x + t.squeeze(-1) * y + n.squeeze(-1) * z
    return F.normalize(wo, eps=1e-7, dim=-1)


@dataclass
class Interaction:
    p: torch.Tensor

    def spawn_rays(self, d):
        return torch.cat([self.p.expand_as(d), d], dim=-1)


@dataclass
class SurfaceInteraction(Interaction):
    uv: torch.Tensor = None
    wi: torch.Tensor = None
    t: torch.Tensor = None
    bsdf: object = None
    obj: object = None
    bidirectional_normals: bool = False
    frame = None
    n: torch.Tensor = None

    def set_normals(self, normals):
        self.n = normals
        self.frame = coordinate_system(normals)

    def to_local(self, wo):
        return to_local(self.frame, wo)

    def from_local(self, v):
        return from_local(self.frame, v)

    def shape(self):
        return self.p.shape

    def device(self):
        return self.p.device


@dataclass
class MixedInteraction(SurfaceInteraction):
    throughput: torch.Tensor = None
    medium_mask = torch.tensor(False)
    with_logits: bool = True

    def mark_mediums(self, medium_mask):
        self.medium_mask = medium_mask

    def surface_interactions(self):
        return ~self.medium_mask


@dataclass
class DirectionSample:
    p: torch.Tensor = None
    n: torch.Tensor = 0
    pdf: torch.Tensor = 1
    delta: torch.Tensor = True
    obj: object = None
    d: torch.Tensor = None
    dist: torch.Tensor = None
