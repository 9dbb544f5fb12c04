"""Volumetric NeRF shapes (shapes/nerf.py).  ``NeRFLE`` (NeRF + point light, or NeRF + envmap
light with envmap=True) renders through ``nrt_nerfle_forward``: sample points, both MLPs and the
reference's compositing on the GPU.  Constructor and RNG consumption follow nerf.py:153-172."""
import random

import torch
import torch.nn.functional as F
import torch.nn as nn

from ... import _lib
from ..differentiable import needs_grad
from ..neural_blocks import SkipConnMLP


class PlainNeRF(nn.Module):
    """A latent-conditioned NeRF (nerf.py:9-74), rendered by ``nrt_plain_nerf_forward``.

    Constructor and RNG order follow nerf.py:10-39 (``first``: 3 (+latent) -> 1 + intermediate,
    ``second``: elev/azim (+intermediate, latent) -> 3, both 5 x 32).  ``forward(rays, lights)``
    draws ``random.random()`` for ``ts = linspace(0.4, 2 + r*0.1, steps)`` and the density noise
    ``randn * 1e-3`` per sample (nerf.py:50, :66; on the device, ``noise=`` injects it) and
    returns ``(rgb + 1) / 2`` with the reference's compositing.  ``lights`` is unused, as there.
    """

    MAX_SAMPLES_PER_CALL = 1 << 22

    def __init__(self, latent_size: int = 32, intermediate_size: int = 32, steps=32,
                 device="cuda"):
        super().__init__()
        self.latent = None
        self.latent_size = latent_size
        self.steps = steps
        self.first = SkipConnMLP(in_size=3, out=1 + intermediate_size, latent_size=latent_size,
                                 num_layers=5, hidden_size=32, device=device).to(device)
        self.second = SkipConnMLP(in_size=2, out=3, latent_size=latent_size + intermediate_size,
                                  num_layers=5, hidden_size=32, device=device).to(device)

    def assign_latent(self, latent):
        assert latent.shape[-1] == self.latent_size
        assert len(latent.shape) == 2, "expected latent in [B, L]"
        self.latent = latent

    def forward(self, rays, lights=None, noise=None):
        assert self.latent is not None
        if not rays.is_cuda:
            raise _lib.NrtError("PlainNeRF renders on the HIP path only: move it and the rays to "
                                "the GPU")
        if needs_grad(self) or (torch.is_grad_enabled() and self.latent.requires_grad):
            raise _lib.NrtError("PlainNeRF is not on the HIP training path: render it under "
                                "torch.no_grad()")
        lead = rays.shape[:-1]
        if len(lead) < 2 or lead[0] != self.latent.shape[0]:
            raise _lib.NrtError(f"PlainNeRF: rays {tuple(rays.shape)} must be [N, ..., 6] with "
                                f"N = latent rows ({self.latent.shape[0]})")
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        dev = flat.device
        S = self.steps
        ts = torch.linspace(0.4, 2 + random.random() * 0.1, S).to(dev)
        if noise is None:
            noise = torch.randn(S, P, device=dev) * 1e-3
        noise = noise.reshape(S, P).float().contiguous()
        latent = self.latent.detach().float().to(dev).contiguous()
        per = P // lead[0]
        lib = _lib.load(require_device=True)
        rgb = torch.empty(P, 3, device=dev)
        # bounded intermediates: chunks of whole cameras, or pieces of one camera's rays (the
        # kernel maps chunk ray p to latent row p / rays_per_latent of the chunk's rows)
        cmax = max(1, self.MAX_SAMPLES_PER_CALL // S)
        first, second = self.first.nrt(), self.second.nrt()
        ws = torch.empty(lib.nrt_plain_nerf_workspace_bytes(first, second, min(cmax, P), S),
                         dtype=torch.uint8, device=dev)
        r0 = 0
        while r0 < P:
            cam = r0 // per
            if per <= cmax:
                n = min((cmax // per) * per, P - r0)
                lat, rpl = latent[cam:cam + n // per], per
            else:
                n = min(cmax, (cam + 1) * per - r0)
                lat, rpl = latent[cam:cam + 1], n
            _lib.call("nrt_plain_nerf_forward", first, second, _lib.ptr(flat[r0:r0 + n]), n,
                      _lib.ptr(ts), S, _lib.ptr(lat.contiguous()), rpl,
                      _lib.ptr(noise[:, r0:r0 + n].contiguous()), _lib.ptr(rgb[r0:r0 + n]),
                      _lib.ptr(ws), _lib.precision_code(), _lib.stream())
            r0 += n
        return rgb.reshape(lead + (3,))


class NeRFLE(nn.Module):
    """NeRF with a point-light emitter input (nerf.py:153-214).

    forward(rays [..., 6], lights) -> rgb [..., 3] with 64 samples at
    ts = linspace(0, 2 + random.random() * 0.1, 64) (nerf.py:178; one ``random.random()`` draw per
    call, as in the reference).  The colour MLP sees the point light's location, or with
    ``envmap=True`` its envmap over bins^2 directions (``nrt_light_envmap``, nerf.py:183-191).
    """

    # workspace bytes per nrt_nerfle_forward call: the unfused path keeps [S*P, 65/70] f32
    # intermediates (~564 B a sample: 4M samples), the fused FP16 kernel 16 B a sample (134M
    # samples: cfg5's 1600^2 x 256 frame in 5 calls instead of 157)
    MAX_WORKSPACE_BYTES = 1 << 31

    def __init__(self, envmap=False, bins=4, device="cuda", steps=64):
        super().__init__()
        self.latent_size = 64
        self.first = SkipConnMLP(num_layers=5, hidden_size=128, in_size=3,
                                 out=1 + self.latent_size, device=device).to(device)
        self.bins = bins
        self.second = SkipConnMLP(in_size=self.latent_size + (6 if not envmap else 3 + bins * bins * 3),
                                  out=3, device=device).to(device)
        self.envmap = envmap
        self.steps = steps  # nerf.py:178 hard-codes 64; BASELINE cfg5 asks 256

    def forward(self, rays, lights):
        if not rays.is_cuda:
            raise _lib.NrtError("NeRFLE renders on the HIP path only: move it and the rays to the GPU")
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        dev = flat.device
        # torch.linspace on the host: the same float32 sequence the CPU reference computes
        ts = torch.linspace(0, 2 + random.random() * 0.1, self.steps).to(dev)
        if needs_grad(self, lights):
            if getattr(self, "envmap", False):
                # nerf.py:183-191: the light's envmap at bins^2 directions (degree values passed
                # as radians, as in the reference), differentiable in the light's parameters
                if not hasattr(lights, "envmap"):
                    raise _lib.NrtError("NeRFLE(envmap=True) needs PointLights (lights.envmap)")
                from ..utils import elev_azim_to_dir
                points = torch.stack(torch.meshgrid(
                    torch.linspace(0, 180, self.bins, device=dev),
                    torch.linspace(0, 45, self.bins, device=dev), indexing="ij"),
                    dim=-1).reshape(-1, 2)
                light = lights.envmap(elev_azim_to_dir(points)).reshape(-1).float()
            else:
                light = lights.location.reshape(-1, 3)[0].detach().float().to(dev)
            return self._forward_train(flat, ts, light).reshape(lead + (3,))
        lib = _lib.load(require_device=True)
        if getattr(self, "envmap", False):
            handle = getattr(lights, "nrt", None)
            if handle is None or not hasattr(lights, "envmap"):
                raise _lib.NrtError("NeRFLE(envmap=True) needs PointLights (lights.envmap, "
                                    "lights.py:81-88)")
            light = torch.empty(3 * self.bins * self.bins, device=dev)
            _lib.call("nrt_light_envmap", handle(), self.bins, _lib.ptr(light), _lib.stream())
        else:
            light = lights.location.reshape(-1, 3)[0].detach().float().to(dev).contiguous()
        rgb = torch.empty(P, 3, device=dev)
        first, second = self.first.nrt(), self.second.nrt()
        prec = _lib.precision_code()
        per_ray = lib.nrt_nerfle_workspace_bytes_for(first, second, 1024, self.steps,
                                                     light.numel(), prec) / 1024
        chunk = max(1, min(P, int(self.MAX_WORKSPACE_BYTES // per_ray)))
        ws = torch.empty(lib.nrt_nerfle_workspace_bytes_for(first, second, chunk, self.steps,
                                                            light.numel(), prec),
                         dtype=torch.uint8, device=dev)
        for r0 in range(0, P, chunk):
            n = min(chunk, P - r0)
            _lib.call("nrt_nerfle_forward", first, second, _lib.ptr(flat[r0:r0 + n]), n,
                      _lib.ptr(ts), self.steps, _lib.ptr(light), light.numel(),
                      _lib.ptr(rgb[r0:r0 + n]),
                      _lib.ptr(ws), prec, _lib.stream())
        return rgb.reshape(lead + (3,))

    def _forward_train(self, flat, ts, light):
        """nerf.py:175-214 with autograd (point light or envmap encoding
        ``light``): both MLPs on the HIP MLP kernels
        with nrt_mlp_backward behind them; the sample points and the rolled-cumprod compositing
        are tensor ops in the reference's order.  FP32 intermediates [S, P, 65 / 70]."""
        o, d = flat[:, :3], flat[:, 3:]
        pts = o.unsqueeze(0) + torch.tensordot(ts, d, dims=0)
        first = self.first(pts)
        latent = first[..., 1:]
        alpha = first[..., 0, None]
        light_enc = light.reshape(1, 1, -1).expand(latent.shape[:-1] + (light.numel(),))
        rgb = self.second(torch.cat([latent, d[None].expand(latent.shape[:-1] + (3,)), light_enc],
                                    dim=-1)).sigmoid()
        sigma = F.relu(alpha).squeeze(-1)
        alpha = 1 - torch.exp(-sigma * ts[:, None].expand_as(sigma))
        cp = torch.cumprod((1 - alpha).clamp(min=1e-10), dim=0)
        cp = torch.roll(cp, 1, 0)
        cp[-1, ...] = 1
        w = alpha * cp
        return (w[..., None] * rgb).sum(dim=0)
