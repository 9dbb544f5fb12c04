"""Lights (lights/lights.py).  Sampling at the hit points runs inside ``nrt_shade_direct``;
the handles below pack the parameters."""
import ctypes
from itertools import chain

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import _lib
from .._handles import _Handle, _host, mlp_handle
from ..interaction import DirectionSample
from ..neural_blocks import SkipConnMLP


class Light(nn.Module):
    def __init__(self):
        super().__init__()

    def sample_direction(self, it, sampler, active=True):
        raise NotImplementedError()

    def intersect(self, _rays):
        return None, False


class PointLights(Light):
    """Point light with constant/linear/quadratic falloff (lights.py:40-110)."""

    def __init__(self, intensity=[1., 1., 1.], location=[0, 1, 0], const=1e-8, linear=1e-8,
                 square=1, scale=1e2, device="cuda"):
        super().__init__()
        self.device = device
        self.scale = torch.tensor(scale, dtype=torch.float, requires_grad=True)
        if type(intensity) is torch.Tensor:
            self.intensity = intensity
        else:
            self.intensity = torch.tensor([intensity], device=device, requires_grad=True, dtype=torch.float)
        if type(location) is torch.Tensor:
            self.location = location
        else:
            self.location = torch.tensor(location, device=device, requires_grad=True, dtype=torch.float)
            if len(self.location.shape) == 1:
                self.location = self.location.unsqueeze(0).detach()
        self.const = torch.tensor(const, dtype=torch.float, requires_grad=True)
        self.linear = torch.tensor(linear, dtype=torch.float, requires_grad=True)
        self.square = torch.tensor(square, dtype=torch.float, requires_grad=True)

    def parameters(self):
        return chain(self.location_parameters(), self.spectrum_parameters())

    def location_parameters(self):
        return [self.location]

    def spectrum_parameters(self):
        return [self.scale, self.intensity, self.const, self.linear, self.square]

    def per_camera(self):
        """None when this is one light for every camera, else the number of lights L: the
        reference broadcasts location[:, None, None, None, :] and intensity (lights.py:91, :106)
        against the hit points [N, W, H, B, 3], so L > 1 distinct lights are one per camera
        (colocate.py:109 moves one light onto each of the N cameras of a batch)."""
        loc = self.location.reshape(-1, 3)
        inten = self.intensity.reshape(-1, 3)
        L = max(loc.shape[0], inten.shape[0])
        for t in (loc, inten):
            if t.shape[0] > 1 and not bool((t == t[:1]).all()):
                return L
        return None

    def camera(self, n):
        """The light camera n sees (a PointLights of location[n], intensity[n]; rows broadcast
        when there is one), sharing the falloff tensors."""
        v = PointLights.__new__(PointLights)
        nn.Module.__init__(v)
        loc = self.location.reshape(-1, 3)
        inten = self.intensity.reshape(-1, 3)
        v.device = self.device
        v.location = loc[n if loc.shape[0] > 1 else 0].reshape(1, 3)
        v.intensity = inten[n if inten.shape[0] > 1 else 0].reshape(1, 3)
        v.scale, v.const, v.linear, v.square = self.scale, self.const, self.linear, self.square
        return v

    def single(self):
        """Raise unless the light is one light for every camera (the HIP shading kernels take
        one light per call; per-camera lights are split per camera by the callers that support
        them, Direct and its training path)."""
        if self.per_camera() is not None:
            raise _lib.NrtError("PointLights with one location / intensity per camera are "
                                "supported by Direct (and its training path), not here")
        return self

    def nrt(self):
        self.single()
        loc = _host(self.location.reshape(-1, 3)[0])
        inten = _host(self.intensity.reshape(-1, 3)[0])
        out = ctypes.c_void_p()
        _lib.check(_lib.load().nrt_light_create_point(
            loc.data_ptr(), inten.data_ptr(), float(self.const), float(self.linear),
            float(self.square), float(self.scale), ctypes.byref(out)), "nrt_light_create_point")
        h = _Handle(out, "nrt_light_destroy")
        object.__setattr__(self, "_nrt_light", h)
        return h.value

    def envmap(self, p):
        d = p[None, ...] - self.location[:, None, None, :]
        dist = torch.linalg.norm(d, dim=-1, keepdim=True)
        spectrum = self.const.clamp(min=1e-6) + self.linear.clamp(min=1e-6) * dist + \
            self.square.clamp(min=1e-6) * dist.square()
        return self.scale * F.normalize(self.intensity, dim=-1) / spectrum.clamp(min=1e-6)


class RendererPointLights(Light):
    """``pytorch3d.renderer.PointLights`` of the reference's PyTorch3D fork (renderer/lighting.py:
    221-304) as a pathtracer light -- the light of utils.sphere_examples / sphere_render_bsdf
    (utils.py:389-431): intensity = ambient_color, sample_direction gives d = (loc - p) inv and
    Le = scale * intensity * inv^2 with inv = 1 / (1e-7 + |loc - p|) (no normalised intensity,
    no constant / linear terms: not the pathtracer's PointLights).  The mesh shader's diffuse /
    specular terms belong to the rasteriser (out of scope).  One light (the reference broadcasts
    a [N, 3] location against the ray bundle axis, so only N = 1 is meaningful there)."""

    def __init__(self, ambient_color=((0.5, 0.5, 0.5),), diffuse_color=((0.3, 0.3, 0.3),),
                 specular_color=((0.2, 0.2, 0.2),), location=((0, 1, 0),), device="cpu",
                 scale=1e-2):
        super().__init__()
        self.device = torch.device(device)

        def t(v):
            v = v.to(self.device) if isinstance(v, torch.Tensor) else \
                torch.tensor(v, device=self.device, dtype=torch.float)
            return v.reshape(-1, 3) if v.dim() < 2 else v
        self.ambient_color = t(ambient_color)
        self.diffuse_color = t(diffuse_color)
        self.specular_color = t(specular_color)
        self.location = t(location)
        if self.location.shape[-1] != 3:
            raise ValueError(f"Expected location to have shape (N, 3); got {tuple(self.location.shape)}")
        self.intensity = torch.tensor(ambient_color, device=self.device) \
            if not isinstance(ambient_color, torch.Tensor) else ambient_color.to(self.device)
        self.scale = scale

    def per_camera(self):
        return None

    def single(self):
        if self.location.reshape(-1, 3).shape[0] != 1 or self.intensity.reshape(-1, 3).shape[0] != 1:
            raise _lib.NrtError("pytorch3d.renderer.PointLights on the pathtracer path: one "
                                "location and one ambient colour")
        return self

    def sample_towards(self, points):
        return F.normalize(self.location - points, dim=-1)

    def sample_direction(self, it, sampler=None, active=True):
        """renderer/lighting.py:285-304 (torch; the HIP kernels do the same in-kernel)."""
        ds = DirectionSample()
        ds.p = self.location
        ds.n = 0
        ds.uv = 0
        ds.obj = self
        ds.delta = torch.tensor(True, device=self.device)
        ds.d = ds.p - it.p
        ds.dist = (ds.d * ds.d).sum(dim=-1, keepdim=True).sqrt()
        inv_dist = (1e-7 + ds.dist).reciprocal()
        ds.d = ds.d * inv_dist
        spectrum = self.scale * self.intensity * inv_dist * inv_dist
        return ds, spectrum

    def nrt(self):
        self.single()
        loc = _host(self.location.reshape(-1, 3)[0])
        inten = _host(self.intensity.reshape(-1, 3)[0].float())
        out = ctypes.c_void_p()
        _lib.check(_lib.load().nrt_light_create_renderer_point(
            loc.data_ptr(), inten.data_ptr(), float(self.scale), ctypes.byref(out)),
            "nrt_light_create_renderer_point")
        h = _Handle(out, "nrt_light_destroy")
        object.__setattr__(self, "_nrt_light", h)
        return h.value

    def diffuse(self, normals, points):
        raise NotImplementedError("PointLights.diffuse belongs to the mesh shader (pytorch3d._C "
                                  "rasteriser, out of scope)")

    def specular(self, normals, points, camera_position, shininess):
        raise NotImplementedError("PointLights.specular belongs to the mesh shader (pytorch3d._C "
                                  "rasteriser, out of scope)")


class LightField(nn.Module):
    """Learned light f(p) -> direction * magnitude, colour sigmoid(c) (lights.py:155-195)."""

    def __init__(self, device="cuda"):
        super().__init__()
        self.light_field_approx = SkipConnMLP(in_size=3, out=3, num_layers=10, hidden_size=256,
                                              device=device).to(device)
        self.color = nn.Parameter(torch.tensor([0., 0., 0.], requires_grad=True, dtype=torch.float,
                                               device=device), requires_grad=True)
        self.device = device

    def nrt(self):
        mh = mlp_handle(self.light_field_approx)
        color = _host(self.color)
        key = (id(mh), tuple(color.tolist()))
        cached = getattr(self, "_nrt_light", None)
        if cached is not None and cached[0] == key:
            return cached[1].value
        out = ctypes.c_void_p()
        _lib.check(_lib.load().nrt_light_create_field(mh.value, color.data_ptr(), ctypes.byref(out)),
                   "nrt_light_create_field")
        h = _Handle(out, "nrt_light_destroy", [mh])
        object.__setattr__(self, "_nrt_light", (key, h))
        return h.value


class Constant(Light):
    """lights.py:114-149: an emitting sphere around the scene.  Its sample_ray reads attributes it
    never sets (broken in the reference); import-resolvable only, not a HIP light."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        self.args, self.kwargs = args, kwargs

    def nrt(self):
        raise _lib.NrtError("Constant light has no HIP implementation (supported: LightField, "
                            "PointLights)")
