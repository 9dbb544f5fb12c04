"""Cameras (cameras/cameras.py).  Primary rays come from the HIP kernel ``nrt_raygen``."""
import ctypes
import math
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ... import _lib


def _cam_struct(kind, size, focal=0.0, mat=None, intrinsic=None, origin=None):
    c = _lib.Camera()
    c.kind = kind
    c.size = int(size)
    c.focal = float(focal)
    if mat is not None:
        m = mat.detach().float().cpu().reshape(-1).tolist()
        for i, v in enumerate(m):
            c.mat[i] = v
    if intrinsic is not None:
        k = intrinsic.detach().float().cpu().reshape(-1).tolist()
        for i, v in enumerate(k):
            c.intrinsic[i] = v
    if origin is not None:
        for i, v in enumerate(origin.detach().float().cpu().reshape(-1).tolist()):
            c.origin[i] = v
    return c


def raygen(structs, x0, y0, W, H, with_noise, noise, positions, device):
    N = len(structs)
    arr = (_lib.Camera * N)(*structs)
    rays = torch.empty(N * W * H, 6, device=device)
    _lib.call("nrt_raygen", ctypes.cast(arr, ctypes.c_void_p), N, int(x0), int(y0), int(W), int(H),
              float(with_noise or 0.0), _lib.ptr(noise), _lib.ptr(positions), _lib.ptr(rays),
              _lib.stream())
    return rays


@dataclass
class Camera:
    camera_to_world = None
    world_to_camera = None

    def sample_positions(self, positions, sampler, bundle_size):
        raise NotImplementedError()


@dataclass
class NeRFCamera(Camera):
    """NeRF-synthetic pinhole camera (cameras.py:16-54)."""
    cam_to_world: torch.Tensor = None
    focal: float = None
    device: str = "cuda"

    def __len__(self):
        return self.cam_to_world.shape[0]

    def _structs(self, size):
        # the matrices go to the host once per (tensor, version, size, focal), not once per tile
        c2w = self.cam_to_world
        key = (c2w.data_ptr(), c2w._version, tuple(c2w.shape), int(size), float(self.focal))
        cached = getattr(self, "_nrt_structs", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        structs = [_cam_struct(_lib.NRT_CAM_NERF, size, self.focal, mat=c2w[n, :3, :4])
                   for n in range(len(self))]
        object.__setattr__(self, "_nrt_structs", (key, structs))
        return structs

    def rays_tile(self, x0, y0, W, H, size, with_noise=False, positions=None):
        """[N, W, H, 1, 6] rays for tile rows x0.. and cols y0.. (u = col, v = row)."""
        dev = self.cam_to_world.device
        noise = None
        if with_noise:
            # two rand_like draws in the reference (u then v): [2, W, H]
            noise = torch.rand(2, W, H, device=dev)
        rays = raygen(self._structs(size), x0, y0, W, H, with_noise, noise, positions, dev)
        return rays.reshape(len(self), W, H, 1, 6)

    def sample_positions(self, position_samples, sampler, bundle_size=4, size=512,
                         with_noise=False, N=1):
        W, H, _ = position_samples.shape
        pos = position_samples.float().contiguous()
        return self.rays_tile(0, 0, W, H, size, with_noise, positions=pos)


def _f32(v, device="cpu"):
    t = v if torch.is_tensor(v) else torch.tensor(v, dtype=torch.float32)
    return t.to(device=device, dtype=torch.float32).reshape(-1)


def look_at_rotation(camera_position, at=((0, 0, 0),), up=((0, 1, 0),), device="cpu"):
    """renderer/cameras.py:1313-1360: world -> view rotations [N, 3, 3] of cameras at
    camera_position looking at ``at`` (columns: x right, y up, z forward)."""
    C = torch.as_tensor(camera_position, dtype=torch.float32).reshape(-1, 3)
    at = torch.as_tensor(at, dtype=torch.float32).reshape(-1, 3)
    up = torch.as_tensor(up, dtype=torch.float32).reshape(-1, 3)
    n = max(C.shape[0], at.shape[0], up.shape[0])
    C, at, up = C.expand(n, 3), at.expand(n, 3), up.expand(n, 3)
    z_axis = F.normalize(at - C, eps=1e-5)
    x_axis = F.normalize(torch.cross(up, z_axis, dim=1), eps=1e-5)
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=1), eps=1e-5)
    is_close = torch.isclose(x_axis, torch.tensor(0.0), atol=5e-3).all(dim=1, keepdim=True)
    if is_close.any():
        x_axis = torch.where(is_close, F.normalize(torch.cross(y_axis, z_axis, dim=1), eps=1e-5),
                             x_axis)
    R = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), dim=1)
    return R.transpose(1, 2).to(device)


def look_at_view_transform(dist=1.0, elev=0.0, azim=0.0, degrees=True, eye=None,
                           at=((0, 0, 0),), up=((0, 1, 0),), device="cpu"):
    """R [N,3,3], T [N,3] of the look-at world -> view transform (renderer/cameras.py:1363-1422,
    with camera_position_from_spherical_angles :1275-1310 and look_at_rotation :1313-1360).
    Host-side float32 math on the camera parameters, as in the reference."""
    at = torch.tensor(at, dtype=torch.float32).reshape(-1, 3)
    up = torch.tensor(up, dtype=torch.float32).reshape(-1, 3)
    if eye is not None:
        C = torch.tensor(eye, dtype=torch.float32).reshape(-1, 3)
    else:
        dist, elev, azim = _f32(dist), _f32(elev), _f32(azim)
        if degrees:
            elev = math.pi / 180.0 * elev
            azim = math.pi / 180.0 * azim
        C = torch.stack([dist * torch.cos(elev) * torch.sin(azim), dist * torch.sin(elev),
                         dist * torch.cos(elev) * torch.cos(azim)], dim=1).view(-1, 3) + at
    n = max(C.shape[0], at.shape[0], up.shape[0])
    C = C.expand(n, 3)
    R = look_at_rotation(C, at, up)
    T = -torch.bmm(R.transpose(1, 2), C[:, :, None])[:, :, 0]
    return R.to(device), T.to(device)


class FoVPerspectiveCameras:
    """OpenGL-style perspective camera used by colocate.py (renderer/cameras.py:314-575).

    Rays (sample_positions, :539-575) come from ``nrt_raygen`` (NRT_CAM_FOV): the inverse of the
    full projection Rotate(R) . Translate(T) . K^T is built on the host in float32 with the
    reference's Transform3d.inverse() order (transforms/transform3d.py:225-272: inv(K^T), then
    Translate(-T), then R^T), and the kernel applies it to (ndc_x, ndc_y, 1) with a homogeneous
    divide and r_d = normalize(point) (the reference normalises the point, not point - centre).
    """

    def __init__(self, znear=1e-2, zfar=1e4, aspect_ratio=1.0, fov=60.0, degrees=True,
                 R=None, T=None, K=None, device="cpu"):
        if K is not None:
            raise NotImplementedError("FoVPerspectiveCameras(K=...) is not on the HIP path")
        self.R = torch.eye(3)[None] if R is None else R
        self.T = torch.zeros(1, 3) if T is None else T
        self.znear, self.zfar, self.aspect_ratio, self.fov = znear, zfar, aspect_ratio, fov
        self.degrees = degrees
        self.device = device

    def __len__(self):
        return self.R.shape[0]

    def compute_projection_matrix(self):
        """[N,4,4] K (renderer/cameras.py:389-439); parameters float32 [N] as TensorProperties
        (renderer/utils.py:91-130) makes them."""
        N = len(self)
        znear, zfar = _f32(self.znear).expand(N), _f32(self.zfar).expand(N)
        aspect, fov = _f32(self.aspect_ratio).expand(N), _f32(self.fov).expand(N)
        if self.degrees:
            fov = (np.pi / 180) * fov
        tan_half = torch.tan(fov / 2)
        max_y = tan_half * znear
        min_y = -max_y
        max_x = max_y * aspect
        min_x = -max_x
        K = torch.zeros((N, 4, 4), dtype=torch.float32)
        K[:, 0, 0] = 2.0 * znear / (max_x - min_x)
        K[:, 1, 1] = 2.0 * znear / (max_y - min_y)
        K[:, 0, 2] = (max_x + min_x) / (max_x - min_x)
        K[:, 1, 2] = (max_y + min_y) / (max_y - min_y)
        K[:, 3, 2] = 1.0 * torch.ones(N)
        K[:, 2, 2] = 1.0 * zfar / (zfar - znear)
        K[:, 2, 3] = -(zfar * znear) / (zfar - znear)
        return K

    def _rt(self):
        R = self.R.detach().float().cpu()
        T = self.T.detach().float().cpu()
        N = R.shape[0]
        rot = torch.eye(4).repeat(N, 1, 1)
        rot[:, :3, :3] = R
        tinv = torch.eye(4).repeat(N, 1, 1)
        tinv[:, 3, :3] = -T
        return rot, tinv

    def get_camera_center(self):
        """renderer/cameras.py:143-149: row 3 of (Rotate . Translate)^-1."""
        rot, tinv = self._rt()
        return torch.bmm(tinv, rot.transpose(1, 2))[:, 3, :3]

    def inverse_full_projection(self):
        rot, tinv = self._rt()
        m = torch.inverse(self.compute_projection_matrix().transpose(1, 2).contiguous())
        return torch.bmm(torch.bmm(m, tinv), rot.transpose(1, 2))

    def _structs(self, size):
        inv = self.inverse_full_projection()
        ctr = self.get_camera_center()
        return [_cam_struct(_lib.NRT_CAM_FOV, size, mat=inv[n], origin=ctr[n])
                for n in range(len(self))]

    def rays_tile(self, x0, y0, W, H, size, with_noise=False, positions=None, noise=None,
                  bundle_size=1, device="cuda"):
        """[N, W, H, B, 6].  noise: [W, H, 2] uniforms (the sampler's draw), drawn here if None."""
        if bundle_size != 1:
            raise NotImplementedError("FoVPerspectiveCameras on the HIP path renders bundle_size 1")
        if with_noise and noise is None:
            noise = torch.rand(W, H, 2, device=device)
        rays = raygen(self._structs(size), x0, y0, W, H, with_noise, noise if with_noise else None,
                      positions, device)
        return rays.reshape(len(self), W, H, 1, 6)

    def sample_positions(self, position_samples, sampler, bundle_size=8, size=512,
                         with_noise=False, N=1):
        """renderer/cameras.py:539-575 (one sampler draw of the jitter, [W, H, B, 2])."""
        W, H, _ = position_samples.shape
        dev = position_samples.device
        noise = None
        if with_noise:
            noise = sampler.sample((W, H, bundle_size, 2), device=dev).reshape(W, H, 2)
        return self.rays_tile(0, 0, W, H, size, with_noise, positions=position_samples.float()
                              .contiguous(), noise=noise, bundle_size=bundle_size, device=dev)


def OpenGLPerspectiveCameras(znear=1.0, zfar=100.0, aspect_ratio=1.0, fov=60.0, degrees=True,
                             R=None, T=None, device="cpu"):
    """renderer/cameras.py:280-311 (deprecated alias with its own defaults)."""
    return FoVPerspectiveCameras(znear=znear, zfar=zfar, aspect_ratio=aspect_ratio, fov=fov,
                                 degrees=degrees, R=R, T=T, device=device)


@dataclass
class DTUCamera(Camera):
    """IDR/DTU camera (cameras.py:149-192); with_noise is ignored like the reference."""
    pose: torch.Tensor = None
    intrinsic: torch.Tensor = None
    device: str = "cuda"

    def __len__(self):
        return self.pose.shape[0]

    def _structs(self, size):
        return [_cam_struct(_lib.NRT_CAM_DTU, size, mat=self.pose[n], intrinsic=self.intrinsic[n])
                for n in range(len(self))]

    def rays_tile(self, x0, y0, W, H, size, with_noise=False, positions=None, bundle_size=1):
        rays = raygen(self._structs(size), x0, y0, W, H, 0.0, None, positions, self.pose.device)
        return rays.reshape(len(self), W, H, 1, 6).expand(len(self), W, H, bundle_size, 6)

    def sample_positions(self, position_samples, sampler, bundle_size=4, size=512,
                         with_noise=False, N=1):
        W, H, _ = position_samples.shape
        pos = position_samples.float().contiguous()
        return self.rays_tile(0, 0, W, H, size, positions=pos, bundle_size=bundle_size)


@dataclass
class NeRVCamera(Camera):
    """cameras.py:103-130 (NeRV dataset): sample_positions returns ``torch.cat([r_o, r_d])`` with
    ``r_o`` never defined (:130), so the camera cannot produce rays in the reference; kept
    import-resolvable (train_nerv, training_utils.py:634)."""
    world_to_cam: torch.Tensor = None
    loc: torch.Tensor = None
    focal: float = None
    device: str = "cuda"

    def __len__(self):
        return self.world_to_cam.shape[0]

    def sample_positions(self, *args, **kwargs):
        raise NotImplementedError("NeRVCamera.sample_positions uses an undefined r_o in the "
                                  "reference (cameras.py:130)")
