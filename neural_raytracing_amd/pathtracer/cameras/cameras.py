"""Cameras (cameras/cameras.py).  Primary rays come from the HIP kernel ``nrt_raygen``."""
import ctypes
from dataclasses import dataclass

import torch

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
        return [_cam_struct(_lib.NRT_CAM_NERF, size, self.focal, mat=self.cam_to_world[n, :3, :4])
                for n in range(len(self))]

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
