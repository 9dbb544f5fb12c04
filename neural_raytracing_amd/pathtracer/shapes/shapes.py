"""Analytic shapes (shapes/shapes.py).  ``Sphere`` intersects on the HIP kernel
``nrt_sphere_intersect`` (quad_solve in the reference's float32 op order) and hands Direct /
Debug / Depth ... the same interaction record as an SDF (hit list included), so the fused
shading runs on its hits; utils.sphere_examples renders every BSDF basis on it."""
import math

import torch

from ... import _lib
from .sdfs import HipInteraction

EPS = 1e-8  # shapes.py:9


class Shape(torch.nn.Module):
    """shapes.py:20-29."""

    def __init__(self):
        super().__init__()

    def intersect(self, rays, max_t=math.inf, active=True):
        raise NotImplementedError()

    def intersect_test(self, rays, max_t=math.inf, active=True):
        return self.intersect(rays, max_t=max_t, active=active)[1]

    def intersect_limits(self, rays, max_t=math.inf, active=True):
        raise NotImplementedError()


class Sphere(Shape):
    """One analytic sphere (shapes.py:31-97).  Like the reference it is a plain object (its
    ``__init__`` never runs nn.Module's), one sphere per instance."""

    def __init__(self, center, radius, device="cuda"):
        self.device = torch.device(device)
        self.center = torch.tensor(center, device=device, dtype=torch.float)
        self.radius = float(radius)
        self.sqr_radius = self.radius * self.radius

    def __len__(self):
        return 1

    def _host_center(self):
        c = self.center.detach().reshape(3).float().cpu().contiguous()
        return c

    def _run(self, rays, want_p=True, want_upper=False, want_list=True):
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        dev = flat.device
        t = torch.empty(P, device=dev)
        hit = torch.empty(P, dtype=torch.uint8, device=dev)
        p = torch.empty(P, 3, device=dev) if want_p else None
        n = torch.empty(P, 3, device=dev) if want_p else None
        upper = torch.empty(P, device=dev) if want_upper else None
        hit_idx = torch.empty(max(P, 1), dtype=torch.int32, device=dev) if want_list else None
        hit_count = torch.zeros(1, dtype=torch.int32, device=dev) if want_list else None
        c = self._host_center()
        _lib.load(require_device=True)
        _lib.call("nrt_sphere_intersect", _lib.ptr(c), float(self.radius), _lib.ptr(flat), P,
                  _lib.ptr(t), _lib.ptr(hit), _lib.ptr(p), _lib.ptr(n), _lib.ptr(upper),
                  _lib.ptr(hit_idx), _lib.ptr(hit_count), _lib.stream())
        return lead, flat, P, t, hit.bool().reshape(lead), p, n, upper, hit_idx, hit_count

    def intersect(self, rays, active=True, primary=True):
        """shapes.py:47-69: SurfaceInteraction(p, t, n, frame, wi = to_local(-d)), mask."""
        if rays.device.type != "cuda":
            raise _lib.NrtError("Sphere.intersect runs on the HIP path: rays must be on the GPU")
        lead, flat, P, t, hit, p, n, _, hit_idx, hit_count = self._run(rays)
        si = HipInteraction(p=p.reshape(lead + (3,)), t=t.reshape(lead), obj=self)
        si.n = n.reshape(lead + (3,))
        frame = torch.empty(P, 9, device=flat.device)
        wi = torch.empty(P, 3, device=flat.device)
        if P:
            _lib.call("nrt_frames", _lib.ptr(flat), _lib.ptr(n), P, _lib.ptr(frame), _lib.ptr(wi),
                      _lib.stream())
        si.frame = frame.reshape(lead + (3, 3))
        si.wi = wi.reshape(lead + (3,))
        si._nrt_hits = (hit_idx, hit_count, flat)
        si._nrt_hit_mask = hit
        return si, hit

    def intersect_test(self, rays, active=True):
        """shapes.py:70-77: the hit mask alone (the reference's signature: no max_t)."""
        if rays.device.type != "cuda":
            raise _lib.NrtError("Sphere.intersect_test runs on the HIP path: rays must be on the GPU")
        return self._run(rays, want_p=False, want_list=False)[4]

    def intersect_limits(self, rays, max_t=math.inf, active=True):
        """shapes.py:78-91: (nearer root, farther root, mask), roots < EPS as inf."""
        if rays.device.type != "cuda":
            raise _lib.NrtError("Sphere.intersect_limits runs on the HIP path: rays must be on the GPU")
        lead, _, _, t, hit, _, _, upper, _, _ = self._run(rays, want_p=False, want_upper=True,
                                                          want_list=False)
        return t.reshape(lead), upper.reshape(lead), hit


class SphereCloud(Shape):
    """SphereCloud (shapes.py:99-206): the nearest of N analytic spheres per ray on the HIP kernel
    ``nrt_sphere_cloud_intersect`` (one thread per ray over the sphere table; quad_solve per
    sphere in the reference's float32 op order, split_n spheres per pass as the reference's
    chunks).  The reference's tensor broadcasting is well-formed for one sphere only; there the
    results are its own bit for bit, and more spheres follow the same per-ray statements."""

    def __init__(self, centers=[[0, 0, 0]], radii=1, device="cuda"):
        self.device = torch.device(device)
        N = len(centers)
        self.centers = torch.zeros([N, 3], dtype=torch.float, device=self.device)
        for i in range(N):
            self.centers[i] = torch.tensor(centers[i], device=device)
        self.radii = torch.full([N], radii, dtype=torch.float, device=self.device)

    def __len__(self):
        return 1

    def _table(self, dev):
        return torch.cat([self.centers.detach().float(), self.radii.detach().float()[:, None]],
                         dim=-1).to(dev).contiguous()

    def _run(self, rays, t_max, split_n, want_p=True, want_list=True):
        if rays.device.type != "cuda":
            raise _lib.NrtError("SphereCloud runs on the HIP path: rays must be on the GPU")
        lead = rays.shape[:-1]
        flat = rays.reshape(-1, 6).float().contiguous()
        P = flat.shape[0]
        dev = flat.device
        table = self._table(dev)
        t = torch.empty(P, device=dev)
        hit = torch.empty(P, dtype=torch.uint8, device=dev)
        p = torch.empty(P, 3, device=dev) if want_p else None
        n = torch.empty(P, 3, device=dev) if want_p else None
        hit_idx = torch.empty(max(P, 1), dtype=torch.int32, device=dev) if want_list else None
        hit_count = torch.zeros(1, dtype=torch.int32, device=dev) if want_list else None
        _lib.load(require_device=True)
        _lib.call("nrt_sphere_cloud_intersect", _lib.ptr(table), table.shape[0], int(split_n),
                  float(t_max), _lib.ptr(flat), P, _lib.ptr(t), _lib.ptr(hit), _lib.ptr(p),
                  _lib.ptr(n), _lib.ptr(hit_idx), _lib.ptr(hit_count), _lib.stream())
        return lead, flat, P, t, hit.bool().reshape(lead), p, n, hit_idx, hit_count

    def intersect(self, rays, active=True, t_max=math.inf, split_n=256):
        """shapes.py:111-179: SurfaceInteraction(p, t, n, frame, wi = to_local(-d)), hit mask."""
        lead, flat, P, t, hit, p, n, hit_idx, hit_count = self._run(rays, t_max, split_n)
        si = HipInteraction(p=p.reshape(lead + (3,)), t=t.reshape(lead), obj=self)
        si.n = n.reshape(lead + (3,))
        frame = torch.empty(P, 9, device=flat.device)
        wi = torch.empty(P, 3, device=flat.device)
        if P:
            _lib.call("nrt_frames", _lib.ptr(flat), _lib.ptr(n), P, _lib.ptr(frame), _lib.ptr(wi),
                      _lib.stream())
        si.frame = frame.reshape(lead + (3, 3))
        si.wi = wi.reshape(lead + (3,))
        si._nrt_hits = (hit_idx, hit_count, flat)
        si._nrt_hit_mask = hit
        return si, hit

    def intersect_test(self, rays, active=True, t_max=math.inf, split_n=256):
        """shapes.py:180-206: the hit mask alone."""
        return self._run(rays, t_max, split_n, want_p=False, want_list=False)[4]
