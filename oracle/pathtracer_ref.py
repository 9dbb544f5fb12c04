"""CPU restatement of the reference ray-march render path (TEST INFRASTRUCTURE ONLY).

This module is the parity oracle for the HIP path in ``neural_raytracing_amd``.  It is
eager PyTorch on the CPU, written from a text reading of
``prashantraina/neural_raytracing`` (``pytorch3d/pathtracer``); the reference itself is never
imported or executed (SURVEY.md §8c records that running it is denied).  Every function names
the reference file:line it restates.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package, and only as the checker.

Parity pin: ``tests/test_oracle.py::test_reference_checksum`` rebuilds the single reference
run recorded in BASELINE.md §2 (same seeds, same construction order, same render call) and
checks ``out.abs().sum() == 4511.5146484375``.  That is the only output of the reference that
exists; everything else is pinned by known-answer tests derived from the code.

Conventions: the reference computes on tensors shaped ``[N, W, H, B, C]`` (cameras, tile
rows, tile cols, bundle, channels).  The restatement keeps those shapes where they change
arithmetic (batched BLAS calls, squeeze quirks) so results match op for op.
"""
import math
import random
import numpy as np

import torch
import torch.nn as nn
import torch.nn.functional as F


# ---------------------------------------------------------------------------------------------
# Fourier-feature skip MLP  (neural_blocks.py:12-86, utils.py:33-40)
# ---------------------------------------------------------------------------------------------

def fourier_encode(x, basis):
    """``[x, sin(xB), cos(xB)]`` -- utils.py:37-40 (fourier2)."""
    proj = x @ basis
    return torch.cat([x, proj.sin(), proj.cos()], dim=-1)


def leaky_relu(x):
    # neural_blocks.py:26 default activation (negative_slope 0.01)
    return F.leaky_relu(x)


def softplus(x):
    # sdfs.py:29 (F.softplus) and nn.Softplus() -- beta 1, threshold 20
    return F.softplus(x)


ACTIVATIONS = {"leaky_relu": leaky_relu, "softplus": softplus, "sigmoid": torch.sigmoid}


class SkipMLP(nn.Module):
    """Restatement of ``SkipConnMLP`` (neural_blocks.py:12-86).

    The RNG consumption order of the constructor is the reference's: the Fourier basis
    (``sigma * randn(freqs, in).T``, utils.py:33-36), then the hidden ``nn.Linear`` list in
    index order (:46-51), then ``init`` (:53), then ``out`` (:55), then the optional zero / xavier
    re-initialisation over ``[init, out, *layers]`` (:56-71).
    """

    def __init__(self, num_layers=8, hidden_size=64, in_size=3, out=3, skip=3, freqs=16,
                 sigma=32, activation="leaky_relu", latent_size=0, zero_init=False,
                 xavier_init=False):
        super().__init__()
        self.in_size = in_size
        self.basis_p = sigma * torch.randn(freqs, in_size).T
        self.dim_p = 2 * freqs + in_size + latent_size
        self.skip = skip
        self.latent_size = latent_size
        self.layers = nn.ModuleList([
            nn.Linear(hidden_size + self.dim_p if self.is_skip(i, num_layers) else hidden_size,
                      hidden_size)
            for i in range(num_layers)
        ])
        self.init = nn.Linear(self.dim_p, hidden_size)
        self.out = nn.Linear(hidden_size, out)
        self.act_name = activation
        ordered = [self.init, self.out, *self.layers]
        if zero_init:
            for lin in ordered:
                nn.init.zeros_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)
        if xavier_init:
            for lin in ordered:
                nn.init.xavier_uniform_(lin.weight)
            for lin in ordered:
                nn.init.zeros_(lin.bias)

    def is_skip(self, i, n=None):
        n = len(self.layers) if n is None else n
        return i != n - 1 and i % self.skip == 0

    def forward(self, p, latent=None):
        act = ACTIVATIONS[self.act_name]
        lead = p.shape[:-1]
        enc = fourier_encode(p.reshape(-1, self.in_size), self.basis_p)
        if latent is not None:
            enc = torch.cat([enc, latent.reshape(-1, self.latent_size)], dim=-1)
        h = self.init(enc)
        for i, lin in enumerate(self.layers):
            if self.is_skip(i):
                h = torch.cat([h, enc], dim=-1)
            h = lin(act(h))
        y = self.out(act(h))
        return y.reshape(lead + (y.shape[-1],))


# ---------------------------------------------------------------------------------------------
# Shapes  (shapes/sdfs.py, utils.py:386-387)
# ---------------------------------------------------------------------------------------------

def smooth_min(v, k: float = 32.0, dim: int = 0):
    """utils.py:385-387: ``-log(clamp(sum(exp(-k v)), 1e-4)) / k``."""
    return -torch.exp(-k * v).sum(dim).clamp(min=1e-4).log() / k


def unit_sphere_sdf(p):
    """SPHERE_SDF, sdfs.py:13."""
    return torch.norm(p, dim=-1) - 1


class SphereBlobSDF(nn.Module):
    """Restatement of ``SphereSDF`` (sdfs.py:16-44).

    ``shift`` is normally ``SkipMLP(8, 128, F=32, softplus, zero_init)``; the ``shift_*``
    arguments let a test or bench substitute a different residual MLP (e.g. 8x256).
    """

    def __init__(self, n=128, shift_layers=8, shift_hidden=128, shift_freqs=32,
                 shift_zero_init=True):
        super().__init__()
        self.centers = nn.Parameter(0.3 * torch.rand(n, 3) - 0.15)
        self.radii = nn.Parameter(0.2 * torch.rand(n) - 0.1)
        self.tfs = nn.Parameter(torch.zeros(n, 3, 3))
        self.shift = SkipMLP(num_layers=shift_layers, hidden_size=shift_hidden, in_size=3, out=1,
                             freqs=shift_freqs, activation="softplus",
                             zero_init=shift_zero_init)

    def spheres(self, p):
        # sdfs.py:37-43
        tfs = self.tfs + torch.eye(3).unsqueeze(0)
        flat = p.reshape(-1, 3).unsqueeze(0)
        q = torch.einsum("ijk,ibk->ibj", tfs, flat.expand(tfs.shape[0], -1, -1))
        q = q - self.centers.unsqueeze(1)
        sd = q.norm(p=2, dim=-1) - self.radii.unsqueeze(-1)
        return smooth_min(sd, k=32.0).reshape(p.shape[:-1])

    def forward(self, p):
        out = self.spheres(p)
        return out + self.shift(p).reshape_as(out)


class MarchedSDF:
    """Restatement of ``SDF`` (sdfs.py:89-277): sphere tracing, coarse scan, normals."""

    def __init__(self, sdf=unit_sphere_sdf, epsilon=1e-3, max_steps=32, dist=2.2,
                 create_graph=False):
        # create_graph=True keeps the normals differentiable, as the reference's autograd_diff
        # does (sdfs.py:184-197) -- used by the training-gradient tests
        self.create_graph = create_graph
        self.sdf = sdf
        self.epsilon = epsilon
        self.max_steps = max_steps
        self.dist = dist

    def __len__(self):
        return 1

    def coarse_scan(self, origin, direction, jitter=None):
        """sdfs.py:232-249.  ``jitter`` replaces the reference's ``random.random()``."""
        n = 128
        if jitter is None:
            jitter = random.random()
        max_t = self.dist + jitter * (2 / n)
        step = max_t / n
        with torch.no_grad():
            best = self.sdf(origin).squeeze(-1)
            idx = torch.zeros_like(best, dtype=torch.long)
            for i in range(n):
                s = self.sdf(origin + step * (i + 1) * direction).squeeze(-1)
                idx = torch.where(s < best, i + 1, idx)
                best = torch.minimum(best, s)
        best_pos = origin + idx.unsqueeze(-1).unsqueeze(-1) * step * direction
        return self.sdf(best_pos), best_pos

    def march(self, origin, direction, max_t=10):
        """Fixed-step sphere tracing, sdfs.py:114-131 (every ray, every step)."""
        t = torch.zeros(origin.shape[:-1] + (1,))
        live = torch.ones(t.shape[:-1], dtype=torch.bool)
        hit = torch.zeros_like(live)
        with torch.no_grad():
            for _ in range(self.max_steps):
                live = live & (t < max_t).squeeze(-1)
                d = self.sdf(origin + direction * t)
                now = live & (d <= self.epsilon)
                hit = hit | now
                live = live & ~now
                t = torch.where(live.unsqueeze(-1), t + d.unsqueeze(-1), t)
        return t, hit

    def gradient(self, p):
        """sdfs.py:184-197 (autograd normal, un-normalised)."""
        with torch.enable_grad():
            p = p.detach().requires_grad_()
            out = self.sdf(p)
            (g,) = torch.autograd.grad(out, p, torch.ones_like(out),
                                       create_graph=self.create_graph)
        return g

    def intersect(self, rays, max_t=10, active=True, primary=True, jitter=None):
        """sdfs.py:111-160.  Returns (interaction dict, hit mask)."""
        origin, direction = rays.split(3, dim=-1)
        t, hit = self.march(origin, direction, max_t)
        p = origin + t * direction
        throughput = 0
        if primary:
            thr, _ = self.coarse_scan(origin, direction, jitter)
            throughput = -1000 * thr
        it = Interaction(p=p, t=t.squeeze(), throughput=throughput)
        n = torch.zeros_like(p)
        if hit.any():
            raw = self.gradient(p[hit])
            it.raw_normals = raw
            n[hit] = F.normalize(raw, eps=1e-6, dim=-1)
            p[hit] = p[hit] + n[hit] * self.epsilon * 5
        it.set_normals(n)
        it.wi = it.to_local(-direction)
        return it, hit

    def intersect_test(self, rays, max_t=10, active=True):
        """Shadow-ray march from t0 = 100*eps, sdfs.py:162-181."""
        origin, direction = rays.split(3, dim=-1)
        t = torch.zeros(origin.shape[:-1] + (1,)) + 1e2 * self.epsilon
        live = torch.ones(t.shape[:-1], dtype=torch.bool)
        with torch.no_grad():
            for _ in range(self.max_steps):
                d = self.sdf(origin + direction * t)
                now = live & (d < self.epsilon)
                t = torch.where(live.unsqueeze(-1), t + d.unsqueeze(-1), t)
                live = live & ~now
        return (t >= max_t).squeeze(-1) | live


# ---------------------------------------------------------------------------------------------
# The analytic Sphere  (shapes/shapes.py:9-97)
# ---------------------------------------------------------------------------------------------

SPHERE_EPS = 1e-8  # shapes.py:9


def quad_solve(a, b, c):
    """shapes.py:11-18: roots [..., 2] of a t^2 + b t + c (sqrt only where the discriminant is
    positive; elsewhere the discriminant itself stands in) and the validity mask."""
    d = b * b - 4 * a * c
    valid = d > 0
    d[valid] = d[valid].sqrt()
    s = torch.stack([d, -d], dim=-1)
    return (-b[..., None] + s) / (2 * a[..., None]), valid


class SphereRef:
    """Sphere, shapes.py:31-97 (one sphere)."""

    def __init__(self, center=(0.0, 0.0, 0.0), radius=1.0):
        self.center = torch.tensor(list(center), dtype=torch.float)
        self.radius = float(radius)
        self.sqr_radius = self.radius * self.radius

    def __len__(self):
        return 1

    def _roots(self, rays):
        r_o, r_d = torch.split(rays, 3, dim=-1)
        fs = r_o - self.center
        a = torch.sum(r_d * r_d, dim=-1)
        b = 2 * torch.sum(r_d * fs, dim=-1)
        c = torch.sum(fs * fs, dim=-1) - self.sqr_radius
        return r_o, r_d, quad_solve(a, b, c)

    def intersect(self, rays, max_t=None, active=True, primary=True, jitter=None):
        """shapes.py:47-69 (no scan, no throughput: a SurfaceInteraction)."""
        r_o, r_d, (ts, mask) = self._roots(rays)
        mask = mask & (ts >= SPHERE_EPS).any(-1)
        ts[ts < SPHERE_EPS] = math.inf
        t, _ = ts.min(dim=-1)
        p = r_o + t[..., None] * r_d
        n = F.normalize(p - self.center, dim=-1)
        p = p + n * 1e-5
        it = Interaction(p=p, t=t)
        it.set_normals(n)
        it.wi = it.to_local(-r_d)
        return it, mask

    def intersect_test(self, rays, max_t=None, active=True):
        """shapes.py:70-77."""
        _, _, (ts, mask) = self._roots(rays)
        return mask & (ts >= SPHERE_EPS).any(-1)

    def intersect_limits(self, rays, max_t=None, active=True):
        """shapes.py:78-91."""
        _, _, (ts, mask) = self._roots(rays)
        mask = mask & (ts >= SPHERE_EPS).any(-1)
        ts[ts < SPHERE_EPS] = math.inf
        return ts.min(dim=-1)[0], ts.max(dim=-1)[0], mask


class SphereCloudRef:
    """SphereCloud, shapes.py:99-206, statement by statement -- including its broadcasting, which
    is well-formed for one sphere only: intersect's `sphere_exp ... .transpose(0, 1)` (:131-132)
    pairs every sphere with every row of rays unless N = 1 and the rays' first dim is 1, and
    intersect_test's `(radii * radii)[..., None]` (:196) aligns [N, 1] with the rays' last two
    dims.  The parity tests run it where it is well-formed; the HIP kernel states the per-ray
    nearest-hit semantics those cases pin (test_gpu_sphere.py)."""

    def __init__(self, centers=((0.0, 0.0, 0.0),), radii=1.0):
        N = len(centers)
        self.centers = torch.zeros([N, 3], dtype=torch.float)
        for i in range(N):
            self.centers[i] = torch.tensor(list(centers[i]), dtype=torch.float)
        self.radii = torch.full([N], radii, dtype=torch.float)

    def __len__(self):
        return 1

    def intersect(self, rays, active=True, t_max=math.inf, split_n=256):
        """shapes.py:111-179."""
        r_o, r_d = torch.split(rays, 3, dim=-1)
        out_active = torch.zeros(r_o.shape[:-1], dtype=torch.bool)
        best_dists = torch.full_like(out_active, t_max, dtype=torch.float)
        best_faces = torch.full_like(out_active, -1, dtype=torch.long)
        r_o_r = r_o.expand(split_n, *r_o.shape)
        r_d_r = r_d.expand_as(r_o_r)
        for spheres, radii in zip(self.centers.split(split_n, dim=0), self.radii.split(split_n, dim=0)):
            batch_size = spheres.shape[0]
            r_o_r, r_d_r = r_o_r[:batch_size], r_d_r[:batch_size]
            sphere_exp = spheres[:, None, None, None].repeat(1, *r_d_r.shape[1:-1], 1).transpose(0, 1)
            radii_exp = radii[:, None, None, None].repeat(1, *r_d_r.shape[1:-1]).transpose(0, 1)
            fs = r_o_r - sphere_exp
            a = torch.sum(r_d_r * r_d_r, dim=-1)
            b = 2 * torch.sum(r_d_r * fs, dim=-1)
            c = torch.sum(fs * fs, dim=-1) - (radii_exp * radii_exp)
            intersections, mask = quad_solve(a, b, c)
            mask = mask & ((intersections >= SPHERE_EPS) & (intersections < t_max)).any(-1)
            intersections[intersections < SPHERE_EPS] = math.inf
            valid_mins = mask.any(0)
            out_active = out_active | valid_mins
            t, _ = intersections.min(dim=-1)
            t[~mask] = math.inf
            min_t, sph_idx = t.min(dim=0)
            lesser = best_dists > min_t
            replace_cond = valid_mins & lesser
            best_dists[replace_cond] = min_t[replace_cond]
            best_faces[replace_cond] = sph_idx[replace_cond]
        p = r_o + best_dists[..., None] * r_d
        n = torch.zeros_like(p, dtype=torch.float)
        n[out_active] = F.normalize(p[out_active] - self.centers[best_faces[out_active]], dim=-1)
        p += n * 1e-5
        it = Interaction(p=p, t=best_dists)
        it.set_normals(n)
        it.wi = it.to_local(-r_d)
        return it, out_active

    def intersect_test(self, rays, active=True, t_max=math.inf, split_n=256):
        """shapes.py:180-206."""
        r_o, r_d = torch.split(rays, 3, dim=-1)
        out_active = torch.zeros(r_o.shape[:-1], dtype=torch.bool)
        r_o_r = r_o.expand(split_n, *r_o.shape)
        r_d_r = r_d.expand_as(r_o_r)
        for spheres, radii in zip(self.centers.split(split_n, dim=0), self.radii.split(split_n, dim=0)):
            batch_size = spheres.shape[0]
            r_o_r, r_d_r = r_o_r[:batch_size], r_d_r[:batch_size]
            sphere_exp = spheres[:, None, None, None].repeat(1, *r_d_r.shape[1:-1], 1)
            fs = r_o_r - sphere_exp
            a = torch.sum(r_d_r * r_d_r, dim=-1)
            b = 2 * torch.sum(r_d_r * fs, dim=-1)
            c = torch.sum(fs * fs, dim=-1) - (radii * radii)[..., None]
            intersections, mask = quad_solve(a, b, c)
            mask = mask & ((intersections >= SPHERE_EPS) & (intersections < t_max)).any(-1)
            out_active = out_active | mask.any(0)
        return out_active


# ---------------------------------------------------------------------------------------------
# Interaction frames  (interaction.py:9-119)
# ---------------------------------------------------------------------------------------------

def shading_frame(n):
    """coordinate_system, interaction.py:9-27: columns [s, t, n]."""
    n = F.normalize(n, eps=1e-7, dim=-1)
    x, y, z = n.split(1, dim=-1)
    sign = torch.where(z >= 0, 1.0, -1.0)
    sz = sign + z
    a = -torch.where(sz.abs() < 1e-6, torch.tensor(1e-6), sz).reciprocal()
    b = x * y * a
    s = torch.cat([(x * x * a * sign) + 1, b * sign, x * -sign], dim=-1)
    s = F.normalize(s, eps=1e-7, dim=-1)
    t = F.normalize(s.cross(n, dim=-1), eps=1e-7, dim=-1)
    s = F.normalize(n.cross(t, dim=-1), eps=1e-7, dim=-1)
    return torch.stack([s, t, n], dim=-1)


def frame_to_local(frame, w):
    """interaction.py:37-41 (the /3 of the mean cancels in the normalize, but is kept)."""
    w = w.unsqueeze(-1).expand_as(frame)
    return F.normalize((frame * w).mean(dim=-2), eps=1e-7, dim=-1)


def frame_from_local(frame, v):
    """interaction.py:44-51."""
    s, t, n = frame.split(1, dim=-1)
    x, y, z = v.split(1, dim=-1)
    w = s.squeeze(-1) * x + t.squeeze(-1) * y + n.squeeze(-1) * z
    return F.normalize(w, eps=1e-7, dim=-1)


class Interaction:
    """MixedInteraction (interaction.py:61-106) as a plain attribute bag."""

    def __init__(self, p, t=None, throughput=None, with_logits=True):
        self.p = p
        self.t = t
        self.throughput = throughput
        self.with_logits = with_logits
        self.n = None
        self.frame = None
        self.wi = None

    def set_normals(self, n):
        self.n = n
        self.frame = shading_frame(n)

    def to_local(self, w):
        return frame_to_local(self.frame, w)

    def from_local(self, v):
        return frame_from_local(self.frame, v)


# ---------------------------------------------------------------------------------------------
# BSDF helpers  (utils.py:43-51, 152-155, 234-258; bsdf/bsdfs.py)
# ---------------------------------------------------------------------------------------------

def nonzero_eps(v, eps: float = 1e-7):
    """utils.py:43-51: values with |v| < eps become +eps."""
    return torch.where(v.abs() < eps, torch.tensor(eps), v)


def rodrigues(v, axis, c, s):
    """rotate_vector, utils.py:152-155."""
    return v * c + axis * (v * axis).sum(dim=-1, keepdim=True) * (1 - c) \
        + torch.cross(axis, v, dim=-1) * s


def rusinkiewicz(wo, wi):
    """param_rusin2, utils.py:233-258 -> [cos(phi_d), cos(theta_h), cos(theta_d)].

    Keeps the reference's ``sqrt(clamp(1 - cos_theta_h, 1e-6))`` (1-cos, not 1-cos^2).
    """
    wo = F.normalize(wo, dim=-1)
    wi = F.normalize(wi, dim=-1)
    ey = torch.tensor([0, 1, 0], dtype=wo.dtype).expand_as(wo)
    ez = torch.tensor([0, 0, 1], dtype=wo.dtype).expand_as(wo)
    h = F.normalize(wo + wi, dim=-1)
    cos_th = h[..., 2]
    r = nonzero_eps(h[..., 1]).hypot(nonzero_eps(h[..., 0])).clamp(min=1e-6)
    c = (h[..., 0] / r).unsqueeze(-1)
    s = -(h[..., 1] / r).unsqueeze(-1)
    tmp = F.normalize(rodrigues(wi, ez, c, s), dim=-1)
    c = h[..., 2].unsqueeze(-1)
    s = -(1 - h[..., 2]).clamp(min=1e-6).sqrt().unsqueeze(-1)
    diff = F.normalize(rodrigues(tmp, ey, c, s), dim=-1)
    cos_td = diff[..., 2]
    cos_pd = torch.atan2(nonzero_eps(diff[..., 1]), nonzero_eps(diff[..., 0])).cos()
    return torch.stack([cos_pd, cos_th, cos_td], dim=-1)


class NeuralBSDFRef(nn.Module):
    """NeuralBSDF, bsdfs.py:613-637: ``act(MLP_6x96,F=64(param_rusin2(it.wi, wo)))``, pdf 1."""

    def __init__(self, activation="sigmoid"):
        super().__init__()
        self.mlp = SkipMLP(in_size=3, out=3, num_layers=6, hidden_size=96, freqs=64)
        self.act_name = activation

    def act(self, x):
        return {"sigmoid": torch.sigmoid, "softplus": F.softplus}[self.act_name](x)

    def eval_and_pdf(self, it, wo, active=True):
        f = self.act(self.mlp(rusinkiewicz(it.wi, wo)))
        return f, torch.ones(f.shape[:-1])

    def joint_eval_pdf(self, it, wo, active=True):
        f, pdf = self.eval_and_pdf(it, wo, active)
        return torch.cat([f, pdf.reshape(f.shape[:-1] + (1,))], dim=-1)


class DiffuseRef(nn.Module):
    """Diffuse, bsdfs.py:78-118 (preprocess default x/pi)."""

    def __init__(self, reflectance=(0.25, 0.2, 0.7), preprocess="div_pi"):
        super().__init__()
        self.reflectance = torch.tensor(list(reflectance))
        self.preproc_name = preprocess

    def preproc(self, x):
        return {"div_pi": lambda v: v / math.pi, "sigmoid": torch.sigmoid,
                "softplus": F.softplus, "identity": lambda v: v}[self.preproc_name](x)

    def eval_and_pdf(self, it, wo, active=True):
        spectrum = self.preproc(wo[..., 2].unsqueeze(-1) * self.reflectance)
        return spectrum, wo[..., 2] / math.pi

    def joint_eval_pdf(self, it, wo, active=True):
        f, pdf = self.eval_and_pdf(it, wo, active)
        return torch.cat([f, pdf.reshape(f.shape[:-1] + (1,))], dim=-1)


def fresnel_conductor(cos_t, eta_r: float, eta_i: float):
    """bsdfs.py:327-341."""
    ct2 = cos_t * cos_t
    st2 = (1 - ct2).clamp(min=1e-10)
    st4 = st2 * st2
    tmp = eta_r * eta_r - eta_i * eta_i - st2
    a2pb2 = (tmp * tmp + 4 * eta_i * eta_i * eta_r * eta_r).clamp(min=1e-10).sqrt()
    a = (0.5 * (a2pb2 + tmp)).clamp(min=1e-10).sqrt()
    t1 = a2pb2 + ct2
    t2 = 2 * cos_t * a
    rs = (t1 - t2) / (t1 + t2)
    t3 = a2pb2 * ct2 + st4
    t4 = t2 * st2
    rp = rs * (t3 - t4) / (t3 + t4)
    return 0.5 * (rs + rp)


class ConductorRef(nn.Module):
    """Conductor, bsdfs.py:345-388."""

    def __init__(self, specular=(1.0, 1.0, 1.0), eta=1.3, k=1.0, activation="sigmoid"):
        super().__init__()
        self.eta = torch.tensor(eta)
        self.k = torch.tensor(k)
        self.specular = torch.tensor(list(specular))
        self.act_name = activation

    def act(self, x):
        return {"sigmoid": torch.sigmoid, "softplus": F.softplus}[self.act_name](x)

    def eval_and_pdf(self, it, wi_unused, active=True):
        wo = wi_unused
        refl = torch.cat([-it.wi[..., :1], -it.wi[..., 1:2], it.wi[..., 2:]], dim=-1)
        thresh = (refl * wo).sum(dim=-1, keepdim=True) > 0.94
        eta = F.softplus(self.eta).item()
        fres = fresnel_conductor(it.wi[..., 2], eta, 0.0).reshape_as(thresh)
        spectrum = torch.where(thresh, fres * self.act(self.specular),
                               torch.zeros(it.p.shape))
        pdf = torch.where(thresh.reshape(it.p.shape[:-1]), 1.0, 0.0)
        if not isinstance(active, bool):
            spectrum = torch.where(active.unsqueeze(-1), spectrum, torch.zeros_like(spectrum))
        return spectrum, pdf

    def joint_eval_pdf(self, it, wo, active=True):
        f, pdf = self.eval_and_pdf(it, wo, active)
        return torch.cat([f, pdf.reshape(f.shape[:-1] + (1,))], dim=-1)


class SpatialMixBSDF(nn.Module):
    """ComposeSpatialVarying, bsdfs.py:482-536.

    ``sp_var_fn = SkipMLP(16, 256, F=128, sigma=128, out=len(bsdfs), xavier)`` is built AFTER
    the component BSDFs (they are constructed in the caller's argument list).
    """

    def __init__(self, bsdfs):
        super().__init__()
        self.bsdfs = nn.ModuleList(bsdfs)
        self.sp_var_fn = SkipMLP(num_layers=16, hidden_size=256, freqs=128, sigma=2 << 6,
                                 in_size=3, out=len(bsdfs), xavier_init=True)

    def weights(self, p):
        w = self.sp_var_fn(p).reshape(p.shape[:-1] + (len(self.bsdfs),))
        return w.sigmoid()

    def eval_and_pdf(self, it, wo, active=True):
        k = self.weights(it.p)
        parts = torch.stack([b.joint_eval_pdf(it, wo, active) for b in self.bsdfs], dim=-1)
        it.normalized_weights = k
        parts = torch.where(active[..., None, None], parts * k.unsqueeze(-2),
                            torch.zeros_like(parts))
        spectrum, pdf = parts.sum(dim=-1).split([3, 1], dim=-1)
        return spectrum, pdf.squeeze(-1)


# ---------------------------------------------------------------------------------------------
# Lights  (lights/lights.py, scene.py:290-324)
# ---------------------------------------------------------------------------------------------

class LightSample:
    def __init__(self, d, pdf, dist=None):
        self.d = d
        self.pdf = pdf
        self.dist = dist


class LightFieldRef(nn.Module):
    """LightField, lights.py:155-195: direction/magnitude from a 10x256 MLP, colour sigmoid."""

    def __init__(self):
        super().__init__()
        self.light_field_approx = SkipMLP(in_size=3, out=3, num_layers=10, hidden_size=256)
        self.color = nn.Parameter(torch.zeros(3))

    def sample_direction(self, it, active):
        v = self.light_field_approx(it.p[active])
        d = torch.zeros_like(it.p)
        d[active] = F.normalize(v, eps=1e-6, dim=-1).clamp(min=1e-6, max=1)
        le = torch.zeros_like(it.p)
        le[active] = torch.linalg.norm(v, ord=2, dim=-1, keepdim=True) * self.color.sigmoid()
        return LightSample(d, torch.ones(it.p.shape[:-1])), le


class PointLightRef(nn.Module):
    """PointLights, lights.py:40-110 (one light)."""

    def __init__(self, intensity=(1.0, 1.0, 1.0), location=(0.0, 1.0, 0.0), const=1e-8,
                 linear=1e-8, square=1.0, scale=1e2):
        super().__init__()
        self.scale = torch.tensor(float(scale))
        self.intensity = torch.tensor([list(intensity)], dtype=torch.float)
        self.location = torch.tensor(list(location), dtype=torch.float).reshape(-1, 3)
        self.const = torch.tensor(float(const))
        self.linear = torch.tensor(float(linear))
        self.square = torch.tensor(float(square))

    def sample_direction(self, it, active):
        # the reference broadcasts location as [L,1,1,1,3] against p [N,W,H,B,3]
        shape = (-1,) + (1,) * (it.p.dim() - 2) + (3,)
        d = self.location.reshape(shape) - it.p
        dist = torch.linalg.norm(d, dim=-1, keepdim=True)
        d = F.normalize(d, eps=1e-6, dim=-1)
        fall = self.const.clamp(min=1e-6) + self.linear.clamp(min=1e-6) * dist \
            + self.square.clamp(min=1e-6) * dist.square()
        color = self.intensity.reshape(shape)
        le = self.scale * F.normalize(color, dim=-1) / fall.clamp(min=1e-6)
        le = le.expand_as(it.p).clone() if le.shape != it.p.shape else le
        le[~active] = 0
        return LightSample(d, 1, dist), le


class RendererPointLightRef(nn.Module):
    """pytorch3d.renderer.PointLights of the reference's fork (renderer/lighting.py:221-304):
    intensity = ambient_color, sample_direction d = (loc - p) inv, Le = scale I inv inv with
    inv = 1 / (1e-7 + |loc - p|)."""

    def __init__(self, ambient_color=((0.5, 0.5, 0.5),), location=((0.0, 1.0, 0.0),), scale=1e-2):
        super().__init__()
        self.location = torch.tensor(location, dtype=torch.float).reshape(-1, 3)
        self.intensity = torch.tensor(ambient_color)
        self.scale = scale

    def sample_direction(self, it, active):
        d = self.location - it.p
        dist = (d * d).sum(dim=-1, keepdim=True).sqrt()
        inv_dist = (1e-7 + dist).reciprocal()
        d = d * inv_dist
        spectrum = self.scale * self.intensity * inv_dist * inv_dist
        le = spectrum.expand_as(it.p).clone() if spectrum.shape != it.p.shape else spectrum
        le[~active] = 0
        return LightSample(d, 1, dist), le


def elev_azim_to_dir(elev_azim):
    """utils.py:478-486."""
    limit = math.pi - 1e-7
    elev, azim = elev_azim.clamp(min=-limit, max=limit).split(1, dim=-1)
    return torch.cat([azim.sin() * elev.cos(), azim.cos() * elev.cos(), elev.sin()], dim=-1)


def point_light_envmap(light, p):
    """PointLights.envmap, lights.py:81-88."""
    d = p[None, ...] - light.location[:, None, None, :]
    dist = torch.linalg.norm(d, dim=-1, keepdim=True)
    fall = light.const.clamp(min=1e-6) + light.linear.clamp(min=1e-6) * dist \
        + light.square.clamp(min=1e-6) * dist.square()
    return light.scale * F.normalize(light.intensity, dim=-1) / fall.clamp(min=1e-6)


def emitter_no_shadow(it, lights, active):
    """sample_emitter_dir_wo_isect, scene.py:321-324."""
    ds, le = lights.sample_direction(it, active)
    le[~active] = 0
    return ds, le


def emitter_shadow_ray(it, shape, lights, active):
    """sample_emitter_dir_w_isect, scene.py:290-298."""
    ds, le = lights.sample_direction(it, active)
    rays = torch.cat([it.p, ds.d], dim=-1)
    visible = shape.intersect_test(rays, max_t=ds.dist.reshape_as(active)[..., None],
                                   active=active)
    le[~visible | ~active] = 0
    return ds, le


def dir_to_elev_azim(direc):
    """utils.py:490-494."""
    x, y, z = F.normalize(direc, dim=-1).clamp(min=-1 + 1e-7, max=1 - 1e-7).split(1, dim=-1)
    elev = z.asin()
    azim = torch.atan2(x, (1 - x.square() - z.square()).clamp(min=1e-10).sqrt())
    return torch.cat([elev, azim], dim=-1)


def emitter_learned_occ(it, shape, lights, occ, active):
    """sample_emitter_dir_w_learned_occ, scene.py:301-319."""
    ds, le = lights.sample_direction(it, active)
    rays = torch.cat([it.p, ds.d], dim=-1)
    visible = shape.intersect_test(rays, max_t=ds.dist.reshape_as(active)[..., None],
                                   active=active)
    occ_rays = torch.cat([it.p, dir_to_elev_azim(ds.d)], dim=-1)
    le = torch.where((~visible)[..., None], occ(occ_rays).sigmoid() * le, le)
    return ds, active[..., None] * le


def emitter(it, shape, lights, active, w_isect):
    """The sample_emitter choice of integrators.py:161-166 / :287-291."""
    if w_isect is True:
        return emitter_shadow_ray(it, shape, lights, active)
    if isinstance(w_isect, SkipMLP):
        return emitter_learned_occ(it, shape, lights, w_isect, active)
    return emitter_no_shadow(it, lights, active)


# ---------------------------------------------------------------------------------------------
# Integrators  (integrators/integrators.py)
# ---------------------------------------------------------------------------------------------

class DirectRef:
    """Direct, integrators.py:139-206 with emitter_samples=1, bsdf_samples=0.

    ``primary`` is always True: ``Direct.__init__`` assigns ``training`` before
    ``nn.Module.__init__`` resets it (:153-154), so the coarse scan always runs.
    """

    def dims(self):
        return 3

    def sample(self, shape, rays, bsdf, lights, w_isect=False, jitter=None):
        result = torch.zeros(*rays.shape[:-1], 3)
        it, active = shape.intersect(rays, primary=True, jitter=jitter)
        if not active.any():
            return result, active, it
        ds, le = emitter(it, shape, lights, active, w_isect)
        ae = active & (torch.as_tensor(ds.pdf) > 0)
        wo = it.to_local(ds.d)
        f, pdf = bsdf.eval_and_pdf(it, wo, active=ae)
        mis = torch.ones_like(pdf.reshape_as(ae))
        val = mis[ae].unsqueeze(-1) * f[ae] * le[ae]
        val = val / 1
        result[ae] = result[ae] + val
        return result, active, it


class NeRFIntegratorRef:
    """NeRFIntegrator, integrators.py:243-257: append sigmoid(throughput) as alpha."""

    def __init__(self, sub):
        self.sub = sub

    def dims(self):
        return self.sub.dims() + 1

    def sample(self, shape, rays, bsdf, lights, w_isect=False, jitter=None):
        rgb, _, it = self.sub.sample(shape, rays, bsdf, lights, w_isect=w_isect, jitter=jitter)
        alpha = it.throughput.unsqueeze(-1)
        if it.with_logits:
            alpha = alpha.sigmoid()
        return torch.cat([rgb, alpha], dim=-1), torch.tensor(True), it


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


def square_to_cos_hemisphere(sample):
    """warps.py:44-49."""
    p = square_to_uniform_disk_concentric(sample)
    z = (1 - (p * p).sum(dim=-1, keepdim=True)).clamp(min=1e-7).sqrt()
    return torch.cat([p, z], dim=-1)


def bsdf_sample_ref(bsdf, it, u_comp, u_sel, active):
    """ComposeSpatialVarying.sample (bsdfs.py:500-513) with NeuralBSDF.sample (:625-633) and
    Diffuse.sample (:90-106) components, randomness injected: u_comp[..., c, :] is component c's
    sampler.sample(shape + (2,)) draw (component order), and the torch.multinomial(k) selection
    is the inverse CDF of k / sum(k) at u_sel (same distribution; torch's internal draw cannot be
    replayed).  Returns (wo_local, spectrum) of the selected component."""
    parts = bsdf.bsdfs if isinstance(bsdf, SpatialMixBSDF) else [bsdf]
    wos, specs = [], []
    for c, b in enumerate(parts):
        wo = F.normalize(square_to_cos_hemisphere(u_comp[..., c, :]), dim=-1)
        if isinstance(b, NeuralBSDFRef):
            spec = b.act(b.mlp(rusinkiewicz(it.wi, wo)))
        elif isinstance(b, DiffuseRef):
            if not ((it.wi[..., 2] > 0) & active).any():  # bsdfs.py:95-96
                wo, spec = torch.zeros_like(it.p), torch.zeros_like(it.p)
            else:
                spec = b.preproc(b.reflectance).expand(it.p.shape).clone()
        else:
            raise NotImplementedError("Conductor.sample crashes in the reference (bsdfs.py:396)")
        wos.append(wo)
        specs.append(spec)
    if isinstance(bsdf, SpatialMixBSDF):
        k = bsdf.weights(it.p)
    else:
        k = torch.ones(it.p.shape[:-1] + (1,))
    cdf = torch.cumsum(k / k.sum(dim=-1, keepdim=True), dim=-1)
    sel = (u_sel.unsqueeze(-1) >= cdf).sum(dim=-1).clamp(max=len(parts) - 1)
    wo = torch.stack(wos, dim=-1).gather(-1, sel[..., None, None].expand(it.p.shape + (1,))).squeeze(-1)
    spec = torch.stack(specs, dim=-1).gather(-1, sel[..., None, None].expand(it.p.shape + (1,))).squeeze(-1)
    return F.normalize(wo, dim=-1), spec


class PathRef:
    """Path.sample (integrators.py:275-354), max_depth 2, no Russian roulette (rr_depth 5 is never
    reached), mis = 1.  ``training`` stays False (set after nn.Module.__init__, :276-278), so the
    primary intersection runs without the coarse scan.  ``uniforms[depth] = (u_comp, u_sel)``
    injects the BSDF-sampling randomness (see bsdf_sample_ref)."""

    def __init__(self, max_depth=2):
        self.max_depth = max_depth

    def dims(self):
        return 3

    def sample(self, shape, rays, bsdf, lights, w_isect=False, jitter=None, uniforms=None):
        throughput = torch.ones(*rays.shape[:-1], 3)
        result = torch.zeros_like(throughput)
        it, active = shape.intersect(rays, primary=False)
        if not active.any():
            return result, active, it
        original_active = active.clone()
        curr = it
        for depth in range(self.max_depth):
            if active.any():
                ds, le = emitter(curr, shape, lights, active, w_isect)
                ae = active & (torch.as_tensor(ds.pdf) > 0)
                wo = curr.to_local(ds.d)
                f, pdf = bsdf.eval_and_pdf(curr, wo, active=ae)
                mis = torch.ones_like(pdf.reshape(ae.shape))
                result = result + torch.where(ae.unsqueeze(-1),
                                              mis.unsqueeze(-1) * throughput * f * le,
                                              torch.zeros_like(result))
            u_comp, u_sel = uniforms[depth]
            wo_l, spec = bsdf_sample_ref(bsdf, curr, u_comp, u_sel, active)
            throughput = spec.clamp(min=1e-10) * throughput
            throughput = throughput.detach()  # "detach to save memory" (integrators.py:336-337)
            active = active & (throughput > 0).any(-1)
            if not active.any():
                break
            d = curr.from_local(wo_l)
            rays = torch.cat([curr.p.expand_as(d), d], dim=-1)
            curr, hits = shape.intersect(rays, primary=False)
            active = active & hits
            if not active.any():
                break
        return result, original_active, it


# ---------------------------------------------------------------------------------------------
# Cameras  (cameras/cameras.py)
# ---------------------------------------------------------------------------------------------

class NeRFCameraRef:
    """NeRFCamera.sample_positions, cameras.py:23-54."""

    def __init__(self, cam_to_world, focal):
        self.cam_to_world = cam_to_world
        self.focal = focal

    def __len__(self):
        return self.cam_to_world.shape[0]

    def sample_positions(self, pos, size, with_noise=0.0, noise=None):
        u, v = pos.split(1, dim=-1)
        if with_noise:
            if noise is None:
                nu, nv = torch.rand_like(u), torch.rand_like(v)
            else:
                nu, nv = noise
            u = u + (nu - 0.5) * with_noise
            v = v + (nv - 0.5) * with_noise
        d = torch.stack([(u - size * 0.5) / self.focal, -(v - size * 0.5) / self.focal,
                         -torch.ones_like(u)], dim=-1)
        r_d = torch.sum(d[..., None, :] * self.cam_to_world[..., :3, :3], dim=-1)
        r_d = F.normalize(r_d, dim=-1).permute(2, 0, 1, 3).unsqueeze(-2)
        r_o = self.cam_to_world[..., :3, -1][:, None, None, None, :].expand_as(r_d)
        return torch.cat([r_o, r_d], dim=-1)


class DTUCameraRef:
    """DTUCamera.sample_positions + lift, cameras.py:132-192 (with_noise ignored)."""

    def __init__(self, pose, intrinsic):
        self.pose = pose
        self.intrinsic = intrinsic

    def __len__(self):
        return self.pose.shape[0]

    def sample_positions(self, pos, size, bundle_size=1):
        r_o = self.pose[:, :3, 3]
        W, H, _ = pos.shape
        N = len(self)
        scale = torch.tensor([1600, 1200], dtype=torch.float) / size
        u, v = (pos * scale).reshape(-1, 2).split(1, dim=-1)
        u = u.reshape(1, -1).expand(N, -1)
        v = v.reshape(1, -1).expand(N, -1)
        K = self.intrinsic
        shape = u.shape
        fx = K[..., 0, 0, None].expand(shape)
        fy = K[..., 1, 1, None].expand(shape)
        cx = K[..., 0, 2, None].expand(shape)
        cy = K[..., 1, 2, None].expand(shape)
        sk = K[..., 0, 1, None].expand(shape)
        z = torch.ones_like(u)
        xl = (u - cx + cy * sk / fy - sk * v / fy) / fx * z
        yl = (v - cy) / fy * z
        pts = torch.stack([xl, yl, z, torch.ones_like(z)], dim=-1)
        world = torch.bmm(self.pose, pts.permute(0, 2, 1)).permute(0, 2, 1)[..., :3]
        r_o = r_o[:, None, :].expand_as(world)
        r_d = F.normalize(world - r_o, dim=-1)
        return torch.cat([r_o, r_d], dim=-1).reshape(N, W, H, 1, 6) \
            .expand(N, W, H, bundle_size, 6)


def look_at_view_transform_ref(dist=1.0, elev=0.0, azim=0.0, degrees=True, at=(0.0, 0.0, 0.0),
                               up=(0.0, 1.0, 0.0)):
    """renderer/cameras.py:1275-1310 (camera_position_from_spherical_angles), :1313-1360
    (look_at_rotation), :1363-1422 (look_at_view_transform) for one camera."""
    dist, elev, azim = (torch.tensor([float(v)]) for v in (dist, elev, azim))
    if degrees:
        elev = math.pi / 180.0 * elev
        azim = math.pi / 180.0 * azim
    x = dist * torch.cos(elev) * torch.sin(azim)
    y = dist * torch.sin(elev)
    z = dist * torch.cos(elev) * torch.cos(azim)
    at_t = torch.tensor([list(at)], dtype=torch.float)
    up_t = torch.tensor([list(up)], dtype=torch.float)
    C = torch.stack([x, y, z], dim=1).view(-1, 3) + at_t
    z_axis = F.normalize(at_t - C, eps=1e-5)
    x_axis = F.normalize(torch.cross(up_t, z_axis, dim=1), eps=1e-5)
    y_axis = F.normalize(torch.cross(z_axis, x_axis, dim=1), eps=1e-5)
    is_close = torch.isclose(x_axis, torch.tensor(0.0), atol=5e-3).all(dim=1, keepdim=True)
    if is_close.any():
        x_axis = torch.where(is_close, F.normalize(torch.cross(y_axis, z_axis, dim=1), eps=1e-5),
                             x_axis)
    R = torch.cat((x_axis[:, None, :], y_axis[:, None, :], z_axis[:, None, :]), dim=1)
    R = R.transpose(1, 2)
    T = -torch.bmm(R.transpose(1, 2), C[:, :, None])[:, :, 0]
    return R, T


class FoVCameraRef:
    """FoVPerspectiveCameras (renderer/cameras.py:314-575) with its Transform3d algebra
    (transforms/transform3d.py:175-324), one camera.

    The full projection is Rotate(R) . Translate(T) . K^T (row vectors, :170-195, :491-494);
    Transform3d.inverse() (invert_composed=False, :225-272) inverts the pieces and composes them in
    reverse: inv(K^T) @ Translate(-T) @ R^T, in that bmm order.  sample_positions (:539-575):
    jitter d*u - d/2, ndc = -2 pos/size + 1, unproject (x, y, 1) with a homogeneous divide and
    r_d = normalize(point) -- the point itself, not point - centre; r_o = the camera centre
    (get_camera_center, :143-149).
    """

    def __init__(self, R, T, znear=1e-2, zfar=1e4, aspect_ratio=1.0, fov=60.0, degrees=True):
        self.R, self.T = R.float(), T.float()
        self.znear, self.zfar, self.aspect, self.fov, self.degrees = znear, zfar, aspect_ratio, fov, degrees

    def __len__(self):
        return 1

    def projection(self):
        # compute_projection_matrix, renderer/cameras.py:389-439; TensorProperties
        # (renderer/utils.py:91-130) has made znear, zfar, aspect_ratio and fov float32 [N]
        f32 = lambda v: torch.tensor([float(v)], dtype=torch.float32)  # noqa: E731
        znear, zfar, aspect, fov = f32(self.znear), f32(self.zfar), f32(self.aspect), f32(self.fov)
        if self.degrees:
            fov = (np.pi / 180) * fov
        tan_half = torch.tan(fov / 2)
        max_y = tan_half * znear
        min_y = -max_y
        max_x = max_y * aspect
        min_x = -max_x
        ones = torch.ones(1, dtype=torch.float32)
        K = torch.zeros((1, 4, 4), dtype=torch.float32)
        K[:, 0, 0] = 2.0 * znear / (max_x - min_x)
        K[:, 1, 1] = 2.0 * znear / (max_y - min_y)
        K[:, 0, 2] = (max_x + min_x) / (max_x - min_x)
        K[:, 1, 2] = (max_y + min_y) / (max_y - min_y)
        K[:, 3, 2] = 1.0 * ones
        K[:, 2, 2] = 1.0 * zfar / (zfar - znear)
        K[:, 2, 3] = -(zfar * znear) / (zfar - znear)
        return K

    def _rot(self):
        M = torch.eye(4).unsqueeze(0).clone()
        M[:, :3, :3] = self.R
        return M

    def _trans(self, sign=1.0):
        M = torch.eye(4).unsqueeze(0).clone()
        M[:, 3, :3] = sign * self.T
        return M

    def inverse_full_projection(self):
        kt = self.projection().transpose(1, 2).contiguous()
        m = torch.inverse(kt)
        m = torch.bmm(m, self._trans(-1.0))                    # Translate._get_matrix_inverse
        m = torch.bmm(m, self._rot().transpose(1, 2))           # Rotate._get_matrix_inverse
        return m

    def center(self):
        # (Rotate . Translate).inverse() = Translate^-1 then Rotate^-1; row 3, :3
        m = torch.bmm(self._trans(-1.0), self._rot().transpose(1, 2))
        return m[:, 3, :3]

    def sample_positions(self, pos, size, with_noise=0.0, noise=None, bundle_size=1):
        ps = pos.unsqueeze(-2).expand(*pos.shape[:-1], bundle_size, 2)
        if with_noise:
            d = with_noise
            ps = ps + (d * noise - d / 2)
        ps = -2 * (ps / size) + 1
        pts = torch.cat([ps, torch.ones(ps.shape[:-1] + (1,))], dim=-1)
        flat = pts.reshape(1, -1, 3)
        hom = torch.cat([flat, torch.ones(1, flat.shape[1], 1)], dim=2)
        out = torch.bmm(hom, self.inverse_full_projection())
        dirs = out[..., :3] / out[..., 3:]
        dirs = F.normalize(dirs.reshape(1, *pts.shape), dim=-1)
        origins = self.center()[:, None, None, None, :].expand_as(dirs)
        return torch.cat([origins, dirs], dim=-1)


# ---------------------------------------------------------------------------------------------
# Renderer  (main.py:13-179)
# ---------------------------------------------------------------------------------------------

def _tile_positions(x0, y0, chunk):
    gx, gy = torch.meshgrid(torch.arange(x0, x0 + chunk, dtype=torch.float),
                            torch.arange(y0, y0 + chunk, dtype=torch.float), indexing="ij")
    return torch.stack([gy, gx], dim=-1)


def render(shape, lights, camera, integrator, bsdf, size, chunk_size, background=1.0,
           with_noise=0.0, crop=None, jitter=None, w_isect=False, camera_noise=None):
    """pathtrace (main.py:13-93) / pathtrace_sample mode="crop" (main.py:97-179).

    ``crop=(u, v, crop_size)`` renders the crop window; ``jitter`` fixes the coarse-scan
    jitter (else ``random.random()`` is drawn per tile like the reference); ``camera_noise``
    is an optional callable ``(u, v) -> (nu, nv)`` replacing the camera's ``rand_like``.
    """
    n_cam = len(camera)
    dims = integrator.dims()
    # main.py:54 / :133 assert before pathtrace_sample clamps the chunk to the crop (:135)
    assert size % chunk_size == 0
    if crop is None:
        u0, v0, extent = 0, 0, size
    else:
        u0, v0, extent = crop
        u0 = max(min(u0, size - extent), 0)
        v0 = max(min(v0, size - extent), 0)
        chunk_size = min(chunk_size, extent)
    out = torch.full([n_cam, extent, extent, dims], float(background))
    xs = list(range(u0, u0 + extent, chunk_size))
    ys = list(range(v0, v0 + extent, chunk_size))
    for ij in range(len(xs) * len(ys)):
        i, j = divmod(ij, len(ys))
        x0, y0 = xs[j], ys[i]
        pos = _tile_positions(x0, y0, chunk_size)
        if isinstance(camera, NeRFCameraRef):
            noise = None if camera_noise is None else camera_noise(pos)
            rays = camera.sample_positions(pos, size, with_noise, noise)
        else:
            rays = camera.sample_positions(pos, size)
        vals, mask, _ = integrator.sample(shape, rays, bsdf, lights, w_isect=w_isect,
                                          jitter=jitter)
        valid = mask.any(dim=-1)
        v = torch.mean(vals, dim=-2)
        v[~valid] = background
        out[:, x0 - u0:x0 - u0 + chunk_size, y0 - v0:y0 - v0 + chunk_size] = v
    if n_cam == 1:
        out = out.squeeze(0)
    return out


# ---------------------------------------------------------------------------------------------
# Volumetric NeRF baselines  (shapes/nerf.py:153-214)
# ---------------------------------------------------------------------------------------------

class NeRFLERef(nn.Module):
    """NeRFLE, nerf.py:153-214 (envmap=False: NeRF+PT; envmap=True: NeRF+LE).

    Reproduces the reference's compositing quirks: ``alpha = 1-exp(-sigma * t)`` with the
    absolute depth, and ``roll(cumprod, 1)`` with the LAST entry set to 1.  With envmap the
    colour MLP sees ``lights.envmap`` at ``bins^2`` directions built from degree values passed
    as radians (:183-191).
    """

    def __init__(self, steps=64, envmap=False, bins=4):
        super().__init__()
        self.latent_size = 64
        self.first = SkipMLP(num_layers=5, hidden_size=128, in_size=3, out=1 + self.latent_size)
        self.bins = bins
        self.second = SkipMLP(in_size=self.latent_size + (6 if not envmap else 3 + bins * bins * 3),
                              out=3)
        self.envmap = envmap
        self.steps = steps

    def forward(self, rays, light_location, jitter=None, light=None):
        r_o, r_d = rays.split([3, 3], dim=-1)
        if jitter is None:
            jitter = random.random()
        ts = torch.linspace(0, 2 + jitter * 0.1, self.steps)
        pts = r_o.unsqueeze(0) + torch.tensordot(ts, r_d, dims=0)
        first = self.first(pts)
        latent = first[..., 1:]
        alpha = first[..., 0, None]
        if self.envmap:
            points = torch.stack(torch.meshgrid(torch.linspace(0, 180, self.bins),
                                                torch.linspace(0, 45, self.bins), indexing="ij"),
                                 dim=-1).reshape(-1, 2)
            enc = point_light_envmap(light, elev_azim_to_dir(points))
            B = latent.shape[1]
            light_enc = enc.reshape(1, B, 1, 1, 1, -1).expand(latent.shape[:-1] + (-1,))
        else:
            light_enc = light_location[None, :, None, None, None, :].expand(
                latent.shape[:-1] + (3,))
        rgb = self.second(torch.cat([latent, r_d[None, ...].expand(latent.shape[:-1] + (3,)),
                                     light_enc], dim=-1)).sigmoid()
        sigma = F.relu(alpha).squeeze(-1)
        alpha = 1 - torch.exp(-sigma * ts[:, None, None, None, None].expand_as(sigma))
        cp = torch.cumprod((1 - alpha).clamp(min=1e-10), dim=0)
        cp = torch.roll(cp, 1, 0)
        cp[-1, ...] = 1
        w = alpha * cp
        return (w[..., None] * rgb).sum(dim=0)


class PlainNeRFRef(nn.Module):
    """PlainNeRF, nerf.py:9-74: a latent-conditioned NeRF.

    ``first = SkipMLP(3 -> 1 + intermediate, latent)`` (5 x 32), ``second = SkipMLP(2 -> 3,
    latent = intermediate + latent)`` (5 x 32) on ``dir_to_elev_azim(r_d)``; ``tanh`` colours,
    ``ts = linspace(0.4, 2 + random()*0.1, steps)``, ``sigma = relu(alpha + randn*1e-3)`` (the
    noise is injectable: ``noise`` [S, N, W, H, B, 1]), the same rolled-cumprod weights as NeRFLE
    and the output ``(rgb + 1) / 2``.  ``latent`` is [N, latent_size]: row n conditions camera n
    (``self.latent[None, :, None, None, None, :]``, :52).
    """

    def __init__(self, latent_size=32, intermediate_size=32, steps=32):
        super().__init__()
        self.latent = None
        self.latent_size = latent_size
        self.steps = steps
        self.first = SkipMLP(in_size=3, out=1 + intermediate_size, latent_size=latent_size,
                             num_layers=5, hidden_size=32)
        self.second = SkipMLP(in_size=2, out=3, latent_size=latent_size + intermediate_size,
                              num_layers=5, hidden_size=32)

    def assign_latent(self, latent):
        assert latent.shape[-1] == self.latent_size and latent.dim() == 2
        self.latent = latent

    def forward(self, rays, lights=None, jitter=None, noise=None):
        r_o, r_d = rays.split([3, 3], dim=-1)
        if jitter is None:
            jitter = random.random()
        ts = torch.linspace(0.4, 2 + jitter * 0.1, self.steps)
        pts = r_o.unsqueeze(0) + torch.tensordot(ts, r_d, dims=0)
        latent = self.latent[None, :, None, None, None, :].expand(pts.shape[:-1] + (-1,))
        first_out = self.first(pts, latent)
        alpha = first_out[..., 0, None]
        intermediate = first_out[..., 1:]
        ea = dir_to_elev_azim(r_d)
        rgb = self.second(ea[None, ...].expand(latent.shape[:-1] + (2,)),
                          torch.cat([intermediate, latent], dim=-1)).tanh()
        if noise is None:
            noise = torch.randn_like(alpha) * 1e-3
        sigma = F.relu(alpha + noise).squeeze(-1)
        alpha = 1 - torch.exp(-sigma * ts[:, None, None, None, None].expand_as(sigma))
        cp = torch.cumprod((1 - alpha).clamp(min=1e-10), dim=0)
        cp = torch.roll(cp, 1, 0)
        cp[-1, ...] = 1
        w = alpha * cp
        rgb_out = (w[..., None] * rgb).sum(dim=0)
        return (rgb_out + 1) / 2
