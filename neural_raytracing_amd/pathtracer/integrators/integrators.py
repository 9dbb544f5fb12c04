"""Integrators (integrators/integrators.py).  ``Direct`` runs the fused HIP path:
nrt_sdf_intersect (march + coarse scan + normals) then nrt_shade_direct (light sample +
spatially varying BSDF) over the compacted hit list."""
import torch
import torch.nn as nn

from ... import _lib
from ..differentiable import direct_sample, needs_grad


class Integrator(nn.Module):
    def __init__(self, max_depth=2, russian_roulette_depth=5, sampler=None, lights=None):
        super().__init__()
        self.max_depth = max_depth
        self.rr_depth = russian_roulette_depth
        self.sampler = sampler
        self.lights = lights

    def dims(self):
        raise NotImplementedError()

    def sample(self, shapes, rays, bsdf, **kwargs):
        raise NotImplementedError()


class Debug(Integrator):
    """Normals as colour (integrators.py:25-35)."""

    def dims(self):
        return 3

    def sample(self, shapes, rays, bsdf, **kwargs):
        si, active = shapes.intersect(rays)
        result = torch.where(active.unsqueeze(-1), (si.n + 1) / 2,
                             torch.tensor(0., device=active.device))
        return result, active, si


class Silhouette(Integrator):
    """1 - hit (integrators.py:38-42)."""

    def dims(self):
        return 1

    def sample(self, shapes, rays, bsdf, **kwargs):
        si, active = shapes.intersect(rays)
        return 1 - active.unsqueeze(-1).float(), active, si


class BasisBRDF(Integrator):
    """The spatial BSDF weights on the hit points (integrators.py:79-90): sigmoid(sp_var_fn(p))
    of a ComposeSpatialVarying, on the HIP MLP kernel."""

    def __init__(self, multi_basis_bsdf):
        super().__init__()
        self.bsdf = multi_basis_bsdf

    def dims(self):
        return len(self.bsdf.bsdfs)

    def sample(self, shapes, rays, bsdf, **kwargs):
        results = torch.zeros(*rays.shape[:-1], self.dims(), device=rays.device)
        it, active = shapes.intersect(rays)
        if not bool(active.any()):
            return results, active, it
        results[active] = self.bsdf.normalized_weights(it.p[active], it)
        return results, active, it


class Illumination(Integrator):
    """Light direction in the shading frame at the hit points (integrators.py:93-111).  The
    reference's signature sample(shapes, rays, lights, sampler) collides with pathtrace's keyword
    call (lights= twice), so it is used by calling sample directly."""

    def dims(self):
        return 3

    def sample(self, shapes, rays, lights, sampler=None, **kwargs):
        from ..differentiable import light_sample
        it, active = shapes.intersect(rays)
        d, _, _, _ = light_sample(lights, it, active)
        res = torch.where(active.unsqueeze(-1),
                          (torch.nn.functional.normalize(it.to_local(d), dim=-1) + 1) / 2,
                          torch.zeros_like(d))
        return (1 + res) / 2, active, it


class Luminance(Integrator):
    """Emitter luminance at the hit points (integrators.py:114-136), with the reference's
    0.2126 r + 0.7152 * 0.0722 b weights."""

    def dims(self):
        return 3

    def sample(self, shapes, rays, lights, sampler=None, **kwargs):
        from ..differentiable import light_sample
        it, active = shapes.intersect(rays)
        d, le, _, _ = light_sample(lights, it, active)
        r, _, b = le.split(1, dim=-1)
        lum = 0.2126 * r + 0.7152 * 0.0722 * b
        return torch.where(active.unsqueeze(-1), lum.expand_as(d), torch.zeros_like(d)), active, it


class NeuralApprox(Integrator):
    """integrators.py:208-240 (a TwoStageMLP light-transport approximation, off the hot path):
    import-resolvable for the drivers (dtu.py:16); sampling raises NrtError."""

    def __init__(self, **kwargs):
        super().__init__(**{k: v for k, v in kwargs.items() if k != "device"})

    def dims(self):
        return 3

    def sample(self, shape, rays, bsdf, **kwargs):
        raise _lib.NrtError("NeuralApprox (TwoStageMLP) has no HIP implementation")


class Mask(Integrator):
    """Adds the hit mask as a channel (integrators.py:45-54)."""

    def __init__(self, sub_integrator, **kwargs):
        super().__init__(**kwargs)
        self.sub_integrator = sub_integrator

    def dims(self):
        return self.sub_integrator.dims() + 1

    def sample(self, density_field, rays, bsdf, **kwargs):
        result, active, si = self.sub_integrator.sample(density_field, rays, bsdf, **kwargs)
        mask = torch.where(active, 1., 0.)
        return torch.cat([result, mask.unsqueeze(-1)], dim=-1), torch.ones_like(active), si


class Depth(Integrator):
    """Ray depths (integrators.py:57-67)."""

    def __init__(self, scale=False, empty_val=-1, **kwargs):
        super().__init__(**kwargs)
        self.empty_val = empty_val
        self.scale = scale

    def dims(self):
        return 1

    def sample(self, shapes, rays, bsdf, **kwargs):
        it, active = shapes.intersect(rays)
        results = torch.where(active, it.t, torch.full_like(it.t, self.empty_val))
        if self.scale:
            results[results != 0] /= results[results != 0].max()
        return results.unsqueeze(-1), active, it


def _light_handle(lights):
    nrt = getattr(lights, "nrt", None)
    if nrt is None:
        raise _lib.NrtError(f"light {type(lights).__name__} has no HIP implementation "
                            "(supported: LightField, PointLights)")
    return nrt()


def _bsdf_handle(bsdf):
    nrt = getattr(bsdf, "nrt", None)
    if nrt is None:
        from ..bsdf import ComposeSpatialVarying
        comp = getattr(bsdf, "_component", None)
        if comp is None:
            raise _lib.NrtError(f"BSDF {type(bsdf).__name__} has no HIP implementation")
        wrapper = getattr(bsdf, "_nrt_single", None)
        if wrapper is None:
            wrapper = ComposeSpatialVarying.__new__(ComposeSpatialVarying)
            nn.Module.__init__(wrapper)
            wrapper.bsdfs = [bsdf]
            wrapper.sp_var_fn = None
            object.__setattr__(bsdf, "_nrt_single", wrapper)
        return wrapper.nrt()
    return nrt()


def _emitter_mode(w_isect):
    """Which sample_emitter_dir_* the reference picks (integrators.py:161-166, :287-291):
    True -> shadow ray (w_isect); a SkipConnMLP -> learned occlusion; anything else -> none.
    Returns (shadow, occlusion-MLP handle or None)."""
    from ..neural_blocks import SkipConnMLP
    if w_isect is True:
        return 1, None
    if type(w_isect) is SkipConnMLP:
        return 1, w_isect.nrt()
    return 0, None


class Direct(Integrator):
    """Direct lighting, one emitter sample, no BSDF sampling (integrators.py:139-206).

    ``training`` is set before ``nn.Module.__init__`` resets it to True (integrators.py:153-154),
    so the coarse scan always runs; that quirk is kept.
    """
    DEFAULT_EMITTER_SAMPLES = 1
    DEFAULT_BSDF_SAMPLES = 0

    def dims(self):
        return 3

    def __init__(self, emitter_samples=DEFAULT_EMITTER_SAMPLES, bsdf_samples=DEFAULT_BSDF_SAMPLES,
                 training=True, **kwargs):
        self.emitter_samples = emitter_samples
        self.bsdf_samples = bsdf_samples
        self.training = training
        super().__init__(**kwargs)

    def sample(self, shapes, rays, bsdf, **kwargs):
        lights = kwargs.get("lights", self.lights)
        shadow, occ = _emitter_mode(kwargs.get("w_isect"))
        if self.emitter_samples != 1 or self.bsdf_samples != 0:
            raise _lib.NrtError("Direct on the HIP path supports emitter_samples=1, bsdf_samples=0")
        it, active = shapes.intersect(rays, primary=self.training)
        from ..shapes.sdfs import is_hip_sdf
        callable_shadow = bool(shadow) and not is_hip_sdf(getattr(shapes, "sdf", None))
        if getattr(it, "_nrt_train", False) or needs_grad(bsdf, lights, kwargs.get("w_isect")) \
                or callable_shadow:
            # (an SDF callable with shadow rays: the shading kernel cannot march the callable, so
            # the composed path shades -- HIP MLPs, the shadow march by intersect_test's
            # nrt_occlusion_callable_step)
            # training: shading with autograd through the HIP MLPs
            return direct_sample(it, active, bsdf, lights, rays.shape[:-1], rays.device, shapes,
                                 kwargs.get("w_isect", False)), active, it
        result = torch.zeros(*rays.shape[:-1], 3, device=rays.device)
        hit_idx, hit_count, flat = it._nrt_hits
        P = flat.shape[0]
        rgb = result.reshape(P, 3)
        # it.normalized_weights / nonnormalized_weights (bsdfs.py:516-536: sigmoid(sp_var_fn(p))
        # on EVERY ray, misses included) are evaluated on first access (HipInteraction), so a
        # render that never reads them pays nothing for them
        it._nrt_spatial = bsdf
        per_cam = getattr(lights, "per_camera", lambda: None)()
        if per_cam is not None:
            # one point light per camera (lights.py:91 broadcasts location[n] over camera n's
            # rays): camera n's rays are the contiguous block n of the [N, W, H, B] order, shaded
            # with its own light over its own hit list
            N = rays.shape[0]
            if per_cam != N or P % N:
                raise _lib.NrtError(f"PointLights with {per_cam} lights for {N} cameras")
            Q = P // N
            act = active.reshape(N, Q)
            for n in range(N):
                idx_n = torch.nonzero(act[n]).reshape(-1).to(torch.int32)
                cnt_n = torch.tensor([idx_n.numel()], dtype=torch.int32, device=rays.device)
                sl = slice(n * Q, (n + 1) * Q)
                args = (_lib.ptr(it.p.reshape(P, 3)[sl]), _lib.ptr(it.n.reshape(P, 3)[sl]),
                        _lib.ptr(it.wi.reshape(P, 3)[sl]), _lib.ptr(idx_n), _lib.ptr(cnt_n), Q,
                        _lib.ptr(rgb[sl]), None)
                self._shade(shapes, bsdf, lights.camera(n), shadow, occ, args, Q, rays.device)
            return result, active, it
        args = (_lib.ptr(it.p.reshape(P, 3)), _lib.ptr(it.n.reshape(P, 3)),
                _lib.ptr(it.wi.reshape(P, 3)), _lib.ptr(hit_idx), _lib.ptr(hit_count), P,
                _lib.ptr(rgb), None)
        self._shade(shapes, bsdf, lights, shadow, occ, args, P, rays.device)
        return result, active, it

    @staticmethod
    def _shade(shapes, bsdf, lights, shadow, occ, args, P, device):
        """nrt_shade_direct[_shadowed | _learned_occ] over one hit list."""
        if shadow:
            # sample_emitter_dir_w_isect (scene.py:290-298): shadow ray to the point light,
            # marched like SDF.intersect_test (sdfs.py:162-181); with an occlusion MLP,
            # sample_emitter_dir_w_learned_occ (scene.py:301-319)
            from ..shapes.sdfs import march_handle
            lib = _lib.load(require_device=True)
            ws = torch.empty(lib.nrt_shadow_workspace_bytes(P), dtype=torch.uint8, device=device)
            head = (_bsdf_handle(bsdf), _light_handle(lights), march_handle(shapes.sdf))
            steps = (int(shapes.max_steps), float(shapes.epsilon))
            if occ is None:
                _lib.call("nrt_shade_direct_shadowed", *head, *steps, *args, None, _lib.ptr(ws),
                          _lib.precision_code(), _lib.stream())
            else:
                _lib.call("nrt_shade_direct_learned_occ", *head, occ, *steps, *args, None,
                          _lib.ptr(ws), _lib.precision_code(), _lib.stream())
        else:
            _lib.call("nrt_shade_direct", _bsdf_handle(bsdf), _light_handle(lights), *args,
                      _lib.precision_code(), _lib.stream())


class Path(Integrator):
    """Light path integrator (integrators.py:275-354): per bounce (max_depth 2) the emitter term
    weighted by the path throughput, then a BSDF sample of the spatially varying mixture and a
    secondary intersection.  Each bounce is one ``nrt_path_bounce`` call plus ``nrt_sdf_intersect``
    of the spawned rays.  ``training`` stays False (the reference sets it after
    ``nn.Module.__init__``), so the primary intersection has no coarse scan.

    Randomness: each BSDF component draws ``sampler.sample(shape + (2,))`` in component order, as
    in the reference; the component selection (torch.multinomial there) is the inverse CDF of the
    spatial weights at one more uniform draw.  ``uniforms=[(u_comp, u_sel), ...]`` (one pair per
    bounce) replaces the draws, for parity tests.
    """

    # secondary intersections march only the rays whose path is still active (compacted on the
    # device; the same per-ray results as marching every spawned ray)
    compact = True

    def __init__(self, training=False, **kwargs):
        super().__init__(**kwargs)
        self.training = training

    def dims(self):
        return 3

    def sample(self, shapes, rays, bsdf, **kwargs):
        from ..shapes.sdfs import sdf_handle
        sampler = kwargs.get("sampler", self.sampler)
        lights = kwargs.get("lights", self.lights)
        shadow, occ = _emitter_mode(kwargs.get("w_isect", False))
        uniforms = kwargs.get("uniforms")
        if needs_grad(shapes, bsdf, lights, kwargs.get("w_isect")):
            # training: the emitter terms with autograd, the BSDF samples on
            # the HIP bounce kernel, the spawned rays rebuilt differentiably
            from ..differentiable import path_sample
            return path_sample(shapes, rays, bsdf, lights, self.max_depth, self.training, sampler,
                               uniforms, kwargs.get("w_isect", False))
        dev = rays.device
        lead = rays.shape[:-1]
        it, active = shapes.intersect(rays, primary=self.training)
        result = torch.zeros(*lead, 3, device=dev)
        if not bool(active.any()):
            return result, active, it
        original_active = active.clone()
        P = active.numel()
        nc = len(getattr(bsdf, "bsdfs", [bsdf]))
        act = active.reshape(-1).to(torch.uint8).contiguous()
        thr = torch.ones(P, 3, device=dev)
        res = result.reshape(P, 3)
        rays_out = torch.empty(P, 6, device=dev)
        lib = _lib.load(require_device=True)
        ws = torch.empty(lib.nrt_path_workspace_bytes(P), dtype=torch.uint8, device=dev)
        sh = sdf_handle(shapes.sdf)
        curr = it
        for depth in range(self.max_depth):
            if uniforms is not None:
                u_comp, u_sel = (u.to(dev).float().reshape(P, -1).contiguous() for u in uniforms[depth])
            else:
                draws = [sampler.sample(tuple(lead) + (2,), device=dev).reshape(P, 1, 2)
                         for _ in range(nc)]
                u_comp = torch.cat(draws, dim=1).contiguous()
                u_sel = sampler.sample((P,), device=dev).contiguous()
            _lib.call("nrt_path_bounce", _bsdf_handle(bsdf), _light_handle(lights), sh,
                      shadow, occ, int(shapes.max_steps), float(shapes.epsilon),
                      _lib.ptr(curr.p.reshape(P, 3).contiguous()),
                      _lib.ptr(curr.n.reshape(P, 3).contiguous()),
                      _lib.ptr(curr.wi.reshape(P, 3).contiguous()), P, _lib.ptr(act),
                      _lib.ptr(thr), _lib.ptr(res), _lib.ptr(u_comp), _lib.ptr(u_sel),
                      _lib.ptr(rays_out), _lib.ptr(ws), _lib.precision_code(), _lib.stream())
            if depth + 1 == self.max_depth:
                break  # the reference's last spawn is never shaded (:309, :342)
            # the spawned rays of the still-active paths only (one host synchronisation, as the
            # reference's act.any()): marching the dead ones would change nothing but the time
            live = torch.nonzero(act).reshape(-1)
            if live.numel() == 0:
                break
            if self.compact and live.numel() < P:
                sub, hits = shapes.intersect(rays_out.index_select(0, live), primary=False)
                curr = _Scattered(sub, live, P, dev)
                act.zero_().index_copy_(0, live, hits.reshape(-1).to(torch.uint8))
            else:
                curr, hits = shapes.intersect(rays_out.reshape(*lead, 6), primary=False)
                act &= hits.reshape(-1).to(torch.uint8)
            if not bool(act.any()):
                break
        return result, original_active, it


class _Scattered:
    """The p / n / wi of a compacted secondary intersection (rays `live` of P) in the full ray
    order nrt_path_bounce reads; rays off the list keep zeros (they are inactive)."""

    def __init__(self, sub, live, P, dev):
        for name in ("p", "n", "wi"):
            full = torch.zeros(P, 3, device=dev)
            full.index_copy_(0, live, getattr(sub, name).reshape(-1, 3))
            setattr(self, name, full)


class NeRFReproduce(Integrator):
    """Runs a volumetric NeRF on the rays (integrators.py:260-267): result = nerf(rays, lights)."""

    def dims(self):
        return 3

    def sample(self, nerf, rays, lights, **kwargs):
        result = nerf(rays, lights)

        class Dummy:
            ...
        return result, torch.tensor(True, device=result.device), Dummy()


_TRUE = {}


def _true(device):
    """The integrator's all-active flag (integrators.py:257) as a cached device tensor: one host
    copy per device instead of one (and a stream sync) per call."""
    t = _TRUE.get(device)
    if t is None:
        t = _TRUE[device] = torch.tensor(True, device=device)
    return t


class NeRFIntegrator(Integrator):
    """Appends sigmoid(throughput) as alpha (integrators.py:243-257)."""

    def __init__(self, sub_integrator, **kwargs):
        super().__init__(**kwargs)
        self.sub_integrator = sub_integrator

    def dims(self):
        return self.sub_integrator.dims() + 1

    def sample(self, density_field, rays, bsdf, **kwargs):
        result, active, mi = self.sub_integrator.sample(density_field, rays, bsdf, **kwargs)
        alpha = mi.throughput.unsqueeze(-1)
        if mi.with_logits:
            alpha = alpha.sigmoid()
        result = torch.cat([result, alpha], dim=-1)
        return result, _true(result.device), mi
