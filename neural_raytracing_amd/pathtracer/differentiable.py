"""Training through the fused path: the differentiable pieces of
``SDF.intersect`` and ``Direct.sample`` for ``loss.backward()``.

Rendering with gradients keeps the reference's split: the march and the 128-step coarse scan
run without gradients (``torch.no_grad`` in sdfs.py:118-131, :239-247) on the fused HIP
kernels; what carries gradients is recomputed at the points they found:

* ``throughput = -1000 * sdf(best_pos)`` (sdfs.py:134-137, :248) -- the SDF MLP forward and
  backward on ``nrt_mlp_forward`` / ``nrt_mlp_backward``;
* ``raw_normals = d sdf / d p`` with ``create_graph=True`` (sdfs.py:184-197) --
  ``nrt_mlp_backward`` for the value, ``nrt_mlp_grad_backward`` for its parameter gradients;
* the shading MLPs (spatial weights, NeuralBSDFs, LightField) -- ``SkipConnMLP`` autograd.

The glue between the MLPs (frames, Rusinkiewicz angles, Fresnel, light falloff, the 128-sphere
smooth-min of ``SphereSDF``) is a few element-wise tensor ops per ray, written here in the
reference's op order so autograd reproduces its gradients.
"""
import math

import torch
import torch.nn.functional as F

from .. import _lib


# ---- interaction frames (interaction.py:9-51) -------------------------------------------------

def coordinate_system(n):
    """Shading frame columns [s, t, n] (interaction.py:9-27), differentiable."""
    n = F.normalize(n, eps=1e-7, dim=-1)
    x, y, z = n.split(1, dim=-1)
    sign = torch.where(z >= 0, 1., -1.)
    s_z = sign + z
    a = -torch.where(s_z.abs() < 1e-6, 1e-6, s_z).reciprocal()
    b = x * y * a
    s = torch.cat([(x * x * a * sign) + 1, b * sign, x * -sign], dim=-1)
    s = F.normalize(s, eps=1e-7, dim=-1)
    t = F.normalize(s.cross(n, dim=-1), eps=1e-7, dim=-1)
    s = F.normalize(n.cross(t, dim=-1), eps=1e-7, dim=-1)
    return torch.stack([s, t, n], dim=-1)


# ---- BSDF helpers (utils.py:43-51, 152-155, 234-258; bsdfs.py:127-129, 327-343) --------------

def nonzero_eps(v, eps: float = 1e-7):
    # a Python scalar branch: no host -> device copy (and no stream sync) per call
    return torch.where(v.abs() < eps, eps, v)


_AXES = {}


def _axis(i, like):
    """Unit axis e_i on like's device, built once per device (no per-call host copy)."""
    key = (like.device, i)
    t = _AXES.get(key)
    if t is None:
        t = torch.zeros(3, device=like.device, dtype=torch.float)
        t[i] = 1.0
        _AXES[key] = t
    return t.expand_as(like)


def rotate_vector(v, axis, c, s):
    return v * c + axis * (v * axis).sum(dim=-1, keepdim=True) * (1 - c) + \
        torch.cross(axis, v, dim=-1) * s


def param_rusin2(wo, wi):
    """[cos phi_d, cos theta_h, cos theta_d] (utils.py:234-258)."""
    wo = F.normalize(wo, dim=-1)
    wi = F.normalize(wi, dim=-1)
    e_1 = _axis(1, wo)
    e_2 = _axis(2, wo)
    H = F.normalize(wo + wi, dim=-1)
    cos_theta_h = H[..., 2]
    r = nonzero_eps(H[..., 1]).hypot(nonzero_eps(H[..., 0])).clamp(min=1e-6)
    c = (H[..., 0] / r).unsqueeze(-1)
    s = -(H[..., 1] / r).unsqueeze(-1)
    tmp = F.normalize(rotate_vector(wi, e_2, c, s), dim=-1)
    c = H[..., 2].unsqueeze(-1)
    s = -(1 - H[..., 2]).clamp(min=1e-6).sqrt().unsqueeze(-1)
    diff = F.normalize(rotate_vector(tmp, e_1, c, s), dim=-1)
    cos_theta_d = diff[..., 2]
    cos_phi_d = torch.atan2(nonzero_eps(diff[..., 1]), nonzero_eps(diff[..., 0])).cos()
    return torch.stack([cos_phi_d, cos_theta_h, cos_theta_d], dim=-1)


def local_reflect(v):
    x, y, z = v.split(1, dim=-1)
    return torch.cat([-x, -y, z], dim=-1)


def fresnel_conductor(cos_t, eta_r: float, eta_i: float):
    ct2 = cos_t * cos_t
    st2 = (1 - ct2).clamp(min=1e-10)
    st4 = st2 * st2
    tmp = eta_r * eta_r - eta_i * eta_i - st2
    a_2_pb_2 = (tmp * tmp + 4 * eta_i * eta_i * eta_r * eta_r).clamp(min=1e-10).sqrt()
    a = (0.5 * (a_2_pb_2 + tmp)).clamp(min=1e-10).sqrt()
    t1 = a_2_pb_2 + ct2
    t2 = 2 * cos_t * a
    r_s = (t1 - t2) / (t1 + t2)
    t3 = a_2_pb_2 * ct2 + st4
    t4 = t2 * st2
    r_p = r_s * (t3 - t4) / (t3 + t4)
    return 0.5 * (r_s + r_p)


# ---- SDF values and gradients with autograd ---------------------------------------------------

def needs_grad(*modules):
    """True when autograd is on and any parameter of the given objects requires a gradient."""
    if not torch.is_grad_enabled():
        return False
    for m in modules:
        params = getattr(m, "parameters", None)
        if params is None:
            continue
        try:
            if any(getattr(q, "requires_grad", False) for q in params()):
                return True
        except (TypeError, AttributeError):
            continue
    return False


SMOOTHMIN_K = 32.0  # sdfs.py:43 / utils.py:386-387
# nrt_sphere_smoothmin_* stage the sphere table (13 floats a sphere) in 64 KB of LDS: larger
# SphereSDFs train on the torch restatement (sphere_part under autograd)
SMOOTHMIN_MAX_SPHERES = 64 * 1024 // (13 * 4)


def _fused_smoothmin(sdf, p):
    return p.is_cuda and sdf.centers.shape[0] <= SMOOTHMIN_MAX_SPHERES


class _SphereSmoothMinFn(torch.autograd.Function):
    """(value, d value / d p) of SphereSDF's smooth-min on nrt_sphere_smoothmin_forward, with the
    sphere parameters' gradients of both outputs from nrt_sphere_smoothmin_backward -- for the
    gradient output that is the double backward of SDF.autograd_diff's create_graph=True normal
    (sdfs.py:184-197).  The points carry no gradient (the reference's hit and scan points come
    from the no-grad march)."""

    @staticmethod
    def forward(ctx, p, centers, radii, tfs):
        P, n = p.shape[0], centers.shape[0]
        value = torch.empty(P, device=p.device)
        grad = torch.empty(P, 3, device=p.device)
        c, r, t = (x.detach().float().contiguous() for x in (centers, radii, tfs))
        _lib.call("nrt_sphere_smoothmin_forward", _lib.ptr(p), P, _lib.ptr(c), _lib.ptr(r),
                  _lib.ptr(t), n, SMOOTHMIN_K, _lib.ptr(value), _lib.ptr(grad), _lib.stream())
        ctx.save_for_backward(p, c, r, t)
        return value, grad

    @staticmethod
    def backward(ctx, dvalue, dgrad):
        if torch.is_grad_enabled():
            raise _lib.NrtError("third derivatives of the SphereSDF smooth-min are not on the "
                                "HIP path")
        p, c, r, t = ctx.saved_tensors
        P, n = p.shape[0], c.shape[0]
        lib = _lib.load(require_device=True)
        dc = torch.empty_like(c) if ctx.needs_input_grad[1] else None
        dr = torch.empty_like(r) if ctx.needs_input_grad[2] else None
        dt = torch.empty_like(t) if ctx.needs_input_grad[3] else None
        dv = None if dvalue is None else dvalue.float().contiguous()
        dg = None if dgrad is None else dgrad.float().contiguous()
        ws = torch.empty(lib.nrt_sphere_smoothmin_workspace_bytes(P), dtype=torch.uint8,
                         device=p.device)
        _lib.call("nrt_sphere_smoothmin_backward", _lib.ptr(p), P, _lib.ptr(c), _lib.ptr(r),
                  _lib.ptr(t), n, SMOOTHMIN_K, _lib.ptr(dv), _lib.ptr(dg), _lib.ptr(dc),
                  _lib.ptr(dr), _lib.ptr(dt), _lib.ptr(ws), _lib.stream())
        return None, dc, dr, dt


def sphere_smoothmin(sdf, p):
    """(value, gradient) of the smooth-min part at points p [..., 3] that carry no gradient, on
    the fused kernels; shapes p.shape[:-1] and p.shape."""
    flat = p.detach().reshape(-1, 3).float().contiguous()
    v, g = _SphereSmoothMinFn.apply(flat, sdf.centers, sdf.radii, sdf.tfs)
    return v.reshape(p.shape[:-1]), g.reshape(p.shape)


def sphere_part(sdf, p):
    """The smooth-min of the transformed spheres of SphereSDF (sdfs.py:37-43, utils.py:386-387)."""
    flat = p.reshape(-1, 3).unsqueeze(0)
    tfs = sdf.tfs + torch.eye(3, device=p.device).unsqueeze(0)
    q = torch.einsum("ijk,ibk->ibj", tfs, flat.expand(tfs.shape[0], -1, -1)) - \
        sdf.centers.unsqueeze(1)
    sd = q.norm(p=2, dim=-1) - sdf.radii.unsqueeze(-1)
    return (-(-32. * sd).exp().sum(dim=0).clamp(min=1e-4).log() / 32.).reshape(p.shape[:-1])


def sdf_value(sdf, p):
    """sdf(p) with gradients for the SDF's parameters."""
    from .neural_blocks import SkipConnMLP
    from .script_modules import resolve
    from .shapes.sdfs import SPHERE_SDF, _is_sphere_sdf
    sdf = resolve(sdf)
    if sdf is SPHERE_SDF:
        return torch.norm(p, dim=-1) - 1
    if isinstance(sdf, SkipConnMLP):
        return sdf(p).reshape(p.shape[:-1])
    if _is_sphere_sdf(sdf):
        if _fused_smoothmin(sdf, p) and not p.requires_grad:
            out = sphere_smoothmin(sdf, p)[0]  # fused forward + parameter backward
        else:  # points with a gradient (an SDF callable warping them): the torch restatement
            out = sphere_part(sdf, p)
        return out + sdf.shift(p).reshape_as(out)
    raise _lib.NrtError(f"SDF callable {type(sdf).__name__} has no HIP training path")


def sdf_gradient(sdf, p):
    """SDF.autograd_diff (sdfs.py:184-197): d sdf / d p, differentiable with respect to the
    SDF's parameters (create_graph=True).  ``p`` itself is not differentiated (the reference's
    hit points come from the no-grad march)."""
    from .neural_blocks import SkipConnMLP, input_gradient
    from .script_modules import resolve
    from .shapes.sdfs import SPHERE_SDF, _is_sphere_sdf
    sdf = resolve(sdf)
    p = p.detach()
    if sdf is SPHERE_SDF:
        return p / torch.norm(p, dim=-1, keepdim=True)
    if isinstance(sdf, SkipConnMLP):
        return input_gradient(sdf, p)
    if _is_sphere_sdf(sdf):
        if _fused_smoothmin(sdf, p):
            g = sphere_smoothmin(sdf, p)[1]  # fused gradient + its double backward
        else:
            with torch.enable_grad():
                q = p.clone().requires_grad_(True)
                out = sphere_part(sdf, q)
                (g,) = torch.autograd.grad(out, q, torch.ones_like(out), create_graph=True)
        return g + input_gradient(sdf.shift, p)
    raise _lib.NrtError(f"SDF callable {type(sdf).__name__} has no HIP training path")


# ---- shading (integrators.py:139-206 with emitter_samples=1, bsdf_samples=0) -----------------

def _per_camera(t, p):
    """A [L, 3] light tensor broadcast like the reference's t[:, None, None, None, :] against
    points p [N, ..., 3]: one row for every camera, or row n for camera n (L == N)."""
    rows = t.reshape(-1, 3).to(p.device)
    if rows.shape[0] == 1 or p.dim() < 2:
        return rows[0]
    if rows.shape[0] != p.shape[0]:
        raise _lib.NrtError(f"PointLights with {rows.shape[0]} locations / intensities for "
                            f"{p.shape[0]} cameras")
    return rows.reshape(rows.shape[0], *([1] * (p.dim() - 2)), 3)


def light_sample(lights, it, active):
    """lights.sample_direction + sample_emitter_dir_wo_isect (scene.py:321-324)
    -> (d, Le, pdf, dist); dist is None for a LightField (lights.py:181-183)."""
    from .lights.lights import LightField, PointLights, RendererPointLights
    p = it.p
    if isinstance(lights, LightField):
        # lights.py:175-195, on the active rows through one integer index (one host sync for
        # its length; the boolean gather and scatters took one each, and their backwards more)
        flat = p.reshape(-1, 3)
        aidx = torch.nonzero(active.reshape(-1)).squeeze(1)
        v = lights.light_field_approx(flat.index_select(0, aidx))
        d = torch.zeros_like(flat).index_put(
            (aidx,), F.normalize(v, eps=1e-6, dim=-1).clamp(min=1e-6, max=1)).reshape(p.shape)
        le = torch.zeros_like(flat).index_put(
            (aidx,), torch.linalg.norm(v, ord=2, dim=-1, keepdim=True) *
            lights.color.sigmoid()).reshape(p.shape)
        pdf = torch.ones(p.shape[:-1], device=p.device)
        dist = None
    elif isinstance(lights, PointLights):
        # lights.py:89-110: location[:, None, None, None, :] against p [N, W, H, B, 3] (one
        # light, or one per camera)
        loc = _per_camera(lights.location, p)
        d = loc - p
        dist = torch.linalg.norm(d, dim=-1, keepdim=True)
        d = F.normalize(d, eps=1e-6, dim=-1)
        fall = lights.const.clamp(min=1e-6).to(p.device) + \
            lights.linear.clamp(min=1e-6).to(p.device) * dist + \
            lights.square.clamp(min=1e-6).to(p.device) * dist.square()
        color = _per_camera(lights.intensity, p)
        le = lights.scale.to(p.device) * F.normalize(color, dim=-1) / fall.clamp(min=1e-6)
        pdf = torch.ones(p.shape[:-1], device=p.device)
    elif isinstance(lights, RendererPointLights):
        # renderer/lighting.py:285-304 (one light): d (loc - p) / (1e-7 + dist), scale I / (..)^2
        lights.single()
        d = lights.location.reshape(-1, 3)[0].to(p.device) - p
        dist = (d * d).sum(dim=-1, keepdim=True).sqrt()
        inv = (1e-7 + dist).reciprocal()
        d = d * inv
        le = lights.scale * lights.intensity.reshape(-1, 3)[0].to(p.device) * inv * inv
        pdf = torch.ones(p.shape[:-1], device=p.device)
    else:
        raise _lib.NrtError(f"light {type(lights).__name__} has no HIP training path")
    le = torch.where(active.unsqueeze(-1), le, torch.zeros_like(le))
    return d, le, pdf, dist


def shadowed_light(shapes, lights, it, active, w_isect):
    """sample_emitter_dir_w_isect / _w_learned_occ (scene.py:290-319) with autograd: the shadow
    march is gradient-free in the reference too (intersect_test runs under no_grad, sdfs.py:
    170-179) and runs on the fused kernel; Le is masked (w_isect=True) or scaled by
    sigmoid(occ([p, dir_to_elev_azim(d)])) where occluded (w_isect=<occlusion MLP>)."""
    from .utils import dir_to_elev_azim
    d, le, pdf, dist = light_sample(lights, it, active)
    if dist is None:
        raise _lib.NrtError("shadow rays need a PointLights (ds.dist, scene.py:296)")
    rays = torch.cat([it.p, d], dim=-1).detach()
    with torch.no_grad():
        visible = shapes.intersect_test(rays, max_t=dist.detach().reshape_as(active)[..., None],
                                        active=active)
    if w_isect is True:
        le = torch.where((~visible | ~active).unsqueeze(-1), torch.zeros_like(le), le)
    else:
        occ_rays = torch.cat([it.p, dir_to_elev_azim(d)], dim=-1)
        le = torch.where((~visible)[..., None], w_isect(occ_rays).sigmoid() * le, le)
        le = active[..., None] * le
    return d, le, pdf


def bsdf_eval(bsdf, it, wo, active, feat=None):
    """eval_and_pdf of the supported BSDFs (bsdfs.py:108-118, 364-388, 515-536, 634-637).
    `feat`: param_rusin2(it.wi, wo) when the caller already has it."""
    from .bsdf.bsdfs import ComposeSpatialVarying, Conductor, Diffuse, NeuralBSDF, identity_div_pi
    from .neural_blocks import mlp_multi, same_shape
    if isinstance(bsdf, ComposeSpatialVarying):
        k = bsdf.sp_var_fn(bsdf.preprocess(it.p)).reshape(it.p.shape[:-1] + (len(bsdf.bsdfs),))
        setattr(it, "nonnormalized_weights", k)
        k = k.sigmoid()
        # every NeuralBSDF of the mixture reads the same Rusinkiewicz features of (wi, wo): the
        # reference recomputes them per component (bsdfs.py:634-637); computing them once gives
        # the same values and the same gradient (autograd sums the components' contributions),
        # with ~40 forward and ~80 backward launches per component fewer
        neural = [b for b in bsdf.bsdfs if isinstance(b, NeuralBSDF)]
        pre = {}
        if len(neural) > 1:
            feat = param_rusin2(it.wi, wo)
            mlps = [b.mlp for b in neural]
            if same_shape(mlps) and not any(m.latent_size for m in mlps):
                # the components' MLPs on the shared features: one batched HIP backward
                pre = {id(b): y for b, y in zip(neural, mlp_multi(mlps, feat))}
        parts = []
        for b in bsdf.bsdfs:
            if id(b) in pre:
                f = b.act(pre[id(b)])
                pdf = torch.ones(f.shape[:-1], device=f.device)
            else:
                f, pdf = bsdf_eval(b, it, wo, active, feat)
            parts.append(torch.cat([f, pdf.reshape(f.shape[:-1] + (1,))], dim=-1))
        spec_pdf = torch.stack(parts, dim=-1)
        setattr(it, "normalized_weights", k)
        spec_pdf = torch.where(active[..., None, None], spec_pdf * k.unsqueeze(-2),
                               torch.zeros_like(spec_pdf))
        f, pdf = spec_pdf.sum(dim=-1).split([3, 1], dim=-1)
        return f, pdf.squeeze(-1)
    if isinstance(bsdf, NeuralBSDF):
        f = bsdf.act(bsdf.mlp(param_rusin2(it.wi, wo) if feat is None else feat))
        return f, torch.ones(f.shape[:-1], device=f.device)
    if isinstance(bsdf, Diffuse):
        refl = bsdf.reflectance.to(wo.device)
        x = wo[..., 2].unsqueeze(-1) * refl
        f = x / math.pi if bsdf.preproc is identity_div_pi else bsdf.preproc(x)
        return f, wo[..., 2] / math.pi
    if isinstance(bsdf, Conductor):
        refl = local_reflect(it.wi)
        thresh = (refl * wo).sum(dim=-1, keepdim=True) > 0.94
        # eta carries no gradient, as in the reference: Conductor.eval_and_pdf passes
        # F.softplus(self.eta) into the @torch.jit.script fresnel_conductor whose eta_r parameter
        # is annotated `float` (bsdfs.py:327-328, 371), so the scripted call receives a plain number
        # and its result has requires_grad=False
        fres = fresnel_conductor(it.wi[..., 2], float(F.softplus(bsdf.eta.detach())), 0.0)
        fres = fres.reshape_as(thresh)
        f = torch.where(thresh, fres * bsdf.act(bsdf.specular.to(wo.device)),
                        torch.zeros_like(it.p))
        pdf = torch.where(thresh.reshape(it.p.shape[:-1]), 1.0, 0.0)
        f = torch.where(active.unsqueeze(-1), f, torch.zeros_like(f))
        return f, pdf
    raise _lib.NrtError(f"BSDF {type(bsdf).__name__} has no HIP training path")


def direct_sample(it, active, bsdf, lights, lead, device, shapes=None, w_isect=False):
    """Direct.sample's shading with autograd (integrators.py:167-189); w_isect as in
    integrators.py:161-166 (True: shadow rays, an MLP: learned occlusion)."""
    from .neural_blocks import SkipConnMLP
    result = torch.zeros(*lead, 3, device=device)
    if not bool(active.any()):
        return result
    if w_isect is True or type(w_isect) is SkipConnMLP:
        d, le, pdf = shadowed_light(shapes, lights, it, active, w_isect)
    else:
        d, le, pdf, _ = light_sample(lights, it, active)
    ae = active & (pdf > 0)
    wo = it.to_local(d)
    f, _ = bsdf_eval(bsdf, it, wo, ae)
    # result[ae] += f[ae] le[ae] without the boolean gathers' host syncs (both are finite and
    # zero outside ae: light_sample / bsdf_eval mask them)
    return torch.where(ae.unsqueeze(-1), result + f * le, result)


def path_sample(shapes, rays, bsdf, lights, max_depth, training, sampler, uniforms=None,
                w_isect=False):
    """Path.sample with autograd (integrators.py:275-354).  Per bounce the emitter term is
    ``direct_sample`` on the current interaction (gradients through its normals and point, the
    BSDF and the light) times the throughput, which the reference detaches after every BSDF
    sample (:335-337).  The BSDF sample itself needs no gradient: ``nrt_path_bounce`` draws it on
    the detached interaction with the same uniforms the no-grad Path uses, and updates the
    (detached) throughput and the active mask.  The spawned rays are then rebuilt with autograd
    -- origin p, direction from_local(wo) through the differentiable frame (:345,
    interaction.py:57) -- so the secondary intersection's points and normals carry gradients as
    in the reference."""
    from .shapes.sdfs import sdf_handle
    from .integrators.integrators import _bsdf_handle, _emitter_mode, _light_handle
    dev = rays.device
    lead = rays.shape[:-1]
    it, active = shapes.intersect(rays, primary=training)
    result = torch.zeros(*lead, 3, device=dev)
    if not bool(active.any()):
        return result, active, it
    original_active = active.clone()
    shadow, occ = _emitter_mode(w_isect)
    P = active.numel()
    nc = len(getattr(bsdf, "bsdfs", [bsdf]))
    act = active.reshape(-1).to(torch.uint8).contiguous()
    thr = torch.ones(P, 3, device=dev)      # detached throughput, updated by the bounce
    scratch = torch.zeros(P, 3, device=dev)  # the bounce's own (gradient-free) emitter sum
    rays_out = torch.empty(P, 6, device=dev)
    lib = _lib.load(require_device=True)
    ws = torch.empty(lib.nrt_path_workspace_bytes(P), dtype=torch.uint8, device=dev)
    sh = sdf_handle(shapes.sdf)
    curr = it
    for depth in range(max_depth):
        cur = act.bool().reshape(lead)
        term = direct_sample(curr, cur, bsdf, lights, lead, dev, shapes, w_isect)
        # a snapshot: autograd keeps this factor for the backward, and the bounce below updates
        # `thr` in place through a raw pointer (no version bump for autograd to catch)
        result = result + thr.clone().reshape(*lead, 3) * term
        if uniforms is not None:
            u_comp, u_sel = (u.to(dev).float().reshape(P, -1).contiguous() for u in uniforms[depth])
        else:
            draws = [sampler.sample(tuple(lead) + (2,), device=dev).reshape(P, 1, 2)
                     for _ in range(nc)]
            u_comp = torch.cat(draws, dim=1).contiguous()
            u_sel = sampler.sample((P,), device=dev).contiguous()
        with torch.no_grad():
            cp = curr.p.detach().reshape(P, 3).contiguous()
            cn = curr.n.detach().reshape(P, 3).contiguous()
            cw = curr.wi.detach().reshape(P, 3).contiguous()
            _lib.call("nrt_path_bounce", _bsdf_handle(bsdf), _light_handle(lights), sh, shadow,
                      occ, int(shapes.max_steps), float(shapes.epsilon), _lib.ptr(cp), _lib.ptr(cn),
                      _lib.ptr(cw), P, _lib.ptr(act), _lib.ptr(thr), _lib.ptr(scratch),
                      _lib.ptr(u_comp), _lib.ptr(u_sel), _lib.ptr(rays_out), _lib.ptr(ws),
                      _lib.precision_code(), _lib.stream())
        if depth + 1 == max_depth or not bool(act.any()):
            break  # the reference's last spawn is never shaded (:309, :342)
        # the sampled local direction carries no gradient in the reference either: NeuralBSDF /
        # Diffuse sample wo from the cosine hemisphere at the sampler's uniforms (bsdfs.py:90-106,
        # 625-633), independent of the geometry; the Conductor's reflect(it.wi) (:396) would, but
        # Conductor.sample fails in the reference and nrt_path_bounce refuses it.  The world
        # direction is rebuilt through the differentiable frame, as spawn_rays(from_local(wo)).
        with torch.no_grad():
            wo = curr.to_local(rays_out[:, 3:].reshape(*lead, 3))
        d = curr.from_local(wo.detach())
        curr, hits = shapes.intersect(curr.spawn_rays(d), primary=False)
        act &= hits.reshape(-1).to(torch.uint8)
        if not bool(act.any()):
            break
    return result, original_active, it
