"""Emitter sampling helpers of scene.py with the reference's names.

``sample_emitter_dir_wo_isect`` / ``_w_isect`` / ``_w_learned_occ`` (scene.py:290-324) run inside
the fused shading entry points (``nrt_shade_direct`` / ``_shadowed`` / ``_learned_occ``), selected
by ``Direct`` / ``Path`` from ``w_isect`` exactly as integrators.py:161-166 does; the functions here
are the autograd restatements (differentiable.py) for callers that use them directly.  The mesh
intersectors (scene.py:10-162, 231-287) belong to the mesh renderer, which is out of scope.
"""
from .differentiable import light_sample, shadowed_light


def sample_emitter_dir_wo_isect(it, shapes=None, lights=None, sampler=None, active=True):
    """scene.py:321-324 -> (DirectionSample-like d, Le)."""
    from .interaction import DirectionSample
    d, le, pdf, dist = light_sample(lights, it, active)
    return DirectionSample(d=d, pdf=pdf, dist=dist), le


def sample_emitter_dir_w_isect(it, shapes, lights, sampler=None, active=True):
    """scene.py:290-298: Le zeroed where the shadow ray toward the light is blocked."""
    from .interaction import DirectionSample
    d, le, pdf = shadowed_light(shapes, lights, it, active, True)
    return DirectionSample(d=d, pdf=pdf), le


def sample_emitter_dir_w_learned_occ(it, shapes, lights, occ_mlp, sampler=None, active=True):
    """scene.py:301-319: occluded Le scaled by sigmoid(occ([p, elev/azim(d)]))."""
    from .interaction import DirectionSample
    d, le, pdf = shadowed_light(shapes, lights, it, active, occ_mlp)
    return DirectionSample(d=d, pdf=pdf), le


def mesh_intersect(*args, **kwargs):
    raise NotImplementedError("mesh_intersect (scene.py:10-110) belongs to the mesh renderer, "
                              "which is out of scope")


def mesh_intersect_test(*args, **kwargs):
    raise NotImplementedError("mesh_intersect_test (scene.py:112-162) belongs to the mesh "
                              "renderer, which is out of scope")
