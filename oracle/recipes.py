"""Seeded scene recipes for the oracle (TEST INFRASTRUCTURE ONLY).

Each builder reproduces the construction order of a reference driver so that the torch RNG
stream -- and therefore every weight -- matches what the reference would draw from the same
seeds.  Builders return plain oracle objects; ``tests/`` copy their weights into the product
classes of ``neural_raytracing_amd`` so both paths see identical parameters.
"""
import math
import random

import numpy as np
import torch

from . import pathtracer_ref as R

LEGO_FOV_X = 0.6911112070083618  # camera_angle_x of nerf_synthetic scenes (rounded in BASELINE.md)


def nerf_focal(size, fov_x=0.6911):
    """scripts/nerf_synthetic.py:49: ``0.5 * SIZE / tan(0.5 * camera_angle_x)``."""
    return float(0.5 * size / np.tan(0.5 * fov_x))


def look_at_c2w(eye, target=(0.0, 0.0, 0.0), up=(0.0, 1.0, 0.0)):
    """A NeRF-convention camera-to-world [3,4] (camera looks down -z)."""
    eye = torch.tensor(eye, dtype=torch.float)
    fwd = torch.nn.functional.normalize(torch.tensor(target) - eye, dim=0)
    right = torch.nn.functional.normalize(torch.cross(fwd, torch.tensor(up), dim=0), dim=0)
    upv = torch.cross(right, fwd, dim=0)
    c2w = torch.zeros(3, 4)
    c2w[:, 0] = right
    c2w[:, 1] = upv
    c2w[:, 2] = -fwd
    c2w[:, 3] = eye
    return c2w


def baseline_checksum_scene():
    """BASELINE.md §2 recipe: the one recorded run of the reference.

    Construction order: SphereSDF(n=128) -> SDF(max_steps=32) ->
    ComposeSpatialVarying([NeuralBSDF(Softplus)]*8) -> LightField -> NeRFIntegrator(Direct).
    """
    torch.manual_seed(0)
    random.seed(0)
    sphere = R.SphereBlobSDF(n=128)
    shape = R.MarchedSDF(sdf=sphere, max_steps=32)
    parts = [R.NeuralBSDFRef(activation="softplus") for _ in range(8)]
    bsdf = R.SpatialMixBSDF(parts)
    lights = R.LightFieldRef()
    integrator = R.NeRFIntegratorRef(R.DirectRef())
    c2w = torch.eye(4)[:3, :4].clone()
    c2w[2, 3] = 1
    camera = R.NeRFCameraRef(c2w.unsqueeze(0), nerf_focal(256))
    return dict(shape=shape, bsdf=bsdf, lights=lights, integrator=integrator, camera=camera)


def baseline_checksum_render(scene=None):
    """Render the BASELINE.md §2 crop; returns the [64,64,4] image."""
    if scene is None:
        scene = baseline_checksum_scene()
    with torch.no_grad():
        return R.render(scene["shape"], scene["lights"], scene["camera"], scene["integrator"],
                        scene["bsdf"], size=256, chunk_size=256, background=0.0,
                        with_noise=1e-2, crop=(96, 96, 64))


BASELINE_ABS_SUM = 4511.5146484375
