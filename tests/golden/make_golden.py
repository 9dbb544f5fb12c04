"""Generate the golden fixtures under tests/golden/ from the CPU restatement (oracle/).

TEST INFRASTRUCTURE: the reference has no tests and cannot be run here
(SURVEY §8c), so these fixtures freeze the restatement itself for the configurations that are
pinned only by reading the reference (NeRFLE, PlainNeRF, Path, FoV + PointLights + Diffuse /
Conductor, DTU camera + render): every case is built from fixed seeds with injected randomness
(scan / depth jitter values, BSDF-sampling uniforms, density noise), and its inputs (rays, noise,
uniforms) and outputs are stored.  tests/test_golden.py rebuilds each case from the same seeds
and asserts the oracle still reproduces the stored outputs, so a later edit of the restatement
cannot drift silently.  The GPU parity tests compare the HIP path with the same oracle.

    python tests/golden/make_golden.py          # rewrite every fixture
"""
import os
import random
import sys

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import pathtracer_ref as R  # noqa: E402
from oracle import recipes  # noqa: E402


def _seeded(s):
    torch.manual_seed(s)
    random.seed(s)


def _weights_sum(*mods):
    """float64 sum of |parameter| over the modules: detects a change of construction order."""
    tot = 0.0
    for m in mods:
        for p in m.parameters():
            tot += float(p.detach().double().abs().sum())
        for v in vars(m).values():
            if isinstance(v, torch.Tensor):
                tot += float(v.detach().double().abs().sum())
    return np.float64(tot)


def _camera_rays(n, seed, eye=(0.0, 0.2, 1.2), spread=0.8):
    g = torch.Generator().manual_seed(seed)
    o = torch.tensor(eye) + 0.05 * torch.randn(1, n, n, 1, 3, generator=g)
    d = F.normalize(torch.cat([torch.rand(1, n, n, 1, 2, generator=g) * spread - spread / 2,
                               -torch.ones(1, n, n, 1, 1)], -1), dim=-1)
    return torch.cat([o, d], -1)


def case_nerfle(steps, envmap=False):
    _seeded(19)
    ref = R.NeRFLERef(steps=steps, envmap=envmap)
    rays = _camera_rays(6 if steps > 64 else 10, 4)
    loc = torch.tensor([[0.3, 1.0, 0.2]])
    light = R.PointLightRef(location=(0.3, 1.0, 0.2)) if envmap else None
    with torch.no_grad():
        out = ref(rays, loc, jitter=0.37, light=light)
    return dict(rays=rays, light_location=loc, jitter=np.float64(0.37), out=out,
                weights=_weights_sum(ref))


def case_plain_nerf():
    _seeded(29)
    ref = R.PlainNeRFRef(steps=32)
    latent = torch.randn(1, ref.latent_size)
    ref.assign_latent(latent)
    rays = _camera_rays(8, 5)
    noise = torch.randn(32, *rays.shape[:-1], 1, generator=torch.Generator().manual_seed(6)) * 1e-3
    with torch.no_grad():
        out = ref(rays, jitter=0.61, noise=noise)
    return dict(rays=rays, latent=latent, noise=noise, jitter=np.float64(0.61), out=out,
                weights=_weights_sum(ref))


def _path_scene(loc=(0.4, 0.9, 0.8)):
    _seeded(31)
    sdf = R.SphereBlobSDF(n=16)
    with torch.no_grad():
        sdf.radii.add_(0.15)
    parts = [R.NeuralBSDFRef(), R.NeuralBSDFRef(), R.DiffuseRef()]
    bsdf = R.SpatialMixBSDF(parts)
    return sdf, bsdf, R.PointLightRef(location=loc, scale=5.0)


def case_path(w_isect):
    # the shadowed case puts the light to the side and behind, so part of the visible surface
    # faces away from it and its shadow rays are blocked
    sdf, bsdf, light = _path_scene((-0.9, 0.2, -0.3) if w_isect else (0.4, 0.9, 0.8))
    shape = R.MarchedSDF(sdf=sdf, max_steps=48)
    c2w = recipes.look_at_c2w((0.1, 0.5, 0.9)).unsqueeze(0)
    cam = R.NeRFCameraRef(c2w, recipes.nerf_focal(16))
    rays = cam.sample_positions(R._tile_positions(0, 0, 16), 16)
    g = torch.Generator().manual_seed(9)
    lead = rays.shape[:-1]
    uniforms = [(torch.rand(*lead, 3, 2, generator=g), torch.rand(*lead, generator=g))
                for _ in range(2)]
    with torch.no_grad():
        out, mask, _ = R.PathRef().sample(shape, rays, bsdf, light, w_isect=w_isect,
                                          uniforms=uniforms)
    return dict(rays=rays, u_comp0=uniforms[0][0], u_sel0=uniforms[0][1],
                u_comp1=uniforms[1][0], u_sel1=uniforms[1][1], out=out, mask=mask,
                weights=_weights_sum(sdf, bsdf))


def _colocate_scene():
    _seeded(13)
    sdf = R.SphereBlobSDF(n=64)
    parts = [R.NeuralBSDFRef(), R.NeuralBSDFRef(),
             R.DiffuseRef(reflectance=torch.rand(3).tolist(), preprocess="softplus"),
             R.ConductorRef(specular=torch.rand(3).tolist(), activation="softplus")]
    bsdf = R.SpatialMixBSDF(parts)
    Rm, Tm = R.look_at_view_transform_ref(dist=1.0, elev=30.0, azim=45.0)
    cam = R.FoVCameraRef(Rm, Tm, znear=1.0, zfar=100.0)
    light = R.PointLightRef(location=(cam.center()[0] * 1.05).tolist(), scale=5.0)
    return sdf, bsdf, cam, light


def case_colocate():
    sdf, bsdf, cam, light = _colocate_scene()
    shape = R.MarchedSDF(sdf=sdf, max_steps=64)
    random.seed(17)
    with torch.no_grad():
        out = R.render(shape, light, cam, R.DirectRef(), bsdf, size=32, chunk_size=16,
                       background=0.5, with_noise=0.0)
    rays = cam.sample_positions(R._tile_positions(8, 8, 8), 32)
    return dict(out=out, rays_crop=rays, weights=_weights_sum(sdf, bsdf))


def _dtu_scene():
    import bench
    _seeded(41)
    sdf = R.SkipMLP(num_layers=8, hidden_size=64, out=1, freqs=16, activation="softplus")
    bench.shape_mlp_sdf(sdf, radius=0.25, copies=8)
    parts = [R.NeuralBSDFRef(activation="sigmoid") for _ in range(3)] + \
            [R.DiffuseRef(reflectance=torch.rand(3).tolist(), preprocess="sigmoid")]
    bsdf = R.SpatialMixBSDF(parts)
    lights = R.LightFieldRef()
    K = torch.eye(4)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = 2890.0, 2890.0, 800.0, 600.0
    pose = torch.eye(4)
    pose[:3, :4] = recipes.look_at_c2w((0.0, 0.5, 0.866))
    pose[:3, 1:3] *= -1  # DTU/IDR cameras look down +z
    return sdf, bsdf, lights, R.DTUCameraRef(pose[None], K[None])


def case_dtu():
    sdf, bsdf, lights, cam = _dtu_scene()
    shape = R.MarchedSDF(sdf=lambda p: sdf(p)[..., 0], max_steps=64)
    random.seed(6)
    with torch.no_grad():
        out = R.render(shape, lights, cam, R.NeRFIntegratorRef(R.DirectRef()), bsdf, size=128,
                       chunk_size=128, background=0.0, crop=(44, 10, 16))
    rays = cam.sample_positions(R._tile_positions(44, 10, 16), 128)
    return dict(out=out, rays=rays, weights=_weights_sum(sdf, bsdf, lights))


CASES = {
    "nerfle_s64": lambda: case_nerfle(64),
    "nerfle_s256": lambda: case_nerfle(256),
    "nerfle_envmap": lambda: case_nerfle(64, envmap=True),
    "plain_nerf": case_plain_nerf,
    "path_2bounce": lambda: case_path(False),
    "path_2bounce_shadow": lambda: case_path(True),
    "colocate_fov_pointlight": case_colocate,
    "dtu_camera_render": case_dtu,
}


def to_numpy(d):
    return {k: (v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v)
            for k, v in d.items()}


def main():
    torch.set_num_threads(1)  # one fixed summation order for the CPU BLAS
    for name, fn in CASES.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **to_numpy(fn()))
        print(f"{name}: {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
