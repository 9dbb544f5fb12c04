"""Dataset and camera loaders of the reference's drivers (host side, no GPU work).

* ``test_nerf_resources`` -- NeRF-synthetic ``transforms_{train,test}.json`` + RGBA PNGs
  (training_utils.py:572-594): focal from ``camera_angle_x`` at the requested size, masks as
  ``ceil(alpha - 1e-5)``, camera-to-world [3, 4] with the translation normalised to unit length.
* ``decompose_projection_matrix`` -- the K, R, camera-centre split of a 3x4 projection that
  ``cv2.decomposeProjectionMatrix`` returns (cv2 is not in this image): an RQ factorisation
  M = K R with R a proper rotation and K upper triangular with K[0,0], K[1,1] > 0 (OpenCV's
  RQDecomp3x3 resolves the sign ambiguity the same way), and the homogeneous camera centre as
  the null vector of P.
* ``KRt_from_P`` / ``load_dtu_cameras`` / ``load_dtu`` -- scripts/dtu.py:50-89: ``cameras.npz``
  world_mat_i @ scale_mat_i, intrinsics K / K[2,2] as a 4x4, pose [R^T | centre], translations
  divided by the largest camera distance; sorted ``mask/`` and ``image/`` directories.
* ``train_nerf`` / ``train_dtu`` -- the per-scene optimisation loops (training_utils.py:211-300,
  347-434): N views per step chosen by a ``LossSampler``, ``pathtrace_sample`` of a crop with
  autograd through the HIP path, ``masked_loss`` + ``extra_loss``, one
  optimiser step, periodic validation renders under ``torch.no_grad``.
* ``test_nerf`` / ``test_dtu`` / ``test`` / ``test_nerv_ptl`` -- the evaluation loops the drivers
  end with (training_utils.py:302-345, 436-485, 487-534, 792-853; nerf_synthetic.py:129,
  dtu.py:179): one ``pathtrace`` per view under ``torch.no_grad`` on the fused HIP kernels,
  ``save_plot``, printed L1 / L2 / PSNR and SSIM (``metrics.ssim``: pytorch_msssim is absent).
* ``train`` / ``train_sample`` / ``train_nerv_ptl`` (training_utils.py:55-121, 123-208, 686-789),
  ``pathtrace_labels`` (:35-51), ``test_colocate_resources`` (:538-570), ``save_image`` /
  ``save_plot`` (:21-33).
"""
import json
import os

import numpy as np
import torch
import torch.nn.functional as F

from .utils import load_image, save_image  # noqa: F401  (training_utils.py:21 re-export)


def save_plot(expected, got, name):
    """training_utils.py:22-33: got | expected side by side, axes off (matplotlib, Agg)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig = plt.figure()
    fig.add_subplot(1, 2, 1)
    plt.imshow(got.detach().squeeze().cpu().numpy())
    plt.grid(False)
    plt.axis("off")
    fig.add_subplot(1, 2, 2)
    plt.imshow(expected.detach().squeeze().cpu().numpy())
    plt.grid(False)
    plt.axis("off")
    plt.savefig(name)
    plt.close(fig)


def _progress(seq):
    from tqdm import tqdm
    return tqdm(seq)


def _summary(l1, l2, psnr):
    print("Avg l1 loss", np.mean(l1))
    print("Avg l2 loss", np.mean(l2))
    print("Avg PSNR loss", np.mean(psnr))


def test_nerf(density_field, integrator, bsdf, lights, cam_to_worlds, focal, exp_imgs, size,
              name_fn=lambda i: f"outputs/test_{i:03}.png"):
    """training_utils.py:302-345: render every test view (pathtrace, chunk min(size, 256),
    background 0, clamped to [0, 1]), save_plot, print average L1 / L2 / PSNR and the SSIM of the
    stacked views."""
    from . import pathtrace
    from .cameras import NeRFCamera
    from .metrics import ssim
    from .utils import mse2psnr
    device = exp_imgs[0].device
    l1, l2, psnr, gots = [], [], [], []
    with torch.no_grad():
        for i, c2w in enumerate(_progress(cam_to_worlds)):
            exp = exp_imgs[i]
            cameras = NeRFCamera(cam_to_world=c2w.unsqueeze(0), focal=focal, device=device)
            got = pathtrace(density_field, size=size, chunk_size=min(size, 256), bundle_size=1,
                            bsdf=bsdf, integrator=integrator, cameras=cameras, lights=lights,
                            device=device, silent=True, background=0)[0].clamp(min=0, max=1)
            save_plot(exp, got, name_fn(i))
            l1.append(F.l1_loss(exp, got).item())
            l2.append(F.mse_loss(exp, got).item())
            psnr.append(mse2psnr(F.mse_loss(exp, got)).item())
            gots.append(got)
    _summary(l1, l2, psnr)
    with torch.no_grad():
        gots = torch.stack(gots, dim=0).permute(0, 3, 1, 2)
        exps = torch.stack(exp_imgs, dim=0).permute(0, 3, 1, 2)
        torch.cuda.empty_cache()
        print("SSIM loss", ssim(gots, exps, data_range=1, size_average=True).item())
    return


def test_dtu(density_field, integrator, bsdf, lights, poses, intrinsics, exp_imgs, exp_masks, size,
             name_fn=lambda i: f"outputs/test_{i:03}.png"):
    """training_utils.py:436-485: DTUCamera per test pose (chunk min(size, 128)); the metrics are
    taken on the masked images."""
    from . import pathtrace
    from .cameras import DTUCamera
    from .metrics import ssim
    from .utils import mse2psnr
    device = exp_imgs[0].device
    l1, l2, psnr, gots, exps = [], [], [], [], []
    with torch.no_grad():
        for i, (pose, intrinsic) in enumerate(zip(_progress(poses), intrinsics)):
            exp = exp_imgs[i]
            mask = exp_masks[i] == 1
            cameras = DTUCamera(pose=pose[None, ...], intrinsic=intrinsic[None, ...], device=device)
            got = pathtrace(density_field, size=size, chunk_size=min(size, 128), bundle_size=1,
                            bsdf=bsdf, integrator=integrator, cameras=cameras, lights=lights,
                            device=device, silent=True, background=0)[0].clamp(min=0, max=1)
            save_plot(exp, got, name_fn(i))
            exp = exp * mask[..., None]
            got = got * mask[..., None]
            l1.append(F.l1_loss(exp, got).item())
            mse = F.mse_loss(exp, got)
            l2.append(mse.item())
            psnr.append(mse2psnr(mse).item())
            gots.append(got)
            exps.append(exp)
    _summary(l1, l2, psnr)
    with torch.no_grad():
        gots = torch.stack(gots, dim=0).permute(0, 3, 1, 2)
        exps = torch.stack(exps, dim=0).permute(0, 3, 1, 2)
        torch.cuda.empty_cache()
        print("SSIM loss", ssim(gots, exps, data_range=1, size_average=True).item())
    return


def no_update(cameras, lights):
    return


def test(density_field, integrator, bsdf, lights, Rs, Ts, exp_imgs, size, max_chunk_size=128,
         light_update=no_update, name_fn=lambda i: f"outputs/test_{i:03}.png", w_isect=False):
    """training_utils.py:487-534 (colocate.py's evaluation): OpenGLPerspectiveCameras per (R, T),
    ``light_update`` moves the light with the camera; SSIM over every third view."""
    from . import pathtrace
    from .cameras import OpenGLPerspectiveCameras
    from .metrics import ssim
    from .utils import mse2psnr
    device = exp_imgs[0].device
    l1, l2, psnr, gots = [], [], [], []
    with torch.no_grad():
        for i, (R, T) in enumerate(zip(_progress(Rs), Ts)):
            exp = exp_imgs[i]
            cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
            light_update(cameras, lights)
            got = pathtrace(density_field, size=size, chunk_size=min(size, max_chunk_size),
                            bundle_size=1, bsdf=bsdf, integrator=integrator, cameras=cameras,
                            lights=lights, device=device, silent=True, background=0,
                            w_isect=w_isect)[0].clamp(min=0, max=1)
            save_plot(exp, got, name_fn(i))
            l1.append(F.l1_loss(exp, got).item())
            l2.append(F.mse_loss(exp, got).item())
            psnr.append(mse2psnr(F.mse_loss(exp, got)).item())
            gots.append(got)
    _summary(l1, l2, psnr)
    with torch.no_grad():
        gots = torch.stack(gots[::3], dim=0).permute(0, 3, 1, 2)
        exps = torch.stack(exp_imgs[::3], dim=0).permute(0, 3, 1, 2)
        torch.cuda.empty_cache()
        print("SSIM loss", ssim(gots, exps, data_range=1, size_average=True).item())
    return


def test_nerv_ptl(density_field, bsdf, integrator, light_locs, cam_to_worlds, focal, exp_imgs, size,
                  name_fn=lambda i: f"outputs/test_{i:03}.png", w_isect=True):
    """training_utils.py:792-853: a NeRFCamera and a PointLights(scale 100) per view, shadow rays
    (w_isect), gamma-2.2 plots, PSNR on the clamped images, MS-SSIM and SSIM of the tone-mapped
    x / (1 + x) stacks."""
    from . import pathtrace
    from .cameras import NeRFCamera
    from .lights import PointLights
    from .metrics import ms_ssim, ssim
    from .utils import mse2psnr
    device = exp_imgs[0].device
    l1, l2, psnr, gots = [], [], [], []
    with torch.no_grad():
        for i, (c2w, lp) in enumerate(zip(_progress(cam_to_worlds), light_locs)):
            exp = exp_imgs[i].clamp(min=0, max=1)
            cameras = NeRFCamera(cam_to_world=c2w.unsqueeze(0), focal=focal, device=device)
            lights = PointLights(intensity=[1, 1, 1], location=lp[None, ...], scale=100,
                                 device=device)
            got = pathtrace(density_field, size=size, chunk_size=min(size, 100), bundle_size=1,
                            bsdf=bsdf, integrator=integrator, background=0, cameras=cameras,
                            lights=lights, device=device, silent=True,
                            w_isect=w_isect)[0].clamp(min=0, max=1)
            save_plot(exp ** (1 / 2.2), got ** (1 / 2.2), name_fn(i))
            l1.append(F.l1_loss(exp, got).item())
            mse = F.mse_loss(exp, got)
            l2.append(mse.item())
            psnr.append(mse2psnr(mse).item())
            gots.append(got)
    _summary(l1, l2, psnr)
    with torch.no_grad():
        gots = torch.stack(gots, dim=0).permute(0, 3, 1, 2)
        tm_gots = gots / (1 + gots)
        exps = torch.stack(exp_imgs, dim=0).permute(0, 3, 1, 2)
        tm_exps = exps / (1 + exps)
        torch.cuda.empty_cache()
        print("MS-SSIM loss", ms_ssim(tm_gots, tm_exps, data_range=1, size_average=True).item())
        print("SSIM loss", ssim(tm_gots, tm_exps, data_range=1, size_average=True).item())
    return


def pathtrace_labels(ref, size, integrator, bsdf, lights, Rs, Ts):
    """training_utils.py:35-51: render ground-truth images and masks of a reference shape with
    Mask(integrator) for every (R, T)."""
    from . import pathtrace
    from .cameras import OpenGLPerspectiveCameras
    from .integrators import Mask
    exp_imgs, exp_masks = [], []
    with torch.no_grad():
        for R, T in zip(Rs, Ts):
            device = R.device
            cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
            expected = pathtrace(ref, size=size, chunk_size=size, bundle_size=1, bsdf=bsdf,
                                 integrator=Mask(integrator), cameras=cameras, lights=lights,
                                 device=device, silent=True)[0].detach()
            exp_imgs.append(expected[..., :-1])
            exp_masks.append(expected[..., -1])
    return exp_imgs, exp_masks


def test_colocate_resources(kind, size=128, dist=1, device="cuda"):
    """training_utils.py:538-570: 4 x 4 camera positions (elev 0..45, azim -90..90) x 3 x 3 light
    positions at 1.05 dist, images gt_{kind}_{i}_{j}_{k}_{l}.png of mitsuba_scenes/cbox_relight."""
    from .cameras import look_at_view_transform

    def elaz_to_xyz(elev, azim, rad):
        elev = torch.deg2rad(elev)
        azim = torch.deg2rad(azim)
        return torch.stack([rad * elev.cos() * azim.sin(), rad * elev.cos() * azim.cos(),
                            rad * elev.sin()], dim=0)

    Rs, Ts, exp_imgs, exp_masks, xyzs = [], [], [], [], []
    for i, elev in enumerate(torch.linspace(0, 45, 4, device=device)):
        for j, azim in enumerate(torch.linspace(-90, 90, 4, device=device)):
            R, T = look_at_view_transform(dist=dist, elev=elev.cpu(), azim=azim.cpu(),
                                          device=device)
            for k, e2 in enumerate(torch.linspace(0, 45, 3, device=device)):
                for l_, a2 in enumerate(torch.linspace(-90, 90, 3, device=device)):
                    Rs.append(R)
                    Ts.append(T)
                    img = load_image(f"mitsuba_scenes/cbox_relight/gt_{kind}_{i:03}_{j:03}_"
                                     f"{k:03}_{l_:03}.png", (size, size)).to(device)
                    exp_imgs.append(img[..., :3])
                    exp_masks.append(img[..., 3])
                    xyzs.append(elaz_to_xyz(e2, a2, dist * 1.05))
    return Rs, Ts, exp_imgs, exp_masks, xyzs


def test_nerf_resources(directory, size=128, kind="test", device="cuda"):
    """training_utils.py:572-594 -> (cam_to_worlds, focal, exp_imgs, exp_masks)."""
    assert kind in ["train", "test"]
    with open(os.path.join(directory, f"transforms_{kind}.json")) as fh:
        tfs = json.load(fh)
    exp_imgs, exp_masks, cam_to_worlds = [], [], []
    focal = 0.5 * size / np.tan(0.5 * float(tfs["camera_angle_x"]))
    for frame in tfs["frames"]:
        img = load_image(os.path.join(directory, frame["file_path"] + ".png"),
                         resize=(size, size)).to(device)
        exp_imgs.append(img[..., :3])
        exp_masks.append((img[..., 3] - 1e-5).ceil())
        tf_mat = torch.tensor(frame["transform_matrix"], dtype=torch.float, device=device)[:3, :4]
        tf_mat[:3, 3] = F.normalize(tf_mat[:3, 3], dim=-1)  # distance 1 from the origin
        cam_to_worlds.append(tf_mat)
    return cam_to_worlds, focal, exp_imgs, exp_masks


def rq3(M):
    """M = K @ R, K upper triangular with K[0,0], K[1,1] > 0, R in SO(3) (float64 numpy)."""
    M = np.asarray(M, dtype=np.float64)
    Pm = np.flipud(np.eye(3))
    q, r = np.linalg.qr((Pm @ M).T)
    K = Pm @ r.T @ Pm
    R = Pm @ q.T
    if np.linalg.det(R) < 0:
        K, R = -K, -R
    if K[0, 0] < 0 and K[1, 1] < 0:
        D = np.diag([-1.0, -1.0, 1.0])
    elif K[0, 0] < 0:
        D = np.diag([-1.0, 1.0, -1.0])
    elif K[1, 1] < 0:
        D = np.diag([1.0, -1.0, -1.0])
    else:
        D = np.eye(3)
    return K @ D, D @ R


def decompose_projection_matrix(P):
    """(K, R, t) of a 3x4 projection as cv2.decomposeProjectionMatrix returns its first three
    outputs: K upper triangular (not normalised), R the world-to-camera rotation, t the
    homogeneous camera centre [4, 1] (P @ t = 0; scale and sign arbitrary)."""
    P = np.asarray(P, dtype=np.float64)
    if P.shape != (3, 4):
        raise ValueError("decompose_projection_matrix: P must be 3x4")
    K, R = rq3(P[:, :3])
    _, _, vt = np.linalg.svd(P)
    t = vt[-1].reshape(4, 1)
    return K, R, t


def KRt_from_P(P, device="cuda"):
    """scripts/dtu.py:70-80 -> (intrinsics [4, 4], pose [4, 4]) float32 tensors."""
    K, R, t = decompose_projection_matrix(P)
    K = K / K[2, 2]
    intrinsics = np.eye(4)
    intrinsics[:3, :3] = K
    pose = np.eye(4, dtype=np.float32)
    pose[:3, :3] = R.transpose()
    pose[:3, 3] = (t[:3] / t[3])[:, 0]
    return (torch.from_numpy(intrinsics).float().to(device),
            torch.from_numpy(pose).float().to(device))


def load_dtu_cameras(path, num_imgs, device="cuda"):
    """scripts/dtu.py:69-89: cameras.npz -> (intrinsics [n, 4, 4], poses [n, 4, 4]) with the
    camera centres scaled so the farthest is at distance 1."""
    tfs = np.load(path)  # allow_pickle stays False
    Ps = [tfs[f"world_mat_{i}"] @ tfs[f"scale_mat_{i}"] for i in range(num_imgs)]
    intrinsics, poses = zip(*[KRt_from_P(p[:3, :4], device) for p in Ps])
    poses = torch.stack(poses, dim=0)
    max_dist = torch.linalg.norm(poses[:, :3, 3], dim=-1).max()
    poses[:, :3, 3] /= max_dist
    return torch.stack(intrinsics, dim=0), poses


def load_dtu(directory, size=512, device="cuda"):
    """scripts/dtu.py:50-89 -> (exp_imgs, exp_masks, intrinsics, poses): masks are the channel
    max, ceiled; files listed in sorted order, skipping AppleDouble ``._*`` entries."""
    exp_masks, exp_imgs = [], []
    mask_dir = os.path.join(directory, "mask")
    for f in sorted(os.listdir(mask_dir)):
        if f.startswith("._"):
            continue
        mask = load_image(os.path.join(mask_dir, f), resize=(size, size)).to(device)
        exp_masks.append(mask.max(dim=-1)[0].ceil())
    image_dir = os.path.join(directory, "image")
    for f in sorted(os.listdir(image_dir)):
        if f.startswith("._"):
            continue
        exp_imgs.append(load_image(os.path.join(image_dir, f), resize=(size, size)).to(device))
    assert len(exp_imgs) == len(exp_masks)
    intrinsics, poses = load_dtu_cameras(os.path.join(directory, "cameras.npz"), len(exp_imgs),
                                         device)
    return exp_imgs, exp_masks, intrinsics, poses


def _train_loop(make_cameras, valid_cameras, shape, bsdf, integrator, lights, exp_imgs, exp_masks,
                opt, size, crop_size, N, iters, num_ckpts, save_freq, valid_freq, max_valid_size,
                extra_loss, save_fn, name_fn, valid_name_fn, uv_select, silent, mask_weight):
    from .. import pathtracer as pt
    from .integrators import NeRFIntegrator
    from .utils import LossSampler, masked_loss, save_image
    train_integrator = NeRFIntegrator(integrator)
    device = exp_imgs[0].device
    ckpt_freq = (iters // num_ckpts) - 1
    losses = []
    selector = LossSampler(len(exp_imgs))
    for i in range(iters):
        idxs = selector.sample(n=N)
        cameras = make_cameras(idxs)
        exp = torch.stack([exp_imgs[j] for j in idxs])
        mask = torch.stack([exp_masks[j] for j in idxs])
        opt.zero_grad()
        (u, v) = uv_select(mask[0], crop_size)
        u, v = int(u), int(v)
        got, mi = pt.pathtrace_sample(shape, size=size, chunk_size=size, bundle_size=1,
                                      crop_size=crop_size, bsdf=bsdf, integrator=train_integrator,
                                      cameras=cameras, lights=lights, device=device, uv=(u, v),
                                      background=0, addition=lambda m: m, squeeze_first=False,
                                      silent=True)
        if save_freq and (i % save_freq) == 0 and name_fn is not None:
            save_image(name_fn(i), got[0])
        exp = exp[:, u:u + crop_size, v:v + crop_size]
        mask = mask[:, u:u + crop_size, v:v + crop_size]
        loss = masked_loss(got[..., :3], exp, mi.throughput.squeeze(-1), mask,
                           mask_weight=mask_weight, with_logits=mi.with_logits) + \
            extra_loss(mi, got, exp, mask)
        if loss.isnan():
            loss.backward()
            opt.step()
            raise Exception("Unexpected NaN")
        loss.backward()
        opt.step()
        loss = loss.detach().item()
        losses.append(loss)
        selector.update_idxs(idxs, loss)
        if silent:
            print(f"{i:06}: {loss:.05}")
        if ((i % ckpt_freq) == 0) and (i != 0):
            save_fn(i)
        if valid_freq and (i % valid_freq) == 0 and valid_name_fn is not None:
            with torch.no_grad():
                validate, _ = pt.pathtrace(shape, size=size, chunk_size=min(size, max_valid_size),
                                           bundle_size=1, bsdf=bsdf, integrator=train_integrator,
                                           cameras=valid_cameras(idxs), lights=lights,
                                           device=device, silent=True)
                save_image(valid_name_fn(i), validate)
    return losses


def train_nerf(shape, bsdf, integrator, lights, cam_to_worlds, focal, exp_imgs, exp_masks, opt,
               size, crop_size, N=3, iters=50_000, num_ckpts=5, save_freq=50, valid_freq=250,
               max_valid_size=128, extra_loss=lambda mi, got, exp, mask: 0,
               save_fn=lambda i: None, name_fn=lambda i: f"outputs/train_{i:05}.png",
               valid_name_fn=lambda i: f"outputs/valid_{i:05}.png", uv_select=None,
               silent=False):
    """training_utils.py:211-300 (NeRF-synthetic scenes, NeRFCamera, mask_weight 15)."""
    from .cameras import NeRFCamera
    from .utils import rand_uv_mask
    device = exp_imgs[0].device

    def cams(idxs):
        c2w = torch.stack([cam_to_worlds[j] for j in idxs], dim=0)
        return NeRFCamera(cam_to_world=c2w, focal=focal, device=device)

    def valid(idxs):
        return NeRFCamera(cam_to_world=cam_to_worlds[idxs[0]].unsqueeze(0), focal=focal,
                          device=device)
    return _train_loop(cams, valid, shape, bsdf, integrator, lights, exp_imgs, exp_masks, opt,
                       size, crop_size, N, iters, num_ckpts, save_freq, valid_freq,
                       max_valid_size, extra_loss, save_fn, name_fn, valid_name_fn,
                       uv_select or rand_uv_mask, silent, 15)


def train_dtu(shape, bsdf, integrator, lights, poses, intrinsics, exp_imgs, exp_masks, opt, size,
              crop_size, N=3, iters=50_000, num_ckpts=5, save_freq=50, valid_freq=250,
              max_valid_size=128, extra_loss=lambda mi, got, exp, mask: 0,
              save_fn=lambda i: None, name_fn=lambda i: f"outputs/train_{i:05}.png",
              valid_name_fn=lambda i: f"outputs/valid_{i:05}.png", uv_select=None,
              silent=False):
    """training_utils.py:347-434 (DTU scans, DTUCamera, mask_weight 10)."""
    from .cameras import DTUCamera
    from .utils import rand_uv_mask
    device = exp_imgs[0].device

    def cams(idxs):
        pose = torch.stack([poses[j] for j in idxs], dim=0)
        intr = torch.stack([intrinsics[j] for j in idxs], dim=0)
        return DTUCamera(pose=pose, intrinsic=intr, device=device)

    def valid(idxs):
        # training_utils.py:421-423: the first drawn pose with intrinsics[0]
        return DTUCamera(pose=poses[idxs[0]][None], intrinsic=intrinsics[0][None], device=device)
    return _train_loop(cams, valid, shape, bsdf, integrator, lights, exp_imgs, exp_masks, opt,
                       size, crop_size, N, iters, num_ckpts, save_freq, valid_freq,
                       max_valid_size, extra_loss, save_fn, name_fn, valid_name_fn,
                       uv_select or rand_uv_mask, silent, 10)


def _silent_update(iterator, silent, every=1):
    if silent:
        return lambda loss, i: print(f"{i:06}: {loss:.05}") if i % every == 0 else None
    return lambda loss, _: iterator.set_postfix(refresh=False, loss=f"{loss:.05}")


def _iterations(iters, silent):
    if silent:
        return range(iters)
    from tqdm import trange
    return trange(iters)


def train(shape, bsdf, integrator, lights, Rs, Ts, exp_imgs, exp_masks, opt, size, N=3,
          iters=50_000, num_ckpts=5, save_freq=50, light_update=no_update,
          save_fn=lambda i: None, name_fn=lambda i: f"outputs/train_{i:05}.png",
          extra_loss=lambda mi, got, exp, mask: 0, silent=True):
    """training_utils.py:55-121: full-frame training with OpenGLPerspectiveCameras, N views per
    step, NeRFIntegrator(integrator), masked_loss (mask_weight 15) + extra_loss; a NaN loss skips
    the step."""
    from . import pathtrace
    from .cameras import OpenGLPerspectiveCameras
    from .integrators import NeRFIntegrator
    from .utils import LossSampler, masked_loss
    integrator = NeRFIntegrator(integrator)
    device = exp_imgs[0].device
    ckpt_freq = (iters // num_ckpts) - 1
    losses = []
    selector = LossSampler(len(exp_imgs))
    iterator = _iterations(iters, silent)
    update = _silent_update(iterator, silent)
    for i in iterator:
        idxs = selector.sample(n=N)
        R = torch.cat([Rs[j] for j in idxs], dim=0)
        T = torch.cat([Ts[j] for j in idxs], dim=0)
        cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
        light_update(cameras, lights)
        opt.zero_grad()
        got, mi = pathtrace(shape, size=size, chunk_size=size, bundle_size=1, bsdf=bsdf,
                            integrator=integrator, cameras=cameras, lights=lights, device=device,
                            background=0, addition=lambda m: m, squeeze_first=False, silent=True)
        if (i % save_freq) == 0:
            save_image(name_fn(i), got[0])
        exp = torch.stack([exp_imgs[j] for j in idxs])
        mask = torch.stack([exp_masks[j] for j in idxs])
        loss = masked_loss(got[..., :3], exp, mi.throughput.squeeze(-1), mask, mask_weight=15,
                           with_logits=mi.with_logits) + extra_loss(mi, got, exp, mask)
        if loss.isnan():
            continue
        loss.backward()
        loss = loss.item()
        selector.update_idxs(idxs, loss)
        losses.append(loss)
        opt.step()
        update(loss, i)
        if ((i % ckpt_freq) == 0) and (i != 0):
            save_fn(i)
    return losses


def train_sample(shape, bsdf, integrator, lights, Rs, Ts, exp_imgs, exp_masks, opt, size,
                 crop_size, N=3, iters=50_000, num_ckpts=5, save_freq=50, valid_freq=250,
                 max_valid_size=128, extra_loss=lambda mi, got, exp, mask: 0,
                 save_fn=lambda i: None, name_fn=lambda i: f"outputs/train_{i:05}.png",
                 valid_name_fn=lambda i: f"outputs/valid_{i:05}.png", uv_select=None,
                 light_update=no_update, silent=False, really_silent=False, w_isect=False):
    """training_utils.py:123-208 (colocate.py:111): crops of N views per step with the integrator
    as given (colocate passes NeRFIntegrator(Direct)), masked_loss (mask_weight 15), w_isect, a
    NaN loss skips the step, validation renders with NeRFIntegrator(integrator).

    Deviation: the reference builds the training cameras with ``mk_camera(R, T, focal, device)``
    (:161), a name defined nowhere in the reference (the call raises NameError); the cameras here
    are ``OpenGLPerspectiveCameras(R=R, T=T)``, the camera its validation renders (:198) and every
    other (R, T) loop of the file use."""
    from . import pathtrace, pathtrace_sample
    from .cameras import OpenGLPerspectiveCameras
    from .integrators import NeRFIntegrator
    from .utils import LossSampler, masked_loss, rand_uv_mask
    uv_select = uv_select or (lambda mask, cs: rand_uv_mask(mask, cs))
    device = exp_imgs[0].device
    ckpt_freq = (iters // num_ckpts) - 1
    losses = []
    selector = LossSampler(len(exp_imgs))
    iterator = _iterations(iters, silent)
    update = _silent_update(iterator, silent or really_silent, 1000 if really_silent else 1)
    for i in iterator:
        idxs = selector.sample(n=N)
        R = torch.cat([Rs[j] for j in idxs], dim=0)
        T = torch.cat([Ts[j] for j in idxs], dim=0)
        exp = torch.stack([exp_imgs[j] for j in idxs])
        mask = torch.stack([exp_masks[j] for j in idxs])
        cameras = OpenGLPerspectiveCameras(device=device, R=R, T=T)
        light_update(cameras, lights)
        opt.zero_grad()
        (u, v) = uv_select(mask[0], crop_size)
        u, v = int(u), int(v)
        got, mi = pathtrace_sample(shape, size=size, chunk_size=size, bundle_size=1,
                                   crop_size=crop_size, bsdf=bsdf, integrator=integrator,
                                   cameras=cameras, lights=lights, device=device, uv=(u, v),
                                   addition=lambda m: m, squeeze_first=False, silent=True,
                                   w_isect=w_isect)
        if (i % save_freq) == 0:
            save_image(name_fn(i), got[0])
        exp = exp[:, u:u + crop_size, v:v + crop_size]
        mask = mask[:, u:u + crop_size, v:v + crop_size]
        loss = masked_loss(got[..., :3], exp, mi.throughput.squeeze(-1), mask, mask_weight=15,
                           with_logits=mi.with_logits) + extra_loss(mi, got, exp, mask)
        if loss.isnan():
            continue
        loss.backward()
        opt.step()
        loss = loss.detach().item()
        losses.append(loss)
        update(loss, i)
        if ((i % ckpt_freq) == 0) and (i != 0):
            save_fn(i)
        if valid_freq and (i % valid_freq) == 0:
            with torch.no_grad():
                cameras = OpenGLPerspectiveCameras(device=device, R=R[0].unsqueeze(0),
                                                   T=T[0].unsqueeze(0))
                light_update(cameras, lights)
                validate, _ = pathtrace(shape, size=size, chunk_size=min(size, max_valid_size),
                                        bundle_size=1, bsdf=bsdf,
                                        integrator=NeRFIntegrator(integrator), cameras=cameras,
                                        lights=lights, device=device, silent=True,
                                        w_isect=w_isect)
                save_image(valid_name_fn(i), validate)
    return losses


def train_nerv_ptl(shape, bsdf, integrator, cam_to_worlds, light_locs, focal, exp_imgs, exp_masks,
                   opt, size, crop_size, N=3, iters=50_000, num_ckpts=3, save_freq=10_000,
                   valid_freq=250, max_valid_size=128, extra_loss=lambda mi, got, exp, mask: 0,
                   save_fn=lambda i: None, name_fn=lambda i: f"outputs/train_{i:05}.png",
                   valid_name_fn=lambda i: f"outputs/valid_{i:05}.png", uv_select=None,
                   silent=False, w_isect=True):
    """training_utils.py:686-789 (path_nerv.py / nerv.py): NeRFCameras with one point light per
    view (PointLights(scale 100) at light_locs), shadow rays, tone-mapped masked_loss
    (mask_weight 10); a NaN loss raises after its step, as in the reference."""
    from . import pathtrace, pathtrace_sample
    from .cameras import NeRFCamera
    from .integrators import NeRFIntegrator
    from .lights import PointLights
    from .utils import LossSampler, masked_loss, rand_uv_mask
    uv_select = uv_select or (lambda mask, cs: rand_uv_mask(mask, cs))
    train_integrator = NeRFIntegrator(integrator)
    device = exp_imgs[0].device
    ckpt_freq = (iters // num_ckpts) - 1
    losses = []
    selector = LossSampler(len(exp_imgs))
    iterator = _iterations(iters, silent)
    update = _silent_update(iterator, silent, 10)
    for i in iterator:
        idxs = selector.sample(n=N)
        c2w = torch.stack([cam_to_worlds[j] for j in idxs], dim=0)
        exp = torch.stack([exp_imgs[j] for j in idxs])
        mask = torch.stack([exp_masks[j] for j in idxs])
        light_pos = torch.stack([light_locs[j] for j in idxs])
        cameras = NeRFCamera(cam_to_world=c2w, focal=focal, device=device)
        lights = PointLights(intensity=[1, 1, 1], location=light_pos, scale=100, device=device)
        opt.zero_grad()
        (u, v) = uv_select(mask[0], crop_size)
        u, v = int(u), int(v)
        got, mi = pathtrace_sample(shape, size=size, chunk_size=size, bundle_size=1,
                                   crop_size=crop_size, bsdf=bsdf, integrator=train_integrator,
                                   cameras=cameras, lights=lights, device=device, uv=(u, v),
                                   background=0, addition=lambda m: m, squeeze_first=False,
                                   silent=True, w_isect=w_isect)
        if (i % save_freq) == 0:
            save_image(name_fn(i), got[0])
        exp = exp[:, u:u + crop_size, v:v + crop_size]
        mask = mask[:, u:u + crop_size, v:v + crop_size]
        loss = masked_loss(got[..., :3], exp, mi.throughput.squeeze(-1), mask, mask_weight=10,
                           with_logits=mi.with_logits, tone_mapping=True) + \
            extra_loss(mi, got, exp, mask)
        if loss.isnan():
            loss.backward()
            opt.step()
            raise Exception("Unexpected NaN")
        loss.backward()
        opt.step()
        loss = loss.detach().item()
        losses.append(loss)
        selector.update_idxs(idxs, loss)
        update(loss, i)
        if ((i % ckpt_freq) == 0) and (i != 0):
            save_fn(i)
        if valid_freq and (i % valid_freq) == 0:
            with torch.no_grad():
                cameras = NeRFCamera(cam_to_world=c2w[0].unsqueeze(0), focal=focal, device=device)
                lights.location = lights.location[0].unsqueeze(0)
                validate, _ = pathtrace(shape, size=size, chunk_size=min(size, max_valid_size),
                                        bundle_size=1, bsdf=bsdf, integrator=train_integrator,
                                        cameras=cameras, lights=lights, device=device,
                                        silent=True, w_isect=w_isect)
                save_image(valid_name_fn(i), validate ** (1 / 2.2))
    return losses


def train_nerv(*args, **kwargs):
    """training_utils.py:597-683 builds ``NeRVCamera``s, whose sample_positions reads an
    undefined ``r_o`` (cameras.py:130) -- the loop cannot run in the reference either."""
    raise NotImplementedError("train_nerv: the reference's NeRVCamera is broken (cameras.py:130 "
                              "uses an undefined r_o); use train_nerv_ptl (NeRFCamera)")
