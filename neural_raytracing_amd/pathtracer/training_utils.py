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
"""
import json
import os

import numpy as np
import torch
import torch.nn.functional as F

from .utils import load_image


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
