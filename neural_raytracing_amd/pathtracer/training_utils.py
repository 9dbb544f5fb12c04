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
