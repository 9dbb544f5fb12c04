"""Host-side loaders and metrics of the reference's drivers, CPU only.

Parity anchors: the reference holds no dataset files, so the loaders are checked on synthetic
files built here with known answers (a projection assembled from chosen K, R, centre; a
transforms json with chosen matrices), and SSIM / MS-SSIM against a direct-summation restatement
of the pytorch_msssim algorithm (explicit window sums, no convolution).
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from neural_raytracing_amd.pathtracer import metrics, training_utils


def _rot(ax, ay, az):
    cx, sx, cy, sy, cz, sz = (math.cos(ax), math.sin(ax), math.cos(ay), math.sin(ay),
                              math.cos(az), math.sin(az))
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _projection(K, R, C, scale):
    return scale * (K @ np.concatenate([R, -R @ C.reshape(3, 1)], axis=1))


@pytest.mark.parametrize("scale", [1.0, -2.5, 1e-3])
def test_decompose_projection_matrix_kat(scale):
    K = np.array([[2890.0, 1.5, 800.0], [0.0, 2880.0, 600.0], [0.0, 0.0, 1.0]])
    R = _rot(0.3, -1.1, 2.0)
    C = np.array([0.4, -1.2, 2.5])
    P = _projection(K, R, C, scale)
    Kd, Rd, t = training_utils.decompose_projection_matrix(P)
    assert Kd[0, 0] > 0 and Kd[1, 1] > 0
    assert np.allclose(np.tril(Kd, -1), 0, atol=1e-9)
    assert np.allclose(Rd @ Rd.T, np.eye(3), atol=1e-12) and np.linalg.det(Rd) > 0
    assert np.allclose(Kd @ Rd, P[:, :3], rtol=1e-10, atol=1e-12 * abs(scale))
    if scale > 0:
        assert np.allclose(Kd / Kd[2, 2], K, rtol=1e-9, atol=1e-7)
        assert np.allclose(Rd, R, atol=1e-10)
    else:  # -K R = (K diag(1,1,-1)) (diag(-1,-1,1) R): the sign convention picks K00, K11 > 0
        assert np.allclose(Rd, np.diag([-1.0, -1.0, 1.0]) @ R, atol=1e-10)
    assert np.allclose(P @ t, 0, atol=1e-9 * max(1.0, abs(scale)))
    assert np.allclose(t[:3, 0] / t[3, 0], C, atol=1e-9)


def test_krt_from_p_pose():
    K = np.array([[1000.0, 0.0, 320.0], [0.0, 1000.0, 240.0], [0.0, 0.0, 1.0]])
    R = _rot(-0.2, 0.5, 0.1)
    C = np.array([0.1, 0.2, -3.0])
    intr, pose = training_utils.KRt_from_P(_projection(K, R, C, 7.0), device="cpu")
    assert intr.shape == (4, 4) and pose.shape == (4, 4)
    assert torch.allclose(intr[:3, :3], torch.tensor(K, dtype=torch.float), rtol=1e-6)
    assert torch.allclose(pose[:3, :3], torch.tensor(R.T, dtype=torch.float), atol=1e-6)
    assert torch.allclose(pose[:3, 3], torch.tensor(C, dtype=torch.float), atol=1e-5)


def test_load_dtu_cameras_normalises_distance(tmp_path):
    K = np.array([[2890.0, 0.0, 800.0], [0.0, 2890.0, 600.0], [0.0, 0.0, 1.0]])
    cams, centres = {}, []
    for i in range(3):
        R = _rot(0.1 * i, 0.7 - 0.3 * i, 0.2)
        C = np.array([1.0 + i, -0.5, 2.0 * i])
        centres.append(C)
        cams[f"world_mat_{i}"] = np.concatenate([_projection(K, R, C, 1.0), [[0, 0, 0, 1]]])
        cams[f"scale_mat_{i}"] = np.eye(4)
    np.savez(tmp_path / "cameras.npz", **cams)
    intr, poses = training_utils.load_dtu_cameras(str(tmp_path / "cameras.npz"), 3, device="cpu")
    dmax = max(np.linalg.norm(c) for c in centres)
    for i, C in enumerate(centres):
        assert torch.allclose(poses[i, :3, 3], torch.tensor(C / dmax, dtype=torch.float),
                              atol=1e-5)
    assert torch.linalg.norm(poses[:, :3, 3], dim=-1).max().item() == pytest.approx(1.0)
    assert torch.allclose(intr[0, :3, :3], torch.tensor(K, dtype=torch.float), rtol=1e-6)


def test_nerf_transforms_loader(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    frames = []
    for i in range(2):
        rgba = rng.integers(0, 256, size=(40, 40, 4), dtype=np.uint8)
        rgba[:10, :, 3] = 0
        Image.fromarray(rgba, "RGBA").save(tmp_path / f"r_{i}.png")
        tf = np.eye(4)
        tf[:3, 3] = [0.0, 3.0 * (i + 1), 4.0 * (i + 1)]
        frames.append({"file_path": f"./r_{i}", "transform_matrix": tf.tolist()})
    with open(tmp_path / "transforms_test.json", "w") as fh:
        json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, fh)
    c2ws, focal, imgs, masks = training_utils.test_nerf_resources(str(tmp_path) + os.sep, size=20,
                                                                  kind="test", device="cpu")
    assert focal == pytest.approx(0.5 * 20 / math.tan(0.5 * 0.6911112070083618))
    assert len(c2ws) == len(imgs) == len(masks) == 2
    assert imgs[0].shape == (20, 20, 3) and masks[0].shape == (20, 20)
    assert torch.allclose(c2ws[1][:3, 3], torch.tensor([0.0, 0.6, 0.8]), atol=1e-6)
    assert set(masks[0].unique().tolist()) <= {0.0, 1.0}
    assert masks[0][:3].sum() == 0  # alpha-0 rows stay masked out (bicubic resize blurs row 4)


def _naive_ssim(X, Y, data_range, K=(0.01, 0.03), win=11, sigma=1.5):
    """Direct-summation SSIM per [N, C] (valid windows), float64 numpy."""
    coords = np.arange(win) - win // 2
    g = np.exp(-(coords ** 2) / (2 * sigma ** 2))
    g /= g.sum()
    w2 = np.outer(g, g)
    C1, C2 = (K[0] * data_range) ** 2, (K[1] * data_range) ** 2
    N, Ch, H, W = X.shape
    out = np.zeros((N, Ch))
    cs_out = np.zeros((N, Ch))
    for n in range(N):
        for c in range(Ch):
            vals, css = [], []
            for i in range(H - win + 1):
                for j in range(W - win + 1):
                    x = X[n, c, i:i + win, j:j + win]
                    y = Y[n, c, i:i + win, j:j + win]
                    mx, my = (w2 * x).sum(), (w2 * y).sum()
                    sx = (w2 * x * x).sum() - mx * mx
                    sy = (w2 * y * y).sum() - my * my
                    sxy = (w2 * x * y).sum() - mx * my
                    cs = (2 * sxy + C2) / (sx + sy + C2)
                    vals.append((2 * mx * my + C1) / (mx * mx + my * my + C1) * cs)
                    css.append(cs)
            out[n, c] = np.mean(vals)
            cs_out[n, c] = np.mean(css)
    return out, cs_out


def test_ssim_matches_direct_summation():
    g = torch.Generator().manual_seed(1)
    X = torch.rand(2, 3, 24, 19, generator=g)
    Y = (X + 0.1 * torch.randn(2, 3, 24, 19, generator=g)).clamp(0, 1)
    want, _ = _naive_ssim(X.double().numpy(), Y.double().numpy(), 1.0)
    got = metrics.ssim(X, Y, data_range=1, size_average=False)
    assert np.allclose(got.numpy(), want.mean(1), atol=1e-5)
    assert metrics.ssim(X, Y, data_range=1).item() == pytest.approx(want.mean(), abs=1e-5)
    assert metrics.ssim(X, X, data_range=1).item() == pytest.approx(1.0, abs=1e-6)


def _pool(x):
    """avg_pool2d(kernel 2, padding = side % 2, count_include_pad) in numpy."""
    N, C, H, W = x.shape
    ph, pw = H % 2, W % 2
    xp = np.zeros((N, C, H + 2 * ph, W + 2 * pw))
    xp[:, :, ph:ph + H, pw:pw + W] = x
    Ho, Wo = (H + 2 * ph) // 2, (W + 2 * pw) // 2
    return xp[:, :, :2 * Ho, :2 * Wo].reshape(N, C, Ho, 2, Wo, 2).mean(axis=(3, 5))


def test_ms_ssim_matches_direct_summation():
    g = torch.Generator().manual_seed(2)
    X = torch.rand(1, 1, 163, 170, generator=g)
    Y = (X + 0.05 * torch.randn(1, 1, 163, 170, generator=g)).clamp(0, 1)
    x, y = X.double().numpy(), Y.double().numpy()
    mcs = []
    for lvl in range(5):
        s, cs = _naive_ssim(x, y, 1.0)
        if lvl < 4:
            mcs.append(np.maximum(cs, 0))
            x, y = _pool(x), _pool(y)
    vals = np.stack(mcs + [np.maximum(s, 0)])
    w = np.array(metrics.MS_SSIM_WEIGHTS).reshape(-1, 1, 1)
    want = np.prod(vals ** w, axis=0).mean()
    got = metrics.ms_ssim(X, Y, data_range=1).item()
    assert got == pytest.approx(want, abs=1e-5)
    with pytest.raises(ValueError):
        metrics.ms_ssim(X[..., :100, :100], Y[..., :100, :100], data_range=1)


def test_mse2psnr():
    assert metrics.mse2psnr(torch.tensor(0.01)).item() == pytest.approx(20.0)
