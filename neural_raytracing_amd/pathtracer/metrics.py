"""Image metrics used by the reference's evaluation loops, without the third-party packages.

The reference imports ``ssim`` / ``ms_ssim`` from ``pytorch_msssim`` (training_utils.py:18, used at
:342, :483, :532, :840) and ``mse2psnr`` from its utils (utils.py:361).  ``pytorch_msssim`` is not
in this image; ``ssim`` / ``ms_ssim`` below restate its published algorithm (Wang et al. 2003/2004
as implemented there): a separable 11-tap Gaussian window (sigma 1.5) applied as a *valid*
convolution per channel, K = (0.01, 0.03), the mean of the SSIM map per channel, then the mean
over channels and batch when ``size_average``; MS-SSIM uses five scales with weights
(0.0448, 0.2856, 0.3001, 0.2363, 0.1333), 2x2 average pooling (padding odd sides) between scales,
relu of the contrast-structure terms and of the last-scale SSIM.

Evaluation utilities, not the render hot path: plain torch ops on whatever device the images
live on.
"""
import torch
import torch.nn.functional as F

from .utils import mse2psnr  # noqa: F401  (re-exported: utils.py:361)

MS_SSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def gaussian_window(size=11, sigma=1.5, device=None, dtype=torch.float32):
    """1-D Gaussian taps, normalised to sum 1 (centred at size // 2)."""
    coords = torch.arange(size, dtype=dtype, device=device) - size // 2
    g = torch.exp(-(coords ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def _filter(x, win):
    """Separable valid convolution of [N, C, H, W] with the 1-D window along H then W."""
    C = x.shape[1]
    k = win.numel()
    wh = win.reshape(1, 1, k, 1).expand(C, 1, k, 1).to(x.dtype)
    ww = win.reshape(1, 1, 1, k).expand(C, 1, 1, k).to(x.dtype)
    x = F.conv2d(x, wh, groups=C)
    return F.conv2d(x, ww, groups=C)


def _ssim_terms(X, Y, data_range, win, K):
    C1 = (K[0] * data_range) ** 2
    C2 = (K[1] * data_range) ** 2
    mu1, mu2 = _filter(X, win), _filter(Y, win)
    mu1_sq, mu2_sq, mu12 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    s1 = _filter(X * X, win) - mu1_sq
    s2 = _filter(Y * Y, win) - mu2_sq
    s12 = _filter(X * Y, win) - mu12
    cs_map = (2 * s12 + C2) / (s1 + s2 + C2)
    ssim_map = ((2 * mu12 + C1) / (mu1_sq + mu2_sq + C1)) * cs_map
    return ssim_map.flatten(2).mean(-1), cs_map.flatten(2).mean(-1)


def _check(X, Y, win_size):
    if X.shape != Y.shape:
        raise ValueError(f"ssim: shapes differ {tuple(X.shape)} vs {tuple(Y.shape)}")
    if X.dim() != 4:
        raise ValueError("ssim: expects [N, C, H, W] images")
    if win_size % 2 != 1:
        raise ValueError("ssim: window size must be odd")


def ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None,
         K=(0.01, 0.03), nonnegative_ssim=False):
    """SSIM of [N, C, H, W] batches (pytorch_msssim.ssim semantics)."""
    _check(X, Y, win_size if win is None else win.numel())
    X, Y = X.float(), Y.float()
    if win is None:
        win = gaussian_window(win_size, win_sigma, device=X.device)
    per_channel, _ = _ssim_terms(X, Y, data_range, win.reshape(-1), K)
    if nonnegative_ssim:
        per_channel = torch.relu(per_channel)
    return per_channel.mean() if size_average else per_channel.mean(1)


def ms_ssim(X, Y, data_range=255, size_average=True, win_size=11, win_sigma=1.5, win=None,
            weights=None, K=(0.01, 0.03)):
    """Multi-scale SSIM of [N, C, H, W] batches (pytorch_msssim.ms_ssim semantics)."""
    ws = win_size if win is None else win.numel()
    _check(X, Y, ws)
    if min(X.shape[-2:]) <= (ws - 1) * (2 ** 4):
        raise ValueError(f"ms_ssim: image sides must exceed {(ws - 1) * 2 ** 4}")
    X, Y = X.float(), Y.float()
    if win is None:
        win = gaussian_window(win_size, win_sigma, device=X.device)
    win = win.reshape(-1)
    w = torch.tensor(MS_SSIM_WEIGHTS if weights is None else weights, dtype=X.dtype,
                     device=X.device)
    mcs = []
    for i in range(w.numel()):
        per_channel, cs = _ssim_terms(X, Y, data_range, win, K)
        if i < w.numel() - 1:
            mcs.append(torch.relu(cs))
            pad = [s % 2 for s in X.shape[2:]]
            X = F.avg_pool2d(X, kernel_size=2, padding=pad)
            Y = F.avg_pool2d(Y, kernel_size=2, padding=pad)
    per_channel = torch.relu(per_channel)
    stacked = torch.stack(mcs + [per_channel], dim=0)
    val = torch.prod(stacked ** w.reshape(-1, 1, 1), dim=0)
    return val.mean() if size_average else val.mean(1)
