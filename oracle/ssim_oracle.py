"""SSIM oracle -- TEST INFRASTRUCTURE ONLY (the checker of gaussian_splatting_lightning_amd/ssim.py).

Parity unpinned: the fused-ssim submodule (rahul-goel/fused-ssim, imported at gs_lightning_module.py:10) is
empty in the reference snapshot and the reference holds no SSIM test or fixture, so this restates the
published SSIM (Wang et al. 2004) as the fused-ssim / original 3DGS loss computes it: 11x11 Gaussian window
with sigma 1.5 (normalised), C1 = 0.01^2, C2 = 0.03^2, per-channel zero-padded "same" filtering, mean of the
map ("valid": map cropped by 5 px).  float64 numpy; the gradient w.r.t. img1 is derived analytically.
"""
from __future__ import annotations

import numpy as np

C1, C2, R = 0.01 ** 2, 0.03 ** 2, 5


def window() -> np.ndarray:
    d = np.arange(11) - R
    g = np.exp(-d * d / (2 * 1.5 ** 2))
    return g / g.sum()


def _filt(img: np.ndarray) -> np.ndarray:
    """Separable zero-padded 'same' filtering of (..., H, W)."""
    w = window()
    H, W = img.shape[-2:]
    p = np.zeros(img.shape[:-2] + (H + 2 * R, W + 2 * R))
    p[..., R:R + H, R:R + W] = img
    h = sum(w[k] * p[..., :, k:k + W] for k in range(11))
    return sum(w[k] * h[..., k:k + H, :] for k in range(11))


def ssim(img1, img2, padding="same"):
    """Returns (mean SSIM, dmean/dimg1) for (B,C,H,W) arrays."""
    x = np.asarray(img1, np.float64)
    y = np.asarray(img2, np.float64)
    mu1, mu2 = _filt(x), _filt(y)
    s11, s22, s12 = _filt(x * x) - mu1 ** 2, _filt(y * y) - mu2 ** 2, _filt(x * y) - mu1 * mu2
    A, B = 2 * mu1 * mu2 + C1, 2 * s12 + C2
    Cc, D = mu1 ** 2 + mu2 ** 2 + C1, s11 + s22 + C2
    m = A * B / (Cc * D)
    mask = np.ones(x.shape[-2:], bool)
    if padding == "valid":
        mask[:] = False
        mask[R:-R, R:-R] = True
    n = m.shape[0] * m.shape[1] * mask.sum()
    mean = float((m * mask).sum() / n)
    g = mask / n
    d12 = 2 * A / (Cc * D)
    d11 = -m / D
    dmu = 2 * mu2 * B / (Cc * D) - 2 * mu1 * m / Cc - 2 * mu1 * d11 - mu2 * d12
    grad = _filt(g * dmu) + 2 * x * _filt(g * d11) + y * _filt(g * d12)
    return mean, grad
