"""Fused SSIM (§8(f) next #1): the HIP kernels against the float64 oracle/ssim_oracle.py, and the oracle's
analytic gradient against finite differences.  Parity unpinned (no reference SSIM fixture, see the oracle)."""
import numpy as np
import pytest
import torch

from oracle import ssim_oracle as SO


def _images(B, C, H, W, seed):
    rng = np.random.default_rng(seed)
    gt = rng.random((B, C, H, W))
    render = np.clip(gt + 0.15 * rng.standard_normal((B, C, H, W)), 0, 1)
    return render.astype(np.float32), gt.astype(np.float32)


@pytest.mark.parametrize("padding", ["same", "valid"])
def test_oracle_gradient_finite_differences(padding):
    x, y = _images(1, 2, 19, 23, 0)
    x = x.astype(np.float64)
    _, g = SO.ssim(x, y, padding)
    rng = np.random.default_rng(1)
    for _ in range(6):
        idx = tuple(rng.integers(0, s) for s in x.shape)
        e = np.zeros_like(x)
        e[idx] = 1e-6
        fd = (SO.ssim(x + e, y, padding)[0] - SO.ssim(x - e, y, padding)[0]) / 2e-6
        assert abs(fd - g[idx]) <= 1e-6 * max(1.0, abs(g[idx])) + 1e-9


def test_identical_images_have_ssim_one():
    x, _ = _images(1, 3, 16, 16, 2)
    m, g = SO.ssim(x, x)
    assert abs(m - 1.0) < 1e-12 and np.abs(g).max() < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("shape,padding", [((1, 3, 100, 150), "same"), ((2, 3, 67, 45), "valid"),
                                           ((1, 1, 11, 11), "same"), ((1, 3, 1080, 1920), "same")])
def test_fused_ssim_matches_oracle(gpu_device, shape, padding):
    from fused_ssim import fused_ssim
    x, y = _images(*shape, seed=3)
    ref_m, ref_g = SO.ssim(x, y, padding)
    xt = torch.tensor(x, device=gpu_device, requires_grad=True)
    m = fused_ssim(xt, torch.tensor(y, device=gpu_device), padding=padding)
    (1 - m).backward()
    assert abs(float(m) - ref_m) <= 2e-6
    got = -xt.grad.cpu().numpy()
    err = np.abs(got - ref_g).max() / np.abs(ref_g).max()
    assert err <= 1e-4, err


@pytest.mark.gpu
def test_fused_ssim_eval_mode_and_3d_input(gpu_device):
    from fused_ssim import fused_ssim
    x, y = _images(1, 3, 40, 52, 4)
    a = fused_ssim(torch.tensor(x[0], device=gpu_device), torch.tensor(y[0], device=gpu_device), train=False)
    assert abs(float(a) - SO.ssim(x, y)[0]) <= 2e-6


@pytest.mark.gpu
@pytest.mark.parametrize("shape,padding", [((1, 3, 100, 150), "same"), ((2, 3, 67, 45), "valid"),
                                           ((1, 1, 11, 11), "same"), ((1, 3, 1080, 1920), "same")])
def test_streaming_ssim_matches_tiled_kernels(gpu_device, shape, padding):
    """The streaming forward (one wave per 64-column x 32-row strip, rows walked once) forms every filter sum in the
    tiled kernel's order: the derivative maps, hence the gradient, are bitwise the tiled ones and the mean equal up
    to the grouping of its partial sums."""
    from fused_ssim import fused_ssim
    from gaussian_splatting_lightning_amd import _native
    x, y = _images(*shape, seed=5)
    out = {}
    try:
        for mode in (0, 1):  # tiled forward, streaming forward (the default)
            _native.set_tuning("ssim_stream", mode)
            xt = torch.tensor(x, device=gpu_device, requires_grad=True)
            m = fused_ssim(xt, torch.tensor(y, device=gpu_device), padding=padding)
            (1 - m).backward()
            out[mode] = (float(m), xt.grad.cpu().numpy())
    finally:
        _native.unset_tuning("ssim_stream")
    assert abs(out[0][0] - out[1][0]) <= 1e-6 * max(1.0, abs(out[0][0]))
    assert np.array_equal(out[0][1], out[1][1])
