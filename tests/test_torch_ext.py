"""The thin torch extension `diff_gaussian_rasterization._C` (csrc_torch/gsr_torch_ext.cpp): the upstream pybind
entry points (rasterize_gaussians / rasterize_gaussians_backward / mark_visible) over the same C ABI
as the Python path.  CPU: the module loads and exports them.  GPU: every output is bitwise the Python path's."""
import os

import numpy as np
import pytest
import torch

from tests.helpers import scene_inputs, upstream

EXT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "diff_gaussian_rasterization", "_C.so")


def test_extension_exports_upstream_entry_points():
    # build() fails when the extension does not build (unless GSR_ALLOW_NO_TORCH_EXT=1), so a missing _C.so is an
    # error here, not a skip: the upstream pybind entry points must not regress silently
    if not os.path.exists(EXT):
        if os.environ.get("GSR_ALLOW_NO_TORCH_EXT") == "1":
            pytest.skip("diff_gaussian_rasterization/_C.so not built (GSR_ALLOW_NO_TORCH_EXT=1)")
        pytest.fail("diff_gaussian_rasterization/_C.so missing: run __graft_entry__.build()")
    from diff_gaussian_rasterization import _C
    for name in ("rasterize_gaussians", "rasterize_gaussians_backward", "mark_visible", "adamUpdate"):
        assert callable(getattr(_C, name)), name


@pytest.mark.gpu
@pytest.mark.parametrize("stress", [0.0, 0.02])
def test_extension_matches_python_path_bitwise(gpu_device, stress):
    from diff_gaussian_rasterization import _C
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    from tests.helpers import settings_for
    n, W, H = 20_000, 320, 240
    inp = scene_inputs(n, W, H, sh_degree=3, seed=44, stress_fraction=stress, bg=(0.2, 0.4, 0.6))
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    dc, di = (torch.as_tensor(a, device=gpu_device) for a in upstream(W, H, seed=44))
    empty = torch.empty(0, device=gpu_device)
    num, color, radii, geom, binning, img, invd = _C.rasterize_gaussians(
        rs.bg, t["means3D"], empty, t["opacities"], t["scales"], t["rotations"], rs.scale_modifier, empty,
        rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, H, W, t["shs"], rs.sh_degree, rs.campos, False, False,
        False)
    grads = _C.rasterize_gaussians_backward(
        rs.bg, t["means3D"], radii, empty, t["opacities"], t["scales"], t["rotations"], rs.scale_modifier, empty,
        rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, dc, di, t["shs"], rs.sh_degree, rs.campos, geom, num,
        binning, img, False, False)
    c2, r2, i2, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    g2 = backward_raw(st, rs, dc, di)
    torch.cuda.synchronize()
    if stress:
        assert st.num_big > 0  # the extension's backward reads the big-Gaussian count on the device
    assert num == st.num_rendered
    for a, b in ((color, c2), (radii, r2), (invd, i2)):
        assert torch.equal(a, b)
    dmeans2D, dcolors, dopac, dmeans3D, dcov, dsh, dscales, drot = grads
    for a, k in ((dmeans2D, "means2D"), (dopac, "opacities"), (dmeans3D, "means3D"), (dsh, "shs"),
                 (dscales, "scales"), (drot, "rotations")):
        assert torch.equal(a, g2[k].reshape(a.shape)), k
    vis = _C.mark_visible(t["means3D"], rs.viewmatrix, rs.projmatrix)
    from gaussian_splatting_lightning_amd.rasterizer import mark_visible
    assert torch.equal(vis, mark_visible(t["means3D"], rs.viewmatrix, rs.projmatrix))
    assert np.any(vis.cpu().numpy())


@pytest.mark.gpu
def test_extension_adam_update_is_the_sparse_adam_step(gpu_device):
    """_C.adamUpdate (upstream adam.h, called by SparseGaussianAdam.step) writes bit for bit what the Python
    SparseGaussianAdam writes for the same group: both launch gsr_sparse_adam_step."""
    from diff_gaussian_rasterization import SparseGaussianAdam, _C
    N, M = 5003, 3
    gen = torch.Generator(device=gpu_device).manual_seed(3)
    p0 = torch.randn(N, M, device=gpu_device, generator=gen)
    g = torch.randn(N, M, device=gpu_device, generator=gen)
    vis = torch.rand(N, device=gpu_device, generator=gen) < 0.5
    a = torch.nn.Parameter(p0.clone())
    a.grad = g.clone()
    opt = SparseGaussianAdam([a], lr=0.01, eps=1e-15)
    opt.step(vis, N)
    opt.step(vis, N)
    b, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for _ in range(2):
        _C.adamUpdate(b, g, m, v, vis, 0.01, 0.9, 0.999, 1e-15, N, M)
    torch.cuda.synchronize()
    assert torch.equal(a.detach(), b)
    assert torch.equal(opt.state[a]["exp_avg"], m) and torch.equal(opt.state[a]["exp_avg_sq"], v)
