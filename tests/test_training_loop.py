"""End-to-end training slice on the GPU: everything a gs_lightning training step calls, on this package.

COLMAP-style points3D.ply -> GaussianModel.initialize (GPU PLY read + exact 3-NN scale init) -> per step:
rasterize (HIP fwd/bwd) + L1/fused-SSIM loss (gs_lightning_module.py:100, :279) -> densification statistics
(update_max_radii2D / update_xyz_gradient) -> GaussianAdam.step -> densify_and_prune with optimizer-state
re-indexing -> save_ply / load_ply.  Checks the initialisation against the oracles exactly and the loop for
a falling loss, finite parameters and a consistent optimizer after densification.
"""
import numpy as np
import pytest
import torch

from oracle import knn_oracle, ply_oracle


def _colmap_points(path, n, seed=0):
    from gaussian_splatting_lightning_amd.synthetic import make_scene
    sc = make_scene(n, sh_degree=0, seed=seed)
    rng = np.random.default_rng(seed)
    arr = np.empty(n, dtype=[("x", "f4"), ("y", "f4"), ("z", "f4"), ("nx", "f4"), ("ny", "f4"), ("nz", "f4"),
                             ("red", "u1"), ("green", "u1"), ("blue", "u1")])
    xyz = sc.means3D.numpy() + rng.normal(size=(n, 3)).astype(np.float32) * 0.02
    for j, k in enumerate("xyz"):
        arr[k] = xyz[:, j]
    for k in ("nx", "ny", "nz"):
        arr[k] = 0
    rgb = rng.integers(0, 256, (n, 3))
    for j, k in enumerate(("red", "green", "blue")):
        arr[k] = rgb[:, j]
    ply_oracle.write_vertex_ply(path, arr)
    return xyz, rgb


@pytest.mark.gpu
def test_initialize_matches_reference_formulae(tmp_path):
    from gaussian_splatting_lightning_amd.gaussian_model import GaussianModel, C0
    p = str(tmp_path / "points3D.ply")
    xyz, rgb = _colmap_points(p, 2000)
    g = GaussianModel(sh_degree=3, colmap_ply=p, spatial_scale=1.0)
    np.testing.assert_array_equal(g._xyz.detach().cpu().numpy(), xyz)
    color = torch.tensor(rgb / 255.).float()                                   # gaussian_model.py:69
    np.testing.assert_allclose(g._features_dc.detach().cpu().numpy()[:, 0], ((color - 0.5) / C0).numpy(), rtol=1e-6)
    assert g._features_rest.shape == (2000, 15, 3) and float(g._features_rest.detach().abs().max()) == 0.0
    d = np.maximum(knn_oracle.mean_dist2(xyz), np.float32(1e-7))
    want = np.log(np.sqrt(d))                                                  # gaussian_model.py:90-91
    np.testing.assert_allclose(g._scaling.detach().cpu().numpy(), np.repeat(want[:, None], 3, 1), rtol=2e-6,
                               atol=1e-6)
    np.testing.assert_allclose(torch.sigmoid(g._opacity).detach().cpu().numpy(), 0.1, rtol=1e-6)
    assert (g._rotation.detach().cpu().numpy() == np.array([1, 0, 0, 0], np.float32)).all()


@pytest.mark.gpu
def test_training_loop_with_densification(tmp_path):
    from gaussian_splatting_lightning_amd.gaussian_model import GaussianModel
    from gaussian_splatting_lightning_amd.optim import GaussianAdam
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, rasterize_gaussians
    from gaussian_splatting_lightning_amd.ssim import fused_ssim
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene

    dev = torch.device("cuda")
    W, H = 160, 120
    cam = make_camera(W, H).to(dev)
    bg = torch.zeros(3, device=dev)
    settings = lambda D: GaussianRasterizationSettings(  # noqa: E731
        image_height=H, image_width=W, tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, bg=bg, scale_modifier=1.0,
        viewmatrix=cam.viewmatrix, projmatrix=cam.projmatrix, sh_degree=D, campos=cam.campos, prefiltered=False,
        debug=False, antialiasing=False)
    gt = make_scene(3000, sh_degree=0, seed=1).to(dev)
    with torch.no_grad():
        target, _, _ = rasterize_gaussians(gt.means3D, torch.zeros_like(gt.means3D), gt.shs, None, gt.opacities,
                                           gt.scales, gt.rotations, None, settings(0))
    p = str(tmp_path / "points3D.ply")
    _colmap_points(p, 1500, seed=2)
    g = GaussianModel(sh_degree=3, colmap_ply=p, spatial_scale=1.0)
    lrs = dict(xyz=1.6e-4, features_dc=2.5e-3, features_rest=1.25e-4, opacity=0.05, scaling=5e-3, rotation=1e-3)
    opt = GaussianAdam([{"params": [getattr(g, f"_{k}")], "lr": lrs[k], "name": k} for k in g.PARAMETER_NAMES],
                       lr=0.0, eps=1e-15)
    losses = []
    n0 = len(g._xyz)
    for step in range(1, 61):
        means2D = torch.zeros_like(g._xyz, requires_grad=True)
        img, radii, _ = rasterize_gaussians(g._xyz, means2D, g.get_features(), None, g.get_opacity(),
                                            g.get_scaling(), g.get_rotation(), None, settings(g.active_sh_degree))
        l1 = (img - target).abs().mean()
        loss = 0.8 * l1 + 0.2 * (1 - fused_ssim(img.unsqueeze(0), target.unsqueeze(0)))
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(float(loss))
        vis = radii > 0
        g.update_max_radii2D(radii.float(), vis)
        g.update_xyz_gradient(means2D.grad, vis)
        if step == 30:
            keep = g.densify_and_prune(0.00002, 0.01, 0.005, 0.5, None, optimizer=opt)
            assert keep.numel() <= n0
            g.reset_max_radii2D()
            g.reset_xyz_gradient()
            for grp in opt.param_groups:
                prm = grp["params"][0]
                assert prm is getattr(g, f"_{grp['name']}")
                assert opt.state[prm]["exp_avg"].shape == prm.shape
        if step % 20 == 0:
            g.step_sh_degree()
    assert len(g._xyz) != n0, "densification changed nothing"
    assert all(np.isfinite(losses))
    assert np.mean(losses[-5:]) < 0.8 * np.mean(losses[:5]), losses
    for k in g.PARAMETER_NAMES:
        assert torch.isfinite(getattr(g, f"_{k}")).all()
    # checkpoint round trip
    out = str(tmp_path / "point_cloud.ply")
    g.save_ply(out)
    h = GaussianModel(sh_degree=3)
    h.load_ply(out)
    for k in g.PARAMETER_NAMES:
        torch.testing.assert_close(getattr(h, f"_{k}"), getattr(g, f"_{k}"), rtol=0, atol=0)
