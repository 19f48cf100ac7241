"""Parity of the HIP path (through the C ABI) against the CPU oracle and the reference's golden vectors.

Bars (DESIGN.md "Parity"), against the oracle's OWN forward on the same inputs:
  * integer state is bit-exact: radii, num_rendered, tiles touched, the sorted instance list
    (tile, depth, index order), the per-tile ranges -- and the per-Gaussian render records (pixel centre, conic,
    opacity, depth bits), since the device evaluates that geometry chain uncontracted like the oracle;
  * n_contrib (last contributor per pixel) is exact on every pixel except the oracle's threshold-flip candidates
    (a decision alpha = 1/255, T = 1e-4 or power = 0 within the fp32 evaluation error, oracle.threshold_margin);
  * colour / inverse depth: |err| <= 1e-5 outside the candidates and <= 2e-2 everywhere (a flip);
  * gradients: relative L2 <= 1e-4 over the Gaussians no candidate pixel touches, and the per-case bar over all;
  * the backward is deterministic: two runs give bitwise identical gradients.
Achieved errors are recorded per case (tests/parity.py; GSR_PARITY_JSON=path writes them).
"""
import os

import numpy as np
import pytest
import torch

from tests import parity

from tests.helpers import (close_fraction, golden_inputs, hip_state_arrays, load_golden, rel_l2, run_hip,
                           run_oracle, scene_inputs, settings_for, upstream)

pytestmark = pytest.mark.gpu

GRADS = ("means3D", "means2D", "opacities", "scales", "rotations", "shs")


# Bars are about 2x the achieved errors recorded in profiles/parity_r3.json (every case of this file, round 3):
FLIP_MARGIN = 1.0    # oracle threshold margin below which a pixel is a threshold-flip candidate (oracle.threshold_margin)
COLOR_TOL = 3e-6     # |colour|, |inverse depth| (relative to max(1, |v|)) on every other pixel; achieved <= 1.31e-6
                     # (SURVEY Appendix A13 asks ~1e-5)
FLIP_TOL = 2e-2      # anywhere (one alpha = 1/255 or T = 1e-4 flip moves a pixel by < alpha T); achieved <= 3.4e-3
GRAD_CLEAN_TOL = 5e-6  # gradient rel-L2 over the Gaussians no flip candidate touches; achieved <= 2.99e-6 (the
                       # long-tile stress cases, walked in 64-instance segments; <= 1.95e-6 elsewhere)
                       # (A13 asks ~1e-4)
GRAD_TOL_ADHOC = 2e-6  # cases checked without flip separation (precomputed inputs, the autograd API); achieved 6.2e-7


def _case():
    return os.environ.get("PYTEST_CURRENT_TEST", "unknown").rsplit("::", 1)[-1].split(" ")[0]


def compare_forward(inp, hip, oracle_out):
    """HIP forward against the oracle's own forward on the same inputs.  Integer state and the per-Gaussian render
    records are bit-exact; pixels are exact in contributor count and within COLOR_TOL in value everywhere except the
    oracle's threshold-flip candidates, which stay within FLIP_TOL.  Achieved errors go to the parity record."""
    color, radii, invd, run = oracle_out
    W, H = inp["image_width"], inp["image_height"]
    hs = hip_state_arrays(hip)
    g = run.geom()
    # integer outputs: bit-exact against the oracle's own preprocess (radii, kept tiles) and binning
    assert np.array_equal(hip["radii"], radii)
    assert hs["num_rendered"] == run.num_rendered
    assert np.array_equal(hs["tiles"], g["tiles_touched"])
    pl, rg = run.point_list(), run.ranges()
    assert np.array_equal(hs["ranges"], rg)
    check_point_list(hs, pl, rg)
    # the render records the compositor reads: the same bits for every rendered Gaussian
    on = radii > 0
    for k in ("xy", "conic_opacity"):
        assert np.array_equal(hs[k][on].view(np.uint32), g[k][on].view(np.uint32)), k
    kept = g["tiles_touched"] > 0
    assert np.array_equal(hs["depths"][kept].view(np.uint32), g["depths"][kept].view(np.uint32))
    # The forward gathers every instance any pixel can reach; for exactly those it writes the sorted id list and the
    # inverse permutation (the backward's row markers), and per tile the key (depth bits << 32 | expansion index) of
    # the last one
    loaded = np.zeros(len(pl), bool)
    for t in np.nonzero(hs["tile_loaded"])[0]:
        loaded[rg[t, 0]: rg[t, 0] + hs["tile_loaded"][t]] = True
    assert np.all(hs["tile_loaded"] >= hs["tile_last"])
    assert np.array_equal(hs["point_list_written"][loaded], pl[loaded])
    su = hs["sorted_u"][loaded].astype(np.int64)
    assert np.array_equal(hs["inv"][su], np.nonzero(loaded)[0].astype(np.uint32))
    # pixels
    _, nc = run.image_state()
    flip = run.threshold_margin() < FLIP_MARGIN
    ok = ~flip
    nc_bad = hs["n_contrib"] != nc
    cerr = np.abs(hip["color"] - color)
    ierr = np.abs(hip["invdepth"] - invd)[0]
    ierr_rel = ierr / np.maximum(np.abs(invd[0]), 1.0)
    rec = dict(W=W, H=H, P=int(len(radii)), num_rendered=int(run.num_rendered), flip_candidates=int(flip.sum()),
               n_contrib_mismatch=int(nc_bad.sum()), n_contrib_mismatch_outside_candidates=int((nc_bad & ok).sum()),
               color_maxabs_clean=float(cerr[:, ok].max(initial=0)), color_maxabs_all=float(cerr.max(initial=0)),
               color_rel_l2=rel_l2(hip["color"], color),
               invdepth_maxrel_clean=float(ierr_rel[ok].max(initial=0)),
               invdepth_maxrel_all=float(ierr_rel.max(initial=0)), invdepth_rel_l2=rel_l2(hip["invdepth"], invd))
    parity.record(_case(), "forward", rec)
    assert rec["n_contrib_mismatch_outside_candidates"] == 0, rec
    assert rec["color_maxabs_clean"] <= COLOR_TOL, rec
    assert rec["invdepth_maxrel_clean"] <= COLOR_TOL, rec
    assert rec["color_maxabs_all"] <= FLIP_TOL, rec
    # Gaussians whose gradient a flip candidate can move: those the pixel's walk reaches on either side
    gx = (W + 15) // 16
    touched = np.zeros(len(radii), bool)
    ys, xs = np.nonzero(flip)
    if len(ys):
        t = (ys // 16) * gx + xs // 16
        n = np.maximum(hs["n_contrib"][ys, xs], nc[ys, xs]).astype(np.int64)
        for tt in np.unique(t):
            m = int(n[t == tt].max())
            touched[pl[rg[tt, 0]: rg[tt, 0] + m]] = True
    run.flip_touched = touched
    run.flip_mask = flip
    return run


def check_point_list(hs, pl, rg):
    """The sorted instance list against the reference order, bit-exact."""
    assert np.array_equal(hs["point_list"], pl)


FLIP_PROPAGATION = 2.0  # a flipped pixel's gradient contribution moves by at most its size before plus after the
                        # flip (the two within 1 / (1 - 1/255) of each other); independent flips add in quadrature,
                        # which the norm of the flip pixels' summed contribution (one backward) measures.  A loose
                        # bound (the flipped pair's alpha is ~1/255, so most of a pixel's terms barely move): the
                        # achieved / bar ratios are in the parity record


def compare_backward(hip, run, dc, di):
    """Gradients against the oracle's backward.  Over the Gaussians no threshold-flip candidate pixel touches (their
    gradients see the same decisions): relative L2 <= GRAD_CLEAN_TOL.  Over all Gaussians the bar is DERIVED from the
    flip census, not fitted: GRAD_CLEAN_TOL + FLIP_PROPAGATION x |g_flip| / |g|, with g_flip the oracle's gradient of
    the candidate pixels alone (its backward with the upstream gradient masked to them) -- what the flips can move."""
    g = run.backward(dc, di)
    touched = getattr(run, "flip_touched", None)
    flip = getattr(run, "flip_mask", None)
    gf = None
    if flip is not None and flip.any():
        m = flip.astype(np.float32)
        gf = run.backward(np.asarray(dc) * m[None], None if di is None else np.asarray(di) * m[None])
    rec = {"touched_gaussians": int(touched.sum()) if touched is not None else None,
           "flip_pixels": int(flip.sum()) if flip is not None else None}
    for k in GRADS:
        if hip["grads"].get(k) is None:
            continue
        a, b = hip["grads"][k], g[k]
        e = {"rel_l2": rel_l2(a, b)}
        nb = float(np.linalg.norm(np.asarray(b, np.float64)))
        e["bar"] = GRAD_CLEAN_TOL + (FLIP_PROPAGATION * float(np.linalg.norm(np.asarray(gf[k], np.float64))) /
                                     max(nb, 1e-30) if gf is not None else 0.0)
        if touched is not None:
            clean = ~touched
            e["rel_l2_clean"] = rel_l2(a[clean], b[clean])
            e["maxabs_clean_over_maxref"] = float(np.abs(a[clean] - b[clean]).max(initial=0) /
                                                  max(np.abs(b).max(initial=0), 1e-30))
        rec[k] = e
    parity.record(_case(), "backward", rec)
    for k in GRADS:
        if k in rec:
            assert rec[k]["rel_l2"] <= rec[k]["bar"], (k, rec[k])
            if "rel_l2_clean" in rec[k]:
                assert rec[k]["rel_l2_clean"] <= GRAD_CLEAN_TOL, (k, rec[k])
    return g


def test_mark_visible_treehill(gpu_device):
    """Port of the reference's only hot-path test, tests/rasterizer_python/test_mark_visible.py:11-21."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    z = load_golden("markvisible_treehill")
    pts = torch.as_tensor(z["points"], device=gpu_device)
    for cam in range(3):
        s = GaussianRasterizationSettings(
            image_height=int(z["image_height"]), image_width=int(z["image_width"]), tanfovx=float(z["tanfovx"]),
            tanfovy=float(z["tanfovy"]), bg=torch.zeros(3, device=gpu_device), scale_modifier=1.0,
            viewmatrix=torch.as_tensor(z["viewmatrix"][cam], device=gpu_device),
            projmatrix=torch.as_tensor(z["projmatrix"][cam], device=gpu_device), sh_degree=3,
            campos=torch.as_tensor(z["campos"][cam], device=gpu_device), prefiltered=False, debug=False,
            antialiasing=False)
        got = GaussianRasterizer(s).markVisible(pts).cpu().numpy()
        assert got.dtype == np.bool_
        assert np.array_equal(got, z["visible"][cam])


@pytest.mark.parametrize("name", ["unsat_sh3_150x100", "unsat_deg1of3_96x80"])
def test_golden_unsaturated_direct(gpu_device, name):
    """HIP against the reference Python rasterizer's own outputs and autograd gradients."""
    z = load_golden(name)
    inp = golden_inputs(z)
    hip = run_hip(inp, gpu_device, z["dL_dcolor"], z["dL_dinvdepth"])
    assert np.abs(hip["color"] - z["ref_color"]).max() <= 1e-5
    assert np.abs(hip["invdepth"] - z["ref_invdepth"]).max() <= 1e-5
    on = hip["radii"] > 0
    assert np.array_equal(hip["radii"][on], z["ref_radii"][on])
    mod = inp["scale_modifier"]
    for k in GRADS:
        ref = z["ref_grad_" + k]
        got = hip["grads"][k] * (mod if k == "scales" else 1.0)
        assert rel_l2(got, ref) <= 1e-4, (k, rel_l2(got, ref))


def test_golden_cfg1_direct(gpu_device):
    z = load_golden("cfg1_10k_256_sh0")
    inp = golden_inputs(z)
    hip = run_hip(inp, gpu_device)
    hs = hip_state_arrays(hip)
    _, _, _, run = run_oracle(inp)
    assert hs["num_rendered"] == run.num_rendered
    keep = hs["final_T"] >= 0.011
    err = np.abs(hip["color"] - z["ref_color"])[:, keep].max(0)
    assert np.mean(err <= 1e-5) >= 0.999 and err.max() <= 5e-3


@pytest.mark.parametrize("name", ["ref_sat_sh3_20k_white", "ref_cfg2_100k_800_sh3"])
def test_saturated_sh3_vs_reference(gpu_device, name):
    """HIP against the reference Python rasterizer's own outputs and autograd gradients on SATURATED SH-3 scenes:
    BASELINE config 2 in full (100k Gaussians, 800x800, SH 3, opacities up to ~1) and a 20k-Gaussian scene on a
    white background (tests/golden/make_golden_ref.py; reference: gs_lightning/rasterize/rasterize.py:28-127, the
    compositing at render_tools.py:141-144 / rasterize.py:245-258).  Radii exact on rendered Gaussians; colour and
    inverse depth within A13's 1e-5 on every pixel the CUDA and Python rules share (the fixture's mask); every
    stopped pixel within its A2/A3 transmittance bound; gradients of a 10k-Gaussian subset within A13's 1e-4
    relative L2 (tests/helpers.py compare_to_reference)."""
    from tests.helpers import compare_to_reference, load_ref_golden
    z = load_ref_golden(name)
    inp = z["inp"]
    hip = run_hip(inp, gpu_device, z["dL_dcolor"], z["dL_dinvdepth"])
    hs = hip_state_arrays(hip)
    rgb_max = float(np.abs(hs["rec"].view(np.float32)[:, 6:9]).max())
    _, _, _, run = run_oracle(inp)  # the checker's threshold margins name the flip-candidate pixels
    compare_to_reference(z, hip["color"], hip["invdepth"], hip["radii"], hs["final_T"], rgb_max,
                         run.threshold_margin(), hip["grads"], record=lambda r: parity.record(_case(), "reference", r))


CASES = {
    # name: (n, W, H, sh_degree, opacity_scale, bg, seed); gradient bars from compare_backward (flip census)
    "unsat_sh3_200x136": (3000, 200, 136, 3, 0.05, (0.3, 0.6, 0.9), 11),
    "cfg1_10k_256_sh0": (10_000, 256, 256, 0, 1.0, (0.0, 0.0, 0.0), 0),
    "sat_sh2_white_333x211": (20_000, 333, 211, 2, 1.0, (1.0, 1.0, 1.0), 7),
    "cfg2_100k_800_sh3": (100_000, 800, 800, 3, 1.0, (0.0, 0.0, 0.0), 0),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_forward_backward_vs_oracle(gpu_device, case):
    n, W, H, deg, osc, bg, seed = CASES[case]
    inp = scene_inputs(n, W, H, sh_degree=deg, seed=seed, opacity_scale=osc, bg=bg)
    dc, di = upstream(W, H, seed)
    hip = run_hip(inp, gpu_device, dc, di)
    run = compare_forward(inp, hip, run_oracle(inp))
    compare_backward(hip, run, dc, di)


def test_no_invdepth_gradient_path(gpu_device):
    inp = scene_inputs(4000, 160, 120, sh_degree=1, seed=21, coeff_degree=3)
    dc, _ = upstream(160, 120, 21)
    hip = run_hip(inp, gpu_device, dc, None)
    out = run_oracle(inp)
    run = compare_forward(inp, hip, out)
    compare_backward(hip, run, dc, None)


def test_big_gaussians_and_partial_tiles(gpu_device):
    """1 % of the Gaussians x10 in scale (BASELINE config 5 stress shape): many instances per Gaussian
    take the block-reduce path (> 64 tiles)."""
    inp = scene_inputs(20_000, 517, 301, sh_degree=3, seed=5, stress_fraction=0.01)
    dc, di = upstream(517, 301, 5)
    hip = run_hip(inp, gpu_device, dc, di)
    run = compare_forward(inp, hip, run_oracle(inp))
    assert int((run.geom()["tiles_touched"] > 64).sum()) > 10
    compare_backward(hip, run, dc, di)


def test_precomputed_colors_and_cov3d(gpu_device):
    inp = scene_inputs(5000, 128, 96, sh_degree=0, seed=9, opacity_scale=0.5, bg=(0.1, 0.2, 0.3))
    rng = np.random.default_rng(0)
    colors = rng.random((5000, 3), dtype=np.float32)
    # cov3D from the same scales/rotations, computed in float64 on the host
    q = inp["rotations"].astype(np.float64)
    w, x, y, z = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    S = inp["scales"].astype(np.float64)
    L = R * S[:, None, :]
    C = L @ L.transpose(0, 2, 1)
    cov = np.stack([C[:, 0, 0], C[:, 0, 1], C[:, 0, 2], C[:, 1, 1], C[:, 1, 2], C[:, 2, 2]], 1).astype(np.float32)
    dc, di = upstream(128, 96, 9)
    hip = run_hip(inp, gpu_device, dc, di, colors_precomp=colors, cov3D_precomp=cov)
    out = run_oracle(inp, colors_precomp=colors, cov3D_precomp=cov)
    run = compare_forward(inp, hip, out)
    g = run.backward(dc, di)
    rec = {k: rel_l2(hip["grads"][k], g[k]) for k in ("colors", "cov3D", "means3D", "means2D", "opacities")}
    parity.record(_case(), "backward", rec)
    for k, e in rec.items():
        assert e <= GRAD_TOL_ADHOC, (k, e)


def test_antialiasing(gpu_device):
    inp = scene_inputs(5000, 144, 144, sh_degree=3, seed=13)
    dc, di = upstream(144, 144, 13)
    hip = run_hip(inp, gpu_device, dc, di, antialiasing=True)
    run = compare_forward(inp, hip, run_oracle(inp, antialiasing=True))
    compare_backward(hip, run, dc, di)


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (16, 16), (17, 33)])
def test_tiny_images(gpu_device, W, H):
    inp = scene_inputs(500, W, H, sh_degree=1, seed=W * 100 + H)
    dc, di = upstream(W, H, 3)
    hip = run_hip(inp, gpu_device, dc, di)
    run = compare_forward(inp, hip, run_oracle(inp))
    compare_backward(hip, run, dc, di)


def test_all_culled_and_empty(gpu_device):
    inp = scene_inputs(300, 64, 48, sh_degree=0, seed=1, bg=(0.25, 0.5, 0.75))
    inp["means3D"] = inp["means3D"] - np.array([0, 0, 50.0], np.float32) @ np.linalg.inv(inp["viewmatrix"][:3, :3])
    dc, di = upstream(64, 48, 1)
    hip = run_hip(inp, gpu_device, dc, di)
    assert hip["state"].num_rendered == 0
    assert np.all(hip["radii"] == 0)
    assert np.allclose(hip["color"], np.array([0.25, 0.5, 0.75], np.float32)[:, None, None])
    for k in GRADS:
        assert not np.any(hip["grads"][k])
    # P == 0: outputs stay zero (no background), like the reference's early return
    empty = {k: (v[:0] if isinstance(v, np.ndarray) and v.ndim >= 2 and k in (
        "means3D", "opacities", "scales", "rotations", "shs") else v) for k, v in inp.items()}
    e = run_hip(empty, gpu_device)
    assert e["color"].shape == (3, 48, 64) and not np.any(e["color"])


def test_backward_is_deterministic(gpu_device):
    inp = scene_inputs(50_000, 640, 480, sh_degree=3, seed=3)
    dc, di = upstream(640, 480, 3)
    a = run_hip(inp, gpu_device, dc, di)
    b = run_hip(inp, gpu_device, dc, di)
    assert np.array_equal(a["color"], b["color"])
    for k in GRADS:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


def test_autograd_api_and_means2d(gpu_device):
    """The training call site (gs_lightning_module.py:316-348): screenspace_points.grad is populated."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from tests.helpers import settings_for
    inp = scene_inputs(8000, 200, 150, sh_degree=3, seed=17)
    dc, di = upstream(200, 150, 17)
    dev = gpu_device
    t = lambda a: torch.as_tensor(a, device=dev).requires_grad_(True)  # noqa: E731
    means, opac, sc, rot, shs = (t(inp[k]) for k in ("means3D", "opacities", "scales", "rotations", "shs"))
    screen = torch.zeros_like(means, requires_grad=True)
    r = GaussianRasterizer(raster_settings=settings_for(inp, dev))
    img, radii, invd = r(means3D=means, means2D=screen, shs=shs, colors_precomp=None, opacities=opac, scales=sc,
                         rotations=rot, cov3D_precomp=None)
    assert radii.dtype == torch.int32 and img.shape == (3, 150, 200) and invd.shape == (1, 150, 200)
    loss = (img * torch.as_tensor(dc, device=dev)).sum() + (invd * torch.as_tensor(di, device=dev)).sum()
    loss.backward()
    _, _, _, run = run_oracle(inp)
    g = run.backward(dc, di)
    rec = {"means2D": rel_l2(screen.grad.cpu().numpy(), g["means2D"]),
           "means3D": rel_l2(means.grad.cpu().numpy(), g["means3D"]), "shs": rel_l2(shs.grad.cpu().numpy(), g["shs"])}
    parity.record(_case(), "backward", rec)
    for k, e in rec.items():
        assert e <= GRAD_TOL_ADHOC, (k, e)
    vis = radii > 0
    assert torch.all(screen.grad[~vis] == 0)


def test_inference_call_with_means2d_none(gpu_device):
    """The render script's call (scripts/render_trained_image.py:115-124): means2D=None, grad-requiring parameters,
    no torch.no_grad().  The outputs are those of the training call, carry a graph, and a backward through them gives
    the training call's parameter gradients (the absent means2D simply gets none)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    from tests.helpers import settings_for
    inp = scene_inputs(6000, 160, 120, sh_degree=3, seed=19)
    dc, di = (torch.as_tensor(a, device=gpu_device) for a in upstream(160, 120, 19))
    r = GaussianRasterizer(raster_settings=settings_for(inp, gpu_device))

    def params():
        return [torch.as_tensor(inp[k], device=gpu_device).clone().requires_grad_(True)
                for k in ("means3D", "opacities", "scales", "rotations", "shs")]

    m, o, sc, rot, shs = params()
    img, radii, invd = r(means3D=m, means2D=None, shs=shs, colors_precomp=None, opacities=o, scales=sc,
                         rotations=rot, cov3D_precomp=None)
    assert img.requires_grad and invd.requires_grad
    m2, o2, sc2, rot2, shs2 = params()
    screen = torch.zeros_like(m2, requires_grad=True)
    img2, radii2, invd2 = r(means3D=m2, means2D=screen, shs=shs2, colors_precomp=None, opacities=o2, scales=sc2,
                            rotations=rot2, cov3D_precomp=None)
    assert torch.equal(img, img2) and torch.equal(radii, radii2) and torch.equal(invd, invd2)
    img.clamp(0, 1)  # the script's post-processing on a graph-carrying output
    ((img * dc).sum() + (invd * di).sum()).backward()
    ((img2 * dc).sum() + (invd2 * di).sum()).backward()
    for a, b in ((m, m2), (o, o2), (sc, sc2), (rot, rot2), (shs, shs2)):
        assert torch.equal(a.grad, b.grad)


def test_cfg3_full_size_properties(gpu_device):
    """BASELINE config 3 (1M Gaussians, 1920x1080, SH3) at full size: exact instance count and sorted
    list against the oracle, image within the forward bars, gradients within 2e-4 relative L2 (5e-6 over the
    Gaussians no threshold flip touches)."""
    inp = scene_inputs(1_000_000, 1920, 1080, sh_degree=3, seed=0)
    dc, di = upstream(1920, 1080, 0)
    hip = run_hip(inp, gpu_device, dc, di)
    out = run_oracle(inp)
    run = compare_forward(inp, hip, out)
    # SURVEY.md §8(d) counted 6,560,987 rect instances with the reference get_covered_tiles in float32; the
    # CUDA-form ndc2Pix (double) moves at most a couple of rects across a tile edge
    from oracle import oracle as O
    g = run.geom()
    full, _, _ = O.bin_instances(g["xy"], out[1], g["depths"], g["conic_opacity"], 1920, 1080, cull=False)
    assert abs(len(full) - 6_560_987) <= 2
    compare_backward(hip, run, dc, di)


def test_cfg5_full_size_properties(gpu_device):
    """BASELINE config 5 (5M Gaussians, 3840x2160, SH3, 1 % bloated "densification-era" Gaussians) at full size:
    48M instances, so the forward takes the radix binning path (depth sort, depth-ordered expansion, stable tile
    sort).  The sorted instance list and tile ranges are bit-exact against the oracle's binning of the same
    preprocess outputs, the image matches within the forward bars and the gradients within the flip-census bar
    (GRAD_CLEAN_TOL over the Gaussians no threshold flip touches)."""
    W, H = 3840, 2160
    inp = scene_inputs(5_000_000, W, H, sh_degree=3, seed=0, stress_fraction=0.01)
    dc, di = upstream(W, H, 0)
    hip = run_hip(inp, gpu_device, dc, di)
    assert hip["state"].num_rendered > 1024 * ((W + 15) // 16) * ((H + 15) // 16)  # above the bucket path's mean
    run = compare_forward(inp, hip, run_oracle(inp))
    # 3914 flip-candidate pixels touch 124k Gaussians (2.5 %) whose long saturated walks carry the flips into the
    # gradients: 4.9e-4 over all Gaussians (scales), 9.0e-7 over the untouched ones (GRAD_CLEAN_TOL)
    compare_backward(hip, run, dc, di)


def test_cfg4_eight_views_full_size(gpu_device):
    """BASELINE config 4 at full size on one device: 1M Gaussians, the 8 orbit views at 1920x1080, each view's
    forward + compact backward, and the multi-view sums the one-view-per-GPU exchange forms (the
    summed gradients == the sum of the 8 single-view gradients).  The 11 non-SH gradient columns are summed per
    view, dL/dshs is expanded once from the 8 views' colour factors and camera positions (gsr_sh_backward_views);
    both match the oracle's per-view gradients summed in float64 within 1e-4 relative L2."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw, sh_backward_views
    W, H, V = 1920, 1080, 8
    keys = ("means3D", "opacities", "scales", "rotations")
    hip_sum, ora_sum, factors, camposes = {}, {}, [], []
    for v in range(V):
        inp = scene_inputs(1_000_000, W, H, sh_degree=3, seed=0, view_index=v, num_views=V)
        dc, di = upstream(W, H, v)
        rs = settings_for(inp, gpu_device)
        t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in keys + ("shs",)}
        _, _, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
        g = backward_raw(st, rs, torch.as_tensor(dc, device=gpu_device), torch.as_tensor(di, device=gpu_device),
                         compact_sh=True)
        for k in keys:
            x = g[k].double().cpu().numpy()
            hip_sum[k] = x if v == 0 else hip_sum[k] + x
        factors.append(g["colors_sh"])
        camposes.append(rs.campos)
        go = run_oracle(inp)[3].backward(dc, di)
        for k in keys + ("shs",):
            x = np.asarray(go[k], np.float64)
            ora_sum[k] = x if v == 0 else ora_sum[k] + x
    torch.cuda.synchronize()
    hip_sum["shs"] = sh_backward_views(t["means3D"], torch.stack(camposes), torch.stack(factors), 3, 16).cpu().numpy()
    rec = {k: rel_l2(hip_sum[k].reshape(ora_sum[k].shape), ora_sum[k]) for k in keys + ("shs",)}
    parity.record(_case(), "backward_view_sums", rec)
    for k, e in rec.items():  # achieved 4.4e-5 (rotations): eight views' threshold flips
        assert e <= 1e-4, (k, e)


def test_exact_culling_is_bitwise_invisible(gpu_device):
    """Culled instances are exactly those that would hit alpha < 1/255 at every pixel of their tile: turning the
    culling off must reproduce every output bit for bit, and the gradient of every Gaussian whose reference rect
    has at most 64 tiles (its rows are summed in row order, so the culled zero rows change nothing).  A bigger
    Gaussian loses rows to its tight rect, which regroups the partial sums of its workgroup reduction: rounding."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(200_000, 1280, 720, sh_degree=3, seed=2)
    dc, di = upstream(1280, 720, 2)
    # segment boundaries are counted in instances, which culling removes: compare one-walk backwards
    try:
        _native.set_tuning("bwd_seg", 0)
        _native.set_tuning("cull", 0)
        full = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("cull", 1)
        cull = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("cull")
        _native.unset_tuning("bwd_seg")
    assert cull["state"].num_rendered < 0.8 * full["state"].num_rendered
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(cull[k], full[k]), k
    small = hip_state_arrays(full)["tiles"] <= 64  # without culling: the reference rect's area
    assert (~small).sum() > 0
    for k in GRADS:
        assert np.array_equal(cull["grads"][k][small], full["grads"][k][small]), k
        # big Gaussians only: float32 rounding of regrouped partial sums (achieved 1.6e-6 for rotations with the
        # backward built without SLP packing, r4p; 2x margin)
        assert rel_l2(cull["grads"][k], full["grads"][k]) <= 3e-6, k


def test_gs_lightning_rasterize_api(gpu_device):
    """rasterize_gaussian / markVisible with gs_lightning/rasterize/rasterize.py:28-46's signature, checked
    against that function's own outputs and autograd gradients (unsaturated golden)."""
    from gaussian_splatting_lightning_amd.rasterize import markVisible, rasterize_gaussian
    z = load_golden("unsat_sh3_150x100")
    t = {k: torch.as_tensor(z[k], device=gpu_device) for k in
         ("means3D", "opacities", "scales", "rotations", "shs", "viewmatrix", "projmatrix", "campos", "bg")}
    leaves = {k: t[k].clone().requires_grad_(True) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    img, radii, depth = rasterize_gaussian(
        leaves["means3D"], leaves["opacities"], leaves["scales"], leaves["rotations"], leaves["shs"],
        float(z["scale_modifier"]), int(z["image_width"]), int(z["image_height"]), float(z["tanfovx"]),
        float(z["tanfovy"]), t["viewmatrix"], t["projmatrix"], t["campos"], t["bg"], int(z["sh_degree"]))
    assert img.shape == z["ref_color"].shape and depth.shape == z["ref_invdepth"].shape
    assert radii.dtype == torch.float32
    assert np.abs(img.detach().cpu().numpy() - z["ref_color"]).max() <= 1e-5
    assert np.abs(depth.detach().cpu().numpy() - z["ref_invdepth"]).max() <= 1e-5
    r = radii.cpu().numpy()
    on = r > 0
    assert np.array_equal(r[on], z["ref_radii"][on])
    (img * torch.as_tensor(z["dL_dcolor"], device=gpu_device)).sum().add_(
        (depth * torch.as_tensor(z["dL_dinvdepth"], device=gpu_device)).sum()).backward()
    for k in ("means3D", "opacities", "scales", "rotations", "shs"):
        assert rel_l2(leaves[k].grad.cpu().numpy(), z["ref_grad_" + k]) <= 1e-4, k
    vis = markVisible(t["means3D"], t["viewmatrix"], t["projmatrix"]).cpu().numpy()
    from oracle import oracle as O
    assert np.array_equal(vis, O.mark_visible(z["means3D"], z["viewmatrix"], z["projmatrix"]))


def test_compact_sh_views_matches_dense(gpu_device):
    """backward_raw(compact_sh=True) + gsr_sh_backward_views over 3 views == the sum of the dense per-view
    dL/dshs; every other gradient of the compact backward is bitwise the dense one."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw, sh_backward_views
    V = 3
    dense_sum, factors, camposes = None, [], []
    for v in range(V):
        inp = scene_inputs(4000, 160, 120, sh_degree=3, seed=5, view_index=v, num_views=V)
        rs = settings_for(inp, gpu_device)
        t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in
             ("means3D", "opacities", "scales", "rotations", "shs")}
        dc, di = (torch.as_tensor(a, device=gpu_device) for a in upstream(160, 120, seed=v))
        _, _, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
        gd = backward_raw(st, rs, dc, di)
        gc = backward_raw(st, rs, dc, di, compact_sh=True)
        assert gc["shs"] is None
        for k in ("means3D", "means2D", "opacities", "scales", "rotations"):
            assert torch.equal(gd[k], gc[k]), k
        dense_sum = gd["shs"].clone() if dense_sum is None else dense_sum + gd["shs"]
        factors.append(gc["colors_sh"])
        camposes.append(rs.campos)
        if v == 0:
            one = sh_backward_views(t["means3D"], rs.campos.view(1, 3), gc["colors_sh"].unsqueeze(0), 3, 16)
            ref1 = gd["shs"].cpu().numpy()
            np.testing.assert_allclose(one.cpu().numpy(), ref1, rtol=1e-5, atol=1e-6 * np.abs(ref1).max())
    got = sh_backward_views(t["means3D"], torch.stack(camposes), torch.stack(factors), 3, 16)
    # summing views cancels: compare at 1e-6 of the largest coefficient gradient
    ds = dense_sum.cpu().numpy()
    np.testing.assert_allclose(got.cpu().numpy(), ds, rtol=1e-5, atol=1e-6 * np.abs(ds).max())
    ref = O_sh_views(t["means3D"], torch.stack(camposes), torch.stack(factors))
    np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max())
    # the chunk-major layout of the chunked exchange's gather (gsr_sh_backward_views_chunked): bitwise the same
    from gaussian_splatting_lightning_amd.multiview import chunk_bounds
    fs = torch.stack(factors)
    for K in (2, 3):
        b = chunk_bounds(fs.shape[1], K)
        flat = torch.cat([fs[:, g0:g1].reshape(-1) for g0, g1 in b])
        chunked = sh_backward_views(t["means3D"], torch.stack(camposes), flat, 3, 16, chunk_len=b[0][1] - b[0][0])
        assert torch.equal(chunked, got), K


def O_sh_views(means3D, campos, factors):
    from oracle import oracle as O
    return O.sh_backward_views(means3D.cpu().numpy(), campos.cpu().numpy(), factors.cpu().numpy(), 3, 16)


def test_densify_stats_from_backward(gpu_device):
    """gsr_backward's densify_stats == torch.linalg.vector_norm(dL/dmeans2D[:, :2]) and radii > 0
    (gaussian_model.py:175-181), so the trainer's per-view statistics need no extra kernels."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    inp = scene_inputs(5000, 200, 150, sh_degree=2, seed=9)
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    dc, di = (torch.as_tensor(a, device=gpu_device) for a in upstream(200, 150, seed=2))
    _, radii, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    stats = torch.full((5000, 2), -1.0, device=gpu_device)
    g = backward_raw(st, rs, dc, di, out={"densify_stats": stats})
    ref = torch.linalg.vector_norm(g["means2D"][:, :2], dim=1)
    assert torch.allclose(stats[:, 0], ref, rtol=1e-6, atol=0)
    assert torch.equal(stats[:, 1], (radii > 0).float())
    # accumulate mode (the reference's add_densification_stats over steps) and the max-radii accumulator
    acc = stats.clone()
    mrad = torch.full((5000,), 3, dtype=torch.int32, device=gpu_device)
    backward_raw(st, rs, dc, di, out={"densify_stats": acc, "max_radii2D": mrad}, accumulate_stats=True)
    assert torch.allclose(acc, 2 * stats, rtol=1e-6, atol=0)
    assert torch.equal(mrad, torch.maximum(radii.to(torch.int32), torch.full_like(mrad, 3)))


@pytest.mark.gpu
def test_per_xcd_lpt_order_is_bitwise_invisible(gpu_device):
    """The per-XCD LPT orders (1080p: 8160 tiles in lpt_append_range; the forward's slot map from the bucket scatter's
    extra workgroup, the backward's per-XCD bucket lists) only change which tile runs where and when: outputs and
    gradients bitwise those of the global LPT order ("xcd_lpt" 0) and of no LPT order at all ("lpt" 0)."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(150_000, 1920, 1080, sh_degree=3, seed=6, bg=(0.3, 0.6, 0.9))
    dc, di = upstream(1920, 1080, 6)
    ref = run_hip(inp, gpu_device, dc, di)
    try:
        _native.set_tuning("xcd_lpt", 0)
        glob = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("lpt", 0)
        none = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("xcd_lpt")
        _native.unset_tuning("lpt")
    for alt in (glob, none):
        for k in ("color", "invdepth", "radii"):
            assert np.array_equal(ref[k], alt[k]), k
        for k in GRADS:
            assert np.array_equal(ref["grads"][k], alt["grads"][k]), k


@pytest.mark.parametrize("knobs", [{"fwd_parts": 1}, {"fwd_parts": 2}, {"fwd_parts": 4}, {"fwd_whole_waves": 6},
                                   {"strip_exact": 0}, {"bwd_parts": 2}, {"bwd_parts": 4},
                                   {"bwd_union": 1}, {"fwd_parts": 1, "bwd_union": 1}, {"fwd_parts": 1, "smask": 0}])
def test_composite_variants_are_bitwise_identical(gpu_device, knobs):
    """Every composite launch shape gives the same bits: a tile composited whole (4 pixels per lane) or in 2 / 4
    row-strip parts gives the same pixels and contributor counts; strip skipping (row-band or exact column-band
    masks) only skips strips where every pixel fails alpha >= 1/255; the backward's n_contrib strip bounds only
    skip strips and compares that cannot contribute; the union walk (pairs formed only from instances that reach a
    strip) gives each instance the same reduction tree whatever its partner; the whole-tile forward's exact strip
    masks ("smask") only skip strips where no pixel took the instance.  Outputs and gradients must match bit
    for bit (with a non-zero background).  The parts backward adds its waves' per-instance sums: gradients agree to
    rounding only."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(200_000, 1280, 720, sh_degree=3, seed=4, bg=(0.3, 0.6, 0.9))
    dc, di = upstream(1280, 720, 4)
    defaults = {"fwd_parts": 0, "fwd_whole_waves": 8, "strip_exact": 1, "bwd_parts": 0, "bwd_union": -1, "smask": 1}
    try:
        _native.set_tuning("bwd_seg", 0)  # 3600 tiles: the default walks segments (test_segmented_backward)
        _native.set_tuning("bwd_parts", 1)  # the reference side: one wave per tile (the default here is 2)
        ref = run_hip(inp, gpu_device, dc, di)
        for k, v in knobs.items():
            _native.set_tuning(k, v)
        alt = run_hip(inp, gpu_device, dc, di)
    finally:
        for k in knobs:
            _native.set_tuning(k, defaults[k])
        _native.unset_tuning("bwd_parts")
        _native.unset_tuning("bwd_seg")
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[k], alt[k]), k
    for k in GRADS:
        if "bwd_parts" in knobs:
            assert rel_l2(alt["grads"][k], ref["grads"][k]) <= 1e-5, k
        else:
            assert np.array_equal(ref["grads"][k], alt["grads"][k]), k


def _seg_rel_errors(alt, ref):
    return {k: rel_l2(alt["grads"][k], ref["grads"][k]) for k in GRADS}


@pytest.mark.parametrize("seg_k", [32, 64, 256])
def test_segmented_backward(gpu_device, seg_k):
    """Small images walk the backward in seg_k-instance segments, each from the forward's checkpoint at its end
    (T and the colour still to come).  The forward's outputs are bitwise those of the plain forward; gradients agree
    with the one-walk backward to rounding (the recursion restarts from the checkpoint's sums)."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(200_000, 1280, 720, sh_degree=3, seed=4, bg=(0.3, 0.6, 0.9))  # 3600 tiles
    dc, di = upstream(1280, 720, 4)
    try:
        _native.set_tuning("bwd_seg", 0)
        _native.set_tuning("bwd_parts", 1)
        ref = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("bwd_seg", 1)
        _native.set_tuning("seg_k", seg_k)
        alt = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("bwd_seg")
        _native.unset_tuning("bwd_parts")
        _native.unset_tuning("seg_k")
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[k], alt[k]), k
    errs = _seg_rel_errors(alt, ref)
    parity.record(f"segmented_backward_k{seg_k}", "backward_vs_one_walk", {"grad_rel_l2": errs})
    for k, e in errs.items():
        assert e <= 1e-5, (k, e)
    # the work list really splits: the longest tile has more than one segment
    assert int(hip_state_arrays(alt)["tile_last"].max()) > seg_k


def test_segmented_backward_without_checkpoints(gpu_device):
    """A backward in segment mode after a forward that wrote no checkpoints (the knob flipped between the two calls)
    walks whole tiles: the forward's flag word, not the host's knob, decides, so no stale checkpoint is ever read."""
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    inp = scene_inputs(50_000, 640, 480, sh_degree=1, seed=6)
    dc, di = upstream(640, 480, 6)
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    dct, dit = torch.as_tensor(dc, device=gpu_device), torch.as_tensor(di, device=gpu_device)
    args = (t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    try:
        _native.set_tuning("bwd_seg", 0)
        _native.set_tuning("bwd_parts", 1)
        _, _, _, st = forward_raw(*args)
        ref = backward_raw(st, rs, dct, dit)
        _native.set_tuning("bwd_seg", 1)  # backward only: the forward wrote no checkpoints
        alt = backward_raw(st, rs, dct, dit)
    finally:
        _native.unset_tuning("bwd_seg")
        _native.unset_tuning("bwd_parts")
    for k in GRADS:
        assert torch.equal(ref[k], alt[k]), k


@pytest.mark.parametrize("n,W,H", [(60_000, 96, 64), (50_000, 32, 32)])
def test_long_tiles_and_depth_ties(gpu_device, n, W, H):
    """Bucket binning on tiles beyond one wave's register sort (> 511 instances: a workgroup's chunk sorts merged in
    LDS; > 2048: 2048-key chunks placed by merge ranks in global memory) and on exact depth ties (duplicated Gaussians:
    proxy-key tie runs of 200 and 300 repaired by odd-even passes to convergence; the
    (tile, depth, index) order falls back to the Gaussian index, as the reference's stable radix sort does)."""
    inp = scene_inputs(n, W, H, sh_degree=1, seed=23)
    for k in ("means3D", "scales", "rotations", "opacities", "shs"):
        inp[k][1000:1200] = inp[k][1000]
        inp[k][5000:5300] = inp[k][5001]
    dc, di = upstream(W, H, 23)
    from gaussian_splatting_lightning_amd import _native
    try:
        _native.set_tuning("bucket", 2)  # bucket binning even for these long tiles (the default picks radix)
        hip = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("bucket")
    run = compare_forward(inp, hip, run_oracle(inp))
    n_tile = np.diff(hip_state_arrays(hip)["ranges"], axis=1)[:, 0]
    if W > 32:
        assert n_tile.max() > 2048 and np.any((n_tile > 511) & (n_tile <= 2048))
    else:
        assert n_tile.max() > 8192
    compare_backward(hip, run, dc, di)


def test_dense_tiles_fall_back_to_radix_after_speculative_count(gpu_device):
    """Default path choice on tiles averaging more than 1024 instances: the bucket count pass has already run
    (it is queued before the instance total is known), then the total selects the radix path, whose outputs must
    not depend on what the count pass left behind."""
    from gaussian_splatting_lightning_amd import _native
    W, H = 96, 64
    inp = scene_inputs(60_000, W, H, sh_degree=1, seed=29)
    dc, di = upstream(W, H, 29)
    hip = run_hip(inp, gpu_device, dc, di)
    T = ((W + 15) // 16) * ((H + 15) // 16)
    assert hip["state"].num_rendered > 1024 * T  # the radix path was chosen
    run = compare_forward(inp, hip, run_oracle(inp))
    compare_backward(hip, run, dc, di)
    try:
        _native.set_tuning("bucket", 2)
        forced = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("bucket")
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(hip[k], forced[k]), k
    for k in GRADS:
        assert np.array_equal(hip["grads"][k], forced["grads"][k]), k


@pytest.mark.parametrize("W,H,onesweep,cscan,xcd,k16", [(1280, 720, 1, 1, 1, 1), (96, 64, 1, 1, 1, 1),
                                                        (1280, 720, 0, 1, 1, 1), (1280, 720, 3, 1, 1, 0),
                                                        (1280, 720, 0, 0, 0, 0)])
def test_binning_paths_are_bitwise_identical(gpu_device, W, H, onesweep, cscan, xcd, k16):
    """The bucket binning (per-tile sorts) and the radix binning (depth sort + stable tile sort) produce the
    same instance order, so every output and gradient is bit for bit the same -- with either radix-sort
    implementation (onesweep 0: the multi-kernel passes for every sort, 3: onesweep for every sort), either count
    scan of the multi-kernel passes (cscan 1: one launch with look-back, 0: three launches), either bucket run
    order (xcd 1: XCD-major, 0: block order) and 16- or 32-bit tile keys in the radix tile sort (k16)."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(200_000 if W > 100 else 60_000, W, H, sh_degree=3, seed=6, stress_fraction=0.01)
    dc, di = upstream(W, H, 6)
    try:
        _native.set_tuning("bucket", 2)
        _native.set_tuning("bk_xcd", xcd)
        ref = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("bucket", 0)
        _native.set_tuning("onesweep", onesweep)
        _native.set_tuning("rs_cscan", cscan)
        _native.set_tuning("tile_key16", k16)
        alt = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("tile_key16")
        _native.unset_tuning("bucket")
        _native.unset_tuning("onesweep")
        _native.unset_tuning("rs_cscan")
        _native.unset_tuning("bk_xcd")
    a, b = hip_state_arrays(ref), hip_state_arrays(alt)
    for k in ("point_list", "ranges", "tiles", "n_contrib", "tile_last", "tile_loaded"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[k], alt[k]), k
    for k in GRADS:
        assert np.array_equal(ref["grads"][k], alt["grads"][k]), k


@pytest.mark.parametrize("db", [4, 5])
def test_tile_sort_digit_width_is_invisible(gpu_device, db):
    """The radix binning's 16-bit tile sort in digits of 4 or 5 bits (3 passes at 1280x720's 12-bit tile ids)
    gives bitwise the instance order of the default 8-bit digits (2 passes)."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(200_000, 1280, 720, sh_degree=3, seed=6, stress_fraction=0.01)
    dc, di = upstream(1280, 720, 6)
    try:
        _native.set_tuning("bucket", 0)
        ref = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("tile_db", db)
        alt = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("bucket")
        _native.unset_tuning("tile_db")
    a, b = hip_state_arrays(ref), hip_state_arrays(alt)
    for k in ("point_list", "ranges", "n_contrib"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[k], alt[k]), k


@pytest.mark.parametrize("n,depth_scale", [(150_000, 1.0), (150_000, 40.0), (2_000, 1.0)])
def test_relative_depth_sort_is_bitwise_the_32bit_one(gpu_device, n, depth_scale):
    """The radix path's depth sort on relative keys (kept keys minus their minimum, culled ones after them; 9-bit
    digits, 3 passes for this scene's ~26-bit span) gives bitwise the order, outputs and gradients of the 4-pass
    32-bit sort.  depth_scale 40 stretches the scene along the view axis (a wider key span), n = 2000 a small one;
    onesweep_max_n = 0 sends every depth sort to the multi-kernel path, where relative keys apply."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(n, 960, 540, sh_degree=1, seed=21)
    if depth_scale != 1.0:
        inp["means3D"] = inp["means3D"] * np.array([1.0, 1.0, depth_scale], np.float32)
    dc, di = upstream(960, 540, 21)
    try:
        _native.set_tuning("bucket", 0)
        _native.set_tuning("onesweep_max_n", 0)
        _native.set_tuning("depth_rel", 0)
        ref = run_hip(inp, gpu_device, dc, di)
        assert _native.get_tuning("stat_depth_passes") == 4
        _native.set_tuning("depth_rel", 1)
        alt = run_hip(inp, gpu_device, dc, di)
        assert 1 <= _native.get_tuning("stat_depth_passes") <= 3  # the relative sort ran
    finally:
        _native.unset_tuning("bucket")
        _native.unset_tuning("onesweep_max_n")
        _native.unset_tuning("depth_rel")
    a, b = hip_state_arrays(ref), hip_state_arrays(alt)
    for key in ("point_list", "ranges", "n_contrib", "tiles"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[key], alt[key]), key
    for key in GRADS:
        assert np.array_equal(ref["grads"][key], alt["grads"][key]), key


def test_beyond_lpt_and_bucket_tile_limits(gpu_device):
    """More than 32768 tiles (8K-class image): the radix binning path."""
    inp = scene_inputs(3000, 4160, 2336, sh_degree=1, seed=31)
    dc, di = upstream(4160, 2336, 31)
    hip = run_hip(inp, gpu_device, dc, di)
    run = compare_forward(inp, hip, run_oracle(inp))
    compare_backward(hip, run, dc, di)


@pytest.mark.parametrize("bucket,os_max", [(0, None), (1, None), (0, 0)])
def test_debug_mode_is_bitwise_identical(gpu_device, bucket, os_max):
    """debug=True synchronises and checks after every stage (notes/rasterizer_note.h:44-53) on both binning
    paths; outputs and gradients are those of the asynchronous run.  os_max = 0 sends every radix sort to the
    multi-kernel path (as sorts above 3M keys go), whose scratch holds no onesweep error word: the debug check must
    not read one."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(20_000, 320, 240, sh_degree=2, seed=41)
    dc, di = upstream(320, 240, 41)
    try:
        _native.set_tuning("bucket", bucket)
        if os_max is not None:
            _native.set_tuning("onesweep_max_n", os_max)
        a = run_hip(inp, gpu_device, dc, di)
        b = run_hip(inp, gpu_device, dc, di, debug=True)
    finally:
        _native.unset_tuning("bucket")
        _native.unset_tuning("onesweep_max_n")
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(a[k], b[k]), k
    for k in GRADS:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.parametrize("bucket,onesweep", [(1, 1), (0, 3), (0, 0)])
def test_lookback_fallback_is_bitwise_invisible(gpu_device, bucket, onesweep):
    """Every decoupled look-back (bucket tile scan, instance scan, onesweep digit look-back) forced onto its
    fallback -- every predecessor's aggregate recomputed from the kernel input instead of read from its status word
    ("lb_force"), the path a look-back takes when a predecessor block is not running -- gives the same bits."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(20_000, 320, 240, sh_degree=2, seed=43, stress_fraction=0.01)
    dc, di = upstream(320, 240, 43)
    try:
        _native.set_tuning("bucket", bucket)
        _native.set_tuning("onesweep", onesweep)
        a = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("lb_force", 1)
        b = run_hip(inp, gpu_device, dc, di)
    finally:
        _native.unset_tuning("lb_force")
        _native.unset_tuning("bucket")
        _native.unset_tuning("onesweep")
    sa, sb = hip_state_arrays(a), hip_state_arrays(b)
    for k in ("point_list", "ranges", "tiles", "n_contrib"):
        assert np.array_equal(sa[k], sb[k]), k
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(a[k], b[k]), k
    for k in GRADS:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.parametrize("force", [0, 1])
@pytest.mark.parametrize("nt", [1024, 2048])
def test_instance_scan_width_is_invisible(gpu_device, force, nt):
    """The radix path's instance scan at 1024 threads x 16 counts per workgroup ("scan_nt" 1024: 4x fewer
    workgroups, a 4x shorter look-back chain) or x 32 ("scan_nt" 2048) gives the 256 x 16 scan's bits, with its look-back on the
    status words and forced onto the recomputed-aggregate fallback."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(70_000, 480, 320, sh_degree=1, seed=47, stress_fraction=0.01)
    dc, di = upstream(480, 320, 47)
    try:
        _native.set_tuning("bucket", 0)
        _native.set_tuning("onesweep", 0)
        _native.set_tuning("lb_force", force)
        _native.set_tuning("scan_nt", 256)
        a = run_hip(inp, gpu_device, dc, di)
        _native.set_tuning("scan_nt", nt)
        b = run_hip(inp, gpu_device, dc, di)
    finally:
        for k in ("scan_nt", "lb_force", "bucket", "onesweep"):
            _native.unset_tuning(k)
    sa, sb = hip_state_arrays(a), hip_state_arrays(b)
    for k in ("point_list", "ranges", "tiles", "n_contrib"):
        assert np.array_equal(sa[k], sb[k]), k
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(a[k], b[k]), k
    for k in GRADS:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs two HIP devices")
def test_render_on_non_current_device():
    """Inputs on cuda:1 while cuda:0 is current (and the reverse afterwards): the library runs on its stream's
    device (per-device readback event and pinned words), so results equal those of a cuda:0 run."""
    inp = scene_inputs(5000, 160, 120, sh_degree=1, seed=51)
    dc, di = upstream(160, 120, 51)
    d0, d1 = torch.device("cuda", 0), torch.device("cuda", 1)
    torch.cuda.set_device(d0)
    a = run_hip(inp, d0, dc, di)
    b = run_hip(inp, d1, dc, di)
    c = run_hip(inp, d0, dc, di)
    for k in ("color", "invdepth", "radii"):
        assert np.array_equal(a[k], b[k]) and np.array_equal(a[k], c[k]), k
    for k in GRADS:
        assert np.array_equal(a["grads"][k], b["grads"][k]), k


@pytest.mark.parametrize("fail_buf", ["GSR_BUF_GEOM", "GSR_BUF_BINNING", "GSR_BUF_BWD_SCRATCH"])
def test_failed_scratch_allocation_is_a_clean_error(gpu_device, fail_buf, monkeypatch):
    """An out-of-memory inside the caller's allocator (here injected for one buffer) surfaces as that exception
    from forward_raw / backward_raw, with nothing launched on a NULL buffer: the next call renders normally."""
    from gaussian_splatting_lightning_amd import _native, rasterizer
    which = getattr(_native, fail_buf)
    inp = scene_inputs(2000, 96, 64, sh_degree=1, seed=41)
    dc, di = upstream(96, 64, 41)
    ref = run_hip(inp, gpu_device, dc, di)

    class Failing(rasterizer._Buffers):
        def __init__(self, device):
            super().__init__(device)
            inner = self._cb

            def alloc(ctx, w, nbytes):
                if w == which:
                    self.errors.append(torch.OutOfMemoryError("injected"))
                    return None
                return inner(ctx, w, nbytes)

            self._keep = inner
            self._cb = _native.ALLOC_FN(alloc)

    monkeypatch.setattr(rasterizer, "_Buffers", Failing)
    with pytest.raises(torch.OutOfMemoryError):
        run_hip(inp, gpu_device, dc, di)
    monkeypatch.undo()
    # the next forward runs on another stream: a preprocess abandoned by the failed call must not publish its
    # readback word over this call's (gsr_forward waits for it before returning the error)
    side = torch.cuda.Stream(device=gpu_device)
    with torch.cuda.stream(side):
        again = run_hip(inp, gpu_device, dc, di)
    side.synchronize()
    assert np.array_equal(ref["color"], again["color"])
    for k in GRADS:
        assert np.array_equal(ref["grads"][k], again["grads"][k]), k


@pytest.mark.parametrize("compact", [False, True])
def test_chunked_backward_is_bitwise_the_single_call(gpu_device, compact):
    """backward_chunked (one compositing call, then the per-Gaussian stage over Gaussian ranges with chunk-relative
    destinations -- the overlapped multi-GPU exchange's backward, multiview.py) writes bit for bit what one
    backward_raw call writes, for ranges on and off the 256-Gaussian block grid, with the statistics accumulated."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_chunked, backward_raw, forward_raw
    n, W, H = 30_000, 320, 240
    inp = scene_inputs(n, W, H, sh_degree=3, seed=12, stress_fraction=0.01)
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    dc, di = (torch.as_tensor(a, device=gpu_device) for a in upstream(W, H, seed=12))
    _, radii, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    assert st.num_big > 0  # the big-Gaussian reduction feeds the chunks too
    stats = torch.ones(n, 2, device=gpu_device)
    mrad = torch.full((n,), 2, dtype=torch.int32, device=gpu_device)
    ref = backward_raw(st, rs, dc, di, out={"densify_stats": stats, "max_radii2D": mrad}, compact_sh=compact,
                       accumulate_stats=True)
    widths = dict(means3D=3, scales=3, rotations=4, opacities=1, means2D=3)
    if compact:
        widths["colors_sh"] = 3
    else:
        widths["shs"] = 48
    bounds = [0, 256, 1000, 7777, 20_480, n]
    chunks, seen = [], []
    stats2 = torch.ones(n, 2, device=gpu_device)
    mrad2 = torch.full((n,), 2, dtype=torch.int32, device=gpu_device)
    for g0, g1 in zip(bounds[:-1], bounds[1:]):
        out = {k: torch.full((g1 - g0, w), float("nan"), device=gpu_device) for k, w in widths.items()}
        out["densify_stats"] = stats2[g0:g1]
        out["max_radii2D"] = mrad2[g0:g1]
        chunks.append((g0, g1, out))
    backward_chunked(st, rs, dc, di, chunks, on_chunk=seen.append, compact_sh=compact, accumulate_stats=True)
    torch.cuda.synchronize()
    assert seen == list(range(len(chunks)))
    for k in widths:
        got = torch.cat([o[k] for _, _, o in chunks], 0)
        want = ref[k].reshape(n, -1)
        assert torch.equal(got, want), k
    assert torch.equal(stats2, stats) and torch.equal(mrad2, mrad)


@pytest.mark.parametrize("W,H,bucket,n", [(1920, 1080, 1, 300_000), (1280, 720, 0, 150_000), (320, 240, 1, 20_000)])
def test_inverse_permutation_marks_exactly_the_loaded_instances(gpu_device, W, H, bucket, n):
    """The backward finds the instances with a gradient row (the ones the forward composite loaded) through the inverse
    permutation: inv[sorted_u[s]] = s over every tile's loaded prefix, INV_NONE for every other instance -- on the
    bucket path (whole tiles at 1080p, row-strip parts at 320x240) and the radix path."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(n, W, H, sh_degree=3, seed=21, stress_fraction=0.01)
    with _native.tuned(bucket=bucket):
        out = run_hip(inp, gpu_device)
    hs = hip_state_arrays(out)
    rg, ld = hs["ranges"].astype(np.int64), hs["tile_loaded"].astype(np.int64)
    pos = np.concatenate([np.arange(a, a + l) for a, l in zip(rg[:, 0], ld) if l > 0])
    assert len(pos) > 0
    u = hs["sorted_u"][pos].astype(np.int64)
    assert np.array_equal(hs["inv"][u], pos.astype(np.uint32))
    rest = np.ones(hs["num_rendered"], bool)
    rest[u] = False
    assert rest.any() and np.all(hs["inv"][rest] == 0xFFFFFFFF)


@pytest.mark.parametrize("W,H,n,stress", [(1920, 1080, 300_000, 0.01), (320, 240, 20_000, 0.0), (1280, 720, 100_000, 0.05),
                                          (1920, 1080, 3_000, 0.0)])
def test_region_scatter_is_bitwise_the_direct_scatter(gpu_device, W, H, n, stress):
    """The bucket scatter through 16-tile regions plus the partition pass ("bk_region" 2: always; 1, default: above
    4096 tiles) fills every tile
    bucket with exactly the instances of the direct scatter (order inside a bucket is free), so the sorted list,
    ranges, outputs and gradients are bitwise the same -- whole tiles, row-strip parts, many big Gaussians, and a sparse
    scene whose partition chunks span more regions than their LDS bins (the per-key fallback)."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(n, W, H, sh_degree=3, seed=33, stress_fraction=stress)
    dc, di = upstream(W, H, 33)
    with _native.tuned(bk_region=0):
        ref = run_hip(inp, gpu_device, dc, di)
    with _native.tuned(bk_region=2):
        alt = run_hip(inp, gpu_device, dc, di)
    a, b = hip_state_arrays(ref), hip_state_arrays(alt)
    for key in ("point_list", "ranges", "tiles", "n_contrib", "tile_last", "tile_loaded", "inv"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[key], alt[key]), key
    for key in GRADS:
        assert np.array_equal(ref["grads"][key], alt["grads"][key]), key


@pytest.mark.parametrize("W,H,n,stress", [(1920, 1080, 2_000, 0.3), (320, 240, 1_500, 0.5), (1280, 720, 40_000, 0.05)])
def test_big_rect_walk_blocks_are_bitwise_the_range_blocks(gpu_device, W, H, n, stress):
    """Few Gaussians with large footprints: the bucket walks add blocks that only walk big rects when the big-Gaussian
    count exceeds the blocks owning Gaussian ranges ("bk_big_blocks", default 256; 0 = the range blocks only).  Every
    tile bucket gets the same instances, so the sorted list, ranges, outputs and gradients are bitwise the same."""
    from gaussian_splatting_lightning_amd import _native
    inp = scene_inputs(n, W, H, sh_degree=3, seed=41, stress_fraction=stress)
    dc, di = upstream(W, H, 41)
    with _native.tuned(bk_big_blocks=0):
        ref = run_hip(inp, gpu_device, dc, di)
    alt = run_hip(inp, gpu_device, dc, di)
    a, b = hip_state_arrays(ref), hip_state_arrays(alt)
    assert a["num_rendered"] == b["num_rendered"] > 0
    for key in ("point_list", "ranges", "tiles", "n_contrib", "tile_last", "tile_loaded", "inv"):
        assert np.array_equal(a[key], b[key]), key
    for key in ("color", "invdepth", "radii"):
        assert np.array_equal(ref[key], alt[key]), key
    for key in GRADS:
        assert np.array_equal(ref["grads"][key], alt["grads"][key]), key


@pytest.mark.parametrize("case", ["cfg1_golden", "big_stress", "cfg3_full", "cfg5_full"])
def test_threshold_guard_band(gpu_device, case):
    """Knob "guard" (off by default): pairs whose alpha lies within 2e-5 (relative) of 1/255, or whose
    T (1 - alpha) within 1e-4 of 1e-4, take their decisions from the oracle's own arithmetic (uncontracted exponent,
    exp in double).  Contributor counts that differ from the oracle's (threshold flips) must not increase with it, and
    the guarded forward + backward keep every bar of the unguarded run; achieved flips and all-Gaussian gradient
    errors of both runs go to the parity record."""
    from gaussian_splatting_lightning_amd import _native
    if case == "cfg1_golden":
        z = load_golden("cfg1_10k_256_sh0")
        inp = golden_inputs(z)
        dc, di = z["dL_dcolor"], z["dL_dinvdepth"]
    elif case == "big_stress":  # test_big_gaussians_and_partial_tiles' scene (unguarded: 1.6e-4)
        inp = scene_inputs(20_000, 517, 301, sh_degree=3, seed=5, stress_fraction=0.01)
        dc, di = upstream(517, 301, 5)
    elif case == "cfg3_full":
        inp = scene_inputs(1_000_000, 1920, 1080, sh_degree=3, seed=0)
        dc, di = upstream(1920, 1080, 0)
    else:
        inp = scene_inputs(5_000_000, 3840, 2160, sh_degree=3, seed=0, stress_fraction=0.01)
        dc, di = upstream(3840, 2160, 0)
    out = run_oracle(inp)
    run = out[3]
    g = run.backward(dc, di)
    _, nc_ref = run.image_state()
    rec = {}
    try:
        for guard in (0, 1):
            _native.set_tuning("guard", guard)
            hip = run_hip(inp, gpu_device, dc, di)
            nc = hip_state_arrays(hip)["n_contrib"]
            e = {"n_contrib_mismatch_pixels": int((nc != nc_ref).sum()),
                 "color_maxabs": float(np.abs(hip["color"] - out[0]).max())}
            for k in GRADS:
                if hip["grads"].get(k) is not None:
                    e[f"grad_rel_l2_{k}"] = rel_l2(hip["grads"][k], g[k])
            rec[f"guard{guard}"] = e
    finally:
        _native.set_tuning("guard", 0)
    parity.record(_case(), "guard_band", rec)
    assert rec["guard1"]["n_contrib_mismatch_pixels"] <= rec["guard0"]["n_contrib_mismatch_pixels"], rec
    # with the guard, SURVEY A13's tolerances hold over ALL pixels and Gaussians (no flip-candidate exclusion):
    # colour <= 1e-4 (achieved <= 3.8e-5, the remaining transmittance flips), every gradient rel-L2 <= 1e-5
    # (achieved <= 1.4e-6; unguarded up to 4.9e-4)
    assert rec["guard1"]["color_maxabs"] <= 1e-4, rec
    for k in GRADS:
        if f"grad_rel_l2_{k}" in rec["guard1"]:
            assert rec["guard1"][f"grad_rel_l2_{k}"] <= 1e-5, rec


@pytest.mark.parametrize("compact_sh", [False, True])
def test_zero_gradients_written_by_the_composite(gpu_device, compact_sh):
    """With "bwd_prezero" (default) the compositing backward zero-fills the per-Gaussian outputs as its workgroups
    exit and preprocess_bwd stores only the Gaussians whose gradient is not identically zero.  Every output must hold
    the values of the full-write path (knob 0) -- also when the outputs start as NaN garbage and sit 4 B off a 16-B
    boundary (each output's unaligned head / tail words go through the odd-word list), and with the compact SH
    gradient of the multi-view exchange."""
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    n, W, H = 60_001, 640, 480
    inp = scene_inputs(n, W, H, sh_degree=3, seed=27, stress_fraction=0.01)
    dc, di = upstream(W, H, 27)
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    dct, dit = torch.as_tensor(dc, device=gpu_device), torch.as_tensor(di, device=gpu_device)
    _, radii, _, st = forward_raw(t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    widths = dict(means3D=3, means2D=3, opacities=1, scales=3, rotations=4)
    widths.update(colors_sh=3) if compact_sh else widths.update(shs=48)

    def outputs():  # NaN-filled, each output 4 B past a 16-B boundary
        o = {}
        for k, w in widths.items():
            buf = torch.full((n * w + 8,), float("nan"), device=gpu_device)
            v = buf[1:1 + n * w]
            o[k] = v.view(n, 16, 3) if k == "shs" else v.view(n, w)
        return o

    res = {}
    for knob in (0, 1):
        out = outputs()
        with _native.tuned(bwd_prezero=knob):
            g = backward_raw(st, rs, dct, dit, out=out, compact_sh=compact_sh)
        torch.cuda.synchronize()
        res[knob] = {k: g[k].detach().cpu().numpy() for k in widths}
    zero = (radii.cpu().numpy() <= 0)
    for k in widths:
        assert not np.isnan(res[1][k]).any(), k
        assert np.array_equal(res[0][k], res[1][k]), k
        assert not np.any(res[1][k].reshape(n, -1)[zero]), k  # culled Gaussians: exact zeros


def test_second_backward_on_one_forward_sees_its_own_rows(gpu_device):
    """The compositing backward marks the Gaussians it stores a non-zero row of (GeomState::live, set-only, cleared
    by the forward) and the per-Gaussian pass gathers only those.  A second backward on the same forward with another
    upstream gradient -- one that is zero on half the image, so the first backward's marks differ from what the
    second needs -- and one run with the marks switched off in its composite must both equal a fresh
    forward + backward."""
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    n, W, H = 50_000, 640, 480
    inp = scene_inputs(n, W, H, sh_degree=3, seed=31, stress_fraction=0.01)
    rs = settings_for(inp, gpu_device)
    t = {k: torch.as_tensor(inp[k], device=gpu_device) for k in ("means3D", "opacities", "scales", "rotations", "shs")}
    args = (t["means3D"], t["shs"], None, t["opacities"], t["scales"], t["rotations"], None, rs)
    d1, i1 = (torch.as_tensor(a, device=gpu_device) for a in upstream(W, H, 31))
    d2, i2 = (torch.as_tensor(a, device=gpu_device) for a in upstream(W, H, 32))
    d1[:, :, W // 2:] = 0.0  # the first backward: rows only from the left half
    i1[:, :, W // 2:] = 0.0

    def grads(g):
        return {k: g[k].detach().cpu().numpy() for k in GRADS}

    _, _, _, st = forward_raw(*args)
    backward_raw(st, rs, d1, i1)
    second = grads(backward_raw(st, rs, d2, i2))
    with _native.tuned(bwd_live=0):
        unmarked = grads(backward_raw(st, rs, d2, i2))
    third = grads(backward_raw(st, rs, d2, i2))  # marks valid again
    _, _, _, st2 = forward_raw(*args)
    fresh = grads(backward_raw(st2, rs, d2, i2))
    torch.cuda.synchronize()
    for k in GRADS:
        assert np.array_equal(second[k], fresh[k]), k
        assert np.array_equal(unmarked[k], fresh[k]), k
        assert np.array_equal(third[k], fresh[k]), k
