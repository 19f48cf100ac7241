"""Shared test helpers: golden fixtures, oracle runs, HIP runs, comparison metrics."""
from __future__ import annotations

import os

import numpy as np
import torch

from gaussian_splatting_lightning_amd.synthetic import Scene, make_camera, make_scene, make_upstream

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GRAD_KEYS = ("means3D", "means2D", "opacities", "scales", "rotations", "shs")


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def golden_inputs(z: dict) -> dict:
    return dict(means3D=z["means3D"], opacities=z["opacities"], scales=z["scales"], rotations=z["rotations"],
                shs=z["shs"], viewmatrix=z["viewmatrix"], projmatrix=z["projmatrix"], campos=z["campos"],
                bg=z["bg"], tanfovx=float(z["tanfovx"]), tanfovy=float(z["tanfovy"]),
                image_height=int(z["image_height"]), image_width=int(z["image_width"]),
                sh_degree=int(z["sh_degree"]), scale_modifier=float(z["scale_modifier"]))


def scene_inputs(n, W, H, sh_degree=3, seed=0, opacity_scale=1.0, bg=(0.0, 0.0, 0.0), view_index=0,
                 num_views=1, stress_fraction=0.0, coeff_degree=None) -> dict:
    sc = make_scene(n, sh_degree=coeff_degree if coeff_degree is not None else sh_degree, seed=seed,
                    opacity_scale=opacity_scale, stress_fraction=stress_fraction)
    cam = make_camera(W, H, view_index=view_index, num_views=num_views)
    return dict(means3D=sc.means3D.numpy(), opacities=sc.opacities.numpy(), scales=sc.scales.numpy(),
                rotations=sc.rotations.numpy(), shs=sc.shs.numpy(), viewmatrix=cam.viewmatrix.numpy(),
                projmatrix=cam.projmatrix.numpy(), campos=cam.campos.numpy(),
                bg=np.asarray(bg, np.float32), tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, image_height=H,
                image_width=W, sh_degree=sh_degree, scale_modifier=1.0)


def upstream(W, H, seed=0):
    dc, di = make_upstream(W, H, seed)
    return dc.numpy(), di.numpy()


def run_oracle(inp: dict, colors_precomp=None, cov3D_precomp=None, antialiasing=False, use_shs=True):
    from oracle import oracle as O
    return O.forward(inp["means3D"], inp["opacities"], None if cov3D_precomp is not None else inp["scales"],
                     None if cov3D_precomp is not None else inp["rotations"],
                     inp["shs"] if (use_shs and colors_precomp is None) else None, inp["viewmatrix"],
                     inp["projmatrix"], inp["campos"], inp["bg"], inp["tanfovx"], inp["tanfovy"],
                     inp["image_height"], inp["image_width"], inp["sh_degree"], inp["scale_modifier"],
                     colors_precomp=colors_precomp, cov3D_precomp=cov3D_precomp, antialiasing=antialiasing)


def settings_for(inp: dict, device, antialiasing=False, debug=False):
    from gaussian_splatting_lightning_amd import GaussianRasterizationSettings
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=device)  # noqa: E731
    return GaussianRasterizationSettings(
        image_height=inp["image_height"], image_width=inp["image_width"], tanfovx=inp["tanfovx"],
        tanfovy=inp["tanfovy"], bg=t(inp["bg"]), scale_modifier=inp["scale_modifier"],
        viewmatrix=t(inp["viewmatrix"]), projmatrix=t(inp["projmatrix"]), sh_degree=inp["sh_degree"],
        campos=t(inp["campos"]), prefiltered=False, debug=debug, antialiasing=antialiasing)


def run_hip(inp: dict, device, dL_dcolor=None, dL_dinvdepth=None, colors_precomp=None, cov3D_precomp=None,
            antialiasing=False, debug=False):
    """HIP forward (+ backward when dL_dcolor is given) through forward_raw/backward_raw."""
    from gaussian_splatting_lightning_amd.rasterizer import backward_raw, forward_raw
    t = lambda a: None if a is None else torch.as_tensor(np.asarray(a, np.float32), device=device)  # noqa: E731
    rs = settings_for(inp, device, antialiasing=antialiasing, debug=debug)
    use_cov = cov3D_precomp is not None
    color, radii, invd, st = forward_raw(
        t(inp["means3D"]), None if colors_precomp is not None else t(inp["shs"]), t(colors_precomp),
        t(inp["opacities"]), None if use_cov else t(inp["scales"]), None if use_cov else t(inp["rotations"]),
        t(cov3D_precomp), rs)
    out = dict(color=color.cpu().numpy(), radii=radii.cpu().numpy(), invdepth=invd.cpu().numpy(), state=st,
               settings=rs)
    if dL_dcolor is not None:
        g = backward_raw(st, rs, t(dL_dcolor), t(dL_dinvdepth))
        out["grads"] = {k: (v.cpu().numpy() if v is not None else None) for k, v in g.items()}
    torch.cuda.synchronize()
    return out


def hip_state_arrays(out: dict) -> dict:
    """Integer binning/image state of a HIP forward, sliced out of its buffers with gsr_state_layout_query."""
    from gaussian_splatting_lightning_amd import _native
    st = out["state"]
    P = st.means3D.shape[0]
    R = st.num_rendered
    H, W = out["color"].shape[1:]
    lay = _native.state_layout(P, R, W, H)
    T = ((W + 15) // 16) * ((H + 15) // 16)

    def view(buf, off, n, dtype):
        nbytes = n * torch.tensor([], dtype=dtype).element_size()
        return buf[off: off + nbytes].view(dtype).cpu().numpy() if n else np.zeros(0)

    i32 = torch.int32
    sorted_u = view(st.binning_buffer, lay["bin_sorted_u"], R, i32).astype(np.int64)
    inst_gid = view(st.binning_buffer, lay["bin_inst_gid"], R, i32).astype(np.uint32)
    ok = (sorted_u >= 0) & (sorted_u < R)
    point_list = np.full(R, 0xFFFFFFFF, np.uint32)
    point_list[ok] = inst_gid[sorted_u[ok]]
    res = dict(
        point_list=point_list,
        point_list_written=view(st.binning_buffer, lay["bin_point_list"], R, i32).astype(np.uint32),
        inv=view(st.binning_buffer, lay["bin_inv"], R, i32).astype(np.uint32),
        sorted_u=sorted_u.astype(np.uint32),
        tile_loaded=view(st.image_buffer, lay["img_tile_loaded"], T, i32).astype(np.uint32),
        tile_last=view(st.image_buffer, lay["img_tile_last"], T, i32).astype(np.uint32),
        ranges=view(st.image_buffer, lay["img_ranges"], 2 * T, i32).astype(np.uint32).reshape(T, 2),
        n_contrib=view(st.image_buffer, lay["img_n_contrib"], W * H, i32).astype(np.uint32).reshape(H, W),
        final_T=view(st.image_buffer, lay["img_final_T"], W * H, torch.float32).reshape(H, W),
        tiles=view(st.geom_buffer, lay["geom_tiles"], P, i32).astype(np.uint32),
        num_rendered=R)
    res["depth_bits"] = view(st.geom_buffer, lay["geom_depth_key"], P, i32).astype(np.uint32)
    # render records: one 48-B (12-float) record per Gaussian, a = floats 0..3, b = 4..7, c = 8..9
    stride = lay["geom_rec_stride"] // 4
    rec = view(st.geom_buffer, lay["geom_rec_a"], stride * P, torch.float32).reshape(P, stride)
    rec_a, rec_b = rec[:, 0:4], rec[:, 4:8]
    depth_bits = view(st.geom_buffer, lay["geom_depth_key"], P, i32)
    res["xy"] = np.ascontiguousarray(rec_a[:, :2])
    res["conic_opacity"] = np.ascontiguousarray(np.concatenate([rec_a[:, 2:4], rec_b[:, 0:2]], 1))
    res["depths"] = depth_bits.view(np.float32)
    # the full record words (a, b, c: position, conic, opacity, colour, inverse depth) and the colour clamp bits of
    # every rendered Gaussian (the others' words are never written)
    on = out["radii"] > 0
    res["rec"] = np.ascontiguousarray(rec[:, :10]).view(np.uint32)[on]
    res["clamped"] = view(st.geom_buffer, lay["geom_clamped"], P, torch.uint8)[on]
    return res


# ---- reference goldens for saturated SH-3 scenes (tests/golden/make_golden_ref.py) ----
T_KEEP = 0.011  # reference transmittance above which the CUDA walk cannot have stopped (make_golden_ref.py)
# oracle threshold margin below which a pixel is left out of a reference fixture's mask: wider than the device-vs-
# oracle flip margin (1.0, tests/test_gpu_parity.py) because the reference forms the geometry in another operation
# order (1 / (w + eps) products, torch matmuls): its exponents differ from the CUDA order's by up to ~1e-5 of the
# quadratic form at the 1/255 edge (flips seen at cfg 2 had margins 4-21)
FLIP_EXCLUDE = 64.0
REF_CASES = {   # name: (n, W, H, sh_degree, seed, opacity_scale, bg)
    # BASELINE.json configs[1]: 100k Gaussians, 800x800, SH degree 3, forward + backward, saturating opacities
    "ref_cfg2_100k_800_sh3": (100_000, 800, 800, 3, 0, 1.0, (0.0, 0.0, 0.0)),
    # a saturated SH-3 mini scene on the training config's white background (configs/train_gs.yaml:40)
    "ref_sat_sh3_20k_white": (20_000, 320, 240, 3, 12, 1.0, (1.0, 1.0, 1.0)),
}
REF_GRAD_SUBSET = 10_000


def case_inputs(name):
    """A reference case's scene, camera, background and upstream gradients as torch CPU tensors, exactly as the
    generator drew them (Gaussians with z_view <= 0.5 dropped: SURVEY Appendix A4)."""
    n, W, H, deg, seed, osc, bg = REF_CASES[name]
    sc = make_scene(n, sh_degree=deg, seed=seed, opacity_scale=osc)
    cam = make_camera(W, H)
    ph = torch.cat([sc.means3D, torch.ones(n, 1)], 1) @ cam.viewmatrix
    keep = ph[:, 2] > 0.5
    sc = Scene(*(t[keep].contiguous() for t in (sc.means3D, sc.scales, sc.rotations, sc.opacities, sc.shs)), deg)
    dc, di = make_upstream(W, H, seed)
    return sc, cam, torch.tensor(bg, dtype=torch.float32), dc, di


# Inputs a reference fixture stores instead of regenerating them: everything the generator forms with more than a
# seeded randn and one rounding (scales = exp(...), opacities = sigmoid(...), rotations = normalize(...), the camera's
# inverse and matrix products) can round differently on another CPU's vector units.  The rest -- means3D, shs and the
# upstream gradients, plain randn (x 0.3) -- is regenerated and checked against the fixture's SHA-256.
REF_STORED_INPUTS = ("scales", "rotations", "opacities", "viewmatrix", "projmatrix", "campos")


def input_hash(sc, cam, dc, di) -> str:
    import hashlib
    h = hashlib.sha256()
    for t in (sc.means3D, sc.shs, dc, di):
        h.update(np.ascontiguousarray(t.numpy(), np.float32).tobytes())
    return h.hexdigest()


def ref_grad_subset(n_gauss: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed + 1000)
    return np.sort(rng.choice(n_gauss, size=min(REF_GRAD_SUBSET, n_gauss), replace=False)).astype(np.int32)


def shuffle_bytes(a) -> np.ndarray:
    """float32 array -> (4, n) uint8 byte planes (compresses about 2x better in an npz)."""
    return np.ascontiguousarray(np.ascontiguousarray(a, np.float32).view(np.uint8).reshape(-1, 4).T)


def unshuffle_bytes(planes, shape) -> np.ndarray:
    return np.ascontiguousarray(planes.T).view(np.float32).reshape(tuple(int(s) for s in shape))


def load_ref_golden(name: str) -> dict:
    """A make_golden_ref.py fixture: the regenerated inputs (their SHA-256 checked against the fixture's), the
    reference outputs, the kept-pixel mask and the masked upstream gradients the reference's backward used."""
    z = load_golden(name)
    out = {k: v for k, v in z.items() if not k.startswith("shape_")}
    for k in z:
        if k.startswith("shape_"):
            out[k[6:]] = unshuffle_bytes(z[k[6:]], z[k])
    sc, cam, bg, dc, di = case_inputs(name)
    h = input_hash(sc, cam, dc, di)
    assert h == str(z["input_sha256"]), f"{name}: regenerated inputs differ from the generator's ({h})"
    n, W, H = REF_CASES[name][:3]
    mask = np.unpackbits(z["mask_bits"])[:W * H].reshape(H, W).astype(bool)
    out["mask"] = mask
    out["inp"] = dict(means3D=sc.means3D.numpy(), shs=sc.shs.numpy(), bg=bg.numpy(),
                      tanfovx=cam.tanfovx, tanfovy=cam.tanfovy, image_height=H, image_width=W,
                      sh_degree=sc.sh_degree, scale_modifier=1.0,
                      **{k: out.pop("input_" + k) for k in REF_STORED_INPUTS})
    out["dL_dcolor"] = (dc * torch.from_numpy(mask.astype(np.float32))).numpy()
    out["dL_dinvdepth"] = (di * torch.from_numpy(mask.astype(np.float32))).numpy()
    return out


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def close_fraction(a, b, atol, rtol=0.0) -> float:
    """Fraction of elements with |a-b| <= atol + rtol*|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.mean(np.abs(a - b) <= atol + rtol * np.abs(b)))


REF_COLOR_TOL = 1e-5   # forward values ~1e-5 relative (relative L2 over the compared pixels)
REF_PIXEL_TOL = 1e-4   # one pixel: each contributor's alpha carries the exponent difference of the two geometry
                       # orders (up to ~5e-5 of the exponent at the 1/255 edge, measured at cfg 2), so a pixel moves by
                       # up to (1 - T) max|colour| x that: 10x A13's figure bounds it with room
REF_GRAD_TOL = 1e-4    # A13: gradients ~1e-4 relative L2
REF_FLIP_TOL = 2e-2    # a threshold-flip candidate pixel: one alpha = 1/255 decision moves it by < alpha T


def compare_to_reference(z: dict, color, invdepth, radii, final_T, rgb_max: float, margin, grads=None,
                         record=None) -> dict:
    """One rasterizer's outputs (the HIP path or the oracle) against a make_golden_ref.py fixture.

    * radii: equal on every Gaussian this rasterizer renders (radius > 0; the reference keeps a nonzero radius on
      some off-screen Gaussians, Appendix A4);
    * colour / inverse depth on the fixture's mask (pixels the CUDA rule never stops, less the threshold-flip
      candidates): relative L2 within REF_COLOR_TOL (A13's forward tolerance) and every pixel within REF_PIXEL_TOL;
    * every other pixel: a pixel the CUDA rule stops with transmittance T left differs from the Python rule's value by
      at most T * max(|colour|, |background|) (A2/A3: the Python walk adds Gaussians whose weights, background
      included, sum to at most T), plus REF_PIXEL_TOL; a threshold-flip candidate (margin < FLIP_EXCLUDE) within
      REF_FLIP_TOL;
    * gradients of the fixture's Gaussian subset (the reference's backward saw upstream gradients only on the mask):
      relative L2 within REF_GRAD_TOL, A13's gradient tolerance."""
    m = z["mask"]
    cerr = np.abs(np.asarray(color) - z["ref_color"]).max(0)
    iref = z["ref_invdepth"][0]
    ierr = np.abs(np.asarray(invdepth)[0] - iref) / np.maximum(np.abs(iref), 1.0)
    on = np.asarray(radii) > 0
    bg_max = float(np.abs(z["inp"]["bg"]).max())
    bound = np.asarray(final_T) * max(rgb_max, bg_max) + REF_PIXEL_TOL
    cand = np.asarray(margin) < FLIP_EXCLUDE
    rest = ~m & ~cand
    rec = dict(pixels=int(m.size), mask_pixels=int(m.sum()), flip_candidates=int(cand.sum()),
               radii_mismatch_rendered=int((np.asarray(radii)[on] != z["ref_radii"][on]).sum()),
               color_maxabs_mask=float(cerr[m].max(initial=0)), invdepth_maxrel_mask=float(ierr[m].max(initial=0)),
               color_rel_l2_mask=rel_l2(np.asarray(color)[:, m], z["ref_color"][:, m]),
               invdepth_rel_l2_mask=rel_l2(np.asarray(invdepth)[0][m], iref[m]),
               stopped_pixels_over_bound=int((cerr[rest] > bound[rest]).sum()),
               stopped_worst_fraction_of_bound=float((cerr[rest] / bound[rest]).max(initial=0)),
               candidate_color_maxabs=float(cerr[cand].max(initial=0)))
    if grads is not None:
        idx = z["grad_idx"]
        for k in GRAD_KEYS:
            rec["grad_" + k] = rel_l2(np.asarray(grads[k])[idx], z["ref_grad_" + k])
    if record is not None:  # before the asserts: a failing case still leaves its achieved errors
        record(rec)
    assert rec["radii_mismatch_rendered"] == 0, rec
    assert rec["color_rel_l2_mask"] <= REF_COLOR_TOL and rec["invdepth_rel_l2_mask"] <= REF_COLOR_TOL, rec
    assert rec["color_maxabs_mask"] <= REF_PIXEL_TOL and rec["invdepth_maxrel_mask"] <= REF_PIXEL_TOL, rec
    assert rec["stopped_pixels_over_bound"] == 0, rec
    assert rec["candidate_color_maxabs"] <= REF_FLIP_TOL, rec
    for k in GRAD_KEYS:
        if "grad_" + k in rec:
            assert rec["grad_" + k] <= REF_GRAD_TOL, (k, rec)
    return rec
