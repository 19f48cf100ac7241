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


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def close_fraction(a, b, atol, rtol=0.0) -> float:
    """Fraction of elements with |a-b| <= atol + rtol*|b|."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.mean(np.abs(a - b) <= atol + rtol * np.abs(b)))
