#!/usr/bin/env python
"""Dump per-tile work statistics of one cfg forward (instances per tile, loaded, last contributor) to npz."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--out", default="gpurun_out/tile_stats.npz")
    args = ap.parse_args()
    import torch
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    _, _, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    torch.cuda.synchronize()
    lay = _native.state_layout(cfg["n"], st.num_rendered, cfg["W"], cfg["H"])
    T = ((cfg["W"] + 15) // 16) * ((cfg["H"] + 15) // 16)
    img = st.image_buffer
    rg = img[lay["img_ranges"]: lay["img_ranges"] + 8 * T].view(torch.int32).view(T, 2).cpu().numpy()
    tl = img[lay["img_tile_last"]: lay["img_tile_last"] + 4 * T].view(torch.int32).cpu().numpy()
    ld = img[lay["img_tile_loaded"]: lay["img_tile_loaded"] + 4 * T].view(torch.int32).cpu().numpy()
    np.savez(args.out, ranges=rg, tile_last=tl, tile_loaded=ld, W=cfg["W"], H=cfg["H"])
    print("tiles", T, "instances", st.num_rendered, "max len", int((rg[:, 1] - rg[:, 0]).max()))


if __name__ == "__main__":
    main()
