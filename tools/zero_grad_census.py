#!/usr/bin/env python
"""Census of Gaussians whose backward gradients are identically zero (culled, or no loaded instance / no contribution)
at a bench config: the share of preprocess_bwd's per-Gaussian stores that only write zeros.

    python tools/zero_grad_census.py [--config cfg3]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    args = ap.parse_args()
    import torch
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    _, radii, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    g = backward_raw(st, rs, dc, di)
    torch.cuda.synchronize()
    n = radii.numel()
    nz = torch.zeros(n, dtype=torch.bool, device=dev)
    for k, v in g.items():
        if v is not None and v.dim() >= 1 and v.shape[0] == n:
            nz |= (v.reshape(n, -1) != 0).any(dim=1)
    out = {"config": args.config, "gaussians": n, "culled": int((radii <= 0).sum()),
           "visible_zero_grad": int(((radii > 0) & ~nz).sum()), "nonzero_grad": int(nz.sum()),
           "fields": sorted(k for k, v in g.items() if v is not None)}
    out["zero_fraction"] = round(1 - out["nonzero_grad"] / n, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
