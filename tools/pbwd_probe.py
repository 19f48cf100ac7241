#!/usr/bin/env python
"""Time preprocess_bwd with and without the dL/dshs writes (compact_sh) on cfg3, interleaved."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    cfg = CONFIGS["cfg3"]
    dev = torch.device("cuda", 0)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    _, _, _, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    res = {}
    for rnd in range(6):
        for mode in ("dense", "compact"):
            _native.reset_stage_times()
            _native.set_profiling(True)
            for _ in range(5):
                backward_raw(st, rs, dc, di, compact_sh=(mode == "compact"))
            torch.cuda.synchronize()
            _native.set_profiling(False)
            t = _native.stage_times()["preprocess_bwd"]
            res.setdefault(mode, []).append(t[0] / t[1])
    print({k: round(float(np.median(v)), 4) for k, v in res.items()})


if __name__ == "__main__":
    main()
