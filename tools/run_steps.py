#!/usr/bin/env python
"""Run K forward+backward steps of a BASELINE config (the profiling target for rocprofv3).

    rocprofv3 --pmc SQ_WAVES ... -- python tools/run_steps.py --config cfg3 --steps 3
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--knob", action="append", default=[])
    args = ap.parse_args()
    import torch
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    for k in args.knob:
        n, v = k.split("=")
        _native.set_tuning(n, int(v))
    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    for _ in range(args.steps):
        c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
        backward_raw(st, rs, dc, di)
    torch.cuda.synchronize()
    print("instances", st.num_rendered)


if __name__ == "__main__":
    main()
