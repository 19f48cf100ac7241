#!/usr/bin/env python
"""Host floor of one forward + backward step: the same calls as bench.py on a scene too small to keep the GPU busy
(the step time is then the host's issue time plus the forward's one readback round trip).

    python tools/host_floor.py [--n 2000] [--steps 50]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    args = ap.parse_args()
    import torch
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    dev = torch.device("cuda", 0)
    sc = make_scene(args.n, 3, seed=0).to(dev)
    cam = make_camera(args.W, args.H).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(args.W, args.H, 0))
    rs = GaussianRasterizationSettings(args.H, args.W, cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, 3, cam.campos, False, False, False)
    res = {}
    for name, bwd in (("fwd", False), ("fwd_bwd", True)):
        for _ in range(10):
            c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
            if bwd:
                backward_raw(st, rs, dc, di)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
            if bwd:
                backward_raw(st, rs, dc, di)
        torch.cuda.synchronize()
        res[name + "_ms"] = 1e3 * (time.perf_counter() - t0) / args.steps
    print(json.dumps(res))


if __name__ == "__main__":
    main()
