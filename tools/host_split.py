#!/usr/bin/env python
"""Where a forward + backward step's host time goes on a scene too small to keep the GPU busy: time spent inside
gsr_forward / gsr_backward (the forward includes its readback wait) against the Python wrapper around them, and
the allocation callback.

    python tools/host_split.py [--n 2000] [--steps 50]
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
    args = ap.parse_args()
    import torch
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd import rasterizer as R
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream
    dev = torch.device("cuda", 0)
    sc = make_scene(args.n, 3, seed=0).to(dev)
    cam = make_camera(1920, 1080).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(1920, 1080, 0))
    rs = R.GaussianRasterizationSettings(1080, 1920, cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                         cam.viewmatrix, cam.projmatrix, 3, cam.campos, False, False, False)
    lib = _native.load()
    acc = {"fwd_lib": 0.0, "bwd_lib": 0.0, "step": 0.0, "alloc": 0.0, "n_alloc": 0}
    f0, b0 = lib.gsr_forward, lib.gsr_backward

    def tf(*a):
        t = time.perf_counter(); r = f0(*a); acc["fwd_lib"] += time.perf_counter() - t; return r

    def tb(*a):
        t = time.perf_counter(); r = b0(*a); acc["bwd_lib"] += time.perf_counter() - t; return r
    lib.gsr_forward, lib.gsr_backward = tf, tb
    orig_get = R._Buffers.__init__

    for it in range(2):
        for k in acc:
            acc[k] = 0.0 if k != "n_alloc" else 0
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            c, r, i, st = R.forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
            R.backward_raw(st, rs, dc, di)
        torch.cuda.synchronize()
        acc["step"] = time.perf_counter() - t0
    out = {k: (1e3 * v / args.steps if isinstance(v, float) else v) for k, v in acc.items()}
    # the library with a null stage: one gsr_forward on the same inputs, timed around the readback alone is not
    # exposed; the stage profiler's readback stage is
    print(json.dumps(out))


if __name__ == "__main__":
    main()
