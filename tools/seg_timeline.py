#!/usr/bin/env python
"""Per-tile timeline of the bucket path's workgroup sorts (long tiles): start, chunk-sort and merge durations.

    python tools/seg_timeline.py --config cfg3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--knob", action="append", default=[], help="name=value tuning knob, repeatable")
    args = ap.parse_args()
    import numpy as np
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
    for kv in args.knob:
        k, v = kv.split("=")
        _native.set_tuning(k, int(v))
    for _ in range(2):
        forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    _native.set_tuning("stamp", 1)
    forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    torch.cuda.synchronize()
    _native.set_tuning("stamp", 0)
    st = _native.wave_stamps(2, 1 << 16).astype(np.int64)
    st = st[st[:, 3] > 0]
    base = st[:, 0].min()
    us = lambda x: x * 10 / 1000.0  # noqa: E731  (100 MHz clock)
    q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 25, 50, 75, 100)]  # noqa: E731
    out = {"long_tiles": int(len(st)), "start_us": q(us(st[:, 0] - base)), "chunk_sort_us": q(us(st[:, 1] - st[:, 0])),
           "merge_us": q(us(st[:, 2] - st[:, 1])), "end_us": q(us(st[:, 2] - base)), "n": q(st[:, 3])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
