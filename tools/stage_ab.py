#!/usr/bin/env python
"""Interleaved A/B of tuning knobs in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/stage_ab.py --config cfg3 --knob bwd_occ4=0,1 [--knob other=0,1] --rounds 5 --steps 5

Every round runs each knob combination for --steps fwd+bwd steps with per-stage hipEvents on; prints the
median per-stage device time per variant and the median wall time per step.
"""
import argparse
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--knob", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch
    from bench import CONFIGS
    from gaussian_splatting_lightning_amd import _native
    from gaussian_splatting_lightning_amd.rasterizer import GaussianRasterizationSettings, backward_raw, forward_raw
    from gaussian_splatting_lightning_amd.synthetic import make_camera, make_scene, make_upstream

    cfg = CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    sc = make_scene(cfg["n"], cfg["deg"], seed=0, stress_fraction=cfg["stress"]).to(dev)
    cam = make_camera(cfg["W"], cfg["H"]).to(dev)
    dc, di = (t.to(dev) for t in make_upstream(cfg["W"], cfg["H"], 0))
    rs = GaussianRasterizationSettings(cfg["H"], cfg["W"], cam.tanfovx, cam.tanfovy, torch.zeros(3, device=dev), 1.0,
                                       cam.viewmatrix, cam.projmatrix, cfg["deg"], cam.campos, False, False, False)
    knobs = []
    for k in args.knob:
        name, vals = k.split("=")
        knobs.append([(name, int(v)) for v in vals.split(",")])
    variants = list(itertools.product(*knobs)) if knobs else [()]

    def step():
        c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
        backward_raw(st, rs, dc, di)

    for _ in range(3):
        step()
    results = {v: {"wall": []} for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            for name, val in v:
                _native.set_tuning(name, val)
            step()
            torch.cuda.synchronize()
            _native.reset_stage_times()
            _native.set_profiling(True)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            results[v]["wall"].append((time.perf_counter() - t0) / args.steps * 1e3)
            _native.set_profiling(False)
            for k, (tot, calls) in _native.stage_times().items():
                if calls:
                    results[v].setdefault(k, []).append(tot / calls)
    out = {}
    for v in variants:
        name = ",".join(f"{n}={x}" for n, x in v) or "default"
        out[name] = {k: round(float(np.median(x)), 4) for k, x in results[v].items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
