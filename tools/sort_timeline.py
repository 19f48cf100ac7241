#!/usr/bin/env python
"""Per-block timeline of the depth sort's multi-histogram and last onesweep pass (diagnostics).

    python tools/sort_timeline.py --config cfg3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--knob", action="append", default=[], help="name=value tuning knob set before the runs")
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
    st_ = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)[3]
    torch.cuda.synchronize()
    _native.set_tuning("stamp", 0)
    n = cfg["n"]
    if cfg["W"] * cfg["H"] > 16384 * 256:  # radix path: the tile sort ran last
        n = st_.num_rendered
    nb = (n + 4095) // 4096
    hb = min((n + 2047) // 2048, 2048)
    out = {}
    for name, which, cnt in (("onesweep_last_pass", 2, nb), ("multi_hist", 3, hb)):
        st = _native.wave_stamps(which, cnt).astype(np.int64)
        base = st[:, 0].min()
        rel = (st[:, :3] - base) * 10 / 1000.0 if which == 3 else (st - base) * 10 / 1000.0  # us
        q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 50, 90, 100)]
        if which == 2:
            out[name] = {"blocks": cnt, "start_us[min,p50,p90,max]": q(rel[:, 0]),
                         "rank_us": q(rel[:, 1] - rel[:, 0]), "lookback_us": q(rel[:, 2] - rel[:, 1]),
                         "scatter_us": q(rel[:, 3] - rel[:, 2]), "end_us": q(rel[:, 3]),
                         "lookback_us_by_block_decile": [round(float(np.mean((rel[:, 2] - rel[:, 1])[i::10])), 2)
                                                         for i in range(10)]}
        else:
            out[name] = {"blocks": cnt, "start_us": q(rel[:, 0]), "loop_us": q(rel[:, 1] - rel[:, 0]),
                         "global_atomics_us": q(rel[:, 2] - rel[:, 1]), "end_us": q(rel[:, 2])}
    out["n"] = n
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
