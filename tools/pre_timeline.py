#!/usr/bin/env python
"""Per-wave phase timeline of the preprocess kernel (diagnostics): one forward with the "stamp" knob, then per wave
the time from its start to the end of the projection + colour (preprocess_gaussian), to the end of the wave-balanced
tile culling, and to its exit (block totals, atomics, ticket), with the resident waves per SIMD over the launch.

    python tools/pre_timeline.py --config cfg3 [--knob name=value ...]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarise(st, n_waves):
    import numpy as np
    a = st[: 2 * n_waves].astype(np.int64).reshape(-1, 2, 4)
    ok = a[:, 0, 3] != 0
    a = a[ok]
    t = a[:, 0, :]
    hw, xcc = a[:, 1, 0], a[:, 1, 1]
    base = t[:, 0].min()
    t = (t - base) * 10.0  # ns (100 MHz clock)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    nsimd = len(np.unique(key))
    span = t[:, 3].max()
    q = lambda x, p: round(float(np.percentile(x, p)) / 1000, 2)  # noqa: E731
    phase = {"proj": t[:, 1] - t[:, 0], "cull": t[:, 2] - t[:, 1], "tail": t[:, 3] - t[:, 2], "wave": t[:, 3] - t[:, 0]}
    bins = np.arange(0, span + 1000, 1000)
    res = np.zeros(len(bins))
    for s, e in zip(t[:, 0], t[:, 3]):
        res[int(s // 1000):int(e // 1000) + 1] += 1
    res /= nsimd
    starts = np.sort(t[:, 0])
    return {
        "waves": int(len(t)), "simds": int(nsimd), "span_us": round(span / 1000, 1),
        "phase_us": {k: {"mean": round(float(v.mean()) / 1000, 2), "p50": q(v, 50), "p90": q(v, 90), "max": q(v, 100)}
                     for k, v in phase.items()},
        "phase_share": {k: round(float(v.sum() / phase["wave"].sum()), 3) for k, v in phase.items() if k != "wave"},
        "start_us_by_decile": [q(starts, p) for p in range(0, 101, 10)],
        "resident_waves_per_simd_by_5us": [round(float(res[i:i + 5].mean()), 2) for i in range(0, len(res), 5)],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--knob", action="append", default=[])
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
    for k in args.knob:
        n, v = k.split("=")
        _native.set_tuning(n, int(v))
    for _ in range(3):
        forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    torch.cuda.synchronize()
    _native.set_tuning("stamp", 1)
    forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    torch.cuda.synchronize()
    _native.set_tuning("stamp", 0)
    n_waves = min((cfg["n"] + 63) // 64, (1 << 16) // 2)
    st = _native.wave_stamps(3, 2 * n_waves)
    print(json.dumps(summarise(st, n_waves), indent=1))


if __name__ == "__main__":
    main()
