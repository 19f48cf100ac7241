#!/usr/bin/env python
"""Per-wave timeline of the composite kernels (diagnostics for the tail / imbalance question).

    python tools/wave_timeline.py --config cfg3 [--knob name=value ...] > gpurun_out/timeline.json

Runs one fwd+bwd step with the "stamp" knob, reads the (start, end, HW_ID, XCC_ID) stamps of every launch
slot and summarises, per kernel: the span, the distribution of wave durations, the busy fraction of the SIMDs
over the span (waves resident per SIMD over time), and how late the last waves finish relative to the point
where fewer than 2 waves per SIMD remain on average.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarise(st, n):
    import numpy as np
    st = st[:n].astype(np.int64)
    t0, t1, hw, xcc = st[:, 0], st[:, 1], st[:, 2], st[:, 3]
    base = t0.min()
    s, e = (t0 - base) * 10.0, (t1 - base) * 10.0  # ns (100 MHz clock)
    dur = e - s
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    span = e.max()
    nsimd = len(np.unique(key))
    # resident waves over time (1 us bins)
    bins = np.arange(0, span + 1000, 1000)
    res = np.zeros(len(bins))
    for a, b in zip(s, e):
        res[int(a // 1000):int(b // 1000) + 1] += 1
    res /= nsimd
    # per-SIMD last finish
    last = {}
    for k, b in zip(key, e):
        last[k] = max(last.get(k, 0), b)
    lasts = np.array(list(last.values()))
    q = lambda x, p: float(np.percentile(x, p))
    return {
        "waves": int(n), "simds": int(nsimd), "span_us": round(span / 1000, 1),
        "wave_us": {"p50": round(q(dur, 50) / 1000, 1), "p90": round(q(dur, 90) / 1000, 1),
                    "max": round(dur.max() / 1000, 1)},
        "first_slots_wave_us_mean(slot<1024)": round(float(dur[:1024].mean()) / 1000, 1),
        "simd_last_finish_us": {"p10": round(q(lasts, 10) / 1000, 1), "p50": round(q(lasts, 50) / 1000, 1),
                                "max": round(lasts.max() / 1000, 1)},
        "resident_waves_per_simd_by_10us": [round(float(res[i:i + 10].mean()), 2) for i in range(0, len(res), 10)],
        "slot_of_longest_waves": [int(i) for i in np.argsort(-dur)[:10]],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--knob", action="append", default=[])
    ap.add_argument("--dump", default="", help="also save the raw stamps, launch orders, ranges and tile_last (.npz)")
    args = ap.parse_args()
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
    for k in args.knob:
        n, v = k.split("=")
        _native.set_tuning(n, int(v))
    for _ in range(2):
        c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
        backward_raw(st, rs, dc, di)
    _native.set_tuning("stamp", 1)
    c, r, i, st = forward_raw(sc.means3D, sc.shs, None, sc.opacities, sc.scales, sc.rotations, None, rs)
    backward_raw(st, rs, dc, di)
    torch.cuda.synchronize()
    _native.set_tuning("stamp", 0)
    T = ((cfg["W"] + 15) // 16) * ((cfg["H"] + 15) // 16)
    # launch slots: whole tiles (render_fwd_v6 <4, 6>) unless the image is small enough for 4 row-strip parts
    # (launch_render_fwd's fwd_part_slots rule)
    nfwd = T * 4 if T * 4 <= 16384 else T
    sf = _native.wave_stamps(0, nfwd)
    # backward slots: one per tile, or one per (tile, segment) work item of the segmented walk (small images); the
    # stamp buffer starts zeroed and slots past the work list never stamp, so the stamped prefix is the launch
    import numpy as np
    sb = _native.wave_stamps(1, 1 << 16)
    nz = np.nonzero(sb[:, 1])[0]
    nbwd = int(nz.max()) + 1 if len(nz) else T
    out = {"fwd": summarise(sf, nfwd), "bwd": summarise(sb, nbwd)}
    print(json.dumps(out, indent=1))
    if args.dump:
        import numpy as np
        lay = _native.state_layout(cfg["n"], st.num_rendered, cfg["W"], cfg["H"])
        img = st.image_buffer.view(torch.uint8)
        al = lambda o: (o + 255) // 256 * 256  # noqa: E731  (Carver alignment)

        def u32(off, n):
            return img[off: off + 4 * n].view(torch.int32).cpu().numpy().view(np.uint32)
        o_fwd = al(lay["img_tile_loaded"] + 4 * (T + 1))
        o_bwd = al(o_fwd + 4 * (T + 1))
        np.savez(args.dump, fwd=np.asarray(sf)[:nfwd], bwd=np.asarray(sb)[:nbwd], order_fwd=u32(o_fwd, T),
                 order_bwd=u32(o_bwd, T), ranges=u32(lay["img_ranges"], 2 * T).reshape(T, 2),
                 tile_last=u32(lay["img_tile_last"], T))


if __name__ == "__main__":
    main()
