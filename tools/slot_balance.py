#!/usr/bin/env python
"""Per-SIMD work balance of the whole-tile forward composite from a wave_timeline.py --dump file.

    python tools/slot_balance.py gpurun_out/tl/a.npz [gpurun_out/tl/b.npz]

Reports how the launch slots of render_fwd were placed on SIMDs (from each wave's HW_ID / XCC_ID), the spread of
the per-SIMD sums of tile weights (range lengths) against the per-SIMD finish times, and, with two dumps, whether
the slot -> CU placement repeats between launches.
"""
import sys

import numpy as np


def simd_keys(st):
    st = st.astype(np.int64)
    hw, xcc = st[:, 2], st[:, 3]
    simd, cu, sh, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
    cu_key = (((xcc & 15) * 8 + se) * 2 + sh) * 16 + cu
    return cu_key * 4 + simd, cu_key


def main():
    d = [np.load(p) for p in sys.argv[1:]]
    for z in d:
        st = z["fwd"].astype(np.int64)
        n = len(st)
        key, cu = simd_keys(st)
        rg = z["ranges"]
        order = z["order_fwd"][:n]
        w = (rg[order, 1] - rg[order, 0]).astype(np.float64)
        end = (st[:, 1] - st[:, 0].min()) * 10.0 / 1000  # us
        u, inv = np.unique(key, return_inverse=True)
        wsum = np.bincount(inv, weights=w)
        fin = np.zeros(len(u))
        np.maximum.at(fin, inv, end)
        cnt = np.bincount(inv)
        print(f"slots {n}, SIMDs {len(u)}, waves/SIMD {cnt.min()}..{cnt.max()}")
        print(f"  per-SIMD weight sum: mean {wsum.mean():.0f} p10 {np.percentile(wsum, 10):.0f} "
              f"p90 {np.percentile(wsum, 90):.0f} max {wsum.max():.0f}")
        print(f"  per-SIMD finish us:  mean {fin.mean():.1f} p10 {np.percentile(fin, 10):.1f} "
              f"p90 {np.percentile(fin, 90):.1f} max {fin.max():.1f}; corr(weight sum, finish) "
              f"{np.corrcoef(wsum, fin)[0, 1]:.2f}")
        wg = np.arange(n) // 4
        cu_of_wg = cu[::4]
        print("  WG -> CU for WG 0..7:", cu_of_wg[:8], " WG 256..263:", cu_of_wg[256:264])
        # same-CU workgroups: how far apart are their WG ids
        first = {}
        gaps = []
        for i, c in enumerate(cu_of_wg):
            if c in first:
                gaps.append(i - first[c])
            first[c] = i
        print("  WG id gap between consecutive WGs on one CU: median", int(np.median(gaps)), "p10",
              int(np.percentile(gaps, 10)), "p90", int(np.percentile(gaps, 90)))
    if len(d) == 2:
        a, b = (simd_keys(z["fwd"].astype(np.int64))[1] for z in d)
        m = min(len(a), len(b))
        print(f"slot -> CU identical between the two launches for {np.mean(a[:m] == b[:m]):.3f} of slots")


if __name__ == "__main__":
    main()
