#!/usr/bin/env python
"""Predicted N-GPU step of bench.py (one view per GPU, cfg 3) from multiview.plan_exchange's cost model.

    python tools/exchange_plan.py [--n 1000000] [--local-ms 0.716] [--efficiency 0.3 0.6 1.0]

local-ms: the measured one-view step without its per-Gaussian backward stage (N = 1 bench line minus
preprocess_bwd), which every rank runs before the exchange.  Prints one row per (world size, bus efficiency).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--local-ms", type=float, default=0.716)
    ap.add_argument("--step1-ms", type=float, default=0.820)
    ap.add_argument("--efficiency", type=float, nargs="+", default=[0.3, 0.6, 1.0])
    args = ap.parse_args()
    from gaussian_splatting_lightning_amd.multiview import EXCHANGE_COSTS, plan_exchange
    rows = []
    for N in (2, 4, 8):
        for eff in args.efficiency:
            p = plan_exchange(args.n, N, costs=dict(bus_efficiency=eff))
            step = args.local_ms + p["end_ms"]
            rows.append({"gpus": N, "bus_efficiency": eff,
                         "bus_GBps": round(EXCHANGE_COSTS["link_GBps"] * EXCHANGE_COSTS["links"] * eff, 1),
                         "plan": f'{p["mode"]} K={p["chunks"]} expand={p["expand"]}', "link_MB_per_rank": p["link_MB"],
                         "comm_ms": p["comm_ms"], "exposed_ms": p["exposed_ms"], "step_ms": round(step, 3),
                         "efficiency_vs_1gpu": round(args.step1_ms / step, 3)})
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
