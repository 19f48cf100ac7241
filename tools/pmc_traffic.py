#!/usr/bin/env python
"""Per-stage HBM traffic of the rasterizer from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py CONFIG OUT.json PMC_DIR...

Writes {CONFIG: {stage: {"hbm_bytes_per_launch", "read_bytes", "write_bytes", "kernel"}}} (merged into OUT.json
if it exists), which bench.py reads for roofline.traffic.  Correction per MI355X_MICROARCH.md §HBM: read bytes =
2 x FETCH_SIZE (KiB), write bytes = WRITE_SIZE (KiB).  Stages (tools/pmc_stages.py) match the library's profiler
stages; multi-kernel stages (the radix sorts, the scans) are per-step sums over their kernels.

The read factor is taken from profiles/pmc_gather_calib.json when present (tools/probes/gather_probe.hip, round 4):
FETCH_SIZE counted exactly 0.50 of 128 B per distinct line for streaming reads, whole random lines, and random 4-B and
16-B gathers alike (0.545 for 48-B records, which straddle lines), so one factor, 1 / 0.50, converts every read
pattern of this path to bytes of 128-B lines fetched.  WRITE_SIZE counted 32 B per random 4- or 8-B store (one
sector) and the full bytes of coalesced stores; the probe's random stores took as long as writing their whole lines.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_stages import stage_totals  # noqa: E402


def main():
    cfg, out_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res, steps = stage_totals(dirs)
    read_factor = 2.0
    calib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                         "pmc_gather_calib.json")
    if os.path.exists(calib):  # the measured streaming factor (the gathers' agree, see above)
        read_factor = 1.0 / json.load(open(calib))["stream16"]["counted_per_line128"]
    table = {}
    for st, cs in res.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = read_factor * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        table[st] = {"kernel": " + ".join(cs["kernels"]), "read_bytes": round(rd), "write_bytes": round(wr),
                     "hbm_bytes_per_launch": round(rd + wr)}
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[cfg] = table
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps({"steps": steps, "stages": table}, indent=1))


if __name__ == "__main__":
    main()
