#!/usr/bin/env python
"""Per-stage HBM traffic of the rasterizer from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py CONFIG OUT.json PMC_DIR...

Writes {CONFIG: {stage: {"hbm_bytes_per_launch", "read_bytes", "write_bytes", "kernel"}}} (merged into OUT.json
if it exists), which bench.py reads for roofline.traffic.  Correction per MI355X_MICROARCH.md §HBM: read bytes =
2 x FETCH_SIZE (KiB), write bytes = WRITE_SIZE (KiB).  Stages (tools/pmc_stages.py) match the library's profiler
stages; multi-kernel stages (the radix sorts, the scans) are per-step sums over their kernels.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_stages import stage_totals  # noqa: E402


def main():
    cfg, out_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res, steps = stage_totals(dirs)
    table = {}
    for st, cs in res.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2.0 * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        table[st] = {"kernel": " + ".join(cs["kernels"]), "read_bytes": round(rd), "write_bytes": round(wr),
                     "hbm_bytes_per_launch": round(rd + wr)}
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[cfg] = table
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps({"steps": steps, "stages": table}, indent=1))


if __name__ == "__main__":
    main()
