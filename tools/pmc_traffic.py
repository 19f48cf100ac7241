#!/usr/bin/env python
"""Per-launch HBM traffic of the rasterizer kernels from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

    python tools/pmc_traffic.py CONFIG OUT.json PMC_DIR...

Writes {CONFIG: {stage: {"hbm_bytes_per_launch", "read_bytes", "write_bytes", "kernel"}}} (merged into OUT.json
if it exists), which bench.py reads for roofline.traffic.  Correction per MI355X_MICROARCH.md §HBM: read bytes =
2 x FETCH_SIZE (KiB), write bytes = WRITE_SIZE (KiB).  Stage names match the library's profiler stages.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load, short  # noqa: E402

STAGE_OF = {
    "render_fwd": "render_fwd", "render_bwd": "render_bwd", "preprocess_kernel": "preprocess",
    "preprocess_bwd": "preprocess_bwd", "expand_kernel": "expand", "big_reduce": "big_reduce",
    "bk_walk_kernel<false": "bucket_count_walk", "bk_walk_kernel<true": "bucket_scatter",
    "bk_columns": "bucket_columns", "seg_sort_kernel": "seg_sort",
}


def stage_of(kernel):
    for k, v in STAGE_OF.items():
        if k in kernel:
            return v
    return None


def main():
    cfg, out_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = load(dirs)
    table = {}
    for name, cs in res.items():
        st = stage_of(short(name))
        if st is None or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        rd = 2.0 * cs["FETCH_SIZE"] * 1024
        wr = cs["WRITE_SIZE"] * 1024
        table[st] = {"kernel": short(name), "read_bytes": round(rd), "write_bytes": round(wr),
                     "hbm_bytes_per_launch": round(rd + wr)}
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[cfg] = table
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()
