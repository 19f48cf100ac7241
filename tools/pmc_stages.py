#!/usr/bin/env python
"""Per-stage, per-step totals of rocprofv3 --pmc counters for the rasterizer pipeline.

The radix binning path launches the same sort / scan kernels for two stages (the depth sort of the P Gaussians and
the tile sort of the R instances), so kernels are attributed to stages by their position in the dispatch stream of
one step rather than by name: after preprocess_kernel, sort and scan kernels belong to the depth sort (the scan
look-back right after it is the instance scan); after expand_kernel they belong to the tile sort.  Counter values
are summed over a stage's dispatches and divided by the number of steps (preprocess_kernel dispatches), i.e. a
per-step figure that equals the per-launch figure for single-kernel stages.

    python tools/pmc_stages.py PMC_DIR...          # prints {stage: {counter: per-step value, "kernels": [...]}}
"""
import collections
import csv
import glob
import json
import os
import sys

FIXED = [  # (substring of the kernel name, stage) for kernels that always belong to one stage
    ("preprocess_kernel", "preprocess"), ("preprocess_color_kernel", "preprocess_color"),
    ("preprocess_bwd_kernel", "preprocess_bwd"),
    ("render_fwd", "render_fwd"), ("render_bwd", "render_bwd"), ("big_reduce", "big_reduce"),
    ("bk_walk_kernel<false", "bucket_count_walk"), ("bk_walk_kernel<true", "bucket_scatter"),
    ("bk_partition_kernel", "bucket_partition"),
    ("bk_columns", "bucket_columns"), ("seg_sort_kernel", "seg_sort"),
    ("expand_owner_kernel", "expand"), ("expand_kernel", "expand"), ("identify_ranges", "tile_ranges"),
    ("tile_order_kernel", "tile_order"), ("sh_backward_views", "sh_views"),
]
SORT_LIKE = ("rs_", "scan_")  # radix sort and scan kernels: stage from the dispatch position


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gsr::", "")


def _rows(dirs):
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            yield from csv.DictReader(open(f))


def stage_totals(dirs):
    disp = {}  # dispatch id -> (kernel, {counter: value summed over instances})
    for row in _rows(dirs):
        did = int(row.get("Dispatch_Id") or row.get("Dispatch-Id"))
        name = short(row.get("Kernel_Name") or row.get("Kernel-Name") or "")
        cname = row.get("Counter_Name") or row.get("Counter-Name")
        val = float(row.get("Counter_Value") or row.get("Counter-Value"))
        k, cs = disp.setdefault(did, (name, collections.defaultdict(float)))
        cs[cname] += val
    totals = collections.defaultdict(lambda: collections.defaultdict(float))
    kernels = collections.defaultdict(set)
    steps = 0
    phase = None  # position inside the forward: None, "after_preprocess", "after_scan", "after_expand"
    for did in sorted(disp):
        name, cs = disp[did]
        stage = None
        for sub, st in FIXED:
            if sub in name:
                stage = st
                break
        if stage == "preprocess":
            steps += 1
            phase = "after_preprocess"
        elif stage == "expand":
            phase = "after_expand"
        elif stage is None and name.startswith(SORT_LIKE):
            if phase == "after_preprocess" and name.startswith("scan_lookback"):
                stage, phase = "instance_scan", "after_scan"
            elif phase == "after_preprocess":
                stage = "depth_sort"
            elif phase == "after_scan":
                stage = "instance_scan"
            elif phase == "after_expand":
                stage = "tile_sort"
        if stage is None:
            continue
        kernels[stage].add(name)
        for c, v in cs.items():
            totals[stage][c] += v
    out = {}
    for st, cs in totals.items():
        out[st] = {c: v / max(steps, 1) for c, v in cs.items()}
        out[st]["kernels"] = sorted(kernels[st])
    return out, steps


if __name__ == "__main__":
    res, steps = stage_totals(sys.argv[1:])
    print(json.dumps({"steps": steps, "stages": res}, indent=1))
