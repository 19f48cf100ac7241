#!/usr/bin/env python
"""Per-stage numbers for DESIGN.md §4 from one round profile: kernel time (rocprofv3 --stats average, or the bench
line's stage events when no trace is given), HBM traffic per launch (profiles/pmc_traffic.json), achieved TB/s and
the VALU issue fraction (profiles/pmc_insts.json priced with the measured issue costs: 1.29 ns per VALU and 3.5 ns
per transcendental wave-instruction per SIMD, 1024 SIMDs).

    python tools/design_table.py cfg3 profiles/pmc_traffic.json profiles/pmc_insts.json [kernel_stats.csv | bench.json]
"""
import csv
import json
import sys

NS_VALU, NS_TRANS, SIMDS = 1.29, 3.5, 1024
# SURVEY.md §8(d) algorithmic bytes per work unit, and the bound, per stage (G Gaussians, I instances, T tiles, M = 16)
ALGO = {
    "preprocess": ("G (40 + 12M) read + 113 write = 345 B/G", "HBM / latency"),
    "bucket_count_walk": ("20 B/G read + 4 B/G offsets + 256 T 4-B count rows", "latency"),
    "bucket_columns": ("2 x the count matrix + 32 B/T", "latency"),
    "bucket_scatter": ("28 B/G read + 16 B/I write (key 8, inst_gid 4, inv 4)", "stores"),
    "bucket_partition": ("8 B/I read + 8 B/I write", "latency"),
    "seg_sort": ("8 B/I read + 4 B/I write", "VALU / LDS"),
    "render_fwd": ("8 B/T + 44 B/I loaded + 24 B/px (+4 B inv + 1 B strip mask per loaded I)", "**VALU issue**"),
    "render_bwd": ("8 B/T + 44 B/I walked + 40 B/I gradient rows + 1 B strip mask + G (56 + 12M) zero fill",
                   "**VALU issue**"),
    "big_reduce": ("rows of > 64-tile Gaussians", "latency"),
    "preprocess_bwd": ("12 B/G + 4 B/I + 40 B/row read; G' (76 read + 56 + 12M write), G' = non-zero Gaussians",
                       "HBM / latency"),
    "depth_sort": ("3 passes x (4 B key + 4 B value) x 2 x G", "HBM / latency"),
    "instance_scan": ("8 B/G", "latency"),
    "expand": ("records 16 B/G + 2 B key, 4 B value, 4 B inv per I", "stores"),
    "tile_sort": ("2 passes x (2 B key + 4 B value) x (read 2 + write 1) per I", "HBM / latency"),
    "tile_ranges": ("2 B/I read", "HBM"),
}


def kernel_times(path):
    """stage -> ms from a rocprofv3 kernel_stats.csv (matched by kernel name), else from a bench line's stages_ms."""
    if path.endswith(".csv"):
        return {r["Name"]: float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(path))}
    t = open(path).read()
    d = json.loads(t[t.index('{"metric'):].splitlines()[0])
    return d.get("stages_ms", {})


def main():
    cfg, traffic, insts = sys.argv[1], json.load(open(sys.argv[2])), json.load(open(sys.argv[3]))
    times = kernel_times(sys.argv[4]) if len(sys.argv) > 4 else {}
    tr, ins = traffic.get(cfg, {}), insts.get(cfg, {})
    print("| stage | kernel | algorithmic bytes | bound | ms | HBM MB / launch | TB/s | VALU issue |")
    print("|---|---|---|---|---|---|---|---|")
    for stage, t in tr.items():
        if not isinstance(t, dict):
            continue
        kern = t.get("kernel", "")
        ms = None
        for name, v in times.items():
            if kern and kern.split("<")[0] in name and (("<" not in kern) or kern.split("<")[1][:8] in name):
                ms = v
                break
        if ms is None:
            ms = times.get(stage)
        mb = t["hbm_bytes_per_launch"] / 1e6
        i = ins.get(stage, {})
        issue = None
        if ms and i:
            per_simd_ms = ((i["valu"] - i["trans"]) * NS_VALU + i["trans"] * NS_TRANS) / SIMDS / 1e6
            issue = per_simd_ms / ms
        algo, bound = ALGO.get(stage, ("", ""))
        head = f"| {stage} | `{kern.split(' + ')[0][:60]}` | {algo} | {bound} "
        print(head + (f"| {ms:.4f} | {mb:.0f} | {mb / 1e3 / ms:.2f} | {issue:.2f} |" if ms and issue is not None
                      else f"| {ms:.4f} | {mb:.0f} | {mb / 1e3 / ms:.2f} | - |" if ms else f"| - | {mb:.0f} | - | - |"))


if __name__ == "__main__":
    main()
