#!/usr/bin/env python
"""Counter calibration per access pattern from tools/probes/gather_probe.hip.

    python tools/pmc_gather_calib.py FETCH_DIR WRITE_DIR [probe_stdout.txt] > profiles/pmc_gather_calib.json

Every probe kernel runs twice (warm-up on other lines, then timed); the counter total of a kernel is divided by its
dispatches.  For each pattern this reports the counted bytes per dispatch, the known bytes (requested bytes and
distinct 128-B lines touched x 128) and their ratios.  MI355X_MICROARCH.md §HBM: FETCH_SIZE is half the bytes of a
coalesced streaming read; the ratio for the gathers says what the same x2 correction means for them.
"""
import collections
import csv
import glob
import json
import os
import sys

# pattern -> (known requested bytes, distinct 128-B lines) per dispatch; must match gather_probe.hip
N = 4 << 20
TABLE = 2 << 30
KNOWN = {
    "stream16": (TABLE / 4, TABLE / 4 / 128),
    "line_full": (N * 16, N / 8),
    "gather4": (N * 4, N),
    "gather16": (N * 16, N),
    "rec48": (N * 48, N * 1.375),
    "scatter4": (N * 4, N),
    "scatter8": (N * 8, N),
    "runs8x2": (N * 8, N / 2),
}


def per_dispatch(d, counter):
    tot, disp = collections.defaultdict(float), collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = (row.get("Kernel_Name") or row.get("Kernel-Name") or "").split("(")[0].replace("void ", "")
            if (row.get("Counter_Name") or row.get("Counter-Name")) != counter:
                continue
            tot[name] += float(row.get("Counter_Value") or row.get("Counter-Value"))
            disp[name].add(row.get("Dispatch_Id") or row.get("Dispatch-Id"))
    return {k: tot[k] / max(1, len(disp[k])) for k in tot}


def main():
    fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write = per_dispatch(sys.argv[2], "WRITE_SIZE")
    timing = {}
    if len(sys.argv) > 3 and os.path.exists(sys.argv[3]):
        for line in open(sys.argv[3]):
            p = line.split()
            if len(p) > 6 and p[0] in KNOWN:
                timing[p[0]] = float(p[p.index("us") - 1])
    out = {}
    for pat, (req, lines) in KNOWN.items():
        counted = fetch.get(pat) if not pat.startswith(("scatter", "runs")) else write.get(pat)
        if counted is None:
            continue
        cb = counted * 1024.0
        e = {"counter": "FETCH_SIZE" if not pat.startswith(("scatter", "runs")) else "WRITE_SIZE",
             "counted_bytes": cb, "requested_bytes": req, "lines_x128": lines * 128,
             "counted_per_requested": cb / req, "counted_per_line128": cb / (lines * 128)}
        if pat in timing:
            e["time_us"] = timing[pat]
            e["lines_x128_TBps"] = lines * 128 / (timing[pat] * 1e-6) / 1e12
        out[pat] = e
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
