#!/usr/bin/env python
"""Split a rocprofv3 kernel trace into steps (a step starts at each preprocess_kernel dispatch) and show where a step's
time goes: per step signature (the count of each kernel kind), the median step span, kernel busy time and the gaps
between consecutive kernels (idle GPU), and one example step's timeline.

    python tools/trace_steps.py run_kernel_trace.csv [--example SIGNATURE_INDEX]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    n = n.replace("gsr::", "")
    return re.sub(r"<.*>", "", n)[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=1.5)
    args = ap.parse_args()
    rows = []
    with open(args.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r.get("Queue_Id", 0))))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith("preprocess_kernel")]
    groups = defaultdict(list)
    for a, b in zip(starts, starts[1:]):
        step = rows[a:b]
        sig = tuple(sorted(defaultdict(int, {}).items()))
        cnt = defaultdict(int)
        for r in step:
            cnt[r[2]] += 1
        sig = tuple(sorted(cnt.items()))
        span = (rows[b][0] - rows[a][0]) / 1e3
        busy, gaps, end = 0.0, [], rows[a][0]
        for s, e, n, q in step:
            if s > end:
                gaps.append(((s - end) / 1e3, n))
            busy += (e - max(s, end)) / 1e3 if e > end else 0.0
            end = max(end, e)
        groups[sig].append((span, busy, gaps, step))
    for gi, (sig, steps) in enumerate(sorted(groups.items(), key=lambda kv: -len(kv[1]))):
        spans = [s[0] for s in steps]
        busy = [s[1] for s in steps]
        print(f"[{gi}] {len(steps)} steps: span median {statistics.median(spans):.1f} us, busy {statistics.median(busy):.1f} us;"
              f" kernels " + ", ".join(f"{n} x{c}" for n, c in sig if c > 1 or 'bwd' in n or 'views' in n or 'adam' in n))
        ex = sorted(steps, key=lambda s: s[0])[len(steps) // 2]
        t0 = ex[3][0][0]
        end = t0
        for s, e, n, q in ex[3]:
            gap = (s - end) / 1e3
            if gap > args.gap_us or any(k in n for k in ("bwd", "views", "adam", "zero", "fill", "copy", "Fill")):
                print(f"      {(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:6.1f} us  gap {gap:6.1f}  q{q}  {n}")
            end = max(end, e)


if __name__ == "__main__":
    main()
