#!/usr/bin/env python
"""One line per bench JSON file (the last JSON line of each file): step time, exchange, train step, p50."""
import json
import sys

for path in sys.argv[1:]:
    d = None
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
    if d is None:
        print(path, "no JSON line")
        continue
    tr = (d.get("train_step") or {}).get("train_step_ms")
    print(f"{path}: {d['ms_per_step']} ms/step, p50 {d.get('step_events_ms', {}).get('p50_ms')}, train_step {tr}, "
          f"{d['config']['parallelism'][:110]}")
