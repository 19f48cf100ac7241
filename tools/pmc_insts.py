#!/usr/bin/env python
"""Per-stage instruction counts of the rasterizer from a rocprofv3 --pmc pass of SQ_INSTS_VALU, SQ_INSTS_SALU and
SQ_INSTS_VALU_TRANS_F32 (wave-instructions, whole GPU).

    python tools/pmc_insts.py CONFIG OUT.json PMC_DIR...

Writes {CONFIG: {stage: {"kernel", "valu", "salu", "trans"}}} (merged into OUT.json if it exists); bench.py turns
it into the composite kernel's VALU issue utilisation with the issue costs tools/probes/valu_rate_probe.hip
measured (plain VALU 1.29 ns, transcendental 3.5 ns per wave-instruction per SIMD with every SIMD issuing).
Stages as tools/pmc_stages.py (per-step sums over a stage's kernels).
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
        if "SQ_INSTS_VALU" not in cs:
            continue
        table[st] = {"kernel": " + ".join(cs["kernels"]), "valu": cs["SQ_INSTS_VALU"], "salu": cs.get("SQ_INSTS_SALU"),
                     "trans": cs.get("SQ_INSTS_VALU_TRANS_F32")}
    out = json.load(open(out_path)) if os.path.exists(out_path) else {}
    out[cfg] = table
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps({"steps": steps, "stages": table}, indent=1))


if __name__ == "__main__":
    main()
