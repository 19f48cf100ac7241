#!/usr/bin/env python
"""Per-launch instruction counts of the rasterizer kernels from a rocprofv3 --pmc pass of SQ_INSTS_VALU,
SQ_INSTS_SALU and SQ_INSTS_VALU_TRANS_F32 (wave-instructions, whole GPU).

    python tools/pmc_insts.py CONFIG OUT.json PMC_DIR...

Writes {CONFIG: {stage: {"kernel", "valu", "salu", "trans"}}} (merged into OUT.json if it exists); bench.py turns
it into the composite kernel's VALU issue utilisation with the issue costs tools/probes/valu_rate_probe.hip
measured (plain VALU 1.29 ns, transcendental 3.5 ns per wave-instruction per SIMD with every SIMD issuing).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load, short  # noqa: E402
from pmc_traffic import stage_of  # noqa: E402


def main():
    cfg, out_path, dirs = sys.argv[1], sys.argv[2], sys.argv[3:]
    res = load(dirs)
    table = {}
    for name, cs in res.items():
        st = stage_of(short(name))
        if st is None or "SQ_INSTS_VALU" not in cs:
            continue
        table[st] = {"kernel": short(name), "valu": cs["SQ_INSTS_VALU"], "salu": cs.get("SQ_INSTS_SALU"),
                     "trans": cs.get("SQ_INSTS_VALU_TRANS_F32")}
    out = {}
    if os.path.exists(out_path):
        out = json.load(open(out_path))
    out[cfg] = table
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()
