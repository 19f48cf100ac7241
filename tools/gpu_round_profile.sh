#!/bin/bash
# One GPU call that produces the round's measurement evidence under gpurun_out/$TAG:
#   1. HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes, no tracing domains) and an SQ
#      instruction-count pass (VALU, SALU, transcendental)
#   2. profiles/pmc_traffic.json and profiles/pmc_insts.json for bench.py's roofline
#   3. the default bench.py line (its roofline reads the two files just written)
#   4. rocprofv3 --kernel-trace --stats over the same bench.py command (kernel averages must agree)
# Usage: tools/gpu_round_profile.sh TAG
set -euo pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" profiles
export TMPDIR=/tmp
pmc() {  # name counter
  timeout -k 10 300 rocprofv3 --pmc $2 -d "$OUT/pmc_$1" -o run --output-format csv -- \
    python tools/run_steps.py --config cfg3 --steps 3 > "$OUT/pmc_$1.log" 2>&1
}
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
pmc insts "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32"
python tools/pmc_traffic.py cfg3 profiles/pmc_traffic.json "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_traffic.log"
python tools/pmc_insts.py cfg3 profiles/pmc_insts.json "$OUT/pmc_insts" > "$OUT/pmc_insts.log"
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
cp profiles/pmc_insts.json "$OUT/pmc_insts.json"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kstats" -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
echo done
