#!/bin/bash
# One GPU call that produces the round's measurement evidence under gpurun_out/$TAG, for every bench config:
#   1. HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE; separate passes, no tracing domains) and an SQ
#      instruction-count pass (VALU, SALU, transcendental), per config
#   2. profiles/pmc_traffic.json and profiles/pmc_insts.json (keyed by config) for bench.py's roofline
#   3. the bench.py line of each config (its roofline reads the two files just written)
#   4. rocprofv3 --kernel-trace --stats over the default (cfg3) bench.py command (kernel averages must agree)
# Usage: tools/gpu_round_profile.sh TAG [CONFIGS...]   (default configs: cfg3 cfg2 cfg5)
set -euo pipefail
TAG=${1:-r3}
shift || true
CONFIGS=${*:-cfg3 cfg2 cfg5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT" profiles
export TMPDIR=/tmp
pmc() {  # config name counters
  timeout -k 10 300 rocprofv3 --pmc $3 -d "$OUT/pmc_$1_$2" -o run --output-format csv -- \
    python tools/run_steps.py --config $1 --steps 3 > "$OUT/pmc_$1_$2.log" 2>&1
}
for c in $CONFIGS; do
  pmc $c fetch FETCH_SIZE
  pmc $c write WRITE_SIZE
  pmc $c insts "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32"
  python tools/pmc_traffic.py $c profiles/pmc_traffic.json "$OUT/pmc_${c}_fetch" "$OUT/pmc_${c}_write" > "$OUT/pmc_traffic_$c.log"
  python tools/pmc_insts.py $c profiles/pmc_insts.json "$OUT/pmc_${c}_insts" > "$OUT/pmc_insts_$c.log"
  echo "pmc $c done"
done
cp profiles/pmc_traffic.json "$OUT/pmc_traffic.json"
cp profiles/pmc_insts.json "$OUT/pmc_insts.json"
for c in $CONFIGS; do
  timeout -k 10 400 python bench.py --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err"
  echo "bench $c done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kstats" -o run --output-format csv -- \
  python bench.py --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
echo done
