#!/bin/bash
# PMC instruction counts (VALU, SALU, transcendental) of every kernel under each knob setting:
#   tools/pmc_ab.sh bwd_lastc=0 bwd_lastc=1 bwd_v=4+bwd_pred=1   -> gpurun_out/pmc_ab/<setting>.json
# (one setting per argument; '+' joins several knobs of one setting)
set -euo pipefail
OUT=gpurun_out/pmc_ab
mkdir -p $OUT
export TMPDIR=/tmp
for kv in "$@"; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VALU_TRANS_F32 -d $OUT/$kv -o run --output-format csv -- python tools/run_steps.py --config cfg3 --steps 3 $(echo "$kv" | tr '+' '\n' | sed 's/^/--knob /') > $OUT/$kv.log 2>&1
  python tools/pmc_summary.py $OUT/$kv > $OUT/$kv.json
done
