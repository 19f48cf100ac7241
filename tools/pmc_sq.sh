#!/bin/bash
# SQ instruction/occupancy counters for the hot kernels (one rocprofv3 pass per counter group, no tracing
# domains).  Usage: tools/pmc_sq.sh OUTDIR [config]; summary in OUTDIR/sq.json
set -euo pipefail
OUT=${1:-gpurun_out/sq}
CFG=${2:-cfg3}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python tools/run_steps.py --config "$CFG" --steps 3 > "$OUT/$name.log" 2>&1
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run p5 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE
python tools/pmc_summary.py "$OUT/p1" "$OUT/p2" "$OUT/p5" > "$OUT/sq.json"
echo done
