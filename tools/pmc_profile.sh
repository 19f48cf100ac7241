#!/bin/bash
# PMC passes over tools/run_steps.py (one rocprofv3 invocation per counter group; --pmc never combined
# with tracing domains).  Usage: tools/pmc_profile.sh OUTDIR [config]
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
CFG=${2:-cfg3}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python tools/run_steps.py --config "$CFG" --steps 3 > "$OUT/$name.log" 2>&1
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run p2 SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run p3 FETCH_SIZE
run p4 WRITE_SIZE
run p5 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE
echo done
