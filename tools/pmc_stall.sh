#!/bin/bash
# Memory-pipeline counters per kernel (one rocprofv3 pass per counter block, no tracing domains):
#   tools/pmc_stall.sh OUTDIR [config]  -> OUTDIR/stall.json
# SQ wave/wait cycles and VMEM issue level; TA busy and stalls behind the texture cache; TCP->TCC request
# counts and their summed latencies (average latency = *_LATENCY / *_REQ).
set -euo pipefail
OUT=${1:-gpurun_out/stall}
CFG=${2:-cfg3}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv -- python tools/run_steps.py --config "$CFG" --steps 3 > "$OUT/$name.log" 2>&1
}
run s1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
run s2 TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES
run s3 TA_DATA_STALLED_BY_TC_CYCLES TA_BUFFER_WAVEFRONTS
run s4 TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_WRITE_REQ
python tools/pmc_summary.py "$OUT/s1" "$OUT/s2" "$OUT/s3" "$OUT/s4" > "$OUT/stall.json"
echo done
