#!/bin/bash
# Stage-time A/B of one tuning knob on the GPU box (results in gpurun_out/ab/TAG.json):
#   gpurun -- bash tools/gpu_ab.sh TAG name=v1,v2[,...] [CONFIG]
set -euo pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python tools/stage_ab.py --config "${3:-cfg3}" --knob "$2" --rounds "${ROUNDS:-3}" --steps 5 \
  > "gpurun_out/ab/$1.json" 2> "gpurun_out/ab/$1.err"
