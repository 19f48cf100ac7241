#!/bin/bash
# Round-4 GPU batch W: region width of the region scatter (library variants, GSR_BK_REGION_LOG2 3 / 5 against 4) at cfg 3.
set -euo pipefail
O=gpurun_out/r4w
mkdir -p $O
export TMPDIR=/tmp
bash tools/lib_ab.sh $O/lib_ab_region8_cfg3.txt variants/libgsrast_head.so variants/libgsrast_r8.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab_region32_cfg3.txt variants/libgsrast_head.so variants/libgsrast_r32.so --config cfg3 --steps 5
echo done
