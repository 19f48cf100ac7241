#!/bin/bash
# Round-4 GPU batch X: regions per partition chunk before the per-key fallback (GSR_PART_MAXR 16 / 64 against 32, then
# 8 against 16), cfg 3.
set -euo pipefail
O=gpurun_out/r4x
mkdir -p $O
export TMPDIR=/tmp
bash tools/lib_ab.sh $O/lib_ab_maxr8_vs16_cfg3.txt variants/libgsrast_m16.so variants/libgsrast_m8.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab2_maxr16_cfg3.txt variants/libgsrast_m16.so variants/libgsrast_head.so --config cfg3 --steps 5
echo done
