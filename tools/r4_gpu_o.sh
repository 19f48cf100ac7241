#!/bin/bash
# Round-4 GPU batch O: whole library built without SLP vectorisation (render_bwd's packed f32 ops) against head.
set -euo pipefail
O=gpurun_out/r4o
mkdir -p $O
export TMPDIR=/tmp
bash tools/lib_ab.sh $O/lib_ab_noslp_cfg3.txt variants/libgsrast_head.so variants/libgsrast_noslp.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab_noslp_cfg5.txt variants/libgsrast_head.so variants/libgsrast_noslp.so --config cfg5 --steps 3
echo done
