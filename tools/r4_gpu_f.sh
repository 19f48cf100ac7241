#!/bin/bash
# Round-4 GPU batch F: the r4a-era library (675e039) against the current one, interleaved, cfg 3 and cfg 5.
set -euo pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
bash tools/lib_ab.sh $O/lib_ab_cfg3.txt variants/libgsrast_r4a.so variants/libgsrast_head.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab_cfg5.txt variants/libgsrast_r4a.so variants/libgsrast_head.so --config cfg5 --steps 3
echo done
