#!/bin/bash
# Round-4 GPU batch Y: the GPU suite with 8-region partition chunks (GSR_PART_MAXR 8), then 4 against 8 at cfg 3.
set -euo pipefail
O=gpurun_out/r4y
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
bash tools/lib_ab.sh $O/lib_ab_maxr4_vs8_cfg3.txt variants/libgsrast_head.so variants/libgsrast_m4.so --config cfg3 --steps 5
echo done
