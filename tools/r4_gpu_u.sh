#!/bin/bash
# Round-4 GPU batch U: region-partition chunk shapes (library variants, GSR_PART_ITEMS / GSR_PART_THREADS) at cfg 3.
set -euo pipefail
O=gpurun_out/r4u
mkdir -p $O
export TMPDIR=/tmp
bash tools/lib_ab.sh $O/lib_ab2_part4_cfg3.txt variants/libgsrast_head.so variants/libgsrast_p4.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab2_part2_cfg3.txt variants/libgsrast_head.so variants/libgsrast_p2.so --config cfg3 --steps 5
bash tools/lib_ab.sh $O/lib_ab3_part4_cfg3.txt variants/libgsrast_p4.so variants/libgsrast_head.so --config cfg3 --steps 5
echo done
