#!/bin/bash
# Round-4 GPU batch H: kernel stats of the cfg 5 step, library at 2c2e231 against the current one (tile_db=8).
set -euo pipefail
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
for L in 2c2e231 head; do
  GSR_LIB=variants/libgsrast_$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$L -o run --output-format csv -- python tools/stage_ab.py --config cfg5 --knob tile_db=8 --rounds 2 --steps 3 > $O/ab_$L.txt 2>&1
done
echo done
