#!/bin/bash
# Round-4 GPU batch G: bisect the cfg 5 tile-sort slowdown over round-4 library builds (tile_db=8 where it exists).
set -euo pipefail
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
for L in r4a 8a9b209 2c2e231 4b483b4 head; do
  echo "== $L" >> $O/bisect_cfg5.txt
  GSR_LIB=variants/libgsrast_$L.so timeout -k 10 200 python tools/stage_ab.py --config cfg5 --knob tile_db=8 --rounds 3 --steps 3 >> $O/bisect_cfg5.txt 2>/dev/null
done
echo done
