#!/bin/bash
# Round-4 GPU batch I: GPU suite (inverse permutation restored, big_reduce split), tile-sort variant without the
# relative-key map (norel) against head at cfg 5, r4a-era library against head at cfg 3.
set -euo pipefail
O=gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for L in norel head; do
  echo "== $L" >> $O/tile_cfg5.txt
  GSR_LIB=variants/libgsrast_$L.so timeout -k 10 200 python tools/stage_ab.py --config cfg5 --knob depth_rel=0 --rounds 3 --steps 3 >> $O/tile_cfg5.txt 2>/dev/null
done
bash tools/lib_ab.sh $O/lib_ab_cfg3.txt variants/libgsrast_r4a.so variants/libgsrast_head.so --config cfg3 --steps 5
echo done
