#!/bin/bash
# Round-4 GPU batch S: extra walk blocks for the big rects of small scenes ("bk_big_blocks"): parity, then the host
# floor probe (2000 / 20000 Gaussians at 1080p) and interleaved knob A/Bs at cfg 2 (cfg 3: 245 range blocks, no extra blocks).
set -euo pipefail
O=gpurun_out/r4s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "big_rect or region_scatter or bucket" > $O/pytest.log 2>&1
for n in 2000 20000; do
  for k in 0 256; do
    GSR_TUNE=bk_big_blocks=$k timeout -k 10 120 python tools/host_floor.py --n $n --steps 30 > $O/host_floor_n${n}_k${k}.json 2>&1
  done
done
for c in cfg2; do
  timeout -k 10 300 python tools/stage_ab.py --config $c --knob bk_big_blocks=0,256 --rounds 4 --steps 5 > $O/ab_bigblocks_$c.txt 2>&1
done
echo done
