#!/bin/bash
# Round-4 GPU batch Q: knob sweeps after the region scatter (walk blocks, per-tile sort occupancy) and render_bwd at
# 6 waves per SIMD (library variant).
set -euo pipefail
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_blocks=192,256,384,512 --rounds 4 --steps 5 > $O/ab_bkblocks_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob seg_minw=5,6,7 --rounds 4 --steps 5 > $O/ab_segminw_cfg3.txt 2>&1
bash tools/lib_ab.sh $O/lib_ab_bwd6_cfg3.txt variants/libgsrast_head.so variants/libgsrast_bwd6.so --config cfg3 --steps 5
echo done
