set -e
O=gpurun_out/r6ai; mkdir -p $O
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob seg_grid=1536,1024,2048,3072 --rounds 6 --steps 5 > $O/seg_grid.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob seg_minw=6,5,7 --rounds 6 --steps 5 > $O/seg_minw.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_blocks=256,192,384 --rounds 6 --steps 5 > $O/bk_blocks.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob fwd_whole_waves=8,6 --rounds 6 --steps 5 > $O/fww.txt 2>&1
