#!/bin/bash
# Round-4 GPU batch C: the whole GPU suite (prefix binning tests), prefix A/B, distributed overhead, the bench.
set -euo pipefail
O=gpurun_out/r4c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_prefix=0,512 --rounds 6 --steps 5 > $O/ab_prefix_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob pre_split=0,1 --rounds 6 --steps 5 > $O/ab_split_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob tile_db=5,8 --rounds 3 --steps 3 > $O/ab_tiledb_cfg5.txt 2>&1
timeout -k 10 300 python tools/dist_overhead.py --config cfg3 --steps 20 > $O/dist_overhead.json 2> $O/dist_overhead.err
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
echo done
