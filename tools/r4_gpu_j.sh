#!/bin/bash
# Round-4 GPU batch J: GPU suite, knob A/Bs after the fixes (tile_key16, tile_db, depth_rel at cfg 5), bench lines,
# kernel stats of cfg 3 and cfg 5.
set -euo pipefail
O=gpurun_out/r4j
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob tile_key16=0,1 --knob tile_db=5,8 --rounds 3 --steps 3 > $O/ab_tile_cfg5.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob depth_rel=0,1 --rounds 3 --steps 3 > $O/ab_rel_cfg5.txt 2>&1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline --steps 20 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_prof3.json 2> $O/bench_prof3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof5 -o run --output-format csv -- python bench.py --config cfg5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_prof5.json 2> $O/bench_prof5.err
echo done
