#!/bin/bash
# Round-4 GPU batch N: late colour with direct row reads (parity, A/B), region partition with wave-parallel region
# search (parity, A/B), kernel stats.
set -euo pipefail
O=gpurun_out/r4n
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "split_colour or forward_backward_vs_oracle or golden or region_scatter or binning_paths or cfg3_full" > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -5 $O/gpu_tests.log; exit 1; fi
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob pre_late=0,2 --knob pre_late_minw=4,6 --rounds 4 --steps 5 > $O/ab_direct_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob pre_late=0,2 --knob pre_late_minw=6 --rounds 3 --steps 3 > $O/ab_direct_cfg5.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_region=0,1 --rounds 6 --steps 5 > $O/ab_region_cfg3.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_prof3.json 2> $O/bench_prof3.err
echo done
