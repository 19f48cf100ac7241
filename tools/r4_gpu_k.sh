#!/bin/bash
# Round-4 GPU batch K: region scatter -- its parity tests, then the A/B against the direct scatter at cfg 3 and cfg 2,
# kernel stats of cfg 3.
set -euo pipefail
O=gpurun_out/r4k
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "region_scatter or binning_paths or forward_backward_vs_oracle or cfg3_full or prefix_binning" > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -5 $O/gpu_tests.log; exit 1; fi
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_region=0,1 --rounds 6 --steps 5 > $O/ab_region_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg2 --knob bk_region=0,2 --rounds 6 --steps 5 > $O/ab_region_cfg2.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof3 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_prof3.json 2> $O/bench_prof3.err
echo done
