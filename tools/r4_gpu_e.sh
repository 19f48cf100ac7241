#!/bin/bash
# Round-4 GPU batch E: GPU suite after restoring the inverse permutation (bwd_inv) and the measured knob defaults,
# knob A/Bs, bench lines.
set -euo pipefail
O=gpurun_out/r4e
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bwd_inv=0,1 --rounds 6 --steps 5 > $O/ab_inv_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob tile_key16=0,1 --rounds 3 --steps 3 > $O/ab_k16_cfg5.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob bwd_inv=0,1 --rounds 3 --steps 3 > $O/ab_inv_cfg5.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --steps 10 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline --steps 20 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
echo done
