#!/bin/bash
# Round-4 GPU batch L: late staged colour -- parity, A/B against the fused preprocess at cfg 3 and cfg 5, occupancy.
set -euo pipefail
O=gpurun_out/r4l
mkdir -p $O
export TMPDIR=/tmp
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread -k "split_colour or forward_backward_vs_oracle or golden or cfg3_full or smoke" > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; tail -5 $O/gpu_tests.log; exit 1; fi
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob pre_late=0,1 --knob pre_late_minw=4,5,6 --rounds 4 --steps 5 > $O/ab_late_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob pre_late=0,1 --rounds 3 --steps 3 > $O/ab_late_cfg5.txt 2>&1
echo done
