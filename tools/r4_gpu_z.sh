#!/bin/bash
# Round-4 GPU batch Z (final code: 4-region partition chunks): the whole GPU suite with the achieved-parity record (profiles/parity_r4.json), then the round
# profile (PMC traffic + instruction passes, bench lines, kernel stats) for cfg 3, cfg 2 and cfg 5.
set -euo pipefail
O=gpurun_out/r4z
mkdir -p $O
export TMPDIR=/tmp
rc=0
GSR_PARITY_JSON=$O/parity_r4.json timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_round_profile.sh r4z cfg3 cfg2 cfg5
echo done
