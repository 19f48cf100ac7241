set -e
O=gpurun_out/r6bc; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_pytest.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_round_profile.sh r6bc cfg3 cfg2 cfg5 > $O/profile.log 2>&1
