set -e
O=gpurun_out/r6ao; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pz1_$i.json 2>&1
  GSR_TUNE=bwd_prezero=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pz0_$i.json 2>&1
done
timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-train-step > $O/pz1_cfg5.json 2>&1
GSR_TUNE=bwd_prezero=0 timeout -k 10 200 python bench.py --config cfg5 --no-cpu-baseline --no-train-step > $O/pz0_cfg5.json 2>&1
