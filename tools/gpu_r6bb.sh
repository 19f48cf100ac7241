set -e
O=gpurun_out/r6bb; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bwd_live=1,0 --rounds 8 --steps 5 > $O/ab_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob bwd_live=1,0 --rounds 4 --steps 3 > $O/ab_cfg5.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg2 --knob bwd_live=1,0 --rounds 8 --steps 5 > $O/ab_cfg2.txt 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/l1_$i.json 2>&1
  GSR_TUNE=bwd_live=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/l0_$i.json 2>&1
done
