set -e
O=gpurun_out/r6ag; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_rccl.py tests/test_train_step.py > $O/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-train-step > $O/n1_$i.json 2>&1
  timeout -k 10 200 python bench.py --force-dist --plan-world 8 --exchange-groups 1 --no-cpu-baseline > $O/g1_$i.json 2>&1
  timeout -k 10 200 python bench.py --force-dist --plan-world 8 --exchange-groups 2 --no-cpu-baseline > $O/g2_$i.json 2>&1
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python bench.py --force-dist --plan-world 8 --no-cpu-baseline --no-train-step --steps 10 > $O/tr.log 2>&1
