set -e
O=gpurun_out/r6ay; mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $O/n1_$i.json 2>&1
  timeout -k 10 200 python bench.py --force-dist --plan-world 8 --no-cpu-baseline > $O/pw8_$i.json 2>&1
done
