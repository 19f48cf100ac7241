set -e
export TMPDIR=/tmp
O=gpurun_out/r6af; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/tr -o run -- python bench.py --force-dist --plan-world 8 --no-cpu-baseline --no-train-step --steps 10 > $O/b.log 2> $O/b.err
