#!/bin/bash
# Round-4 GPU batch B: where the distributed step's extra time goes (one-rank RCCL group), kernel trace of it.
set -euo pipefail
O=gpurun_out/r4b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/dist_overhead.py --config cfg3 --steps 20 > $O/dist_overhead.json 2> $O/dist_overhead.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_fd -o run --output-format csv -- python bench.py --force-dist --steps 10 --warmup 3 --no-cpu-baseline --no-stage-events > $O/bench_fd_prof.json 2> $O/bench_fd_prof.err
echo done
