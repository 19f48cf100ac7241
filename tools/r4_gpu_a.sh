#!/bin/bash
# Round-4 GPU batch A: the one-rank RCCL path, the XCD-major bucket layout A/B (time and WRITE_SIZE), the bench.
set -euo pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rccl.py -x -v --timeout 120 --timeout-method thread > $O/rccl.log 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "binning_paths or lookback or debug_mode or dense_tiles or means2d_none" > $O/parity_sel.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 1 --force-dist --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_fd.json 2> $O/bench_fd.err
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob bk_xcd=0,1 --rounds 6 --steps 5 > $O/ab_xcd.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg5 --knob rs_cscan=0,1 --knob tile_key16=0,1 --rounds 3 --steps 3 > $O/ab_cscan_cfg5.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob pre_sh_lds=0,1 --rounds 6 --steps 5 > $O/ab_shlds_cfg3.txt 2>&1
timeout -k 10 300 python tools/stage_ab.py --config cfg3 --knob rb_spin=0,1 --knob cull=0,1 --rounds 4 --steps 5 > $O/ab_rbspin_cfg3.txt 2>&1
for v in 0 1; do
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw$v -o run --output-format csv -- python tools/run_steps.py --config cfg3 --steps 3 --knob bk_xcd=$v > $O/pmcw$v.log 2>&1
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 120 ./tools/probes/bin/gather_probe > $O/gather_probe.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/probe_fetch -o run --output-format csv -- ./tools/probes/bin/gather_probe > $O/probe_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/probe_write -o run --output-format csv -- ./tools/probes/bin/gather_probe > $O/probe_write.log 2>&1
echo done
