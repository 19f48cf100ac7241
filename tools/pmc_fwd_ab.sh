set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_fwd
mkdir -p $OUT
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/v${v}_p1 -o run --output-format csv -- python tools/run_steps.py --config cfg3 --steps 2 --knob fwd_v4=$v > $OUT/v${v}_p1.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 -d $OUT/v${v}_p2 -o run --output-format csv -- python tools/run_steps.py --config cfg3 --steps 2 --knob fwd_v4=$v > $OUT/v${v}_p2.log 2>&1
done
echo ok
