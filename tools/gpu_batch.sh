#!/bin/bash
# One parametrised GPU batch (replaces the per-call r4_gpu_*.sh scripts): run named steps in order under
# gpurun_out/TAG, each under its own time limit, stopping at the first step that fails.
#
#   tools/gpu_batch.sh TAG STEP [STEP ...]
#
# Steps (arguments after ':' separated by ':'):
#   tests[:EXPR]              pytest -m gpu (optionally -k EXPR, "+" for " or "); writes parity.json
#   rccl                      tests/test_rccl.py (one-rank RCCL group)
#   smoke                     __graft_entry__.smoke()
#   bench[:CFG[:ARGS]]        bench.py --config CFG (ARGS: extra flags, ',' for spaces)
#   forcedist[:CFG[:ARGS]]    torchrun --nproc-per-node 1 bench.py --force-dist (the N > 1 path on one rank)
#   distov[:CFG]              tools/dist_overhead.py, and the same under rocprofv3 --kernel-trace --stats
#   ab:CFG:KNOBS[:ROUNDS]     tools/stage_ab.py interleaved knob A/B (KNOBS: name=v1,v2[+name=...])
#   libab:CFG:LIBA:LIBB       tools/lib_ab.sh interleaved library A/B
#   kstats[:CFG]              rocprofv3 --kernel-trace --stats over bench.py --config CFG
#   pmc:CFG:NAME:COUNTERS     one rocprofv3 --pmc pass over tools/run_steps.py (COUNTERS: ',' for spaces)
#   round[:CFGS]              tools/gpu_round_profile.sh TAG (PMC passes, bench lines, kernel stats; CFGS ',')
#   py:SCRIPT[:ARGS]          python SCRIPT ARGS (ARGS: ',' for spaces), 300 s limit
set -uo pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
n=0
run() {  # limit name cmd...: run one step, stop the batch on failure (pytest's "tests failed" rc 1 continues)
  local lim=$1 name=$2
  shift 2
  echo "[$(date +%T)] $name" | tee -a "$O/batch.log"
  timeout -k 10 "$lim" "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a "$O/batch.log"
  if [ $rc -ne 0 ]; then
    if [ "${ALLOW_RC1:-0}" = 1 ] && [ $rc -eq 1 ]; then return 0; fi
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}
for step in "$@"; do
  n=$((n + 1))
  IFS=':' read -r kind a1 a2 a3 a4 <<< "$step"
  case $kind in
    tests)
      sel=()
      [ -n "${a1:-}" ] && sel=(-k "${a1//+/ or }")
      ALLOW_RC1=1 GSR_PARITY_JSON=$O/parity.json run 600 "tests" python -u -m pytest tests/ -m gpu -v \
        --timeout 120 --timeout-method thread "${sel[@]}" > "$O/gpu_tests_$n.log" 2>&1
      tail -2 "$O/gpu_tests_$n.log" ;;
    rccl)
      run 300 rccl python -u -m pytest tests/test_rccl.py -v --timeout 120 --timeout-method thread \
        > "$O/rccl_$n.log" 2>&1 ;;
    smoke)
      run 200 smoke python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench)
      cfg=${a1:-cfg3}; extra=${a2:-}
      run 400 "bench $cfg" python bench.py --config "$cfg" ${extra//,/ } > "$O/bench_${cfg}_$n.json" 2> "$O/bench_${cfg}_$n.err"
      cat "$O/bench_${cfg}_$n.json" | cut -c1-400 ;;
    forcedist)
      cfg=${a1:-cfg3}; extra=${a2:-}
      run 400 "forcedist $cfg" python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --config "$cfg" --gpus 1 --force-dist \
        --no-cpu-baseline ${extra//,/ } > "$O/forcedist_${cfg}_$n.json" 2> "$O/forcedist_${cfg}_$n.err"
      cat "$O/forcedist_${cfg}_$n.json" | cut -c1-400 ;;
    distov)
      cfg=${a1:-cfg3}
      run 300 "distov $cfg" python tools/dist_overhead.py --config "$cfg" > "$O/distov_${cfg}_$n.json" 2> "$O/distov_${cfg}_$n.err"
      cat "$O/distov_${cfg}_$n.json"
      run 300 "distov-trace $cfg" rocprofv3 --kernel-trace --stats -d "$O/distov_trace_$n" -o run \
        --output-format csv -- python tools/dist_overhead.py --config "$cfg" --steps 10 \
        > "$O/distov_trace_${cfg}_$n.json" 2> "$O/distov_trace_${cfg}_$n.err" ;;
    ab)
      knobs=()
      IFS='+' read -ra ks <<< "$a2"
      for k in "${ks[@]}"; do knobs+=(--knob "$k"); done
      run 400 "ab $a1 $a2" python tools/stage_ab.py --config "$a1" "${knobs[@]}" --rounds "${a3:-5}" --steps 5 \
        > "$O/ab_${a1}_$n.txt" 2>&1
      tail -30 "$O/ab_${a1}_$n.txt" ;;
    libab)
      run 900 "libab $a1" bash tools/lib_ab.sh "$O/libab_${a1}_$n.txt" "$a2" "$a3" --config "$a1"
      cat "$O/libab_${a1}_$n.txt" ;;
    kstats)
      cfg=${a1:-cfg3}
      run 300 "kstats $cfg" rocprofv3 --kernel-trace --stats -d "$O/kstats_${cfg}_$n" -o run --output-format csv -- \
        python bench.py --config "$cfg" --no-cpu-baseline > "$O/kstats_bench_${cfg}_$n.json" 2> "$O/kstats_${cfg}_$n.err" ;;
    pmc)
      run 120 "pmc $a1 $a2" rocprofv3 --pmc ${a3//,/ } -d "$O/pmc_${a1}_${a2}" -o run --output-format csv -- \
        python tools/run_steps.py --config "$a1" --steps 3 > "$O/pmc_${a1}_${a2}.log" 2>&1 ;;
    round)
      run 1100 round bash tools/gpu_round_profile.sh "$TAG" ${a1//,/ } ;;
    py)
      run 300 "py $a1" python "$a1" ${a2//,/ } > "$O/py_$n.log" 2>&1
      tail -20 "$O/py_$n.log" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "batch $TAG done"
