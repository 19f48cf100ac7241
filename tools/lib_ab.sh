#!/bin/bash
# Interleaved A/B of two library builds (separate processes): tools/lib_ab.sh OUT LIB_A LIB_B [stage_ab args]
set -euo pipefail
OUT=$1; A=$2; B=$3; shift 3
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in 1 2; do
  for L in "$A" "$B"; do
    echo "== $L" >> "$OUT"
    GSR_LIB="$L" timeout -k 10 200 python tools/stage_ab.py --rounds 3 "$@" >> "$OUT" 2>/dev/null
  done
done
