#!/bin/bash
# Interleaved A/B of several library builds (separate processes): tools/lib_ab_multi.sh OUT CONFIG LIB...
set -euo pipefail
OUT=$1; CFG=$2; shift 2
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
for r in 1 2; do
  for L in "$@"; do
    echo "== $L" >> "$OUT"
    GSR_LIB="$L" timeout -k 10 200 python tools/stage_ab.py --rounds 2 --config "$CFG" >> "$OUT" 2>/dev/null
  done
done
