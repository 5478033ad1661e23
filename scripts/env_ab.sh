#!/bin/bash
# Interleaved A/B of one library build under two MGMC_DISABLE settings: REPS x (A, B) bench lines.
#   A="" B="jsweep" REPS=3 OUT=gpurun_out/env_ab.jsonl bash scripts/env_ab.sh --plain --steps 100
set -e
OUT=${OUT:-gpurun_out/env_ab.jsonl}
: > "$OUT"
for r in $(seq ${REPS:-3}); do
  for tag in A B; do
    val=${!tag}
    echo "== $tag ($val) rep $r" >&2
    MGMC_DISABLE=$val timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" | sed "s/^/$tag /" >> "$OUT"
  done
done
