#!/bin/bash
# A/B of library builds on a bench.py configuration: for each build (0 = product, else
# build/libmgmc_<x>.so; "<x>+VAR=value" adds an environment switch, e.g. 0+MGMC_DISABLE=xzero) and each
# rep, one bench line (JSON) into $OUT.
#   LIBS="w0 w512" REPS=2 OUT=gpurun_out/ab.jsonl bash scripts/lib_bench_ab.sh --posterior 8 --chains 8
set -e
OUT=${OUT:-gpurun_out/ab.jsonl}
: > "$OUT"
for r in $(seq ${REPS:-1}); do
  for ent in ${LIBS:-0}; do
    x=${ent%%+*}; extra=""; [ "$ent" != "$x" ] && extra=${ent#*+}
    if [ "$x" = "0" ]; then lib=""; else lib="$PWD/build/libmgmc_$x.so"; fi
    echo "== $ent rep $r" >&2
    env $extra MGMC_LIBRARY=$lib timeout -k 10 240 python -u bench.py --no-cpu-baseline "$@" | sed "s/^/$ent /" >> "$OUT"
  done
done
