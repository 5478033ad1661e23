# A/B of environment settings on a bench.py configuration: for each rep and each setting ("-" = none,
# else NAME=VALUE), one bench line (JSON) into $OUT, prefixed with the setting.
#   ENVS="- MGMC_GRAPH_UNROLL=2" REPS=3 OUT=gpurun_out/env_ab.jsonl bash scripts/env_bench_ab.sh --steps 100
set -e
OUT=${OUT:-gpurun_out/env_ab.jsonl}
: > "$OUT"
for r in $(seq ${REPS:-1}); do
  for e in ${ENVS:--}; do
    echo "== $e rep $r" >&2
    if [ "$e" = "-" ]; then
      timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" | sed "s/^/$e /" >> "$OUT"
    else
      env "$e" timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" | sed "s/^/$e /" >> "$OUT"
    fi
  done
done
