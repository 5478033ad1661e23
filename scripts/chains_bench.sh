#!/bin/bash
# Batched-chain throughput (bench.py --chains K): one JSON line per (workload, K) into $OUT.
# Usage (GPU box): OUT=gpurun_out/chains.jsonl KS="1 4 8 16" bash scripts/chains_bench.sh
set -e
OUT=${OUT:-gpurun_out/chains.jsonl}
KS=${KS:-"1 8"}
: > "$OUT"
run() {
    for K in $KS; do
        echo "== $* --chains $K" >&2
        timeout -k 10 240 python -u bench.py --no-cpu-baseline --chains "$K" "$@" >> "$OUT"
    done
}
run --posterior 8 --measure-global --steps 100 --warmup 10
run --posterior 8 --steps 200 --warmup 10
run --n 256 --nlevel 6 --steps 200 --warmup 10
run --dim 2 --n 1024 --nlevel 5 --steps 1000 --warmup 50
if [ -n "$WITH512" ]; then run --steps 50 --warmup 5; fi
