# Fine-sweep kernel times under timing-experiment builds (build/libmgmc_exp<N>.so; never the product)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/eprof && export TMPDIR=/tmp
for e in ${EXPS:-0 7 8}; do
  lib=""; [ "$e" != 0 ] && lib=build/libmgmc_exp$e.so
  MGMC_LIBRARY=$lib K=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eprof/e$e -o e$e -- python3 scripts/vcycle_once.py > gpurun_out/eprof/e$e.log 2>&1 || exit 3
  python3 - "$e" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/eprof/e{sys.argv[1]}/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "zsweep" in r["Name"]:
        print(sys.argv[1], r["Name"][12:60], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
