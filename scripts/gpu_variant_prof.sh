# Kernel times of the fine pre-sweep and the fused post-sweep per z-sweep tile variant (512^3 V-cycles)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/vprof && export TMPDIR=/tmp
for v in ${VARIANTS:-0 9 1 3 8}; do
  MGMC_ZS_VARIANT=$v K=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof/v$v -o v$v -- python3 scripts/vcycle_once.py > gpurun_out/vprof/v$v.log 2>&1 || exit 3
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/vprof/v{sys.argv[1]}/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "zsweep" in r["Name"]:
        print(sys.argv[1], r["Name"][12:60], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
  tail -1 gpurun_out/vprof/v$v.log
done
