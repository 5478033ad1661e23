# zres kernel times (512^3 V-cycles) under MGMC_ZR_KZ / MGMC_ZR_VARIANT settings
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/zr && export TMPDIR=/tmp
for cfgs in ${ZCFGS:-"kz8:MGMC_ZR_KZ=8" "kz4:MGMC_ZR_KZ=4" "kz2:MGMC_ZR_KZ=2" "v1:MGMC_ZR_VARIANT=1" "v3:MGMC_ZR_VARIANT=3" "v1kz8:MGMC_ZR_VARIANT=1,MGMC_ZR_KZ=8" "v3kz8:MGMC_ZR_VARIANT=3,MGMC_ZR_KZ=8" "def:"}; do
  name=${cfgs%%:*}; envs=${cfgs#*:}
  env $(echo $envs | tr ',' ' ') K=10 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/zr/$name -o $name -- python3 scripts/vcycle_once.py > gpurun_out/zr/$name.log 2>&1 || exit 3
  python3 - "$name" <<'PY'
import csv, glob, sys, collections
f = glob.glob(f"gpurun_out/zr/{sys.argv[1]}/*kernel_trace.csv")[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "zresrestrict" in r["Kernel_Name"] or "residual_restrict" in r["Kernel_Name"]:
        key = (r["Kernel_Name"][12:50], r["Grid_Size_X"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -max(kv[1])):
    print(sys.argv[1], k[0], k[1], round(sum(v) / len(v), 1), "us", len(v))
PY
  tail -1 gpurun_out/zr/$name.log
done
