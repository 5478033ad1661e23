# V-cycle kernel traces under a list of environment settings (ENVS="A=1,B=2 C=3 ..." ; "-" = none):
# the top kernels per setting
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/envs && export TMPDIR=/tmp
i=0
for E in ${ENVS:--}; do
  i=$((i+1))
  rm -rf gpurun_out/envs/$i
  if [ "$E" = "-" ]; then EV=""; else EV=$(echo $E | tr ',' ' '); fi
  env $EV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/envs/$i -o vt -- python3 scripts/vcycle_once.py > gpurun_out/envs/$i.log 2>&1 || exit 3
  echo "== $E: $(grep vcycle gpurun_out/envs/$i.log)"
  python3 scripts/kstats.py $(find gpurun_out/envs/$i -name "*kernel_trace.csv" | head -1) 13 > gpurun_out/envs/$i.txt
  head -${TOP:-4} gpurun_out/envs/$i.txt
done
