# fine-sweep tile study: time (product) and FETCH_SIZE / WRITE_SIZE per z-sweep variant
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tiles && export TMPDIR=/tmp
timeout -k 10 600 python scripts/exp_bench.py ${VARIANTS:-0,11,12,13} 0 > gpurun_out/tiles/time.log 2>&1; echo "time rc=$?"; cat gpurun_out/tiles/time.log
for V in $(echo ${VARIANTS:-0,11,12,13} | tr ',' ' '); do
  MGMC_ZS_VARIANT=$V K=4 timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/tiles/f$V -o f --output-format csv -- python3 scripts/sweep_once.py > gpurun_out/tiles/f$V.log 2>&1 || exit 3
done
exit 0
