# cache-policy study of the fine sweep: time and FETCH_SIZE for product / nt-store / nt-store+f builds
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/nt && export TMPDIR=/tmp
timeout -k 10 600 python scripts/exp_bench.py 0 0,7,8,9 > gpurun_out/nt/time.log 2>&1; echo "time rc=$?"; cat gpurun_out/nt/time.log
for X in 0 7 9; do
  if [ $X = 0 ]; then export MGMC_LIBRARY=; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$X.so; fi
  K=4 timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/nt/f$X -o f --output-format csv -- python3 scripts/sweep_once.py > gpurun_out/nt/f$X.log 2>&1 || exit 3
done
exit 0
