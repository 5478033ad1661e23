# Round-2 fine-sweep tile study: product vs memory skeleton (exp5) per tile shape and z-chunk depth,
# then FETCH_SIZE / WRITE_SIZE per shape (sweep_once.py, 4 sweeps).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tiles2 && export TMPDIR=/tmp
O=gpurun_out/tiles2
TZS=32,64 timeout -k 10 600 python scripts/exp_bench.py 0,11,12,13 0,5 > $O/time.log 2>&1; rc=$?; echo "time rc=$rc"; cat $O/time.log; [ $rc -eq 0 ] || exit $rc
for V in 0 11 12 13; do
  for c in FETCH_SIZE WRITE_SIZE; do
    MGMC_ZS_VARIANT=$V K=4 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/p${V}_$c -o p --output-format csv -- python3 scripts/sweep_once.py > $O/p${V}_$c.log 2>&1 || exit 3
  done
done
exit 0
