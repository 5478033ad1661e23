# Round 4 timing-only experiment (build/libmgmc_exprevhack.so gives WRONG results, never the product):
# the level-1 second half-sweep's rows in mirrored memory order, i.e. the access order of a downward
# j-march, to see whether the half-sweep after the first gains from the Infinity Cache.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4j && export TMPDIR=/tmp
O=gpurun_out/r4j
for v in 0 revhack; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; tail -2 $O/kt_$v.log
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "jsweep|zresrestrict<27, 64" $O/kstats_$v.txt
done
exit 0
