# Round 4 timing experiments (builds in build/, never the product): pre-sweep z-chunk depths that fill
# the last round of workgroups (TZ 44: 2496 tiles = 4.875 rounds of 512 slots; 22: 9.75; 30: 7.3;
# product 32: 6.5) and level-1 residual + restriction chunk depths (kz 11: 768 tiles = one round of
# 768 slots; 6: 1.83 rounds; product 4: 2.67).  Per-kernel traces, then interleaved cycle times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4g && export TMPDIR=/tmp
O=gpurun_out/r4g
V="0 s20x6x44 s20x6x22 s20x6x30 zk11 zk6"
for lib in $V; do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$lib.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$lib -o kt -- python3 scripts/vcycle_once.py > $O/kt_$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$lib/kt_kernel_trace.csv 13 > $O/kstats_$lib.txt; echo "== $lib"; head -8 $O/kstats_$lib.txt; grep zresrestrict $O/kstats_$lib.txt
done
unset MGMC_LIBRARY
REPS=3 timeout -k 10 900 python scripts/lib_cycle_bench.py $(echo $V | tr ' ' ,) > $O/cycle.log 2>&1; rc=$?
echo "cycle rc=$rc"; cat $O/cycle.log
exit $rc
