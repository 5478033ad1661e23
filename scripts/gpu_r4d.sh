# Round 4 timing experiments on the level-1 kernels (builds in build/, never the product): per-kernel
# times (rocprofv3 kernel trace of scripts/vcycle_once.py, summarised by grid with scripts/kstats.py)
# for the j-sweep prefetch depth / rounds and the 27-point residual + restriction tile height / chunk
# depth, then interleaved cycle times.   VARS="0 jd2 ..." overrides the list.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4d && export TMPDIR=/tmp
O=gpurun_out/r4d
for lib in ${VARS:-0 jd2 jd4 jr2 zc3 zc8 zk2 zk8}; do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$lib.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$lib -o kt -- python3 scripts/vcycle_once.py > $O/kt_$lib.log 2>&1
  rc=$?; echo "$lib rc=$rc"; [ $rc -eq 0 ] || exit 3
  f=$(ls $O/kt_$lib/*/kt_kernel_trace.csv 2>/dev/null || ls $O/kt_$lib/kt_kernel_trace.csv)
  python3 scripts/kstats.py $f 13 > $O/kstats_$lib.txt; echo "== $lib"; head -14 $O/kstats_$lib.txt; tail -1 $O/kstats_$lib.txt
done
unset MGMC_LIBRARY
REPS=2 timeout -k 10 700 python scripts/lib_cycle_bench.py $(echo ${VARS:-0 jd2 jd4 jr2 zc3 zc8 zk2 zk8} | tr ' ' ,) > $O/cycle.log 2>&1; rc=$?
echo "cycle rc=$rc"; cat $O/cycle.log
exit $rc
