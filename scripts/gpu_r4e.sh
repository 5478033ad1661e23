# Round 4 timing experiments on the fine sweeps (builds in build/, never the product): HBM traffic per
# launch (separate FETCH_SIZE / WRITE_SIZE passes, scripts/pmc_by_kernel.py) and interleaved cycle
# times for the pre-sweep z-chunk depth (s20x6x48/64/128) and the tile orders (o1: y fastest, o2: no
# XCD remap).   VARS="0 s20x6x64 ..." overrides the list.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4e && export TMPDIR=/tmp
O=gpurun_out/r4e
V=${VARS:-0 s20x6x48 s20x6x64 s20x6x128 o1 o2}
for lib in $V; do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$lib.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    K=4 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/${lib}_$c -o pmc -- python3 scripts/vcycle_once.py > $O/${lib}_$c.log 2>&1
    rc=$?; echo "$lib $c rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
  python3 scripts/pmc_by_kernel.py $O/${lib}_FETCH_SIZE $O/${lib}_WRITE_SIZE 512 > $O/pmc_$lib.txt 2>&1; echo "== $lib"; head -8 $O/pmc_$lib.txt
done
unset MGMC_LIBRARY
REPS=2 timeout -k 10 700 python scripts/lib_cycle_bench.py $(echo $V | tr ' ' ,) > $O/cycle.log 2>&1; rc=$?
echo "cycle rc=$rc"; cat $O/cycle.log
exit $rc
