# Fine-sweep tile-order experiment (timing builds, never the product): PMC FETCH_SIZE / WRITE_SIZE per
# fine-sweep launch in V-cycles and in-cycle sweep times for LIBS (0 = product, else
# build/libmgmc_exp<name>.so).  Build first: VARIANTS="expo1=-DMGMC_ZS_ORDER=1 expo2=-DMGMC_ZS_ORDER=2" bash scripts/build_exp.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/order && export TMPDIR=/tmp
O=gpurun_out/order
for lib in $(echo ${LIBS:-0} | tr ',' ' '); do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$lib.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    K=6 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/${lib}_$c -o pmc --output-format csv -- python3 scripts/vcycle_once.py > $O/${lib}_$c.log 2>&1
    rc=$?; echo "$lib $c rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
done
unset MGMC_LIBRARY
REPS=${REPS:-3} timeout -k 10 600 python scripts/lib_cycle_bench.py ${LIBS:-0} > $O/cycle.log 2>&1; rc=$?
echo "cycle rc=$rc"; cat $O/cycle.log
exit $rc
