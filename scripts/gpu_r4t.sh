# Round 4: level-1 j-sweep with a 6-row LDS ring (one more barrier per step; 40 KB, 4 workgroups per CU
# at <= 128 VGPRs): JS_D 3 (build/libmgmc_expjs6.so) and 2 (expjs6d2.so) against the product --
# parity modules, kernel traces, cycle times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4t && export TMPDIR=/tmp
O=gpurun_out/r4t
for v in js6 js6d2; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 js6 js6d2; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "jsweep|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,js6,js6d2 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
