# Round 4: the symmetric 27-point residual + restriction on 48-wide tiles (441 residual items = 2 rounds
# of 256 threads instead of 585 = 3; build/libmgmc_expzrcx48.so) -- parity modules, kernel traces at
# 512^3 / 256^3, cycle times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4u && export TMPDIR=/tmp
O=gpurun_out/r4u
MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_expzrcx48.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_config3.py --deselect tests/test_gpu_headline.py::test_headline_kernel_instances --deselect tests/test_gpu_config3.py::test_config3_kernel_instances "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_cx48.log 2>&1; rc=$?
echo "pytest cx48 rc=$rc"; tail -2 $O/pytest_cx48.log; [ $rc -eq 0 ] || exit $rc
for v in 0 zrcx48; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "zresrestrict<27|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,zrcx48 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,zrcx48 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log
exit $rc
