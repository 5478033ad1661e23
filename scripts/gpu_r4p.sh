# Round 4: residual + restriction workgroup sizes -- the 255^3 -> 127^3 27-point instance with 320
# threads and <= 128 VGPRs (3 workgroups of 5 waves per CU; build/libmgmc_expzr27w4.so), the fine 7-point
# instance with 576 threads (2 rounds of residual items instead of 3; expzr7nt576.so) -- and the 127^3 /
# 63^3 prolongation with 4 planes per thread (exppz4.so): parity modules, kernel traces, cycle times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4p && export TMPDIR=/tmp
O=gpurun_out/r4p
for v in zr27w4 zr7nt576; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py --deselect tests/test_gpu_headline.py::test_headline_kernel_instances "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 zr27w4 zr7nt576; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "zresrestrict|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,zr27w4,zr7nt576,pz4 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,zr27w4,zr7nt576,pz4 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
