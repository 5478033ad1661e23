# Round 4: quad passes on the 63^3 / 31^3 levels with smaller workgroups (512 threads: 93 / 15
# workgroups per launch at 512^3) -- 256 / 128 / 64 threads (build/libmgmc_expq3n*.so): parity modules,
# kernel traces, cycle times at 512^3 / 256^3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4v && export TMPDIR=/tmp
O=gpurun_out/r4v
for v in q3n128 q3n64; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_config3.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 q3n256 q3n128 q3n64; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "quads|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,q3n256,q3n128,q3n64 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,q3n256,q3n128,q3n64 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
