# Round 4: the nx = 128 level (level 2 at 512^3, level 1 at 256^3) as j-marching half-sweeps
# (build/libmgmc_expjs128.so) or as quad passes on rows of 64 pairs (build/libmgmc_expqm64.so), against
# the pair passes (product) -- parity modules on each, per-kernel traces, cycle times
# at 512^3 / 256^3 (state digests must agree).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4m && export TMPDIR=/tmp
O=gpurun_out/r4m
for v in js128 qm64; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py --deselect tests/test_gpu_headline.py::test_headline_kernel_instances "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in js128 qm64; do
  export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "jsweep|pairs|quads|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,js128,qm64 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,js128,qm64 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log
exit $rc
