# Round 4: small-level launch shapes -- the 127^3 -> 63^3 residual + restriction on 16 x 4 tiles
# (build/libmgmc_expzrs64.so) and the 127^3 prolongation with 4 / 2 planes per thread
# (build/libmgmc_exppz4.so, exppz2.so), with the product's 256-thread quads on 64-pair rows: parity modules, per-kernel traces, cycle times (digests agree).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4o && export TMPDIR=/tmp
O=gpurun_out/r4o
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_config3.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" "tests/test_gpu_parity.py::test_level_kernels_labels" > $O/pytest_0.log 2>&1; rc=$?
echo "pytest 0 rc=$rc"; tail -2 $O/pytest_0.log; [ $rc -eq 0 ] || exit $rc
for v in zrs64 pz4; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py --deselect tests/test_gpu_headline.py::test_headline_kernel_instances "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 zrs64 pz4 pz2; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "zresrestrict<27|prolongate|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
N=256 NLEVEL=6 K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt256 -o kt -- python3 scripts/vcycle_once.py > $O/kt256.log 2>&1; rc=$?
echo "kt256 rc=$rc"; [ $rc -eq 0 ] || exit 3
python3 scripts/kstats.py $O/kt256/kt_kernel_trace.csv 13 > $O/kstats256.txt; cat $O/kstats256.txt
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,zrs64,pz4,pz2 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,zrs64,pz4,pz2 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
