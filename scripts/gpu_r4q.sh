# Round 4: the 256^3 fine level -- the plain sweep on 16-row tiles (512 workgroups = one round of the
# 2 x 256 slots, build/libmgmc_exps16x6.so) and the 7-point residual + restriction with the rounds x
# depth chunk rule (build/libmgmc_expzr7kz.so): parity modules, 256^3 kernel traces, cycle times.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4q && export TMPDIR=/tmp
O=gpurun_out/r4q
for v in s16x6 zr7kz; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_config3.py --deselect tests/test_gpu_config3.py::test_config3_kernel_instances "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 s16x6 zr7kz; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  N=256 NLEVEL=6 K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "zsweep|zresrestrict<7|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,s16x6,zr7kz > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,s16x6 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
