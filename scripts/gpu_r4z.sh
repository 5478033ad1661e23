# Round 4: quad-pass workgroups one step smaller again -- 127^3 rows with 128 threads (T = 1;
# build/libmgmc_expqw128.so) and 2D with 64 threads (build/libmgmc_expq2n64.so): parity modules,
# cycle times (256^3 / 512^3), config-2 bench lines, interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4z && export TMPDIR=/tmp
O=gpurun_out/r4z
for v in qw128 q2n64; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,qw128 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,qw128 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 q2n64; do
    if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
    timeout -k 10 120 python bench.py --dim 2 --n 1024 --nlevel 5 --steps 2000 --warmup 50 --no-cpu-baseline > $O/b_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || exit $rc
    echo "$v $r $(tail -1 $O/b_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
