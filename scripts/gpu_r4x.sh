# Round 4: 2D Galerkin quad passes with 256 / 1024 threads (build/libmgmc_expq2n*.so) against 512 --
# 2D parity modules, then config-2 bench lines (2D 1024^2, 5 levels), interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4x && export TMPDIR=/tmp
O=gpurun_out/r4x
for v in q2n256 q2n1024; do
  MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" tests/test_gpu_configs.py > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 $O/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in 0 q2n256 q2n1024; do
    if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
    timeout -k 10 120 python bench.py --dim 2 --n 1024 --nlevel 5 --steps 2000 --warmup 50 --no-cpu-baseline > $O/b_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || exit $rc
    echo "$v $r $(tail -1 $O/b_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
