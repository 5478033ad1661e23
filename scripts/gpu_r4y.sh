# Round 4 final: smoke(), parity modules with the product's 256-thread 2D quad passes, config-2 bench
# lines against 128 threads (build/libmgmc_expq2n128.so), interleaved.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4y && export TMPDIR=/tmp
O=gpurun_out/r4y
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" "tests/test_gpu_parity.py::test_level_kernels_labels" tests/test_gpu_configs.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 q2n128; do
    if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
    timeout -k 10 120 python bench.py --dim 2 --n 1024 --nlevel 5 --steps 2000 --warmup 50 --no-cpu-baseline > $O/b_${v}_$r.log 2>&1; rc=$?
    [ $rc -eq 0 ] || exit $rc
    echo "$v $r $(tail -1 $O/b_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
