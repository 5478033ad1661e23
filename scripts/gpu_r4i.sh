# Round 4: the coarse level's first pre-sweep takes x_{l+1} = 0 as constants (xzero) -- parity modules,
# then per-kernel traces and interleaved cycle times against MGMC_DISABLE=xzero.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4i && export TMPDIR=/tmp
O=gpurun_out/r4i
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_config3.py tests/test_gpu_fem.py tests/test_gpu_batch.py tests/test_gpu_configs.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 noxz; do
  if [ "$v" = noxz ]; then export MGMC_DISABLE=xzero; else unset MGMC_DISABLE; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; head -9 $O/kstats_$v.txt
done
unset MGMC_DISABLE
REPS=3 timeout -k 10 600 python scripts/lib_cycle_bench.py 0,0+MGMC_DISABLE=xzero > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
