# Round evidence on the GPU box: (optional) gpu tests, the default bench (with the CPU baseline),
# rocprofv3 stats of the bench command, PMC traffic of both fine sweeps inside V-cycles (separate
# FETCH_SIZE / WRITE_SIZE passes).
#   RUN_PYTEST=1 bash scripts/profile_round.sh     BENCH_ARGS="--steps 100"
#   RUN_SMOKE=1: __graft_entry__.smoke();  RUN_POISON=1: the headline cycle / same-seed tests under MGMC_POISON=1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/round && export TMPDIR=/tmp
O=gpurun_out/round
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > $O/cpu.txt
if [ -n "$RUN_PYTEST" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$RUN_SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 $O/smoke.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$RUN_POISON" ]; then
  MGMC_POISON=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_headline.py -k "same_seed or cycle_and_qoi" > $O/headline_poison.log 2>&1; rc=$?
  echo "headline poison rc=$rc"; tail -3 $O/headline_poison.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -2 $O/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  for c in FETCH_SIZE WRITE_SIZE; do
    K=6 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o pmc -- python3 scripts/vcycle_once.py > $O/pmc_$c.log 2>&1; rc=$?
    echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
