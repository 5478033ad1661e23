#!/bin/bash
# GPU-box check: smoke, gpu tests, short bench, rocprofv3 kernel trace.  Stops at the first
# fault / abort / timeout (exit codes other than 0 and 1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS=${STEPS:-30}
echo "== smoke" ; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; ok $rc || exit $rc
echo "== pytest -m gpu"; timeout -k 10 1200 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/pytest_gpu.log; ok $rc || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -5 $OUT/bench.log; ok $rc || exit $rc
if [ -n "$PROFILE" ]; then
  echo "== rocprofv3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
  find $OUT/prof -name "*stats*" | head
fi
exit 0
