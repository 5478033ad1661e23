# Kernel A/B on the GPU box: a parity subset of the -m gpu suite, then interleaved in-cycle timing of
# the product against experiment builds.   LIBS=0,expold,... PYTEST_K='...' bash scripts/gpu_ab.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/ab/pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
REPS=${REPS:-3} timeout -k 10 600 python scripts/lib_cycle_bench.py ${LIBS:-0} > gpurun_out/ab/cycle.log 2>&1; rc=$?
grep -v "^ \|Traceback" gpurun_out/ab/cycle.log; exit $rc
