# the -m gpu suite on the box (one process), log under gpurun_out/tests
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tests && export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} --durations=15 > gpurun_out/tests/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/tests/pytest.log; exit $rc
