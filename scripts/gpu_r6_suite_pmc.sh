# the -m gpu suite (one process) then the round-6 per-kernel PMC passes
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6s
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > gpurun_out/r6s/pytest.log 2>&1; rc=$?
tail -4 gpurun_out/r6s/pytest.log
[ $rc -eq 0 ] || exit $rc
[ -n "$SKIP_PMC" ] || TAG=r6pmc bash scripts/gpu_r6_pmc.sh
