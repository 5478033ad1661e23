# round-6 evidence, part 1: the whole -m gpu suite (one process), smoke(), the headline determinism tests
# under MGMC_POISON=1
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6final} && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
MGMC_POISON=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py -k "same_seed or cycle_and_qoi" > $O/headline_poison.log 2>&1; rc=$?
echo "headline poison rc=$rc"; tail -2 $O/headline_poison.log
exit $rc
