# Round-2 baseline check on the GPU box: gpu tests, then the headline bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r2a && export TMPDIR=/tmp
O=gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $O/b512.log 2>&1 || exit 3
tail -1 $O/b512.log
