cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "zsweep or smoke" > gpurun_out/pytest_z.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_z.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python scripts/sweep_bench.py 512 7 > gpurun_out/sweep_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/sweep_bench.log
