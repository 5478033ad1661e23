# iteration check: full gpu tests, rng + sweep micro-benchmarks
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 ./scripts/rng_bench > gpurun_out/rng_bench.log 2>&1; rc=$?; echo "rng rc=$rc"; cat gpurun_out/rng_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python scripts/sweep_bench.py 512 7 > gpurun_out/sweep_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/sweep_bench.log
