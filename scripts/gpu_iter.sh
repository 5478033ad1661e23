# iteration check: full gpu tests, micro-benchmarks, per-kernel V-cycle trace
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1; else timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; fi; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python scripts/sweep_bench.py 512 7 > gpurun_out/sweep_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; cat gpurun_out/sweep_bench.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
rm -rf gpurun_out/vtrace; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vtrace -o vt -- python3 scripts/vcycle_once.py > gpurun_out/vtrace.log 2>&1; rc=$?; echo "trace rc=$rc"
python3 scripts/kstats.py $(find gpurun_out/vtrace -name "*kernel_trace.csv" | head -1) 13
