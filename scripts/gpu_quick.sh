# quick iteration on the GPU box: selected gpu tests (PYTEST_K), then a rocprofv3 kernel trace of
# a few 512^3 V-cycles summarised per kernel
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/q && export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/q/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 gpurun_out/q/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
rm -rf gpurun_out/q/vt; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/q/vt -o vt -- python3 scripts/vcycle_once.py > gpurun_out/q/vt.log 2>&1; rc=$?; echo "trace rc=$rc"; tail -2 gpurun_out/q/vt.log
[ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py $(find gpurun_out/q/vt -name "*kernel_trace.csv" | head -1) 13
