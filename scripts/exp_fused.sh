cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/fused
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread > gpurun_out/fused/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/fused/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fused/tr -o tr -- python3 scripts/fused_once.py > gpurun_out/fused/tr.log 2>&1; rc=$?
tail -1 gpurun_out/fused/tr.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py $(find gpurun_out/fused/tr -name "*kernel_trace.csv" | head -1) 1 | head -5
