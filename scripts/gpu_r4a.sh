# Round 4, first box call: the 512^3 determinism evidence (oracle-pinned same-seed handles, plain and
# with MGMC_POISON=1), the headline and config-3 parity modules, the default bench and a rocprofv3
# kernel trace of the same bench command whose timed window is summarised separately.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4a && export TMPDIR=/tmp
O=gpurun_out/r4a
PYT="python -u -m pytest -x -v --timeout 900 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_headline.py > $O/headline.log 2>&1; rc=$?
echo "headline rc=$rc"; tail -3 $O/headline.log; [ $rc -eq 0 ] || exit $rc
MGMC_POISON=1 timeout -k 10 600 $PYT tests/test_gpu_headline.py -k "same_seed or cycle_and_qoi" > $O/headline_poison.log 2>&1; rc=$?
echo "headline poison rc=$rc"; tail -3 $O/headline_poison.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $PYT tests/test_gpu_config3.py > $O/config3.log 2>&1; rc=$?
echo "config3 rc=$rc"; tail -3 $O/config3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 $PYT tests/test_gpu_smoother.py "tests/test_gpu_cholesky.py::test_dense_lowrank_column_band_unsupported" > $O/smoother.log 2>&1; rc=$?
echo "smoother rc=$rc"; tail -3 $O/smoother.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
