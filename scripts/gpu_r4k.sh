# Round 4: k_tail window reads as single ds_read_b64 (no read2 pairing) and xzero on 3D quad-pass levels --
# tail phase times (timing build), parity modules, interleaved cycle times at 512^3 / 256^3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4k && export TMPDIR=/tmp
O=gpurun_out/r4k
MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exptprof.so timeout -k 10 120 python scripts/tail_prof.py 512 7 > $O/tail_prof512.log 2>&1; rc=$?
echo "tail prof rc=$rc"; tail -9 $O/tail_prof512.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_config3.py tests/test_gpu_configs.py tests/test_gpu_lowrank.py tests/test_gpu_batch.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,0+MGMC_DISABLE=xzero > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,0+MGMC_DISABLE=xzero > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log
exit $rc
