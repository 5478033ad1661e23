# Round 4 final head: parity modules (kernel-instance tests included), 256^3 cycle, then the round
# evidence (bench line with CPU baseline, rocprofv3 stats of the bench command, PMC FETCH / WRITE passes).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4w && export TMPDIR=/tmp
O=gpurun_out/r4w
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_config3.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" "tests/test_gpu_parity.py::test_level_kernels_labels" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 200 python scripts/lib_cycle_bench.py 0 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_round.sh
