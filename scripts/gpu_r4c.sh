# Round 4, re-entry box call: the whole -m gpu suite at the head (symmetric-stencil kernels, chunk
# clamps, z-marching prolongation), interleaved cycle A/B of those switches at 512^3 and 256^3, the
# default bench (with the CPU baseline) and a rocprofv3 kernel trace of the bench command.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4c && export TMPDIR=/tmp
O=gpurun_out/r4c
# k_tail phase times (timing build with wall-clock stamps; never the product)
MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exptprof.so timeout -k 10 120 python scripts/tail_prof.py 512 7 > $O/tail_prof512.log 2>&1; rc=$?
echo "tail prof rc=$rc"; cat $O/tail_prof512.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 600 python scripts/lib_cycle_bench.py 0,noclamp,0+MGMC_DISABLE=sym,0+MGMC_DISABLE=prolong_z > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=2 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,noclamp,0+MGMC_DISABLE=sym,0+MGMC_DISABLE=prolong_z > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
