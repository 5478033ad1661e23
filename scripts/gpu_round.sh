# Round check on the GPU box: the full -m gpu suite, in-cycle A/B of the product against build/libmgmc_<LIBS>.so
# (512^3 and 256^3, scripts/lib_cycle_bench.py), and a rocprofv3 kernel trace of a short bench.
#   TAG=r5b LIBS=prev bash scripts/gpu_round.sh
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/${TAG:-round} && export TMPDIR=/tmp
O=gpurun_out/${TAG:-round}
if [ -z "$SKIP_PYTEST" ]; then  # PYTEST_K: a subset
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py ${LIBS:-prev},0 > $O/ab512.log 2>&1; rc=$?; grep -v "^ " $O/ab512.log | tail -8; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py ${LIBS:-prev},0 > $O/ab256.log 2>&1; rc=$?; grep -v "^ " $O/ab256.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; exit $rc
