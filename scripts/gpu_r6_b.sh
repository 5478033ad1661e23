# round-6 batch b: the -m gpu suite, in-cycle A/B of the product against build/libmgmc_<AB>.so, per-kernel
# A/B of timing-only variants (KAB), rocprof kernel trace of a short bench
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6b} && mkdir -p $O
if [ -z "$SKIP_PYTEST" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$AB" ]; then
  REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py $AB > $O/ab512.log 2>&1; rc=$?; cat $O/ab512.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$KAB" ]; then
  TAG=${TAG:-r6b}/kab LIBS="$KAB" REPS=${KREPS:-1} timeout -k 10 600 bash scripts/gpu_kab.sh > $O/kab.txt 2>&1; rc=$?
  grep -E "^==|jsweep|quads|zresrestrict<27|tail|total" $O/kab.txt; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -1 $O/prof.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
