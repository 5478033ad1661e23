# Round-3 evidence on the GPU box: default bench line, rocprofv3 --kernel-trace --stats of the bench
# command, and per-kernel FETCH_SIZE / WRITE_SIZE passes over 512^3 V-cycles (separate --pmc runs).
#   OUT=gpurun_out/r3 bash scripts/gpu_r3_profile.sh
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
O=${OUT:-gpurun_out/r3}; mkdir -p $O
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $O/bench.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 $O/prof.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    K=6 timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o pmc -- python3 scripts/vcycle_once.py > $O/pmc_$c.log 2>&1; rc=$?
    echo "pmc $c rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
