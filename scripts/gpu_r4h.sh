# Round 4: fine pre-sweep z-chunk pairs marching towards each other (zpairs) -- parity modules first,
# then HBM traffic per launch (separate FETCH_SIZE / WRITE_SIZE passes) and interleaved cycle times
# against MGMC_DISABLE=zpairs at 512^3 and 256^3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4h && export TMPDIR=/tmp
O=gpurun_out/r4h
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_config3.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 nozp; do
  if [ "$v" = nozp ]; then export MGMC_DISABLE=zpairs; else unset MGMC_DISABLE; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    K=4 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/${v}_$c -o pmc -- python3 scripts/vcycle_once.py > $O/${v}_$c.log 2>&1
    rc=$?; echo "$v $c rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
  python3 scripts/pmc_by_kernel.py $O/${v}_FETCH_SIZE $O/${v}_WRITE_SIZE 512 > $O/pmc_$v.txt 2>&1; echo "== $v"; head -6 $O/pmc_$v.txt
done
unset MGMC_DISABLE
REPS=3 timeout -k 10 600 python scripts/lib_cycle_bench.py 0,0+MGMC_DISABLE=zpairs > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log; [ $rc -eq 0 ] || exit $rc
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,0+MGMC_DISABLE=zpairs > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log
exit $rc
