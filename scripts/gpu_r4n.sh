# Round 4: quad passes on the 127^3 levels (rows of 64 pairs; product: 512-thread workgroups) -- the
# parity modules that name or vary the level kernels, per-kernel traces and cycle times against
# 256- / 1024-thread workgroups (build/libmgmc_expqw256.so, build/libmgmc_expqw1024.so).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4n && export TMPDIR=/tmp
O=gpurun_out/r4n
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_config3.py tests/test_gpu_configs.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 qw256 qw1024; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "quads|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
N=256 NLEVEL=6 REPS=3 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,qw256,qw1024 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log; [ $rc -eq 0 ] || exit $rc
REPS=2 timeout -k 10 300 python scripts/lib_cycle_bench.py 0,qw256,qw1024 > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
