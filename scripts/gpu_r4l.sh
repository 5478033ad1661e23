# Round 4: j-sweep window reads as single ds_read_b64 (product) against the compiler's ds_read2_b64 pairing
# (build/libmgmc_expread2.so); pair / quad windows from lane shuffles (product) against three loads per row
# (build/libmgmc_expnoshfl.so) -- per-kernel traces and interleaved cycle times; k_tail's index loops
# without integer divisions (tail phase times); parity modules.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4l && export TMPDIR=/tmp
O=gpurun_out/r4l
MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exptprof.so timeout -k 10 120 python scripts/tail_prof.py 512 7 > $O/tail_prof512.log 2>&1; rc=$?
echo "tail prof rc=$rc"; tail -9 $O/tail_prof512.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" "tests/test_gpu_parity.py::test_mgmc_cycles_bitwise" tests/test_gpu_config3.py tests/test_gpu_configs.py tests/test_gpu_lowrank.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 read2 noshfl; do
  if [ "$v" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$v.so; fi
  K=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 scripts/vcycle_once.py > $O/kt_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; [ $rc -eq 0 ] || exit 3
  python3 scripts/kstats.py $O/kt_$v/kt_kernel_trace.csv 13 > $O/kstats_$v.txt; echo "== $v"; grep -E "jsweep|pairs|quads|total" $O/kstats_$v.txt
done
unset MGMC_LIBRARY
REPS=3 timeout -k 10 400 python scripts/lib_cycle_bench.py 0,read2,noshfl > $O/cycle512.log 2>&1; rc=$?
echo "cycle512 rc=$rc"; cat $O/cycle512.log
exit $rc
