# Round 4 timing experiments (builds in build/, never the product): fine-sweep tile orders (o1, o2:
# PMC traffic per fine-sweep launch + in-cycle times) and the 27-point residual + restriction tile
# height (zc3, zc3k4: cycle times).  Interleaved repetitions in one box call.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r4b && export TMPDIR=/tmp
O=gpurun_out/r4b
# k_tail phase times (timing build with wall-clock stamps; never the product)
MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exptprof.so timeout -k 10 120 python scripts/tail_prof.py 512 7 > $O/tail_prof512.log 2>&1; rc=$?
echo "tail prof rc=$rc"; cat $O/tail_prof512.log; [ $rc -eq 0 ] || exit $rc
# correctness first: the symmetric-stencil kernels (k_jsweep_half<128,.,true>, k_tail<3,true>) at the
# headline and config-3 sizes and their MGMC_DISABLE=sym variants, bitwise against the oracle
timeout -k 10 600 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_config3.py "tests/test_gpu_parity.py::test_variant_cycles_bitwise" -k "headline or config3 or sym or prolong_z or fuse_prolong" > $O/sym_parity.log 2>&1; rc=$?
echo "sym parity rc=$rc"; tail -3 $O/sym_parity.log; [ $rc -eq 0 ] || exit $rc
for lib in 0 noclamp o1; do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$lib.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    K=6 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $O/${lib}_$c -o pmc --output-format csv -- python3 scripts/vcycle_once.py > $O/${lib}_$c.log 2>&1
    rc=$?; echo "$lib $c rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
done
unset MGMC_LIBRARY
REPS=2 timeout -k 10 800 python scripts/lib_cycle_bench.py 0,noclamp,0+MGMC_DISABLE=sym,jrole0,pz0,pz16,o1,o2,zc3,jd4,jr2 > $O/cycle.log 2>&1; rc=$?
echo "cycle rc=$rc"; cat $O/cycle.log; [ $rc -eq 0 ] || exit $rc
# config 3 (256^3, 6 levels): fine-sweep tile heights / chunk depths (the 512^3-tuned TY 20, TZ 32 leaves
# 416 tiles on 512 workgroup slots at 256^3)
N=256 NLEVEL=6 REPS=3 timeout -k 10 500 python scripts/lib_cycle_bench.py 0,noclamp,pz0,s16x6,s16x6x24,s20x6x16 > $O/cycle256.log 2>&1; rc=$?
echo "cycle256 rc=$rc"; cat $O/cycle256.log
exit $rc
