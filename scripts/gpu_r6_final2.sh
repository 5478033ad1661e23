# round-6 evidence, part 2: the default bench line (CPU baseline included), rocprofv3 --stats of a bench
# run, per-kernel HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes over V-cycles), the SQ wave-cycle
# split, and the BASELINE.md section 4 configuration table
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6final} && mkdir -p $O
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS'))" > $O/cpu.txt
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  K=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o pmc -- python3 scripts/vcycle_once.py > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
K=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $O/sq -o sq --output-format csv -- python3 scripts/vcycle_once.py > $O/sq.log 2>&1 || { echo "pmc sq failed"; exit 1; }
python3 scripts/pmc_by_kernel.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE 512 > $O/pmc_by_kernel.txt 2>&1
if [ -n "$CONFIG_TABLE" ]; then
  timeout -k 10 900 python scripts/config_table.py $O/config_table.jsonl > $O/config_table.log 2>&1; rc=$?
  echo "config table rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
exit 0
