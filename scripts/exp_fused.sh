# fused cycle boundaries: parity tests, kernel trace of the fused launch, plain-replay bench A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/fused
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread > gpurun_out/fused/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/fused/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fused/tr -o tr -- python3 scripts/fused_once.py > gpurun_out/fused/tr.log 2>&1; rc=$?
tail -1 gpurun_out/fused/tr.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/kstats.py $(find gpurun_out/fused/tr -name "*kernel_trace.csv" | head -1) 1 | head -4
for v in fused nofused; do
  d=""; [ $v = nofused ] && d=fuse_cycles
  MGMC_DISABLE=$d timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --plain > gpurun_out/fused/bench_$v.json 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fused/bench_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
