# k_tail's Box-Muller pairs drawn by spare workgroups of the restriction before it: 3D parity tests
# (tails, batched chains, low-rank tails), the 256^3 / 512^3 cycles against the previous library build,
# then BASELINE.md's config table
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tn && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest --maxfail 3 tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_lowrank.py \
  tests/test_gpu_headline.py -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-3d or tail or headline}" \
  > gpurun_out/tn/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/tn/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="0 prev" REPS=3 OUT=gpurun_out/tn/ab256.jsonl bash scripts/lib_bench_ab.sh --n 256 --nlevel 6 --steps 500 --warmup 20 \
  --plain || exit 1
LIBS="0 prev" REPS=2 OUT=gpurun_out/tn/ab512.jsonl bash scripts/lib_bench_ab.sh --steps 100 --warmup 10 --plain || exit 1
python -c "
import json
for f in ('ab256', 'ab512'):
    for l in open('gpurun_out/tn/%s.jsonl' % f):
        t, j = l.split(' ', 1); d = json.loads(j); print(f, t, d['value'], d['ms_per_step'])
"
[ -n "$NO_TABLE" ] || timeout -k 10 900 python -u scripts/config_table.py gpurun_out/tn/config_table.jsonl > gpurun_out/tn/ct.log 2>&1
