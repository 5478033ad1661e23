# 2D fused kernel (k_quads_restrict2d): parity tests, an interleaved
# A/B of the BASELINE config-2 cycle (2D 1024^2, 5 levels) against MGMC_DISABLE=<token> (AB_LIST),
# the default (segment-timed) bench lines of configs 2 and 3, and a rocprof kernel trace of config 2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qr && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail 3 tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_configs.py \
  tests/test_gpu_cholesky.py tests/test_gpu_adapter.py -q --timeout 300 --timeout-method thread \
  -k "${PYTEST_K:-qr or 2d}" > gpurun_out/qr/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/qr/pytest.log; [ $rc -eq 0 ] || exit $rc
for b in ${AB_LIST:-qrestrict}; do
  A="" B="$b" REPS=${REPS:-3} OUT=gpurun_out/qr/ab2d_$b.jsonl bash scripts/env_ab.sh --dim 2 --n 1024 \
    --nlevel 5 --steps 2000 --warmup 50 --plain || exit 1
  B=$b python - <<'PY'
import json, os
for l in open("gpurun_out/qr/ab2d_%s.jsonl" % os.environ["B"]):
    tag, js = l.split(" ", 1)
    d = json.loads(js)
    print(os.environ["B"], tag, d["value"], d["ms_per_step"])
PY
done
timeout -k 10 200 python bench.py --dim 2 --n 1024 --nlevel 5 --steps 2000 --warmup 50 --no-cpu-baseline > gpurun_out/qr/b2d.json || exit 1
timeout -k 10 200 python bench.py --n 256 --nlevel 6 --steps 500 --warmup 20 --no-cpu-baseline > gpurun_out/qr/b256.json || exit 1
python -c "
import json
for f in ('b2d', 'b256'):
    d = json.loads(open('gpurun_out/qr/%s.json' % f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d.get('segments_ms_per_step'), d['roofline']['frac'] if d.get('roofline') else None)
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qr/prof -o p2d -- python3 bench.py --dim 2 --n 1024 --nlevel 5 --steps 200 --warmup 10 --no-cpu-baseline --plain > gpurun_out/qr/prof.log 2>&1
