# 2D fused last pre-sweep + residual + restriction (k_quads_restrict2d): parity tests, then an
# interleaved A/B of the BASELINE config-2 cycle (2D 1024^2, 5 levels) against MGMC_DISABLE=qrestrict
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qr && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 300 \
  --timeout-method thread -k "qr or 2d or qp" > gpurun_out/qr/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/qr/pytest.log; [ $rc -eq 0 ] || exit $rc
A="" B="qrestrict,qprolong" REPS=${REPS:-4} OUT=gpurun_out/qr/ab2d.jsonl bash scripts/env_ab.sh --dim 2 --n 1024 --nlevel 5 \
  --steps 2000 --warmup 50 --plain || exit 1
python - <<'PY'
import json
for l in open("gpurun_out/qr/ab2d.jsonl"):
    tag, js = l.split(" ", 1)
    d = json.loads(js)
    print(tag, d["value"], d["ms_per_step"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qr/prof -o p2d -- python3 bench.py --dim 2 --n 1024 --nlevel 5 --steps 200 --warmup 10 --no-cpu-baseline --plain > gpurun_out/qr/prof.log 2>&1
