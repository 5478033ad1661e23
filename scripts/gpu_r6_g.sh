# round-6 batch g: low-rank GPU tests (xzero / tail-drawn noise on low-rank quad levels), config 5 / 3 A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6g} && mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lowrank.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-lowrank or posterior or config5 or variant or tail_drawn}" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="0 0+MGMC_DISABLE=xzero,post_noise" REPS=3 OUT=$O/ab_cfg5.jsonl timeout -k 10 600 bash scripts/lib_bench_ab.sh --posterior 8 --steps 200 --warmup 20 || exit 1
LIBS="0 0+MGMC_DISABLE=post_noise" REPS=3 OUT=$O/ab_cfg3.jsonl timeout -k 10 600 bash scripts/lib_bench_ab.sh --n 256 --nlevel 6 --steps 200 --warmup 20 || exit 1
python3 - << 'PY'
import json, os
O = os.environ.get("TAG", "r6g")
for f in ("ab_cfg5", "ab_cfg3"):
    for line in open(f"gpurun_out/{O}/{f}.jsonl"):
        tag, _, js = line.partition(" ")
        d = json.loads(js)
        print(f, tag, d["value"], d["ms_per_step"])
PY
exit 0
