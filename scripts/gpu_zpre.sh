# the coarse SSOR sampler's noise drawn by spare workgroups of the fused restriction before it: 2D
# parity tests, then the config-2 cycle against the previous library build (build/libmgmc_expprev.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/zp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail 3 tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_configs.py \
  tests/test_gpu_cholesky.py tests/test_gpu_qoi_vector.py -q --timeout 300 --timeout-method thread -k "qr or 2d or nonfinite" > gpurun_out/zp/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/zp/pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="0 prev" REPS=3 OUT=gpurun_out/zp/ab.jsonl bash scripts/lib_bench_ab.sh --dim 2 --n 1024 --nlevel 5 --steps 2000 \
  --warmup 50 --plain || exit 1
python -c "
import json
for l in open('gpurun_out/zp/ab.jsonl'):
    t, j = l.split(' ', 1); d = json.loads(j); print(t, d['value'], d['ms_per_step'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zp/prof -o p2d -- python3 bench.py --dim 2 --n 1024 --nlevel 5 --steps 200 --warmup 10 --no-cpu-baseline --plain > gpurun_out/zp/prof.log 2>&1
