mkdir -p gpurun_out/r3 && export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/r3/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r3/b512.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --n 256 --nlevel 6 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r3/b256.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --posterior 8 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r3/p256.log 2>&1 || exit 5
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r3/prof.log 2>&1 || exit 6
for f in gpurun_out/r3/b512.log gpurun_out/r3/b256.log gpurun_out/r3/p256.log; do tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"; done
