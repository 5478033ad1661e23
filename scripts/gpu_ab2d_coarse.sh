cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && export TMPDIR=/tmp
for r in 1 2 3; do
  for L in 0 c1; do
    if [ $L = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_exp$L.so; fi
    timeout -k 10 120 python bench.py --dim 2 --n 1024 --nlevel 5 --steps 3000 --warmup 200 --no-cpu-baseline > gpurun_out/ab/b2d_$L.log 2>&1 || exit 3
    echo "$L $(tail -1 gpurun_out/ab/b2d_$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
