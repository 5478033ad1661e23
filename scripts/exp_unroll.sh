cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/exp1
for v in "timed::" "plain:--plain:" "plain4:--plain:4" "plain8:--plain:8" "timed2:::"; do
  IFS=: read -r name flag unroll <<< "$v"
  MGMC_GRAPH_UNROLL=$unroll timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline $flag > gpurun_out/exp1/$name.json 2> gpurun_out/exp1/$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp1/$name.json'));print('$name', d['value'], d['ms_per_step'])"
done
