# kernel traces of the 256^3 configurations (3: prior, 5: posterior with 8 points) through bench.py, and
# per-(kernel, grid) summaries (scripts/kstats.py)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-cfgprof} && mkdir -p $O
for c in "prior:" "post8:--posterior 8"; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$name -o kt -- python3 bench.py --n 256 --nlevel 6 $args --steps 60 --warmup 5 --no-cpu-baseline > $O/bench_$name.log 2>&1 || { echo "trace $name failed"; exit 1; }
  f=$(ls $O/kt_$name/*/*kernel_trace.csv $O/kt_$name/*kernel_trace.csv 2>/dev/null | head -1)
  python3 scripts/kstats.py "$f" 65 > $O/kstats_$name.txt
  echo "== $name: $(tail -1 $O/bench_$name.log | cut -c1-200)"
  cat $O/kstats_$name.txt
done
exit 0
