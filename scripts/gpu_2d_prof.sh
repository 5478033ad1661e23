# kernel trace of the 2D 1024^2 configuration (BASELINE config 2) through bench.py, per-(kernel, grid) summary
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-prof2d} && mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --dim 2 --n 1024 --nlevel 5 --steps 400 --warmup 20 --no-cpu-baseline > $O/bench.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(ls $O/kt/*/*kernel_trace.csv $O/kt/*kernel_trace.csv 2>/dev/null | head -1)
python3 scripts/kstats.py "$f" 420 > $O/kstats.txt; cat $O/kstats.txt
exit 0
