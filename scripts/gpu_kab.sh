# Per-kernel A/B of library builds on the box: for each of LIBS (0 = the product, else
# build/libmgmc_<name>.so; "<lib>+VAR=value" adds an environment switch, e.g. 0+MGMC_DISABLE=post_noise)
# a rocprofv3 kernel trace of K V-cycles of N^3 (scripts/vcycle_once.py), then the per-(kernel, grid)
# averages (scripts/kstats.py).  Interleaved REPS times.
#   TAG=r6x LIBS="0 zr27w4" N=512 NLEVEL=7 bash scripts/gpu_kab.sh
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-kab} && mkdir -p $O
for r in $(seq 1 ${REPS:-1}); do
  for ent in ${LIBS:-0}; do
    lib=${ent%%+*}; extra=""; [ "$ent" != "$lib" ] && extra=${ent#*+}
    name=$(echo "$ent" | tr '+=,' '___')
    if [ "$lib" = "0" ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=build/libmgmc_$lib.so; fi
    K=${K:-10} timeout -k 10 180 env $extra rocprofv3 --kernel-trace --output-format csv -d $O/kt_${name}_$r -o kt -- python3 scripts/vcycle_once.py > $O/kt_${name}_$r.log 2>&1 || { echo "trace $ent failed"; exit 1; }
    f=$(ls $O/kt_${name}_$r/*/*kernel_trace.csv $O/kt_${name}_$r/*kernel_trace.csv 2>/dev/null | head -1)
    echo "== $ent rep $r: $(grep 'vcycle ms' $O/kt_${name}_$r.log)"
    python3 scripts/kstats.py "$f" $(( ${K:-10} + 3 )) > $O/kstats_${name}_$r.txt
    head -26 $O/kstats_${name}_$r.txt
  done
done
unset MGMC_LIBRARY
exit 0
