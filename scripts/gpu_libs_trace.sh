# V-cycle kernel traces for a list of experiment builds (LIBS="name ..." -> build/libmgmc_<name>.so;
# "product" = the in-tree library): top kernels per build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/libs && export TMPDIR=/tmp
# an entry may carry a z-sweep tile variant: name:variant (MGMC_ZS_VARIANT)
for E in ${LIBS:-product}; do
  L=${E%%:*}; V=${E#*:}; [ "$V" = "$E" ] && V=0
  export MGMC_ZS_VARIANT=$V
  if [ "$L" = product ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$PWD/build/libmgmc_$L.so; fi
  L=$L-v$V
  rm -rf gpurun_out/libs/$L; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/libs/$L -o vt -- python3 scripts/vcycle_once.py > gpurun_out/libs/$L.log 2>&1 || exit 3
  echo "== $L $(tail -1 gpurun_out/libs/$L.log)"
  python3 scripts/kstats.py $(find gpurun_out/libs/$L -name "*kernel_trace.csv" | head -1) 13 > gpurun_out/libs/$L.txt
  head -4 gpurun_out/libs/$L.txt
done
