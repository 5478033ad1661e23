# PMC stall/instruction picture of the fine sweeps for several library builds (LIBS=0,old,...; 0 =
# product, else build/libmgmc_<name>.so), one counter group per rocprofv3 run, kernel-trace only
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcab && export TMPDIR=/tmp
for lib in $(echo ${LIBS:-0} | tr ',' ' '); do
  if [ "$lib" = 0 ]; then unset MGMC_LIBRARY; else export MGMC_LIBRARY=$GRAFT_REPO_ROOT/build/libmgmc_$lib.so; fi
  for g in "w:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES" \
           "l:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"; do
    n=${g%%:*}; c=${g#*:}
    K=3 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmcab/${lib}_$n -o p --output-format csv -- python3 scripts/vcycle_once.py > gpurun_out/pmcab/${lib}_$n.log 2>&1
    rc=$?; echo "$lib $n rc=$rc"; [ $rc -eq 0 ] || exit 3
  done
done
exit 0
