# PMC passes (kernel-trace only) for z-sweep variants: issue / stall / LDS counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc2 && export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc2/counters.txt 2>&1 || true
run() {  # name variant counters...
  local name=$1; shift; local v=$1; shift
  MGMC_ZS_VARIANT=$v K=4 timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc2/$name -o $name --output-format csv -- python3 scripts/sweep_once.py > gpurun_out/pmc2/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
for V in ${VARIANTS:-0 3}; do
  run v${V}_a $V SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 3
  run v${V}_b $V SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY || echo "b failed"
  run v${V}_c $V SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_IFETCH || echo "c failed"
done
exit 0
