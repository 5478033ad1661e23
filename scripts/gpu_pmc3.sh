# PMC passes (kernel-trace only): busy / wait / issue counters of z-sweep variants
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc3 && export TMPDIR=/tmp
run() {  # name variant counters...
  local name=$1; shift; local v=$1; shift
  MGMC_ZS_VARIANT=$v K=4 timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc3/$name -o $name --output-format csv -- python3 scripts/sweep_once.py > gpurun_out/pmc3/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
for V in ${VARIANTS:-0 5 11}; do
  run v${V}_a $V VALUBusy SALUBusy || echo "a failed"
  run v${V}_b $V SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 || echo "b failed"
  run v${V}_c $V SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE || echo "c failed"
done
exit 0
