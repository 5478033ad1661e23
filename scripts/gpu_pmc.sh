# PMC passes (kernel-trace only, no sys-trace) for the fine sweep kernels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc && export TMPDIR=/tmp
run() {  # name env counters...
  local name=$1; shift; local envs=$1; shift
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$name -o $name --output-format csv -- python3 scripts/sweep_once.py > gpurun_out/pmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
for V in colour:MGMC_NO_ZSWEEP=1 zs4:MGMC_ZS_VARIANT=4 zs0:MGMC_ZS_VARIANT=0; do
  nm=${V%%:*}; ev=${V#*:}
  run ${nm}_a "$ev" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 3
  run ${nm}_b "$ev" FETCH_SIZE || exit 3
  run ${nm}_c "$ev" WRITE_SIZE || exit 3
  run ${nm}_d "$ev" SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_ANY SQ_WAIT_ANY || echo "d failed (counter names?)"
done
exit 0
