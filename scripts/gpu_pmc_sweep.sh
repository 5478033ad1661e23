# PMC passes over a few 512^3 V-cycles for the stall picture of the fine sweeps (one counter group
# per rocprofv3 run, kernel-trace only)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcs && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  K=4 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcs/$name -o $name --output-format csv -- python3 scripts/vcycle_once.py > gpurun_out/pmcs/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run w SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES || exit 3
run l SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 3
run t TCC_HIT_sum TCC_MISS_sum || exit 3
exit 0
