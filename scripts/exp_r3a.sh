# round-3 measurements: graph replay modes (timed / plain / unrolled) and VALU counters of the cycle
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/exp1 gpurun_out/pmcc
bash scripts/exp_unroll.sh || exit 1
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcc/$name -o $name --output-format csv -- python3 scripts/vcycle_once.py > gpurun_out/pmcc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run a VALUBusy SALUBusy || exit 3
run b SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE || exit 3
python3 scripts/pmc_table.py gpurun_out/pmcc > gpurun_out/pmcc/table.txt
exit 0
