# PMC passes (kernel-trace only) over a few 512^3 V-cycles: per-kernel busy / LDS / traffic counters
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcc && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmcc/$name -o $name --output-format csv -- python3 scripts/vcycle_once.py > gpurun_out/pmcc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run a VALUBusy SALUBusy || exit 3
run b SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE || exit 3
run c FETCH_SIZE || exit 3
run d WRITE_SIZE || exit 3
exit 0
