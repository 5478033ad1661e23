# One PMC pass (kernel-trace only) over 512^3 V-cycles: where the waves' cycles go per kernel
# (SQ_WAIT_ANY = parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls, SQ_ACTIVE_INST_ANY =
# issuing; MI355X_MICROARCH.md: the three are disjoint and sum to SQ_WAVE_CYCLES)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmcs && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmcs/s -o s \
  --output-format csv -- python3 scripts/vcycle_once.py > gpurun_out/pmcs/s.log 2>&1
