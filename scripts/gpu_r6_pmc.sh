# Round-6 per-kernel PMC at the current head over 512^3 V-cycles (scripts/vcycle_once.py): HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md HBM section), wave-cycle split and LDS.
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6pmc} && mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  K=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o pmc -- python3 scripts/vcycle_once.py > $O/pmc_$c.log 2>&1 || exit 1
done
K=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU -d $O/s -o s --output-format csv -- python3 scripts/vcycle_once.py > $O/s.log 2>&1 || exit 1
K=6 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD \
  -d $O/l -o l --output-format csv -- python3 scripts/vcycle_once.py > $O/l.log 2>&1 || exit 1
python3 scripts/pmc_by_kernel.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE 512 > $O/pmc_by_kernel.txt 2>&1
exit 0
