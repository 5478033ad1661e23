# BASELINE.md section 4 rows at the round-6 head (scripts/config_table.py: configs 1, 2, 3, 5, 5' with CPU
# baselines) and config 2's kernel trace
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6cfg} && mkdir -p $O
timeout -k 10 1000 python scripts/config_table.py $O/config_table.jsonl > $O/config_table.log 2>&1; rc=$?
echo "config table rc=$rc"; tail -3 $O/config_table.log; [ $rc -eq 0 ] || exit $rc
exit 0
