# BASELINE.md section 4 rows 1-3, 5 at the head (scripts/config_table.py); a heartbeat file under
# gpurun_out/ while the bench subprocesses (CPU baselines included) run with their output captured.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ct && export TMPDIR=/tmp
(while true; do date > gpurun_out/ct/heartbeat.txt; sleep 30; done) &
hb=$!
timeout -k 10 1100 python -u scripts/config_table.py gpurun_out/ct/config_table.jsonl > gpurun_out/ct/config_table.log 2>&1; rc=$?
kill $hb
echo "config table rc=$rc"; cat gpurun_out/ct/config_table.log | cut -c1-400
exit $rc
