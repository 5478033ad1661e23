# round-6 fix run: the LDS-race stress of the standalone fine sweep (pre-fix build against the product),
# then the whole -m gpu suite, smoke, poisoned headline (gpu_r6_final1.sh) and the bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6fix} && mkdir -p $O
REPS=40 timeout -k 10 500 python -u scripts/race_stress.py prefix 0 > $O/race_stress.txt 2>&1; rc=$?
echo "race stress rc=$rc"; cat $O/race_stress.txt; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r6fix} bash scripts/gpu_r6_final1.sh || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json | cut -c1-400
exit $rc
