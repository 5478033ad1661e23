# round-6 fix run: the whole -m gpu suite, smoke, poisoned headline (gpu_r6_final1.sh), then the bench line
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && O=gpurun_out/${TAG:-r6fix} && mkdir -p $O
TAG=${TAG:-r6fix} bash scripts/gpu_r6_final1.sh || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; cat $O/bench.json | cut -c1-400
exit $rc
