# round-6 first GPU batch: the -m gpu suite, per-kernel PMC, the grid-barrier microbenchmark, per-kernel A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6s
bash scripts/gpu_r6_suite_pmc.sh || exit 1
timeout -k 10 60 ./scripts/ubench/grid_barrier > gpurun_out/r6s/grid_barrier.txt 2>&1 || exit 1
cat gpurun_out/r6s/grid_barrier.txt
TAG=r6kab LIBS="0 zr27w4 zr27cy3" REPS=2 bash scripts/gpu_kab.sh > gpurun_out/r6s/kab.txt 2>&1; rc=$?
grep -E "^==|zresrestrict<27, 64" gpurun_out/r6s/kab.txt; exit $rc
