# round-6 batch 2: the -m gpu suite (quads LANES in), per-kernel PMC, grid-barrier microbenchmark, A/B
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r6s
timeout -k 10 60 ./scripts/ubench/grid_barrier > gpurun_out/r6s/grid_barrier.txt 2>&1 || exit 1
cat gpurun_out/r6s/grid_barrier.txt
TAG=r6kab LIBS="0 nolanes zr27w4" REPS=2 bash scripts/gpu_kab.sh > gpurun_out/r6s/kab.txt 2>&1 || exit 1
grep -E "^==|zresrestrict<27, 64|sweep_quads" gpurun_out/r6s/kab.txt | head -60
bash scripts/gpu_r6_suite_pmc.sh
