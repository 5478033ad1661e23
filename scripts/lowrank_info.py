"""Per-level low-rank sizes of BASELINE config 5 at 256^3 (GPU box): unknowns, (m, B_bar rows) per
sweep direction, and the kernels / low-rank path of each level (mgmc_level_kernels)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg
lat = mg.Lattice3d(256, 256, 256)
op = mg.synthetic_posterior(mg.ShiftedLaplaceFDOperator(lat, 25.0), 8, 0.0, False)
s = mg.MultigridMCSampler(op, 1, mg.MultigridParameters(nlevel=6))
B = op.get_B()
print("fine nnz", len(B.rows), "m", B.m)
for l in range(6):
    print(l, s.level_desc(l)["ndof"], [s.lowrank_info(l, d) for d in (mg.FORWARD, mg.BACKWARD)], s.level_kernels(l))
s.close()
