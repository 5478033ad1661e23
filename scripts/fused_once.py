"""A few fused post+pre fine sweeps at n^3 (rocprofv3 kernel traces: k_zsweep2_rb7 against the two
k_zsweep_rb7 launches of the cycle)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
n = int(os.environ.get("N", "512"))
lat = mg.Lattice3d(n, n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=2))
n0, n1 = s.level_desc(0)["ndof"], s.level_desc(1)["ndof"]
rng = np.random.default_rng(1)
x, f, xc = rng.standard_normal(n0), rng.standard_normal(n0), rng.standard_normal(n1)
for k in range(int(os.environ.get("K", "3"))):
    x, cap = s.fused_sweeps_apply(3, 0, k, 1.0, xc, f, x, n0 // 2)
print("fused ok", cap, float(np.std(x)))
