"""Run K fine-level sweeps at 512^3 (for rocprofv3 counter collection)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
n = int(os.environ.get("N", "512"))
lat = mg.Lattice3d(n, n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=7))
print("ms/sweep", s.time_fine_sweeps(int(os.environ.get("K", "6"))) / int(os.environ.get("K", "6")))
