"""Run a few 512^3 7-level V-cycles (for rocprofv3 kernel traces)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
n = int(os.environ.get("N", "512"))
lat = mg.Lattice3d(n, n, n) if os.environ.get("DIM", "3") == "3" else mg.Lattice2d(n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=int(os.environ.get("NLEVEL", "7")),
                                                                                   ncoarsesmooth=int(os.environ.get("NCS", "1"))))
s.sample(3)
_t = s.sample_timed(int(os.environ.get("K", "10"))); tot, fine, nfine = _t["total_ms"], _t["pre_ms"], _t["npre"]
print("vcycle ms", tot / int(os.environ.get("K", "10")))
