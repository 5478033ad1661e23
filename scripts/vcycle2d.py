"""A few 2D 1024^2 5-level V-cycles (FD or FEM prior, FEM=1) for kernel traces."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
n = int(os.environ.get("N", "1024"))
lat = mg.Lattice2d(n, n)
cls = mg.ShiftedLaplaceFEMOperator if os.environ.get("FEM") == "1" else mg.ShiftedLaplaceFDOperator
s = mg.MultigridMCSampler(cls(lat, 25.0), 1, mg.MultigridParameters(nlevel=int(os.environ.get("NLEVEL", "5"))))
s.sample(3)
k = int(os.environ.get("K", "10"))
_t = s.sample_timed(k); tot, fine, nfine = _t["total_ms"], _t["pre_ms"], _t["npre"]
print("vcycle ms", tot / k)
