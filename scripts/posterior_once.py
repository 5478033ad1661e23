"""A few 256^3 posterior V-cycles (BASELINE config 5, 8 point measurements) for kernel traces."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
import bench  # noqa: E402

lat = mg.Lattice3d(256, 256, 256)
op = bench.posterior_operator(mg.ShiftedLaplaceFDOperator(lat, 25.0), int(os.environ.get("M", "8")), 0.0, False)
s = mg.MultigridMCSampler(op, 1, mg.MultigridParameters(nlevel=6))
s.sample(3)
_t = s.sample_timed(10); tot, fine, nfine = _t["total_ms"], _t["pre_ms"], _t["npre"]
print("vcycle ms", tot / 10)
