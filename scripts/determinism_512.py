"""Determinism of the 512^3 7-level cycle: REPS handles with the same (seed, chain) run 4 QoI samples
each; prints the series and whether they agree bit for bit (MGMC_LIBRARY selects the build)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402

shape = (512, 512, 512)
lat = mg.Lattice(*shape)
q = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
p = mg.MultigridParameters(nlevel=7, smoother="SOR", coarse_solver="SSOR")
ref = None
for r in range(int(os.environ.get("REPS", "3"))):
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 5418513, p, device=0)
    z = s.sample(4, q)
    x = s.get_state()
    h = hash(x.tobytes())
    s.close()
    same = ref is None or (np.array_equal(z, ref[0]) and h == ref[1])
    print(os.environ.get("MGMC_LIBRARY", "head"), r, z.tolist(), "state", h, "same" if same else "DIFFERENT", flush=True)
    if ref is None:
        ref = (z, h)
