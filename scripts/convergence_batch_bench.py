"""Wall time of measure_convergence's chains (driver_mgmc.cc:236-254), sequential against batched
on cloned handles.  python scripts/convergence_batch_bench.py [nsamples nsteps]"""
import os
import sys
import time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402
from multigridmc_amd.driver import convergence_series  # noqa: E402

ns = int(sys.argv[1]) if len(sys.argv) > 1 else 200
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for shape, nlevel, cycle in (((64, 64), 4, 2), ((256, 256), 5, 1), ((64, 64, 64), 4, 1)):
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 5418513, mg.MultigridParameters(nlevel=nlevel, cycle=cycle))
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    s.fix_rhs(np.zeros(lat.Nvertex))
    convergence_series(s, 4, nsteps, [q], [1.0], batch=4)  # warm
    for batch in (1, 4, 8, 16):
        t0 = time.perf_counter()
        convergence_series(s, ns, nsteps, [q], [1.0], batch=batch)
        dt = time.perf_counter() - t0
        print(f"{lat.shape} nlevel {nlevel} cycle {cycle}: {ns} chains x {nsteps} cycles, batch {batch:2d}: "
              f"{dt:7.3f} s  ({ns * nsteps / dt:9.1f} cycles/s)", flush=True)
    s.close()
