"""Throughput of C independent chains per GPU, each handle on its own HIP stream (graph replays
overlap across streams).  python scripts/multichain_bench.py N NLEVEL K C1 C2 ...
THREADS=1: one host thread per chain."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402

n, nlevel, K = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
lat = mg.Lattice3d(n, n, n) if n > 0 else mg.Lattice2d(-n, -n)
q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
for C in [int(c) for c in sys.argv[4:]]:
    ss = [mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 5418513, mg.MultigridParameters(nlevel=nlevel),
                                chain_id=c) for c in range(C)]
    for s in ss:
        s.sample(5, q)
    t0 = time.perf_counter()
    if os.environ.get("THREADS") == "1":
        # one host thread per chain: the graph launches (host-side AQL packets, a few us per kernel
        # node) of different chains are enqueued concurrently; ctypes releases the GIL
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(len(ss)) as ex:
            list(ex.map(lambda s: (s.sample_async(K, q), s.synchronize()), ss))
    else:
        for s in ss:
            s.sample_async(K, q)
        for s in ss:
            s.synchronize()
    dt = time.perf_counter() - t0
    print(f"lattice {lat.shape} chains {C}: {C * K / dt:10.1f} samples/s  ({dt / K * 1e3:.3f} ms per round)", flush=True)
    for s in ss:
        s.close()
