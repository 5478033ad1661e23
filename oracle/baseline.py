"""CPU baseline of bench.py -- TEST INFRASTRUCTURE (the cpu_baseline leg only, never the product).

Times the FAITHFUL oracle (oracle/refcpu.cpp: the reference algorithm -- lexicographic SOR Gibbs
sweeps, one mt19937_64 + a normal_distribution per sampler object, CSR operators, the recursion of
multigridmc_sampler.cc:103-138; g++ -O3 as the reference's Release build) on the same hierarchy as
the GPU bench, in the loop shape of driver_mgmc.cc:66-78:

  single core : one chain, `--warmup` untimed + `--samples` timed applications after the setup
  all cores   : the hierarchy is built once, then `--chains` processes are forked (copy-on-write:
                the CSR operators are shared, every chain owns its vectors and its re-seeded
                mt19937_64); all chains start together after their warm-up, and the aggregate rate
                is chains x samples / (the slowest chain's timed interval)

bench.py runs this as a child process (python oracle/baseline.py ...), so nothing here shares a
process with the GPU, and prints one JSON line.  Run by hand: python oracle/baseline.py --n 64
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SEED = 5418513  # driver_mgmc.cc:448


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share() -> int:
    """Cores this process may use: the affinity mask, capped by OMP_NUM_THREADS when it is set (the
    GPU box exports the per-GPU CPU share there; its nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def mem_available() -> int:
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


_ORACLE = None   # built in the parent before the fork, inherited copy-on-write
_BARRIER = None  # the chains start their timed samples together


def _chain(chain, warmup, samples, q):
    o = _ORACLE
    o.L.orc_reseed(o.h, SEED, chain)
    o.time_samples(warmup)
    _BARRIER.wait()
    q.put(o.time_samples(samples))


def main():
    global _ORACLE, _BARRIER
    ap = argparse.ArgumentParser()
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--nlevel", type=int, default=7)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--samples", type=int, default=5)
    ap.add_argument("--chains", type=int, default=0, help="all-cores chains (0 = the CPU share, 1 = skip)")
    ap.add_argument("--agg-warmup", type=int, default=1)
    ap.add_argument("--agg-samples", type=int, default=2)
    ap.add_argument("--posterior", type=int, default=0, help="m point measurements (bench.py posterior_operator)")
    ap.add_argument("--radius", type=float, default=0.0)
    ap.add_argument("--measure-global", action="store_true")
    a = ap.parse_args()

    import multigridmc_amd as mg  # host classes only (the HIP library is never loaded here)
    from tests import oracle_lib as O

    p = mg.MultigridParameters(nlevel=a.nlevel, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                               ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    t0 = time.perf_counter()
    o = O.Oracle.fd((a.n,) * a.dim, p, kappa_sq=25.0, mode=O.FAITHFUL, seed=SEED, galerkin=1)
    if a.posterior:
        lat = mg.Lattice(*((a.n,) * a.dim))
        op = mg.synthetic_posterior(mg.ShiftedLaplaceFDOperator(lat, 25.0), a.posterior, a.radius, a.measure_global)
        o.set_lowrank(op.get_B())
        o.time_samples(1)  # B_bar of every smoother is set up on first use: keep it out of the timing
    setup = time.perf_counter() - t0
    if a.warmup > 0:
        o.time_samples(a.warmup)
    secs = o.time_samples(a.samples)
    out = {
        "value": a.samples / secs,
        "unit": "samples/s",
        "cores": 1,
        "kind": "port",
        "setup_s": round(setup, 1),
        "timed_s": round(secs, 2),
        "warmup": a.warmup,
        "samples": a.samples,
        "cpu_model": cpu_model(),
    }
    chains = a.chains if a.chains > 0 else cpu_share()
    # every forked chain writes its own x, f, r and sampler scratch (about 6 N0 doubles at this size)
    per_chain = 6 * 8 * (a.n - 1) ** a.dim * 8 // 7
    avail = mem_available()
    if avail:
        chains = max(1, min(chains, int(0.6 * avail) // max(per_chain, 1)))
    if chains > 1 and a.agg_samples > 0:
        _ORACLE = o
        ctx = mp.get_context("fork")
        _BARRIER = ctx.Barrier(chains)
        q = ctx.Queue()
        procs = [ctx.Process(target=_chain, args=(c + 1, a.agg_warmup, a.agg_samples, q)) for c in range(chains)]
        for pr in procs:
            pr.start()
        t_agg = [q.get() for _ in procs]
        for pr in procs:
            pr.join()
        out["cores_aggregate"] = chains
        out["value_aggregate"] = chains * a.agg_samples / max(t_agg)
        out["aggregate_warmup"] = a.agg_warmup
        out["aggregate_samples"] = a.agg_samples
        out["aggregate_timed_s_max"] = round(max(t_agg), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
