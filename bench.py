#!/usr/bin/env python3
"""MGMC V-cycle benchmark (BASELINE.json metric): samples/s of the 3D 512^3 shifted-Laplace
7-level V-cycle, one independent chain per GPU, plus the fine-smoother HBM roofline and the CPU
oracle baseline.

  python bench.py --gpus N --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE from the environment).  Each rank runs an
independent chain (Philox key = (seed, chain = rank)).  The device-side collectives (barrier,
max-over-ranks time, the final all-gather of the per-chain QoI moments) run on an RCCL
communicator owned by the C-ABI library on the sampler's own HIP stream; torch.distributed (gloo,
CPU) only ships the RCCL unique id.  torch.cuda is never initialised: the library and torch bundle
different HIP runtimes, and the library's stream synchronisation replaces torch.cuda.synchronize().
A step is one MGMC V-cycle; the K timed steps are bracketed by barrier + device synchronisation on
both sides and the max over ranks is used.

Rank 0 prints ONE JSON line.  Field notes:
  value      = chains x K / max-over-ranks time (whole job, samples/s)
  roofline   = fine-level (level 0) Gibbs sweep: algorithmic 24 B/unknown (read x, read f,
               write x) x N0 / average sweep time, measured with HIP events on the library's
               stream around the fine pre-sampler graph segment (plain sweep kernel) inside the
               timed region
  cpu_baseline = the CPU oracle (oracle/refcpu.cpp, FAITHFUL mode = the reference algorithm,
               1 thread) timed on a bounded sample of the same workload on rank 0 at N=1
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Load the HIP library (ROCm 7.2 runtime) before torch so one runtime serves the process.
import multigridmc_amd as mg  # noqa: E402

mg.load_library()

METRIC = "MGMC V-cycle samples/sec + fine-smoother HBM GB/s, 512³ lattice, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 5418513         # driver_mgmc.cc:448


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--n", type=int, default=512, help="cells per direction")
    ap.add_argument("--dim", type=int, default=3, choices=(2, 3),
                    help="2: BASELINE config 2 (2D n^2 lattice, e.g. --dim 2 --n 1024 --nlevel 5); not the headline line")
    ap.add_argument("--nlevel", type=int, default=7)
    ap.add_argument("--cpu-samples", type=int, default=1, help="V-cycles timed for the CPU baseline (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--plain", action="store_true", help="time the single-graph loop instead of the segmented one")
    ap.add_argument("--posterior", type=int, default=0, metavar="M",
                    help="BASELINE config 5: posterior operator with M point measurements (default lattice 256^3, "
                         "6 levels); not the headline line")
    ap.add_argument("--fem", action="store_true",
                    help="ShiftedLaplaceFEMOperator prior (27/9-point fine level); no CPU baseline")
    ap.add_argument("--radius", type=float, default=0.0, help="measurement radius (--posterior)")
    ap.add_argument("--measure-global", action="store_true", help="add the global average measurement (--posterior)")
    return ap.parse_args()


def cpu_info():
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model


def cpu_baseline(n, nlevel, nsamples, posterior=None, dim=3):
    """FAITHFUL oracle (reference algorithm: lexicographic SOR Gibbs sweeps, mt19937_64 +
    normal_distribution, CSR operators; with a posterior operator the reference's dense
    lexicographic B_bar fix) on the same hierarchy, 1 thread."""
    from tests import oracle_lib as O
    p = mg.MultigridParameters(nlevel=nlevel, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                               ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    t0 = time.perf_counter()
    o = O.Oracle.fd((n,) * dim, p, kappa_sq=25.0, mode=O.FAITHFUL, seed=SEED, galerkin=1)
    if posterior is not None:
        o.set_lowrank(posterior.get_B())
        o.time_samples(1)  # B_bar setup of every smoother happens on first use: keep it out of the timing
    setup = time.perf_counter() - t0
    secs = o.time_samples(nsamples)
    del o
    return {
        "value": nsamples / secs,
        "unit": "samples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{nsamples} V-cycles of the same {dim}D {n}^{dim} {nlevel}-level hierarchy after a {setup:.0f} s setup "
                  f"(oracle/refcpu.cpp FAITHFUL mode: lexicographic SOR Gibbs, mt19937_64, CSR; g++ -O2, 1 thread); "
                  f"{secs:.1f} s timed; host CPU: {cpu_info()}",
    }


class Collectives:
    """The bench's three collectives (barrier, max of the timed interval, all-gather of the per-chain
    QoI moments -- 24 B per chain).  N > 1: RCCL on the library's stream, with the unique id shipped
    by torch.distributed gloo on the CPU; if the RCCL communicator cannot be created (e.g. ranks
    sharing one device), the same three host-side collectives run on gloo."""

    def __init__(self, sampler, rank, world):
        self.s, self.rank, self.world, self.rccl = sampler, rank, world, False
        if world == 1:
            return
        import torch.distributed as dist
        self.dist = dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        obj = [None]
        if rank == 0:
            try:
                obj[0] = mg.comm_unique_id()
            except mg.MgmcError as e:
                print(f"rank 0: no RCCL unique id ({e})", file=sys.stderr)
        dist.broadcast_object_list(obj, src=0)
        try:
            if obj[0] is None:
                raise mg.MgmcError(-2, "no RCCL unique id")
            sampler.comm_init(world, rank, obj[0])
            ok = 1
        except mg.MgmcError as e:
            print(f"rank {rank}: RCCL communicator unavailable ({e}); host collectives on gloo", file=sys.stderr)
            ok = 0
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        self.rccl = all(f == 1 for f in flags)
        if not self.rccl and ok:
            sampler.comm_destroy()

    def barrier(self):
        if self.rccl or self.world == 1:
            self.s.comm_barrier()  # RCCL all-reduce + device synchronisation
        else:
            self.s.synchronize()
            self.dist.barrier()

    def max(self, v):
        if self.rccl or self.world == 1:
            return self.s.comm_allreduce_max(v)
        out = [None] * self.world
        self.dist.all_gather_object(out, v)
        return max(out)

    def allgather_moments(self):
        if self.rccl or self.world == 1:
            return self.s.comm_allgather_moments(self.world)
        import numpy as np
        out = [None] * self.world
        self.dist.all_gather_object(out, list(self.s.qoi_moments()))
        return np.array(out)


def posterior_operator(prior, m, radius, measure_global):
    """BASELINE config 5: m measurements at fixed pseudo-random interior locations with the
    variances of measurements_template.cfg's scale (~1e-6), optional global average
    (parameters_template.cfg: variance_global 0.01)."""
    import numpy as np
    from multigridmc_amd.parameters import MeasurementParameters
    rng = np.random.default_rng(20250219)
    mp = MeasurementParameters(radius=radius, variance_scaling=1.0, measure_global=measure_global,
                               variance_global=0.01)
    mp.measurement_locations = [list(rng.uniform(0.1, 0.9, 3)) for _ in range(m)]
    mp.variance = list(1e-6 * (1.0 + rng.random(m)))
    return mg.MeasuredOperator(prior, mp)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))

    n, nlevel = args.n, args.nlevel
    if args.posterior and "--n" not in sys.argv:
        n = 256
    if args.posterior and "--nlevel" not in sys.argv:
        nlevel = 6
    lat = mg.Lattice3d(n, n, n) if args.dim == 3 else mg.Lattice2d(n, n)
    prior_cls = mg.ShiftedLaplaceFEMOperator if args.fem else mg.ShiftedLaplaceFDOperator
    op = prior_cls(lat, kappa_sq=1.0 / 0.2 ** 2)  # Lambda = 0.2 (parameters_template.cfg)
    if args.posterior:
        op = posterior_operator(op, args.posterior, args.radius, args.measure_global)
    params = mg.MultigridParameters(nlevel=nlevel, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                                    ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    t_setup = time.perf_counter()
    # MGMC_BENCH_DEVICE pins every rank to one device (rehearsing the N>1 path on a 1-GPU box)
    device = int(os.environ.get("MGMC_BENCH_DEVICE", local_rank))
    sampler = mg.MultigridMCSampler(op, SEED, params, device=device, chain_id=rank)
    t_setup = time.perf_counter() - t_setup
    qoi = mg.measurement_vector_index(lat, [0.5] * args.dim)
    n0 = lat.Nvertex

    coll = Collectives(sampler, rank, world)

    # warmup (prior: f = 0, x0 = 0 -- driver_mgmc.cc:61-69 with mean_x_exact = xbar = 0)
    sampler.sample(args.warmup, qoi)
    sampler.reset_moments()
    coll.barrier()  # barrier + device synchronisation
    t0 = time.perf_counter()
    if args.plain:
        sampler.sample_async(args.steps, qoi)
        sampler.synchronize()
        fine_ms, nfine = float("nan"), 0
    else:
        _, fine_ms, nfine = sampler.sample_timed(args.steps, qoi)
    sampler.synchronize()
    t1 = time.perf_counter()
    coll.barrier()
    elapsed = coll.max(t1 - t0)

    from multigridmc_amd.distributed import merge_moments
    parts = coll.allgather_moments()
    nq, mean, m2 = merge_moments([tuple(r) for r in parts])

    if rank == 0:
        value = world * args.steps / elapsed
        roof = None
        if nfine > 0:
            t_sweep = fine_ms / nfine * 1e-3
            bytes_sweep = 24.0 * n0
            achieved = bytes_sweep / t_sweep / 1e9
            traffic = None
            if os.path.exists(args.traffic_file):
                try:
                    tj = json.load(open(args.traffic_file))
                    if tj.get("n") == n and args.dim == 3 and not args.fem:
                        traffic = tj.get("fine_sweep_hbm_bytes_per_launch")
                except (OSError, ValueError):
                    traffic = None
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": "fine-level (level 0) multicolour Gibbs sweep",
                    "bytes_per_launch": bytes_sweep, "avg_launch_ms": round(t_sweep * 1e3, 4)}
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.cpu_samples > 0 and not args.fem:
            cpu = cpu_baseline(n, nlevel, args.cpu_samples, op if args.posterior else None, args.dim)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: prior (f = 0), x0 = 0, Philox4x32-10 counter-based Gaussian noise",
            "config": {"workload": f"{args.dim}D {n}^{args.dim} shifted-Laplace {'FEM' if args.fem else 'FD'} "
                                   f"prior (kappa^2 = 25), "
                                   f"{nlevel}-level V-cycle, SOR Gibbs 1/1, SSOR coarse 1, omega 1, "
                                   f"one independent chain per GPU",
                       "lattice": [n] * args.dim, "unknowns": n0, "nlevel": nlevel, "chains": world,
                       "parallelism": f"chains{world} (independent MCMC chains, 1 per GPU; "
                                      f"{'RCCL' if coll.rccl or world == 1 else 'gloo'} all-gather of QoI moments)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "qoi": {"index": qoi, "samples": nq, "mean": mean, "variance": m2 / nq if nq else None, "chains": len(parts)},
        }
        if args.dim == 2:
            line["metric"] = "MGMC V-cycle samples/sec, 2D (BASELINE config 2)"
        if args.posterior:
            m = op.get_m_lowrank()
            rows = [sampler.lowrank_info(lv, mg.FORWARD)[1] for lv in range(nlevel)]
            line["metric"] = "MGMC V-cycle samples/sec, 3D posterior (low-rank measurement update)"
            line["data"] = ("synthetic: posterior operator, f = 0, x0 = 0, Philox4x32-10 noise; "
                            f"{args.posterior} measurements of radius {args.radius}"
                            + (" + global average" if args.measure_global else ""))
            line["config"]["workload"] = (f"BASELINE config 5: 3D {n}^3 posterior Q = A + B Sigma^-1 B^T (m = {m}), "
                                          f"{nlevel}-level V-cycle, SOR Gibbs 1/1 with the B_bar fix, SSOR coarse 1")
            line["config"]["m_lowrank"] = m
            line["config"]["bbar_rows_forward_per_level"] = rows
            line["config"]["setup_s"] = round(t_setup, 2)
            if roof:
                roof["kernel"] = "fine pre-sampler segment: Gibbs sweep + low-rank noise patch + B_bar fix"
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()
    sampler.close()


if __name__ == "__main__":
    main()
