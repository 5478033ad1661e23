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
  roofline   = the dominant fine-level kernel (the longer of the two level-0 Gibbs sweeps of a cycle);
               roofline.per_kernel holds both:
                 pre_sweep : algorithmic 24 B/unknown (read x, read f, write x) x N0 / average time,
                 post_sweep: 24 B x N0 + 8 B x N1 (the fused prolongation reads x_1) / average time,
               each timed with HIP events on the library's stream around its graph segment of the
               timed cycles (mgmc_sample_timed); `traffic` = rocprofv3 PMC bytes per launch from the
               committed profiles/pmc_traffic.json (a stored figure; `traffic_source` names it)
  config.collectives / rccl_ranks = what the final all-gather ran on and how many ranks the RCCL
               communicator spans (ncclCommCount); a failed communicator exits non-zero
  cpu_baseline = the CPU oracle (oracle/refcpu.cpp, FAITHFUL mode = the reference algorithm,
               g++ -O3) run as a child process (oracle/baseline.py) on rank 0 at N=1: 1 core
               (3 warm-up + 5 timed cycles) and the all-cores aggregate
"""
from __future__ import annotations

import argparse
import json
import math
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
    ap.add_argument("--cpu-samples", type=int, default=5, help="V-cycles timed for the 1-core CPU baseline (0 = skip)")
    ap.add_argument("--cpu-warmup", type=int, default=3, help="untimed V-cycles before them")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--plain", action="store_true", help="time the single-graph loop instead of the segmented one")
    ap.add_argument("--timing-stride", type=int, default=0,
                    help="time the fine-sweep segments (HIP event nodes) of every N-th cycle of the timed loop; the "
                         "other cycles replay the plain graph.  0 (default): N = max(4, ceil(10 ms / cycle)), the "
                         "cycle estimated from the warm-up, so the event nodes (about 0.05-0.1 ms per timed cycle) "
                         "stay near 1% of the loop: 4 at 512^3, 21 at 256^3, ~100 for the 2D 1024^2 cycle")
    ap.add_argument("--posterior", type=int, default=0, metavar="M",
                    help="BASELINE config 5: posterior operator with M point measurements (default lattice 256^3, "
                         "6 levels); not the headline line")
    ap.add_argument("--fem", action="store_true",
                    help="ShiftedLaplaceFEMOperator prior (27/9-point fine level); no CPU baseline")
    ap.add_argument("--radius", type=float, default=0.0, help="measurement radius (--posterior)")
    ap.add_argument("--measure-global", action="store_true", help="add the global average measurement (--posterior)")
    ap.add_argument("--chains", type=int, default=1, metavar="K",
                    help="independent chains per GPU, batched in one handle (mgmc_create_batch): every kernel "
                         "of the cycle covers all K, chain ids rank * K .. rank * K + K - 1")
    return ap.parse_args()


def cpu_baseline(dim, n, nlevel, warmup, samples, posterior_args=None):
    """The CPU oracle in FAITHFUL mode (the reference algorithm, oracle/refcpu.cpp, g++ -O3) on the same
    hierarchy, run as a GPU-free child process (oracle/baseline.py): one core (warmup + samples
    timed applications after the setup) and the all-cores aggregate (one forked chain per core of
    this process's CPU share, all timed together)."""
    import subprocess
    cmd = [sys.executable, os.path.join(ROOT, "oracle", "baseline.py"), "--dim", str(dim), "--n", str(n),
           "--nlevel", str(nlevel), "--warmup", str(warmup), "--samples", str(samples)]
    if posterior_args:
        cmd += posterior_args
    # a progress line on stderr every 30 s: the CPU baseline runs for minutes at 512^3, and a GPU box
    # takes a command that stays silent for 3 minutes to be hung
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.perf_counter()
    while True:
        try:
            stdout, stderr = proc.communicate(timeout=30)
            break
        except subprocess.TimeoutExpired:
            el = time.perf_counter() - t0
            print(f"bench: CPU baseline running ({el:.0f} s)", file=sys.stderr, flush=True)
            if el > 1500:
                proc.kill()
                stdout, stderr = proc.communicate()
                raise RuntimeError("CPU baseline timed out")
    if proc.returncode != 0:
        raise RuntimeError(f"CPU baseline failed (rc {proc.returncode}): {stderr[-800:]}")
    b = json.loads(stdout.strip().splitlines()[-1])
    agg = ""
    if "cores_aggregate" in b:
        agg = (f"; all cores: {b['cores_aggregate']} chains forked after the setup (shared CSR operators, own "
               f"state and mt19937_64 stream each), {b['aggregate_warmup']} warm-up + {b['aggregate_samples']} "
               f"timed cycles each, aggregate = chains x cycles / slowest chain ({b['aggregate_timed_s_max']} s)")
    out = {
        "value": b["value"],
        "unit": "samples/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{dim}D {n}^{dim} {nlevel}-level hierarchy, oracle/refcpu.cpp FAITHFUL mode (reference algorithm: "
                  f"lexicographic SOR Gibbs, mt19937_64 + normal_distribution, CSR; g++ -O3); setup {b['setup_s']} s "
                  f"excluded; 1 core: {b['warmup']} warm-up + {b['samples']} timed cycles ({b['timed_s']} s){agg}; "
                  f"host CPU: {b['cpu_model']}",
    }
    if "cores_aggregate" in b:
        out["cores_aggregate"] = b["cores_aggregate"]
        out["value_aggregate"] = b["value_aggregate"]
    return out


class CommError(RuntimeError):
    pass


class Collectives:
    """The bench's three collectives: barrier, max of the timed interval, all-gather of the per-chain
    QoI moments (24 B per chain).  N > 1 on distinct devices: RCCL on the library's stream (the
    unique id is shipped by torch.distributed gloo on the CPU); a communicator that cannot be
    created, or one that does not span every rank, is an error (exit non-zero), never a silent
    fallback.  Ranks that share one device (MGMC_BENCH_DEVICE, a rehearsal of the N > 1 path on a
    1-GPU box, where RCCL cannot run) use gloo collectives, and the line says so."""

    def __init__(self, sampler, rank, world):
        self.s, self.rank, self.world = sampler, rank, world
        self.kind, self.rccl_ranks, self.n_devices = "none", 0, 1
        if world == 1:
            return
        import threading
        import torch.distributed as dist
        self.dist = dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        buses = [None] * world
        dist.all_gather_object(buses, sampler.comm_info()["pci_bus_id"])
        self.n_devices = len(set(buses))  # distinct GPUs the ranks run on
        if len(set(buses)) < world:
            if os.environ.get("MGMC_BENCH_DEVICE") is None:
                raise CommError(f"ranks share GPUs (PCI bus ids {buses}): RCCL cannot run and the line would "
                                f"claim {world} GPUs; set MGMC_BENCH_DEVICE only to rehearse the N > 1 host path")
            self.kind = "gloo"
            return
        obj = [None]
        if rank == 0:
            try:
                obj[0] = mg.comm_unique_id()
            except mg.MgmcError as e:
                obj[0] = f"rank 0: no RCCL unique id ({e})"
        dist.broadcast_object_list(obj, src=0)
        if not isinstance(obj[0], bytes):
            raise CommError(str(obj[0]))
        # ncclCommInitRank is collective: if another rank failed before reaching it, this one would
        # wait forever -- a watchdog turns that into a non-zero exit
        done = threading.Event()

        def watchdog():
            if not done.wait(float(os.environ.get("MGMC_COMM_INIT_TIMEOUT", "300"))):
                print(f"rank {rank}: ncclCommInitRank did not return; exiting", file=sys.stderr, flush=True)
                os._exit(3)
        threading.Thread(target=watchdog, daemon=True).start()
        try:
            sampler.comm_init(world, rank, obj[0])
        finally:
            done.set()
        info = sampler.comm_info()
        if info["rccl_ranks"] != world or info["rccl_rank"] != rank:
            raise CommError(f"rank {rank}: the RCCL communicator spans {info['rccl_ranks']} ranks (rank "
                            f"{info['rccl_rank']}), expected {world}")
        counts = [None] * world
        dist.all_gather_object(counts, info["rccl_ranks"])
        self.kind, self.rccl_ranks = "rccl", min(counts)

    def barrier(self):
        if self.kind == "gloo":
            self.s.synchronize()
            self.dist.barrier()
        else:
            self.s.comm_barrier()  # RCCL all-reduce + device synchronisation (world 1: synchronisation)

    def max(self, v):
        if self.kind == "gloo":
            out = [None] * self.world
            self.dist.all_gather_object(out, v)
            return max(out)
        return self.s.comm_allreduce_max(v)

    def allgather_moments(self):
        if self.kind == "gloo":
            import numpy as np
            out = [None] * self.world
            self.dist.all_gather_object(out, [list(self.s.qoi_moments(c)) for c in range(self.s.nchains)])
            return np.array(out).reshape(-1, 3)
        return self.s.comm_allgather_moments(self.world)


def stored_traffic(path, n, key):
    """Per-launch HBM bytes of one fine-sweep kernel from a committed rocprofv3 PMC summary
    (scripts/pmc_traffic.py): a stored figure, with its provenance, not a measurement of this run."""
    try:
        tj = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if tj.get("n") != n or key not in tj:
        return None, None
    return tj[key]["hbm_bytes_per_launch"], {"file": os.path.relpath(path, ROOT), "head": tj.get("head"),
                                              "date": tj.get("date"), "method": tj.get("correction")}


def sweep_roofline(ms, nsweeps, bytes_sweep, traffic, provenance, kernel):
    t = ms / nsweeps * 1e-3
    achieved = bytes_sweep / t / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": provenance,
            "kernel": kernel, "bytes_per_launch": bytes_sweep, "avg_launch_ms": round(t * 1e3, 4)}


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
        op = mg.synthetic_posterior(op, args.posterior, args.radius, args.measure_global)
    params = mg.MultigridParameters(nlevel=nlevel, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                                    ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    t_setup = time.perf_counter()
    # MGMC_BENCH_DEVICE pins every rank to one device (rehearsing the N>1 host path on a 1-GPU box)
    device = int(os.environ.get("MGMC_BENCH_DEVICE", local_rank))
    K = args.chains
    sampler = mg.MultigridMCSampler(op, SEED, params, device=device, chain_id=rank * K, nchains=K)
    t_setup = time.perf_counter() - t_setup
    if rank == 0:
        print(f"bench: setup {t_setup:.1f} s", file=sys.stderr, flush=True)
    qoi = mg.measurement_vector_index(lat, [0.5] * args.dim)
    n0 = lat.Nvertex

    try:
        coll = Collectives(sampler, rank, world)
    except (CommError, mg.MgmcError) as e:
        print(f"rank {rank}: {e}", file=sys.stderr, flush=True)
        sampler.close()
        sys.exit(2)

    # warmup (prior: f = 0, x0 = 0 -- driver_mgmc.cc:61-69 with mean_x_exact = xbar = 0)
    if args.warmup // 2 > 0:
        sampler.sample(args.warmup // 2, qoi)
    stride = args.timing_stride
    if args.warmup - args.warmup // 2 > 0:  # the second half of the warm-up estimates the cycle time
        tw = time.perf_counter()
        sampler.sample(args.warmup - args.warmup // 2, qoi)
        sampler.synchronize()
        est_ms = (time.perf_counter() - tw) * 1e3 / (args.warmup - args.warmup // 2)
    else:
        est_ms = 1.0
    if stride <= 0:
        stride = max(4, int(math.ceil(10.0 / max(est_ms, 1e-3))))
    sampler.reset_moments()
    coll.barrier()  # barrier + device synchronisation
    t0 = time.perf_counter()
    if args.plain:
        sampler.sample_async(args.steps, qoi)
        sampler.synchronize()
        timed = None
    else:
        timed = sampler.sample_timed(args.steps, qoi, stride=stride)
    sampler.synchronize()
    t1 = time.perf_counter()
    coll.barrier()
    elapsed = coll.max(t1 - t0)

    from multigridmc_amd.distributed import merge_moments
    parts = coll.allgather_moments()
    nq, mean, m2 = merge_moments([tuple(r) for r in parts])

    if rank == 0:
        value = world * K * args.steps / elapsed
        roof, per_kernel = None, {}
        if timed and timed["npre"] > 0:
            plain3d = args.dim == 3 and not args.fem and not args.posterior
            tr_pre, prov = stored_traffic(args.traffic_file, n, "pre_sweep") if plain3d else (None, None)
            tr_post, prov2 = stored_traffic(args.traffic_file, n, "post_sweep") if plain3d else (None, None)
            kern = sampler.level_kernels(0)  # the kernels level 0 really runs on (mgmc_level_kernels)
            n1 = mg.Lattice(*((n // 2,) * args.dim)).Nvertex
            pre = sweep_roofline(timed["pre_ms"], timed["npre"], 24.0 * n0 * K, tr_pre if K == 1 else None, prov,
                                 f"fine pre-sweep {kern['sweep']} (one Gibbs sweep of level 0)")
            per_kernel["pre_sweep"] = pre
            if timed["npost"] > 0:
                fused = "post_sweep" in kern
                post = sweep_roofline(timed["post_ms"], timed["npost"], (24.0 * n0 + (8.0 * n1 if fused else 0.0)) * K,
                                      tr_post if K == 1 else None, prov2,
                                      f"fine post-sweep {kern.get('post_sweep', kern['sweep'])} "
                                      + ("(prolongate-add of level 1 fused, 24 B per fine + 8 B per coarse unknown; "
                                         "its own segment of the cycle graph)" if fused else
                                         "(one Gibbs sweep of level 0; the prolongation is a separate pass)"))
                per_kernel["post_sweep"] = post
            # the dominant kernel (the longer of the two) is the headline roofline
            roof = dict(max(per_kernel.values(), key=lambda r: r["avg_launch_ms"]))
            roof["per_kernel"] = per_kernel
            if args.posterior:
                for r in (roof, pre):
                    r["kernel"] += " + low-rank noise patch and B_bar fix (same segment)"
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.cpu_samples > 0 and not args.fem:
            pa = None
            if args.posterior:
                pa = ["--posterior", str(args.posterior), "--radius", str(args.radius)]
                if args.measure_global:
                    pa.append("--measure-global")
            cpu = cpu_baseline(args.dim, n, nlevel, args.cpu_warmup, args.cpu_samples, pa)
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "n_devices": coll.n_devices,
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
                                   + ("one independent chain per GPU" if K == 1 else
                                      f"{K} independent chains per GPU batched in one handle"),
                       "lattice": [n] * args.dim, "unknowns": n0, "nlevel": nlevel, "chains": world * K,
                       "parallelism": f"chains{world * K} (independent MCMC chains, {K} per GPU, no data-path "
                                      f"collective; final QoI-moment all-gather over {coll.kind})",
                       "collectives": coll.kind, "rccl_ranks": coll.rccl_ranks},
            "roofline": roof,
            "cpu_baseline": cpu,
            "qoi": {"index": qoi, "samples": nq, "mean": mean, "variance": m2 / nq if nq else None, "chains": len(parts)},
        }
        if timed:
            # pre / post: summed over the timed cycles only (every stride-th), so per timed cycle
            nct = timed["ncycles_timed"]
            line["segments_ms_per_step"] = {"pre": round(timed["pre_ms"] / nct, 4),
                                            "post": round(timed["post_ms"] / nct, 4),
                                            "total": round(timed["total_ms"] / args.steps, 4),
                                            "timing_stride": stride, "timed_cycles": nct,
                                            "timed_pre_sweeps": timed["npre"]}
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
                                          f"{nlevel}-level V-cycle, SOR Gibbs 1/1 with the B_bar fix, SSOR coarse 1"
                                          + (f", {K} chains per GPU batched" if K > 1 else ""))
            line["config"]["m_lowrank"] = m
            line["config"]["bbar_rows_forward_per_level"] = rows
            line["config"]["setup_s"] = round(t_setup, 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        coll.dist.barrier()
        coll.dist.destroy_process_group()
    sampler.close()


if __name__ == "__main__":
    main()
