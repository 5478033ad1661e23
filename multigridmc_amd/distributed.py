"""Multi-GPU chains: one independent MCMC chain per rank (one process per GPU), and the one
collective of the path -- the final QoI mean/variance reduction (driver_mgmc.cc:86-94).

Each rank holds Welford moments (n, mean, M2) of its chain's QoI time series.  They are
all-gathered (24 bytes per chain; RCCL over xGMI with backend "nccl", gloo on CPU) and merged
in rank order with Chan et al.'s pairwise update, so the pooled result does not depend on the
arrival order of the ranks.
"""
from __future__ import annotations

import numpy as np


def merge_moments(parts) -> tuple:
    """Chan/Welford merge of [(n, mean, M2), ...] in the given order."""
    n, mean, m2 = 0.0, 0.0, 0.0
    for nb, mb, m2b in parts:
        nb = float(nb)
        if nb == 0:
            continue
        if n == 0:
            n, mean, m2 = nb, float(mb), float(m2b)
            continue
        tot = n + nb
        delta = float(mb) - mean
        mean = mean + delta * nb / tot
        m2 = m2 + float(m2b) + delta * delta * n * nb / tot
        n = tot
    return n, mean, m2


def moments_of(series) -> tuple:
    s = np.asarray(series, dtype=np.float64)
    if s.size == 0:
        return 0.0, 0.0, 0.0
    mean = float(s.mean())
    return float(s.size), mean, float(((s - mean) ** 2).sum())


def allgather_moments(local, device=None) -> list:
    """All-gather (n, mean, M2) of every rank; returns the list in rank order."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in local], dtype=torch.float64, device=device)
    if not (dist.is_available() and dist.is_initialized()):
        return [tuple(t.cpu().tolist())]
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [tuple(o.cpu().tolist()) for o in out]


def pooled_statistics(local, device=None) -> dict:
    """Pooled QoI mean / variance over all ranks' chains (variance with the reference's
    E[z^2] - E[z]^2 normalisation, driver_mgmc.cc:86-93)."""
    parts = allgather_moments(local, device)
    n, mean, m2 = merge_moments(parts)
    var = m2 / n if n > 0 else float("nan")
    return {"n": n, "mean": mean, "variance": var, "error": float(np.sqrt(var / n)) if n > 0 else float("nan"),
            "chains": len(parts)}
