"""Test launcher (tests/test_host.py::test_bench_world2_through_torchrun): bench.py's main() under the
driver's own N > 1 launch line, on a host without a GPU.

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port P tests/bench_rehearsal.py --gpus 2 --steps K --warmup W

Everything of bench.main() runs for real -- argument parsing, RANK / LOCAL_RANK / WORLD_SIZE, the
Collectives class (gloo process group, the PCI-bus-id check, the RCCL unique-id broadcast and the
communicator checks), the timed loop's barriers and max-over-ranks, the moment all-gather and the
JSON line -- except the device sampler, which this launcher replaces with a stand-in recording the
calls (MGMC_FAKE_MODE: "shared" = both ranks report one PCI bus id, "distinct" = one each, with a
communicator whose collectives run over the gloo group the way RCCL computes them).  Test
infrastructure only: bench.py itself has no such switch and fails loudly without a GPU.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


class RehearsalSampler:
    def __init__(self, op, seed, params, device=0, chain_id=0, nchains=1):
        self.rank = int(os.environ["RANK"])
        self.device, self.chain_id, self.nchains = device, chain_id, nchains
        self.mode = os.environ.get("MGMC_FAKE_MODE", "shared")
        self.comm = False
        self.n = 0

    def sample(self, n, qoi):
        self.n += n
        time.sleep(0.001 * n)

    def synchronize(self):
        pass

    def reset_moments(self):
        self.n = 0

    def sample_timed(self, steps, qoi, stride=1):
        self.sample(steps, qoi)
        ncyc = sum(1 for s in range(steps) if s % stride == 0 or s == steps - 1)
        return {"total_ms": 1.0 * steps, "pre_ms": 0.5 * ncyc, "npre": ncyc, "post_ms": 0.5 * ncyc, "npost": ncyc,
                "ncycles_timed": ncyc}

    def level_kernels(self, level):
        return {"sweep": "k_zsweep_rb7<32,20,...,0>", "post_sweep": "k_zsweep_rb7<32,16,...,PROLONG>"}

    def qoi_moments(self, chain=0):
        return np.array([float(self.n), 0.1 * (self.rank + 1), 1.0])

    def comm_info(self):
        shared = self.mode == "shared"
        return {"rccl_ranks": 2 if self.comm else 0, "rccl_rank": self.rank if self.comm else -1,
                "pci_bus_id": 7 if shared else 7 + self.rank}

    def comm_init(self, world, rank, uid):
        assert len(uid) == 128
        self.comm = True

    def comm_barrier(self):
        import torch.distributed as dist
        dist.barrier()

    def comm_allreduce_max(self, v):
        import torch.distributed as dist
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, v)
        return max(out)

    def comm_allgather_moments(self, world):
        import torch.distributed as dist
        out = [None] * world
        dist.all_gather_object(out, [list(self.qoi_moments(c)) for c in range(self.nchains)])
        return np.array(out).reshape(-1, 3)

    def close(self):
        pass


if __name__ == "__main__":
    bench.mg.MultigridMCSampler = RehearsalSampler
    bench.mg.comm_unique_id = lambda: bytes(128)
    bench.main()
