"""The library's RCCL path on hardware (-m gpu), one rank.

SURVEY §8(e): chains are independent; the only collective is the end-of-run all-gather of each
chain's (n, mean, M2) (driver_mgmc.cc:86-94 computes those moments for one chain), merged in rank
order.  bench.py also uses the communicator for its barrier and the max-over-ranks time.  Every
N > 1 CPU test runs with gloo fakes, so this test runs the real calls on one MI355X with a 1-rank
communicator: ncclGetUniqueId, ncclCommInitRank, ncclCommCount / ncclCommUserRank, the packing
hipMemcpy2DAsync plus ncclAllGather, ncclAllReduce (max and the barrier's sum), ncclCommDestroy and
a second init on the same handle.
"""
import numpy as np
import pytest

import multigridmc_amd as mg

pytestmark = pytest.mark.gpu

SEED = 5418513


def _batch(nchains):
    lat = mg.Lattice(64, 64, 64)
    p = mg.MultigridParameters(nlevel=4)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=3,
                              nchains=nchains)
    return s, mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])


@pytest.mark.parametrize("nchains", [1, 4])
def test_rccl_one_rank_communicator(hip_device, nchains):
    s, q = _batch(nchains)
    s.sample(7, q, chain=None)
    s.sample(5, q, chain=None)
    local = np.stack([s.qoi_moments(c) for c in range(nchains)])
    assert local[0, 0] > 0 and np.all(local[:, 0] == local[0, 0]) and np.all(np.isfinite(local))

    # no communicator: the all-gather is the handle's own chains, rccl_ranks reports 0
    assert s.comm_info()["rccl_ranks"] == 0
    assert np.array_equal(s.comm_allgather_moments(1), local)

    for attempt in range(2):  # init, use, destroy, and a second init on the same handle
        uid = mg.comm_unique_id()
        assert len(uid) == 128
        s.comm_init(1, 0, uid)
        info = s.comm_info()
        assert info["rccl_ranks"] == 1 and info["rccl_rank"] == 0, info
        g = s.comm_allgather_moments(1)
        assert g.shape == (nchains, 3)
        assert np.array_equal(g, local), (attempt, g, local)  # packed (n, mean, M2) per chain, bitwise
        for v in (0.0, -3.25, 2.390625e-3, 1e300):
            assert s.comm_allreduce_max(v) == v
        s.comm_barrier()
        # the communicator leaves the chains alone: more cycles, then the gather again
        s.sample(3, q, chain=None)
        local = np.stack([s.qoi_moments(c) for c in range(nchains)])
        assert np.array_equal(s.comm_allgather_moments(1), local)
        s.comm_destroy()
        assert s.comm_info()["rccl_ranks"] == 0
    s.close()
