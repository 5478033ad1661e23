"""The fused fine sweeps (mgmc_zsweep2.hpp, -m gpu): one launch = the backward post-sweep of cycle n
(with the prolongation of the coarse correction) and the forward pre-sweep of cycle n+1, bit for bit
the oracle's prolongate_add + SORSampler::apply backward (tag_post, sample s) + forward (tag_pre,
sample s + 1) (sampler/sor_sampler.cc:37-59, multigridmc_sampler.cc:117-128), and the captured
post-sweep value at the QoI vertex."""
import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513


@pytest.mark.parametrize("shape,alpha,omega", [((128, 128, 128), 1.0, 1.0), ((128, 64, 96), 0.9, 1.1),
                                               ((192, 48, 40), 1.0, 1.0), ((64, 34, 18), 2.0, 0.8)])
def test_fused_sweeps_bitwise(hip_device, shape, alpha, omega):
    lat = mg.Lattice(*shape)
    p = mg.MultigridParameters(nlevel=2, omega=omega)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=3)
    st = np.concatenate([s.level_desc(level)["stencil"] for level in range(2)])
    o = O.Oracle.fd(lat.shape, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=3, override_stencils=st)
    rng = np.random.default_rng(17)
    n0, n1 = s.level_desc(0)["ndof"], s.level_desc(1)["ndof"]
    x = rng.standard_normal(n0)
    f = rng.standard_normal(n0)
    xc = rng.standard_normal(n1)
    for q, (tag_post, tag_pre, sample) in zip([n0 // 2, 7, n0 - 3], [(5, 0, 11), (2, 0, 2 ** 33 + 4), (9, 1, 0)]):
        d, cap = s.fused_sweeps_apply(tag_post, tag_pre, sample, alpha, xc, f, x, q)
        y = o.prolongate_add(0, alpha, xc, x)
        y = o.sor_sampler_apply(0, mg.BACKWARD, tag_post, sample, f, y)
        assert cap == y[q]
        y = o.sor_sampler_apply(0, mg.FORWARD, tag_pre, sample + 1, f, y)
        assert np.array_equal(d, y), f"max diff {np.max(np.abs(d - y))} at {np.argmax(np.abs(d - y))}"
    s.close()


FUSE_CONFIGS = {
    "3d128": ((128, 128, 128), dict(nlevel=3)),
    "3d128_4lvl_w2": ((128, 64, 96), dict(nlevel=4, coarse_scaling=0.9, omega=1.2)),
    "3d192": ((192, 48, 40), dict(nlevel=2)),
}


@pytest.mark.parametrize("name", list(FUSE_CONFIGS))
@pytest.mark.parametrize("nsteps", [2, 5, 8])
def test_fused_sample_loop_bitwise(hip_device, monkeypatch, name, nsteps):
    """The sample loop with fused cycle boundaries (MGMC_FUSE_CYCLES=1 forces them below 4 M
    unknowns): QoI series, final state and sample index equal the oracle's sequential cycles, for odd
    and even numbers of boundaries (the exchanged-buffer graph), and a following apply() / sample(1)
    continues the same chain."""
    monkeypatch.setenv("MGMC_FUSE_CYCLES", "1")
    shape, kw = FUSE_CONFIGS[name]
    lat = mg.Lattice(*shape)
    p = mg.MultigridParameters(**{"smoother": "SOR", "coarse_solver": "SSOR", **kw})
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=1)
    st = np.concatenate([s.level_desc(level)["stencil"] for level in range(p.nlevel)])
    o = O.Oracle.fd(lat.shape, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=1, override_stencils=st)
    f = np.random.default_rng(5).standard_normal(lat.Nvertex)
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    s.fix_rhs(f)
    o.set_rhs(f)
    assert np.array_equal(s.sample(nsteps, q), o.sample(nsteps, q))
    assert np.array_equal(s.get_state(), o.get_state())
    assert s.get_sample_index() == nsteps
    assert np.array_equal(s.sample(1, q), o.sample(1, q))  # one cycle: no boundary to fuse
    s.sample(3)  # guard-vertex mode (no QoI recorded), fused
    o.sample(3)
    assert np.array_equal(s.get_state(), o.get_state())
    n, mean, m2 = s.qoi_moments()
    assert n == nsteps + 1
    s.close()


def test_fused_batched_chains_bitwise(hip_device, monkeypatch):
    monkeypatch.setenv("MGMC_FUSE_CYCLES", "1")
    lat = mg.Lattice(128, 128, 64)
    p = mg.MultigridParameters(nlevel=3)
    b = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, chain_id=2, nchains=3)
    q = mg.measurement_vector_index(lat, [0.5] * 3)
    zb = b.sample(6, q, chain=None)
    monkeypatch.setenv("MGMC_DISABLE", "fuse_cycles")
    for c in range(3):
        s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, chain_id=2 + c)
        assert np.array_equal(s.sample(6, q), zb[c])
        assert np.array_equal(s.get_state(), b.get_state(c))
        s.close()
    b.close()
