"""Batched chains (-m gpu): one handle carrying nchains independent chains (mgmc_create_batch).

Every kernel of a cycle covers all chains of the batch (grid.z / blockIdx.x = chain, vectors
L.nstore apart, the low-rank B_bar rows read once for all chains).  Chain c of a batch created with
chain0 draws the Philox stream of chain id chain0 + c, so it must reproduce a one-chain handle with
chain_id = chain0 + c BIT FOR BIT: QoI series, final state and moments.  The reference runs its
chains one after another (driver_mgmc.cc:236-254 measure_convergence, one MGMCSampler per chain);
the batch is the MI355X way of running them, and this test pins that it changes nothing.
"""
import numpy as np
import pytest

import multigridmc_amd as mg
from tests import test_gpu_lowrank as LR
from tests import test_gpu_parity as PAR

pytestmark = pytest.mark.gpu

SEED = 5418513
CHAIN0 = 11

PRIOR = ["3d128_zsweep", "3d_aniso_zsweep_ssor", "3d_zres27", "3d64_4lvl", "2d64_template_W", "2d_aniso_ssor",
         "2d256_global_coarse", "2d64_chol_W", "3d32_chol_ssor", "3d8_1lvl", "2d_qr_aniso_ssor_W"]
POSTERIOR = ["2d32_point_global", "3d32_ball_global", "3d128_zsweep_points", "3d_aniso_zres_points",
             "2d32_point_global_chol", "3d32_points_tail_W", "2d128_points_tail", "3d_jsweep_points_ssor",
             "3d128_global_inplace_W"]


def _prior(name, nchains=1, chain=0):
    shape, kw = PAR.CONFIGS[name]
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    lat = mg.Lattice(*shape)
    op = mg.ShiftedLaplaceFDOperator(lat, 25.0)
    return mg.MultigridMCSampler(op, SEED, p, device=0, chain_id=chain, nchains=nchains), lat


def _posterior(name, nchains=1, chain=0):
    shape, kw, (radius, nmeas, glob) = LR.CONFIGS[name]
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    op, lat = LR.measured(shape, 25.0, radius, nmeas, glob)
    return mg.MultigridMCSampler(op, SEED, p, device=0, chain_id=chain, nchains=nchains), lat


def _check_batch(make, name, nchains=3, nsteps=5):
    b, lat = make(name, nchains=nchains, chain=CHAIN0)
    assert b.nchains == nchains and b.lib.mgmc_nchains(b.handle) == nchains
    rng = np.random.default_rng(17)
    f = rng.standard_normal(lat.Nvertex)
    x0 = 0.1 * rng.standard_normal(lat.Nvertex)
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    b.fix_rhs(f)
    b.set_state(x0)
    zb = b.sample(nsteps, qoi, chain=None)
    for c in range(nchains):
        s, _ = make(name, chain=CHAIN0 + c)
        s.fix_rhs(f)
        s.set_state(x0)
        z = s.sample(nsteps, qoi)
        assert np.all(np.isfinite(z))
        assert np.array_equal(zb[c], z), f"chain {c}: QoI series"
        assert np.array_equal(b.get_state(c), s.get_state()), f"chain {c}: state"
        assert np.array_equal(b.qoi_moments(c), s.qoi_moments()), f"chain {c}: moments"
        s.close()
    # chains with different ids differ
    assert not np.array_equal(zb[0], zb[1])
    b.close()


@pytest.mark.parametrize("name", PRIOR)
def test_batched_prior_chains_bitwise(hip_device, name):
    _check_batch(_prior, name)


@pytest.mark.parametrize("name", POSTERIOR)
def test_batched_posterior_chains_bitwise(hip_device, name):
    _check_batch(_posterior, name)


@pytest.mark.parametrize("paths,name", [(PAR.ALL_PATHS, "3d128_zsweep"), (PAR.ALL_PATHS, "2d64_template_W"),
                                        ("tail", "3d_zres27"), ("lr_small,lr_merge,tail", "3d32_points_tail_W"),
                                        ("lr_small,tail", "2d32_point_global")])
def test_batched_chains_on_fallback_paths(hip_device, monkeypatch, paths, name):
    """The generic launches (one chain per launch inside the batch) give the same chains."""
    monkeypatch.setenv("MGMC_DISABLE", paths)
    _check_batch(_posterior if name in LR.CONFIGS else _prior, name, nchains=2, nsteps=4)


def test_batched_chain_state_accessors_and_growth(hip_device):
    """Per-chain set_state / get_state, a series that grows between calls (the graphs carry the
    chain stride of the series) and the unrolled sample loop."""
    b, lat = _prior("3d64_4lvl", nchains=4, chain=0)
    rng = np.random.default_rng(5)
    xs = [rng.standard_normal(lat.Nvertex) for _ in range(4)]
    for c, x in enumerate(xs):
        b.set_state(x, chain=c)
    for c, x in enumerate(xs):
        assert np.array_equal(b.get_state(c), x)
    qoi = mg.measurement_vector_index(lat, [0.25] * lat.dim)
    za = b.sample(3, qoi, chain=None)
    zb = b.sample(37, qoi, chain=None)  # grows the series past its first capacity
    for c in (0, 3):
        s, _ = _prior("3d64_4lvl", chain=c)
        s.set_state(xs[c])
        assert np.array_equal(s.sample(3, qoi), za[c])
        assert np.array_equal(s.sample(37, qoi), zb[c])
        assert np.array_equal(s.get_state(), b.get_state(c))
        s.close()
    b.close()


def test_batched_chain_argument_validation(hip_device):
    for bad in (0, 17):
        with pytest.raises(mg.MgmcError):
            _prior("3d16", nchains=bad)
    b, lat = _prior("3d16", nchains=2)
    with pytest.raises(mg.MgmcError):
        b.get_state(2)
    with pytest.raises(mg.MgmcError):
        b.set_state(np.zeros(lat.Nvertex), chain=5)
    with pytest.raises(mg.MgmcError):
        b.qoi_moments(-1)
    b.close()


def test_batched_config5_global_at_256_cubed(hip_device):
    """BASELINE config 5 with the global average (the dense-column path) at full size, 2 chains in
    one handle: each chain's QoI series and state bitwise equal to its one-chain handle."""
    from tests.test_gpu_configs import _config5
    lat, op, p = _config5(True)
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    b = mg.MultigridMCSampler(op, SEED, p, chain_id=CHAIN0, nchains=2)
    zb = b.sample(3, qoi, chain=None)
    for c in range(2):
        s = mg.MultigridMCSampler(op, SEED, p, chain_id=CHAIN0 + c)
        assert np.array_equal(s.sample(3, qoi), zb[c])
        assert np.array_equal(s.get_state(), b.get_state(c))
        s.close()
    b.close()
