"""Parity at BASELINE config 3 itself (-m gpu): 3D 256^3 shifted-Laplace prior, 6-level V-cycle, one
chain -- the hierarchy `bench.py --n 256 --nlevel 6` times.

The kernel instances this configuration selects differ from the 512^3 ones (mgmc_capi.hip): the fine
z-sweeps run 256-wide rows in shorter z chunks, the fine residual + restriction is the 64 x 4
`k_zresrestrict<7,64,4>` (the coarse level has fewer than 16 K tile planes), level 1 (127^3, 64-pair
rows) runs colour-pair passes, not j-marching half-sweeps, level 2 (63^3) runs quad passes and
k_tail takes the 15^3 and 7^3 levels.  One V-cycle from x = 0 plus a 3-sample QoI series are compared
bit for bit (np.array_equal) with the CPU oracle's MULTICOLOUR replay (its OWN Galerkin hierarchy:
the stencil-mode RAP from its FD row, no device stencil fed in; Philox key (5418513, 0)); component kernels at this width are compared too.
"""
import sys
import time

import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

SEED = 5418513
SHAPE = (256, 256, 256)
NLEVEL = 6


def _log(msg):
    sys.__stderr__.write(f"[config 3, 256^3] {msg}\n")
    sys.__stderr__.flush()


@pytest.fixture(scope="module")
def config3(hip_device):
    t0 = time.time()
    lat = mg.Lattice(*SHAPE)
    p = mg.MultigridParameters(nlevel=NLEVEL, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                               ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=0)
    O.set_threads(O.cpu_share())
    orc = O.Oracle.fd_own(SHAPE, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=0)
    _log(f"device handle + oracle hierarchy {time.time() - t0:.1f} s")
    yield s, orc, lat, p
    s.close()
    del orc
    O.set_threads(1)


def test_config3_kernel_instances(config3):
    """The instances this configuration runs (mgmc_level_kernels)."""
    s, orc, lat, p = config3
    k0 = s.level_kernels(0)
    assert k0["sweep"].startswith("k_zsweep_rb7<") and k0["post_sweep"].endswith("PROLONG>")
    assert k0["residual_restrict"] == "k_zresrestrict<7,64,4>"
    # levels 1-3 (quad passes): pre-sweep noise drawn by the restriction launch before them (level 1: the
    # fine 7-point residual, which does not), post-sweep noise by the tail launch's spare workgroups
    assert s.level_kernels(1) == {"sweep": "k_sweep_quads<3>", "residual_restrict": "k_zresrestrict<27,64,4>",
                                  "noise": "tail"}
    assert s.level_kernels(2)["sweep"] == "k_sweep_quads<3>" and s.level_kernels(2)["noise"] == "restriction+tail"
    assert s.level_kernels(NLEVEL - 1)["sweep"] == "k_tail<3>"


@pytest.mark.parametrize("level", [0, 1])
def test_config3_residual_restrict_bitwise(config3, level):
    """R (f - A x) at 256^3 (CSR order) and 127^3 (class-folded) against the MULTICOLOUR oracle, bit for bit."""
    s, orc, lat, p = config3
    rng = np.random.default_rng(300 + level)
    n = s.level_desc(level)["ndof"]
    f = rng.standard_normal(n)
    x = rng.standard_normal(n)
    assert np.array_equal(s.residual_restrict(level, f, x), orc.residual_restrict(level, f, x))


@pytest.mark.parametrize("level,direction", [(0, mg.BACKWARD), (1, mg.FORWARD), (2, mg.BACKWARD)])
def test_config3_noisy_sweep_bitwise(config3, level, direction):
    """One Gibbs sweep (SORSampler::apply, sor_sampler.cc:37-59) at full width on levels 0-2."""
    s, orc, lat, p = config3
    rng = np.random.default_rng(400 + level)
    n = s.level_desc(level)["ndof"]
    f = rng.standard_normal(n)
    x = rng.standard_normal(n)
    d = s.sor_sampler_apply(level, direction, 5 + level, 17, f, x)
    o = orc.sor_sampler_apply(level, direction, 5 + level, 17, f, x)
    assert np.array_equal(d, o)


def test_config3_cycle_and_qoi_series_bitwise(config3):
    """Sampler::apply (one 6-level V-cycle from x = 0, multigridmc_sampler.cc:132-138) with a random
    right-hand side, then the device-resident measure_sampling_time loop (driver_mgmc.cc:66-78) for 3
    samples with the QoI at the lattice centre: state, QoI series and final state equal the oracle's."""
    s, orc, lat, p = config3
    f = np.random.default_rng(13).standard_normal(lat.Nvertex)
    x_dev = np.zeros(lat.Nvertex)
    x_orc = np.zeros(lat.Nvertex)
    t0 = time.time()
    s.apply(f, x_dev)
    orc.apply(f, x_orc)
    _log(f"apply: {time.time() - t0:.1f} s")
    assert np.all(np.isfinite(x_dev)) and np.std(x_dev) > 0
    assert np.array_equal(x_dev, x_orc)
    qoi = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    s.fix_rhs(f)
    s.set_state(x_dev)
    orc.set_rhs(f)
    orc.set_state(x_orc)
    z_dev = s.sample(3, qoi)
    z_orc = orc.sample(3, qoi)
    assert np.array_equal(z_dev, z_orc)
    assert np.array_equal(s.get_state(), orc.get_state())
    assert s.get_sample_index() == 4


def test_config3_prior_series_from_zero_bitwise(config3):
    """The bench's own workload: the prior (f = 0) from x = 0, 4 cycles, QoI at the centre."""
    s, orc, lat, p = config3
    qoi = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    zero = np.zeros(lat.Nvertex)
    s.fix_rhs(zero)
    s.set_state(zero)
    s.set_sample_index(0)
    orc.set_rhs(zero)
    orc.set_state(zero)
    orc.set_sample_index(0)
    z_dev = s.sample(4, qoi)
    z_orc = orc.sample(4, qoi)
    assert np.all(z_dev != 0)
    assert np.array_equal(z_dev, z_orc)
    assert np.array_equal(s.get_state(), orc.get_state())
