"""Parity at the headline configuration itself (-m gpu): BASELINE config 4, 3D 512^3, 7-level
V-cycle, one chain -- the hierarchy bench.py times.

The kernel instances this configuration selects exist only at this size (mgmc_capi.hip): the fine
residual + restriction `k_zresrestrict<7,64,8,512>` (chosen when the coarse level has >= 16 K tile
planes), the fused-prolongation post-sweep's 128-plane z chunks, the level-1 j-marching half-sweeps (k_jsweep_half) at
their full 128-pair row width and the 512^3 `k_tail`.  Every one of them is compared here bit for
bit (np.array_equal) with the CPU oracle's MULTICOLOUR replay, which builds its OWN Galerkin
hierarchy (the stencil-mode RAP from its FD row; no device stencil is fed in) with Philox key
(5418513, 0).  The level-0 residual + restriction is also the FAITHFUL arithmetic (the reference's
`A_sparse * x` then `f - r`, linear_operator.hh:66-76, multigridmc_sampler.cc:118-120, in CSR
order); level 1 and below take the class-folded sum (fold27), which the MULTICOLOUR oracle replays.

The oracle runs its row-parallel loops on the CPU share (tests/oracle_lib.set_threads; bitwise the
serial oracle's results): setup about 30 s and 4-8 s per cycle on 16 cores.  Progress lines go to
the real stderr so a long step is visibly alive.
"""
import sys
import time

import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

SEED = 5418513
SHAPE = (512, 512, 512)
NLEVEL = 7


def _log(msg):
    sys.__stderr__.write(f"[headline 512^3] {msg}\n")
    sys.__stderr__.flush()


@pytest.fixture(scope="module")
def headline(hip_device):
    t0 = time.time()
    lat = mg.Lattice(*SHAPE)
    p = mg.MultigridParameters(nlevel=NLEVEL, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                               ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=0)
    _log(f"device handle {time.time() - t0:.1f} s")
    O.set_threads(O.cpu_share())
    orc = O.Oracle.fd_own(SHAPE, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=0)
    _log(f"oracle hierarchy ({O.cpu_share()} threads) {time.time() - t0:.1f} s")
    yield s, orc, lat, p
    s.close()
    del orc
    O.set_threads(1)


def test_headline_fine_stencil_is_the_reference_operator(headline):
    """The device's level-0 stencil is the reference FD row (shiftedlaplace_fd_operator.cc:9-57):
    the oracle's own assembly of the 512^3 operator has it on an interior row."""
    s, orc, lat, p = headline
    st = s.level_desc(0)["stencil"]
    row = lat.Nvertex // 2 + 511 * 5 + 7  # an interior vertex
    cols, vals = orc.csr_row(0, row)
    n = 511
    expect = {row - n * n: st[4], row - n: st[10], row - 1: st[12], row: st[13], row + 1: st[14], row + n: st[16],
              row + n * n: st[22]}
    assert dict(zip(cols.tolist(), vals.tolist())) == expect


@pytest.mark.parametrize("level", [0, 1])
def test_headline_residual_restrict_bitwise(headline, level):
    """R (f - A x) at 512^3 (level 0: k_zresrestrict<7,64,8,512>, the CSR order) and 255^3 (level 1: the
    27-point fold instance) against the MULTICOLOUR oracle, bit for bit."""
    s, orc, lat, p = headline
    rng = np.random.default_rng(100 + level)
    n = s.level_desc(level)["ndof"]
    f = rng.standard_normal(n)
    x = rng.standard_normal(n)
    t0 = time.time()
    d = s.residual_restrict(level, f, x)
    o = orc.residual_restrict(level, f, x)
    _log(f"residual_restrict level {level}: {time.time() - t0:.1f} s")
    assert np.array_equal(d, o)


@pytest.mark.parametrize("level,direction", [(0, mg.FORWARD), (1, mg.BACKWARD)])
def test_headline_noisy_sweep_bitwise(headline, level, direction):
    """One Gibbs sweep (SORSampler::apply, sor_sampler.cc:37-59) at full width: the fine z-marching
    red-black sweep (512^3) and the level-1 j-marching half-sweeps (255^3, 128-pair rows)."""
    s, orc, lat, p = headline
    rng = np.random.default_rng(200 + level)
    n = s.level_desc(level)["ndof"]
    f = rng.standard_normal(n)
    x = rng.standard_normal(n)
    t0 = time.time()
    d = s.sor_sampler_apply(level, direction, 3 + level, 41, f, x)
    o = orc.sor_sampler_apply(level, direction, 3 + level, 41, f, x)
    _log(f"sor_sampler_apply level {level}: {time.time() - t0:.1f} s")
    assert np.array_equal(d, o)


def test_headline_cycle_and_qoi_series_bitwise(headline):
    """Sampler::apply (one 7-level V-cycle from x = 0, multigridmc_sampler.cc:132-138), then the
    device-resident measure_sampling_time loop (driver_mgmc.cc:66-78) for 3 samples with the QoI at
    the lattice centre: cycle state, QoI series and final state equal the oracle's exactly.  This
    runs the benchmark's graph: fused-prolongation post-sweep (128-plane chunks), k_zresrestrict
    <7,64,8,512>, the level-1 j-marching half-sweeps, the level-2 colour-pair passes, the 512^3 k_tail and
    the QoI record."""
    s, orc, lat, p = headline
    f = np.random.default_rng(11).standard_normal(lat.Nvertex)
    x_dev = np.zeros(lat.Nvertex)
    x_orc = np.zeros(lat.Nvertex)
    t0 = time.time()
    s.apply(f, x_dev)
    orc.apply(f, x_orc)
    _log(f"apply: {time.time() - t0:.1f} s")
    assert np.all(np.isfinite(x_dev)) and np.std(x_dev) > 0
    assert np.array_equal(x_dev, x_orc)
    qoi = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    assert qoi == lat.Nvertex // 2  # vertex (256, 256, 256)
    s.fix_rhs(f)
    s.set_state(x_dev)
    orc.set_rhs(f)
    orc.set_state(x_orc)
    del x_dev, x_orc
    t0 = time.time()
    z_dev = s.sample(3, qoi)
    z_orc = orc.sample(3, qoi)
    _log(f"3-sample series: {time.time() - t0:.1f} s")
    assert np.array_equal(z_dev, z_orc)
    assert np.array_equal(s.get_state(), orc.get_state())
    assert s.get_sample_index() == 4


def test_headline_same_seed_handles_match_oracle(headline):
    """Determinism at the headline size, pinned to the oracle: three fresh handles
    with the same (seed, chain) -- each allocated after the previous one was freed, so each runs on
    recycled device memory -- start from one state (x, f, sample index) and run 4 prior cycles of the
    benchmark graph; every QoI series and final state equals the MULTICOLOUR oracle's, not just each
    other.  With MGMC_POISON=1 (scripts/determinism_512.py) unzeroed buffers and the LDS start as NaN."""
    s, orc, lat, p = headline
    qoi = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    rng = np.random.default_rng(12)
    x0 = 0.01 * rng.standard_normal(lat.Nvertex)
    f = np.zeros(lat.Nvertex)  # prior (driver_mgmc configs 2-4: f = 0)
    t0 = time.time()
    orc.set_rhs(f)
    orc.set_state(x0)
    orc.set_sample_index(7)
    z_orc = orc.sample(4, qoi)
    x_orc = orc.get_state()
    _log(f"oracle 4 cycles: {time.time() - t0:.1f} s")
    for r in range(3):
        h = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=0)
        h.fix_rhs(f)
        h.set_state(x0)
        h.set_sample_index(7)
        z = h.sample(4, qoi)
        same_z, same_x = bool(np.array_equal(z, z_orc)), bool(np.array_equal(h.get_state(), x_orc))
        _log(f"handle {r}: series {'==' if same_z else '!='} oracle, state {'==' if same_x else '!='} oracle")
        h.close()
        assert same_z and same_x, (r, z.tolist(), z_orc.tolist())


def test_headline_kernel_instances(headline):
    """The instances the tests above ran are the benchmark's (mgmc_level_kernels): the fused z-sweep
    pair on level 0 with the 64 x 8 residual + restriction, j-marching half-sweeps on level 1, k_tail below."""
    s, orc, lat, p = headline
    k0 = s.level_kernels(0)
    assert k0["sweep"].startswith("k_zsweep_rb7<") and k0["post_sweep"].endswith("PROLONG>")
    assert k0["residual_restrict"] == "k_zresrestrict<7,64,8>"
    # the 255^3 Galerkin stencil is reflection-symmetric bit for bit: the folded instance (stencil_coef)
    assert s.level_kernels(1) == {"sweep": "k_jsweep_half<128,sym>", "residual_restrict": "k_zresrestrict<27,64,4>"}
    assert s.level_kernels(2)["sweep"] == "k_sweep_quads<3>"  # 64-pair rows: quad passes
    # levels 2-4: the first pre-sweep reads the Box-Muller pairs the restriction launch drew, the post-sweep
    # those the tail launch's spare workgroups drew
    assert all(s.level_kernels(l).get("noise") == "restriction+tail" for l in range(2, NLEVEL - 2))
    assert s.level_kernels(NLEVEL - 1)["sweep"] == "k_tail<3>"
