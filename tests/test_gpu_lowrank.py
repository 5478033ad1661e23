"""GPU parity of the low-rank posterior path (-m gpu): Q = A + B Sigma^{-1} B^T.

T2 (bitwise, np.array_equal) against the oracle's MULTICOLOUR replay of the same arithmetic order
(mgmc_lowrank.hpp header): posterior operator apply, SOR smoother with the B_bar fix
(sor_smoother.cc:41-53), SOR sampler with the low-rank noise (sor_sampler.cc:48-56), posterior
residual + restriction, and whole MGMC cycles on every level with B_c = R B.  Columns of B cover
radius-0 point measurements, radius > 0 ball averages (measured_operator.cc:92-170) and the dense
global column.  T3: the device chain's mean / covariance against the exact posterior Q^-1.
"""
import numpy as np
import pytest

import multigridmc_amd as mg
from multigridmc_amd.parameters import MeasurementParameters
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513

# shape, multigrid parameters, (radius, number of measurements, measure_global)
CONFIGS = {
    "2d32_point_global": ((32, 32), dict(nlevel=3), (0.0, 3, True)),
    "2d64_ball_ssor_W": ((64, 64), dict(nlevel=4, cycle=2, smoother="SSOR", omega=0.9), (0.06, 4, False)),
    "3d32_ball_global": ((32, 32, 32), dict(nlevel=3, ncoarsesmooth=2), (0.1, 2, True)),
    "3d128_zsweep_points": ((128, 128, 128), dict(nlevel=3, smoother="SSOR"), (0.0, 8, False)),
    "3d_aniso_zres_points": ((256, 40, 48), dict(nlevel=2, omega=1.1), (0.0, 5, False)),
    "2d32_point_global_chol": ((32, 32), dict(nlevel=3, coarse_solver="Cholesky"), (0.0, 3, True)),
    "3d32_ball_chol_ssor": ((32, 32, 32), dict(nlevel=3, smoother="SSOR", coarse_solver="Cholesky"), (0.1, 2, False)),
    # levels whose sub-cycle runs in one k_tail workgroup, low-rank part included
    "3d32_points_tail_W": ((32, 32, 32), dict(nlevel=4, cycle=2, ncoarsesmooth=2), (0.0, 6, False)),
    "3d48_ball_tail_ssor": ((48, 48, 48), dict(nlevel=4, smoother="SSOR"), (0.1, 3, False)),
    "2d128_points_tail": ((128, 128), dict(nlevel=5), (0.0, 4, False)),
    # dense-column path on the fine level (> 4096 vertices), the global column as an entry list below
    "2d128_point_global_W": ((128, 128), dict(nlevel=4, cycle=2), (0.0, 4, True)),
    # j-marching half-sweeps on level 1 (128-pair rows) with the low-rank patch / fix around them
    "3d_jsweep_points_ssor": ((512, 24, 20), dict(nlevel=3, smoother="SSOR"), (0.0, 5, False)),
    # the fine z-sweep level with the constant global column: right-hand side read in place, the
    # column's term split off (LowRankDev::rhs_inplace, lr_row_patch); two pre- / post-sweeps, W-cycle
    "3d128_global_inplace_W": ((128, 128, 128), dict(nlevel=3, cycle=2, npresmooth=2, npostsmooth=2),
                               (0.0, 5, True)),
    # ... the global average alone (m = 1: no local rows, every patch is the kernels' e)
    "3d128_global_only_inplace": ((128, 128, 128), dict(nlevel=3), (0.0, 0, True)),
}
TAIL_CONFIGS = ["2d64_ball_ssor_W", "3d32_points_tail_W", "3d48_ball_tail_ssor", "2d128_points_tail"]


def measured(shape, kappa_sq, radius, nmeas, glob, seed=1212417, scale=1e-3):
    rng = np.random.default_rng(seed)
    lat = mg.Lattice(*shape)
    mp = MeasurementParameters(radius=radius, variance_scaling=scale, measure_global=glob, variance_global=0.02)
    mp.measurement_locations = [list(rng.uniform(0.15, 0.85, len(shape))) for _ in range(nmeas)]
    mp.variance = list(1.0 + 2.0 * rng.random(nmeas))
    return mg.MeasuredOperator(mg.ShiftedLaplaceFDOperator(lat, kappa_sq), mp), lat


def make(name, kappa_sq=25.0, chain=0):
    shape, kw, (radius, nmeas, glob) = CONFIGS[name]
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    op, lat = measured(shape, kappa_sq, radius, nmeas, glob)
    s = mg.MultigridMCSampler(op, SEED, p, device=0, chain_id=chain)
    mc = O.Oracle.fd_own(lat.shape, p, kappa_sq, mode=O.MULTICOLOUR, seed=SEED, chain=chain)
    mc.set_lowrank(op.get_B())
    return s, mc, p, lat, op


@pytest.mark.parametrize("name", list(CONFIGS))
def test_lowrank_components_bitwise(hip_device, name):
    s, mc, p, lat, op = make(name)
    rng = np.random.default_rng(3)
    for level in range(p.nlevel):
        n = s.level_desc(level)["ndof"]
        x = rng.standard_normal(n)
        b = rng.standard_normal(n)
        assert np.array_equal(s.operator_apply(level, x), mc.operator_apply(level, x)), f"level {level} apply"
        for direction in (mg.FORWARD, mg.BACKWARD):
            d = s.smoother_apply(level, direction, 2, b, x)
            o = mc.smoother_apply(level, direction, 2, b, x)
            assert np.array_equal(d, o), f"level {level} dir {direction} smoother"
            d = s.sor_sampler_apply(level, direction, 9 + level, 31, b, x)
            o = mc.sor_sampler_apply(level, direction, 9 + level, 31, b, x)
            assert np.array_equal(d, o), f"level {level} dir {direction} sampler"
        if level + 1 < p.nlevel:
            assert np.array_equal(s.residual_restrict(level, b, x), mc.residual_restrict(level, b, x)), \
                f"level {level} residual"
    s.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_lowrank_cycles_bitwise(hip_device, name):
    s, mc, p, lat, op = make(name)
    if name in ("3d128_global_inplace_W", "3d128_global_only_inplace"):  # the path these configurations are here for
        assert s.level_kernels(0)["lowrank"] == "dense,rhs_inplace"
        assert s.level_kernels(1)["lowrank"] == "dense"
    rng = np.random.default_rng(11)
    f = rng.standard_normal(lat.Nvertex)
    x_dev = np.zeros(lat.Nvertex)
    x_orc = np.zeros(lat.Nvertex)
    for _ in range(2):
        s.apply(f, x_dev)
        mc.apply(f, x_orc)
        assert np.array_equal(x_dev, x_orc)
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    s.fix_rhs(f)
    s.set_state(x_dev)
    mc.set_rhs(f)
    mc.set_state(x_orc)
    assert np.array_equal(s.sample(4, qoi), mc.sample(4, qoi))
    assert np.array_equal(s.get_state(), mc.get_state())
    s.close()


def test_bbar_rows_stay_local_for_point_measurements(hip_device):
    """Multicolour splitting: B_bar of a point measurement lives on a few vertices around it (the
    reference's lexicographic B_bar is dense, N rows)."""
    s, mc, p, lat, op = make("3d128_zsweep_points")
    m = op.get_m_lowrank()
    for level in range(p.nlevel):
        for direction in (mg.FORWARD, mg.BACKWARD):
            mm, rows = s.lowrank_info(level, direction)
            assert mm == m
            assert 0 < rows <= m * 200, f"level {level}: {rows} B_bar rows"
    s.close()


def test_set_lowrank_validation_and_reset(hip_device):
    s, mc, p, lat, op = make("2d32_point_global")
    lr = op.get_B()
    bad = mg.LowRankUpdate.__new__(mg.LowRankUpdate)  # bypass host validation: the C-ABI must check
    bad.__dict__.update(lr.__dict__)
    bad.sigma = lr.sigma.copy()
    bad.sigma[0] = -1.0
    with pytest.raises(mg.MgmcError):
        s.set_lowrank(bad)
    bad.sigma = lr.sigma.copy()
    bad.rows = lr.rows.copy()
    bad.rows[0] = lat.Nvertex
    with pytest.raises(mg.MgmcError):
        s.set_lowrank(bad)
    # m = 0 restores the prior: cycles equal the prior oracle
    s.set_lowrank(None)
    assert s.lowrank_info(0, mg.FORWARD) == (0, 0)
    prior = O.Oracle.fd_own(lat.shape, p, 25.0, mode=O.MULTICOLOUR, seed=SEED)
    f = np.random.default_rng(5).standard_normal(lat.Nvertex)
    xd = np.zeros(lat.Nvertex)
    xo = np.zeros(lat.Nvertex)
    s.apply(f, xd)
    prior.apply(f, xo)
    assert np.array_equal(xd, xo)
    s.close()


@pytest.mark.parametrize("shape,kw,glob,nsamples,tol", [
    ((8, 8), dict(nlevel=3, smoother="SSOR", coarse_solver="Cholesky"), False, 40000, 0.04),
    ((8, 8), dict(nlevel=3), True, 40000, 0.04),
    ((8, 8, 8), dict(nlevel=2, ncoarsesmooth=2), True, 20000, 0.07),
])
def test_posterior_statistics_vs_exact_covariance(hip_device, shape, kw, glob, nsamples, tol):
    """sampler/test_sampler.hh:260-323 on the device chain with the posterior operator (4 ball
    measurements, radius 0.05 in 2D / 0.15 in 3D, Sigma = 1e-2 (1 + 2u), optional global
    measurement): sample mean and covariance against the exact Q^-1 f and Q^-1, relative to
    max|Q^-1| (tolerances as for the prior chain, test_gpu_parity.py)."""
    radius = 0.05 if len(shape) == 2 else 0.15
    op, lat = measured(shape, 4.0, radius, 4, glob, scale=1e-2)
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    s = mg.MultigridMCSampler(op, SEED, p)
    orc = O.Oracle.fd(lat.shape, p, 4.0, mode=O.FAITHFUL)
    Q = orc.csr_matrix(0).toarray() + op.get_B().precision_update()
    mu = np.random.default_rng(1342517).random(lat.Nvertex)
    s.fix_rhs(Q @ mu)
    s.sample(500)
    n = lat.Nvertex
    ex = np.zeros(n)
    exx = np.zeros((n, n))
    for k in range(nsamples):
        s.sample(1)
        x = s.get_state()
        ex += (x - ex) / (k + 1)
        exx += (np.outer(x, x) - exx) / (k + 1)
    cov = exx - np.outer(ex, ex)
    Qinv = np.linalg.inv(Q)
    scale = np.max(np.abs(Qinv))
    assert np.max(np.abs(ex - mu)) < 2 * tol * scale
    assert np.max(np.abs(cov - Qinv)) < tol * scale
    s.close()


@pytest.mark.parametrize("name,paths", [(n, "tail") for n in TAIL_CONFIGS] +
                         [(n, q) for n in ("3d32_points_tail_W", "2d32_point_global", "3d_aniso_zres_points")
                          for q in ("lr_small", "lr_merge", "lr_small,lr_merge,tail")] +
                         [(n, "lr_dense") for n in ("2d128_point_global_W", "3d32_ball_global")] +
                         [("3d128_global_inplace_W", q) for q in ("lr_merge", "lr_dense")])
def test_lowrank_paths_match(hip_device, name, paths, monkeypatch):
    """Low-rank kernel paths switched off (MGMC_DISABLE): tail = the coarse levels' sub-cycle as
    separate launches instead of k_tail (low-rank patches, fix and residual in LDS); lr_small = the
    generic fix / patch / restore launches instead of the single-workgroup k_lr_small; lr_merge =
    separate restore and patch launches around the residual + restriction; lr_dense = the row lists over every vertex for a dense column (the
    global average measurement) instead of streaming B_g / Y_g with the patched right-hand side in
    a separate vector.  QoI series and state bitwise against the oracle, on and off."""
    out = []
    for env in (paths, None):
        if env:
            monkeypatch.setenv("MGMC_DISABLE", env)
        else:
            monkeypatch.delenv("MGMC_DISABLE", raising=False)
        s, mc, p, lat, op = make(name)
        qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
        z = s.sample(5, qoi)
        assert np.array_equal(z, mc.sample(5, qoi))
        out.append(s.get_state())
        assert np.array_equal(out[-1], mc.get_state())
        s.close()
    assert np.array_equal(out[0], out[1])


def test_failed_rollback_refuses_cycle_until_reinstall(hip_device):
    """mgmc_set_lowrank's failure path: a coarse Cholesky factor that cannot be built
    after the argument checks leaves the prior operator; if restoring the prior's factor fails as
    well, the handle refuses every call that runs the cycle or needs the factor (sample, apply,
    solve, per-level calls) with the reason, keeps the state / QoI calls, and a later successful
    mgmc_set_lowrank clears it -- after which the chain equals a fresh posterior handle's."""
    s, mc, p, lat, op = make("2d32_point_global_chol")
    q = mg.measurement_vector_index(lat, [0.5, 0.5])
    B = op.get_B()
    s.sample(2, q)
    # one injected failure: the posterior factor fails, the prior's is rebuilt -> usable prior handle
    assert s.lib.mgmc_debug_fail_coarse_factor(s.handle, 1) == 0
    with pytest.raises(mg.MgmcError, match="injected failure"):
        s.set_lowrank(B)
    assert s.lowrank_info(0, mg.FORWARD)[0] == 0
    s.sample(2, q)
    # two: the restore fails too -> unusable
    assert s.lib.mgmc_debug_fail_coarse_factor(s.handle, 2) == 0
    with pytest.raises(mg.MgmcError, match="unusable"):
        s.set_lowrank(B)
    for call in (lambda: s.sample(1, q), lambda: s.apply(np.zeros(lat.Nvertex), np.zeros(lat.Nvertex)),
                 lambda: s.solve(np.ones(lat.Nvertex), method="cg"), lambda: s.operator_apply(0, np.zeros(lat.Nvertex))):
        with pytest.raises(mg.MgmcError, match="unusable"):
            call()
    x = s.get_state()  # state calls stay available
    s.set_state(x)
    # a successful install clears it; the chain then equals a fresh posterior handle's
    s.set_lowrank(B)
    ref, _, _, _, _ = make("2d32_point_global_chol")
    f = np.random.default_rng(5).standard_normal(lat.Nvertex)
    for h in (s, ref):
        h.fix_rhs(f)
        h.set_state(x)
        h.set_sample_index(40)
    assert np.array_equal(s.sample(3, q), ref.sample(3, q))
    assert np.array_equal(s.get_state(), ref.get_state())
    s.close()
    ref.close()
