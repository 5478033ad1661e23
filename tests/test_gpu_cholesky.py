"""Coarse Cholesky above 8,192 unknowns (-m gpu): the blocked banded solves (mgmc_cholesky.hpp
k_coarse_chol_blocked) of CholeskySampler (sampler/cholesky_sampler.cc:26-41, x = L^-T (xi + L^-1 f))
and of the multigrid preconditioner's exact coarse solve (multigrid_preconditioner.cc:76-80).

T2: whole cycles bitwise against the oracle's blocked mode (refcpu.cpp DenseCholeskySampler, the same
banded factor, blocks and fma order), which it selects by itself above 8,192 unknowns and by
set_chol_blocked for the small cases of MGMC_DISABLE=chol_dense.  T3: the exact sampler's mean and
covariance against Q^-1 f and Q^-1 (the blocked solves on a small lattice, several blocks), and the
preconditioned CG with the blocked coarse solve against a sparse direct solve."""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import multigridmc_amd as mg
from multigridmc_amd import _native
from tests import oracle_lib as O
from tests import test_gpu_lowrank as LR

pytestmark = pytest.mark.gpu

SEED = 5418513

# shape, parameters; the coarsest level has more than 8,192 unknowns
CONFIGS = {
    "2d256_nl2": ((256, 256), dict(nlevel=2)),  # 127^2 = 16,129 coarse unknowns, bandwidth 128
    "2d256_nl2_ssor": ((256, 256), dict(nlevel=2, smoother="SSOR", npresmooth=2, omega=0.9)),
    "3d48_nl2": ((48, 48, 48), dict(nlevel=2)),  # 23^3 = 12,167, bandwidth 553 (blocks of 576)
    "2d_aniso_nl1": ((160, 96), dict(nlevel=1)),  # the fine level itself: 15,105 unknowns
}


def _make(shape, kw, kappa_sq=25.0, chain=0, nchains=1):
    p = mg.MultigridParameters(**{"nlevel": 2, "smoother": "SOR", "coarse_solver": "Cholesky", **kw})
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, kappa_sq), SEED, p, device=0, chain_id=chain,
                              nchains=nchains)
    return s, p, lat


def _oracle(s, p, lat, kappa_sq=25.0, chain=0):
    return O.Oracle.fd_own(lat.shape, p, kappa_sq, mode=O.MULTICOLOUR, seed=SEED, chain=chain)


@pytest.mark.parametrize("name", list(CONFIGS))
def test_blocked_coarse_cholesky_cycles_bitwise(hip_device, name):
    shape, kw = CONFIGS[name]
    s, p, lat = _make(shape, kw)
    assert s.level_desc(p.nlevel - 1)["ndof"] > 8192
    assert s.level_kernels(p.nlevel - 1)["sweep"] == "k_coarse_chol_blocked"
    mc = _oracle(s, p, lat)
    f = np.random.default_rng(11).standard_normal(lat.Nvertex)
    x_dev, x_orc = np.zeros(lat.Nvertex), np.zeros(lat.Nvertex)
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


def test_blocked_coarse_cholesky_posterior_bitwise(hip_device):
    """B_c Sigma^-1 B_c^T of point measurements widens the band by each column's row span."""
    LR.CONFIGS["2d256_points_chol_blocked"] = ((256, 256), dict(nlevel=2, coarse_solver="Cholesky"),
                                               (0.0, 3, False))
    try:
        s, mc, p, lat, op = LR.make("2d256_points_chol_blocked")
    finally:
        del LR.CONFIGS["2d256_points_chol_blocked"]
    assert s.level_kernels(p.nlevel - 1)["sweep"] == "k_coarse_chol_blocked"
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    f = np.random.default_rng(2).standard_normal(lat.Nvertex)
    s.fix_rhs(f)
    mc.set_rhs(f)
    assert np.array_equal(s.sample(3, qoi), mc.sample(3, qoi))
    assert np.array_equal(s.get_state(), mc.get_state())
    s.close()


def test_blocked_coarse_cholesky_batched_chains(hip_device):
    shape, kw = CONFIGS["2d256_nl2"]
    b, p, lat = _make(shape, kw, chain=3, nchains=3)
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    zb = b.sample(3, q, chain=None)
    for c in range(3):
        s, _, _ = _make(shape, kw, chain=3 + c)
        assert np.array_equal(s.sample(3, q), zb[c])
        assert np.array_equal(s.get_state(), b.get_state(c))
        s.close()
    b.close()


def test_dense_lowrank_column_band_unsupported(hip_device):
    """A global-average measurement couples every coarse unknown: a bandwidth of n - 1 has no blocked
    factor above 8,192 unknowns (MGMC_E_UNSUPPORTED naming the bandwidth), nor has a lattice whose
    rows are longer than 4,096; a 3D level whose banded factor would take the host hours is refused
    too."""
    op, lat = LR.measured((256, 256), 25.0, 0.0, 2, True)
    p = mg.MultigridParameters(nlevel=2, coarse_solver="Cholesky")
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p)
    with pytest.raises(mg.MgmcError, match="bandwidth") as e:
        s.set_lowrank(op.get_B())
    assert e.value.code == _native.MGMC_E_UNSUPPORTED
    # the failed call leaves the prior: the handle samples exactly what a fresh prior handle
    # samples -- no posterior smoothers left on the levels with a prior-only coarse factor
    q = mg.measurement_vector_index(lat, [0.5, 0.5])
    z = s.sample(5, q)
    x = s.get_state()
    s.close()
    fresh = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p)
    assert np.array_equal(z, fresh.sample(5, q))
    assert np.array_equal(x, fresh.get_state())
    fresh.close()
    with pytest.raises(mg.MgmcError, match="bandwidth"):  # lexicographic band of 8191 unknowns
        _make((8192, 8), dict(nlevel=1))
    with pytest.raises(mg.MgmcError, match="host work limit"):  # 63^3 unknowns, bandwidth 4033
        _make((128, 128, 128), dict(nlevel=2))


@pytest.mark.parametrize("shape,nlevel,tol", [((16, 16), 1, 0.04), ((32, 32), 2, 0.05)])
def test_blocked_cholesky_statistics_vs_exact_covariance(hip_device, monkeypatch, shape, nlevel, tol):
    """sampler/test_sampler.hh:113-153 with the blocked solves forced on a small coarsest level
    (225 unknowns, bandwidth 15: four blocks of 64): mean and covariance against Q^-1 f and Q^-1,
    relative to max|Q^-1|.  nlevel 1 is the exact sampler (independent draws: 5 sigma of the max
    entry error ~ 0.03 at n = 40000); nlevel 2 the MGMC chain on 961 unknowns (IACT ~ 1.5, the max
    over ~460,000 entries: 0.05)."""
    monkeypatch.setenv("MGMC_DISABLE", "chol_dense")
    s, p, lat = _make(shape, dict(nlevel=nlevel), kappa_sq=4.0)
    assert s.level_kernels(nlevel - 1)["sweep"] == "k_coarse_chol_blocked"
    orc = O.Oracle.fd(lat.shape, p, 4.0, mode=O.FAITHFUL)
    Q = orc.csr_matrix(0).toarray()
    mu = np.random.default_rng(1342517).random(lat.Nvertex)
    n, nsamples = lat.Nvertex, 40000
    s.fix_rhs(Q @ mu)
    s.sample(100)
    ex = np.zeros(n)
    exx = np.zeros((n, n))
    chunk = 1000
    for k0 in range(0, nsamples, chunk):  # states in chunks: one download per sample
        X = np.empty((chunk, n))
        for k in range(chunk):
            s.sample(1)
            X[k] = s.get_state()
        ex += X.sum(axis=0)
        exx += X.T @ X
    ex /= nsamples
    cov = exx / nsamples - np.outer(ex, ex)
    Qinv = np.linalg.inv(Q)
    scale = np.max(np.abs(Qinv))
    assert np.max(np.abs(ex - mu)) < 2 * tol * scale
    assert np.max(np.abs(cov - Qinv)) < tol * scale
    s.close()


def test_cg_with_blocked_coarse_solve(hip_device):
    """The preconditioner's exact coarse solve through the blocked solves (noise off)."""
    shape, kw = CONFIGS["2d256_nl2"]
    s, p, lat = _make(shape, kw)
    orc = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL)
    b = np.random.default_rng(3).standard_normal(lat.Nvertex)
    x_ref = spla.spsolve(orc.csr_matrix(0).tocsc(), b)
    x, it, rn = s.solve(b, method="cg", rtol=1e-13, maxiter=200)
    assert it < 200
    assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) < 1e-10
    s.close()
