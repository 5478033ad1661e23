"""Pin the CPU oracle (oracle/refcpu.cpp) against the reference's own known answers, identities
and statistical tests (CPU only, no GPU).

The reference cannot be compiled here (Eigen / libconfig / GoogleTest absent, DESIGN.md
"Oracle"), so the oracle is pinned by:
  * the known answers of lattice/test_lattice.hh,
  * the libstdc++ normal stream head of the reference's RNG plumbing,
  * the prolongation / adjointness identities of intergrid/test_intergrid.hh,
  * the smoother fixed-point test of smoother/test_smoother.hh,
  * the mean / covariance statistical tests of sampler/test_sampler.hh,
  * the Galerkin stencil values of SURVEY.md Appendix A.
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

from tests import oracle_lib as O
from multigridmc_amd.parameters import MultigridParameters

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_known_answers.json")))
LATS = {k: v for k, v in GOLD["lattices"].items() if not k.startswith("_")}


def _dim(name):
    return len(LATS[name])


# ---------------------------------------------------------------- lattice (test_lattice.hh)
@pytest.mark.parametrize("case", GOLD["vertex_linear2euclidean"], ids=lambda c: c["cite"])
def test_vertex_linear2euclidean(case):
    n = LATS[case["lattice"]]
    idx = (O.ctypes.c_int * 3)()
    O.lib().orc_lattice_lin2euc(len(n), O.ivec(n), case["ell"], idx)
    assert list(idx)[: len(n)] == case["idx"]


@pytest.mark.parametrize("case", GOLD["vertex_euclidean2linear"], ids=lambda c: c["cite"])
def test_vertex_euclidean2linear(case):
    n = LATS[case["lattice"]]
    assert O.lib().orc_lattice_euc2lin(len(n), O.ivec(n), O.ivec(case["idx"] + [0] * (3 - len(n)))) == case["ell"]


@pytest.mark.parametrize("case", GOLD["shift_vertexidx"], ids=lambda c: c["cite"])
def test_shift_vertexidx(case):
    n = LATS[case["lattice"]]
    sh = case["shift"] + [0] * (3 - len(n))
    assert O.lib().orc_lattice_shift(len(n), O.ivec(n), case["ell"], O.ivec(sh)) == case["result"]


@pytest.mark.parametrize("case", GOLD["fine_vertex_idx"], ids=lambda c: c["cite"])
def test_fine_vertex_idx(case):
    n = LATS[case["lattice"]]
    assert O.lib().orc_lattice_fine_vertex_idx(len(n), O.ivec(n), case["ell"]) == case["result"]


# ---------------------------------------------------------------- RNG
def test_mt19937_normal_stream_head():
    g = GOLD["rng_stream_head"]
    np.testing.assert_array_equal(O.mt_normals(g["seed"], 4), np.array(g["values"]))


@pytest.mark.parametrize("kat", GOLD["philox4x32_10_kat"]["vectors"], ids=str)
def test_philox_kat(kat):
    conv = lambda v: int(v, 16) if isinstance(v, str) else int(v)  # noqa: E731
    out = O.philox_raw([conv(v) for v in kat["ctr"]], [conv(v) for v in kat["key"]])
    assert out == [conv(v) for v in kat["out"]]


def test_philox_normals_distribution():
    from scipy import stats
    z = O.philox_normals(5418513, 3, 0, 400000, 7, 11)
    assert abs(z.mean()) < 5 * np.sqrt(1 / len(z))
    assert abs(z.var() - 1) < 5 * np.sqrt(2 / len(z))
    assert stats.kstest(z, "norm").pvalue > 1e-4
    # distinct tags / samples / chains give independent streams
    z2 = O.philox_normals(5418513, 3, 0, 2000, 8, 11)
    z3 = O.philox_normals(5418513, 4, 0, 2000, 7, 11)
    assert abs(np.corrcoef(z[:2000], z2)[0, 1]) < 0.1 and abs(np.corrcoef(z[:2000], z3)[0, 1]) < 0.1


def test_oracle_math_accuracy():
    import ctypes
    import math
    us = np.random.default_rng(0).random(20000)
    us[0], us[1], us[2] = 1.0, 2.0 ** -52, 1.0 - 2.0 ** -52
    rel, ab = 0.0, 0.0
    for u in us:
        if u <= 0:
            continue
        d = abs(O.lib().orc_ln_unit(float(u)) - math.log(u))
        if abs(math.log(u)) > 1e-3:
            rel = max(rel, d / abs(math.log(u)))
        else:
            ab = max(ab, d)
    assert rel < 5e-16 and ab < 1e-16
    c, s = ctypes.c_double(), ctypes.c_double()
    e = 0.0
    ts = list(np.random.default_rng(1).random(20000))
    # exact quadrant points and the rounding boundaries k/64 +- 1/128 of the table reduction
    ts += [0.0, 0.25, 0.5, 0.75, 1.0 - 2.0 ** -52] + [(k + 0.5) / 64 for k in range(64)]
    ts += [(k + 0.5) / 64 - 2.0 ** -52 for k in range(64)]
    for t in ts:
        O.lib().orc_cos_sin_2pi(float(t), ctypes.byref(c), ctypes.byref(s))
        e = max(e, abs(c.value - math.cos(2 * math.pi * t)), abs(s.value - math.sin(2 * math.pi * t)))
    assert e < 2e-15
    for t, (ce, se) in ((0.0, (1.0, 0.0)), (0.25, (0.0, 1.0)), (0.5, (-1.0, 0.0)), (0.75, (0.0, -1.0))):
        O.lib().orc_cos_sin_2pi(t, ctypes.byref(c), ctypes.byref(s))
        assert (c.value, s.value) == (ce, se)


# ---------------------------------------------------------------- intergrid (test_intergrid.hh)
def _fd_oracle(shape, nlevel=2, mode=O.FAITHFUL, **kw):
    p = MultigridParameters(nlevel=nlevel, **kw)
    return O.Oracle.fd(shape, p, kappa_sq=25.0, mode=mode)


@pytest.mark.parametrize("shape", [(8, 8), (8, 8, 8)])
def test_prolongation_is_multilinear_interpolation(shape):
    o = _fd_oracle(shape)
    nc = o.ndof(1)
    xc = np.random.default_rng(1212417).standard_normal(nc)
    xp = o.prolongate_add(0, 1.0, xc, np.zeros(o.ndof(0)))
    # manual interpolation on the full (n+1)^d grid with zero boundary
    cshape = tuple(v // 2 for v in shape)
    grid_c = np.zeros(tuple(v + 1 for v in reversed(cshape)))
    inner = tuple(slice(1, v) for v in reversed(cshape))
    grid_c[inner] = xc.reshape(tuple(v - 1 for v in reversed(cshape)))
    fine = grid_c
    for ax in range(len(shape)):
        m = fine.shape[ax]
        out_shape = list(fine.shape)
        out_shape[ax] = 2 * (m - 1) + 1
        out = np.zeros(out_shape)
        sl = [slice(None)] * len(shape)
        sl[ax] = slice(0, None, 2)
        out[tuple(sl)] = fine
        sl[ax] = slice(1, None, 2)
        lo = [slice(None)] * len(shape)
        hi = [slice(None)] * len(shape)
        lo[ax] = slice(0, m - 1)
        hi[ax] = slice(1, m)
        out[tuple(sl)] = 0.5 * (fine[tuple(lo)] + fine[tuple(hi)])
        fine = out
    ref = fine[tuple(slice(1, v) for v in reversed(shape))].ravel()
    assert np.linalg.norm(xp - ref) < 1e-12


@pytest.mark.parametrize("shape", [(8, 8), (8, 8, 8)])
def test_restriction_is_adjoint_of_prolongation(shape):
    o = _fd_oracle(shape)
    rng = np.random.default_rng(1212417)
    xc = rng.standard_normal(o.ndof(1))
    r = rng.standard_normal(o.ndof(0))
    xp = o.prolongate_add(0, 1.0, xc, np.zeros(o.ndof(0)))
    rc = o.restrict(0, r)
    assert abs(xc @ rc - xp @ r) < 1e-12


# ---------------------------------------------------------------- Galerkin coarsening
def test_galerkin_appendix_a_values():
    a = GOLD["galerkin_3d_n16_units_of_h"]
    o = _fd_oracle((16, 16, 16), nlevel=2)
    A = o.csr_matrix(1).toarray() * 16.0
    # interior row (2,2,2) of the 7^3 coarse lattice
    r = (1 * 7 + 1) * 7 + 1
    centre = A[r, r]
    assert centre == pytest.approx(a["centre"], abs=5e-6)
    assert A[r, r + 1] == pytest.approx(a["face"], abs=5e-6)
    assert A[r, r + 1 + 7] == pytest.approx(a["edge"], abs=5e-6)
    assert A[r, r + 1 + 7 + 49] == pytest.approx(a["corner"], abs=5e-6)


@pytest.mark.parametrize("shape", [(16, 16), (32, 16), (16, 16, 16), (16, 8, 32)])
def test_galerkin_levels_are_truncated_constant_stencils(shape):
    """Every Galerkin level is symmetric and is the interior stencil truncated at the boundary;
    the oracle's stencil mode (used at 512^3) is bitwise equal to the full SpGEMM."""
    nlevel = 3
    full = _fd_oracle(shape, nlevel=nlevel)
    p = MultigridParameters(nlevel=nlevel)
    sten = O.Oracle.fd(shape, p, kappa_sq=25.0, galerkin=1)
    for lev in range(nlevel):
        A = full.csr_matrix(lev)
        B = sten.csr_matrix(lev)
        assert (A != A.T).nnz == 0
        assert (A != B).nnz == 0, f"level {lev}: stencil mode differs from SpGEMM"


# ---------------------------------------------------------------- smoother fixed point
@pytest.mark.parametrize("mode", [O.FAITHFUL, O.MULTICOLOUR])
@pytest.mark.parametrize("shape", [(32, 32), (16, 16, 16)])
def test_ssor_smoother_leaves_solution_invariant(mode, shape):
    """smoother/test_smoother.hh:90-101 (omega = 0.8), FD operator."""
    o = O.Oracle.fd(shape, MultigridParameters(nlevel=2, omega=0.8), kappa_sq=25.0, mode=mode)
    for lev in (0, 1):
        x_exact = np.random.default_rng(1212417).standard_normal(o.ndof(lev))
        b = o.operator_apply(lev, x_exact)
        x = o.smoother_apply(lev, 1, 1, b, x_exact)
        x = o.smoother_apply(lev, 2, 1, b, x)
        assert np.linalg.norm(x - x_exact) / np.linalg.norm(x_exact) < 1e-12


@pytest.mark.parametrize("shape,tol", [((512, 512), 2e-4), ((64, 64, 64), 7e-3)])
def test_fd_operator_manufactured_solution(shape, tol):
    """linear_operator/test_linear_operator.hh:212-244 (FD, relative L2 error of A u against
    h^d (-lap u + kappa^2 u); 2D 512^2 tol 2e-4, 3D 64^3 tol 7e-3), constant kappa^2."""
    o = _fd_oracle(shape, nlevel=1)
    dim = len(shape)
    h = 1.0 / shape[0]
    axes = [np.arange(1, n) / n for n in reversed(shape)]
    grids = np.meshgrid(*axes, indexing="ij")  # slowest axis first
    ks = [1.0, 2.0, 1.0][:dim]
    u = np.ones_like(grids[0])
    for d in range(dim):
        u = u * np.sin(ks[d] * np.pi * grids[dim - 1 - d])
    rhs_exact = (np.pi ** 2 * sum(k * k for k in ks) + 25.0) * u * h ** dim
    rhs = o.operator_apply(0, u.ravel())
    assert np.linalg.norm(rhs - rhs_exact.ravel()) / np.linalg.norm(rhs) < tol


# ---------------------------------------------------------------- statistical tests (test_sampler.hh)
def _test_operator_1d():
    n = 7
    rowptr, col, val = [0], [], []
    for i in range(n):
        for j in (i - 1, i, i + 1):
            if 0 <= j < n:
                col.append(j)
                val.append(6.0 if i == j else -1.0)
        rowptr.append(len(col))
    return np.array(rowptr), np.array(col), np.array(val)


def _mean_cov_error(oracle, Q, nsamples, nwarmup=1000):
    rng = np.random.default_rng(1342517)
    mu = rng.random(Q.shape[0])
    f = Q @ mu
    ex, cov = oracle.mean_cov(f, nwarmup, nsamples)
    return np.max(np.abs(ex - mu)), np.max(np.abs(cov - np.linalg.inv(Q)))


def test_mgmc_1d_statistics_faithful():
    """sampler/test_sampler.hh:224-256: 3 levels, SSOR smoother, Cholesky coarse, tol 2e-3."""
    case = GOLD["sampler_tests"]["TestMultigridMCSampler1d"]
    rowptr, col, val = _test_operator_1d()
    p = MultigridParameters(nlevel=3, smoother="SSOR", coarse_solver="Cholesky", omega=1.0, cycle=1)
    o = O.Oracle.csr((8,), p, rowptr, col, val, seed=case["seed"])
    Q = sp.csr_matrix((val, col, rowptr)).toarray()
    em, ec = _mean_cov_error(o, Q, case["nsamples"])
    assert em < case["tolerance"] and ec < case["tolerance"]


def test_ssor_sampler_1d_statistics_faithful():
    """sampler/test_sampler.hh:201-218 as a one-level MGMC (coarse SSOR sampler, omega 0.8)."""
    case = GOLD["sampler_tests"]["TestSSORSampler1d"]
    rowptr, col, val = _test_operator_1d()
    p = MultigridParameters(nlevel=1, coarse_solver="SSOR", ncoarsesmooth=1, omega=case["omega"])
    o = O.Oracle.csr((8,), p, rowptr, col, val, seed=case["seed"])
    Q = sp.csr_matrix((val, col, rowptr)).toarray()
    em, ec = _mean_cov_error(o, Q, case["nsamples"])
    assert em < case["tolerance"] and ec < case["tolerance"]


@pytest.mark.parametrize("mode", [O.FAITHFUL, O.MULTICOLOUR])
@pytest.mark.parametrize("smoother,cycle", [("SOR", 1), ("SSOR", 1), ("SOR", 2)])
def test_mgmc_2d_fd_statistics(mode, smoother, cycle):
    """sampler/test_sampler.hh:260-323 (fast mode: 8x8, 10000 samples, tol 2e-2) with the FD prior
    (FEM / periodic kappa are out of scope).  The kappa^2 = 1 operator has O(1e-2) covariance
    entries at this resolution, scaled so the tolerance is as demanding as the reference's."""
    case = GOLD["sampler_tests"]["TestMultigridMCSampler2d_fast"]
    p = MultigridParameters(nlevel=3, smoother=smoother, coarse_solver="SSOR", ncoarsesmooth=2, cycle=cycle)
    o = O.Oracle.fd((case["nx"], case["ny"]), p, kappa_sq=1.0, mode=mode, seed=1212417)
    Q = o.csr_matrix(0).toarray()
    em, ec = _mean_cov_error(o, Q, 4 * case["nsamples"])
    scale = np.max(np.abs(np.linalg.inv(Q)))
    assert em < case["tolerance"] * scale * 2 and ec < case["tolerance"] * scale


@pytest.mark.parametrize("mode", [O.FAITHFUL, O.MULTICOLOUR])
def test_mgmc_3d_fd_statistics(mode):
    p = MultigridParameters(nlevel=2, smoother="SOR", coarse_solver="SSOR", ncoarsesmooth=2)
    o = O.Oracle.fd((8, 8, 8), p, kappa_sq=4.0, mode=mode, seed=31841287)
    Q = o.csr_matrix(0).toarray()
    em, ec = _mean_cov_error(o, Q, 20000, nwarmup=200)
    scale = np.max(np.abs(np.linalg.inv(Q)))
    # infinity norm over 343^2 covariance entries of a 20000-sample estimate: ~4 sigma of
    # sqrt(2/n) * max|Q^-1| * sqrt(IACT) ~ 0.04-0.05 relative; tolerance 0.07
    assert em < 0.05 * scale and ec < 0.07 * scale


def test_host_code_clean_under_address_sanitizer():
    """`make -C oracle asan`: the product's host-side hierarchy setup (mgmc_hierarchy.cpp) and the
    whole oracle C API (both modes, FD / FEM / CSR, low-rank sparse and dense columns, dense
    Cholesky coarse sampler) under AddressSanitizer + UBSan, no report."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"], check=True)
    r = subprocess.run([os.path.join(root, "oracle", "build", "asan_host")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "asan_host OK" in r.stdout


# ---------------------------------------------------------------- blocked banded Cholesky
@pytest.mark.parametrize("shape,nlevel", [((16, 16), 1), ((32, 32), 2), ((8, 8, 8), 1), ((12, 10), 1)])
def test_blocked_cholesky_equals_dense_products(shape, nlevel):
    """The oracle's two multicolour Cholesky sampler forms (refcpu.cpp DenseCholeskySampler): the
    dense products x = G f + U xi (up to 8,192 unknowns) and the blocked banded solves (above, or
    forced) compute the same x = L^-T (xi + L^-1 f) from the same Philox xi: equal to rounding."""
    p = MultigridParameters(nlevel=nlevel, coarse_solver="Cholesky")
    f = np.random.default_rng(5).standard_normal(int(np.prod([n - 1 for n in shape])))
    out = []
    for blocked in (False, True):
        O.set_chol_blocked(blocked)
        try:
            o = O.Oracle.fd(shape, p, kappa_sq=4.0, mode=O.MULTICOLOUR, seed=77)
        finally:
            O.set_chol_blocked(False)
        x = np.zeros_like(f)
        o.apply(f, x)
        out.append(x)
    assert np.max(np.abs(out[0] - out[1])) <= 1e-12 * np.max(np.abs(out[0]))
    assert not np.array_equal(out[0], np.zeros_like(f))


def test_blocked_cholesky_is_exact_sampler():
    """Above 8,192 unknowns (2D 128^2, one level: 16,129, the blocked mode by size) the oracle's
    Cholesky sampler is exact: 400 independent draws of the centre vertex against (Q^-1)_cc and
    (Q^-1 f)_c (5 sigma)."""
    p = MultigridParameters(nlevel=1, coarse_solver="Cholesky")
    o = O.Oracle.fd((128, 128), p, kappa_sq=25.0, mode=O.MULTICOLOUR, seed=3)
    Q = o.csr_matrix(0).tocsc()
    import scipy.sparse.linalg as spla
    n = Q.shape[0]
    c = n // 2
    f = np.random.default_rng(1).standard_normal(n)
    e = np.zeros(n)
    e[c] = 1.0
    var, mean = spla.spsolve(Q, e)[c], spla.spsolve(Q, f)[c]
    o.set_rhs(f)
    z = o.sample(400, c)
    assert abs(z.mean() - mean) < 5 * np.sqrt(var / 400)
    assert abs(z.var() - var) < 5 * var * np.sqrt(2.0 / 400)


# ---------------------------------------------------------------- class-folded residual (fold levels)
@pytest.mark.parametrize("shape,nlevel,folds", [((16, 16, 16), 3, [False, True]), ((32, 16, 16), 2, [False]),
                                                 ((64, 64, 64), 4, [False, True, True]),
                                                 ((512, 16, 24), 3, [False, False]), ((32, 32), 3, [False, False])])
def test_folded_residual_matches_reference_order_to_rounding(shape, nlevel, folds):
    """The MULTICOLOUR oracle's residual on a fold level (3D, 27-point, bitwise reflection-symmetric
    stencil: the device's fold27, mgmc_kernels.hpp) sums by coefficient class.  It equals the reference's
    CSR order (FAITHFUL, linear_operator.hh:66-76) to 1e-14 of R(|f| + |A||x|) and differs from it in
    the last bits (the fold is real); on every other level the two are bitwise equal."""
    import multigridmc_amd as mg
    p = MultigridParameters(nlevel=nlevel)
    # the device's decision (host-only mgmc_describe) is the same as the oracle's
    desc = mg.describe(mg.make_config(mg.ShiftedLaplaceFDOperator(mg.Lattice(*shape), 25.0), p))
    assert [O.fold_level(d) for d in desc[:len(folds)]] == folds
    fa = O.Oracle.fd(shape, p, 25.0, mode=O.FAITHFUL)
    mc = O.Oracle.fd(shape, p, 25.0, mode=O.MULTICOLOUR)
    rng = np.random.default_rng(5)
    for level, fold in enumerate(folds):
        n = fa.ndof(level)
        x, f = rng.standard_normal(n), rng.standard_normal(n)
        a, b = fa.residual_restrict(level, f, x), mc.residual_restrict(level, f, x)
        if fold:
            assert not np.array_equal(a, b)
            assert O.residual_tolerance_ok(b, a, fa.csr_matrix(level), f, x, lambda v: fa.restrict(level, v))
        else:
            assert np.array_equal(a, b)


# ---------------------------------------------------------------- split column (constant dense column)
@pytest.mark.parametrize("shape,split", [((24, 24, 24), True), ((128, 128), True), ((12, 12, 12), False)])
def test_split_column_patch_matches_reference_order_to_rounding(shape, split):
    """A posterior level whose one dense column is a single number (the fine level's global average,
    measured_operator.cc:31-45) adds that column's term of B t last and on its own in the MULTICOLOUR
    oracle (lr_patch_mc, the device's lr_row_patch: mgmc_lowrank.hpp), which lets the device add it
    inside the sweep / residual kernels.  The posterior residual + restriction still equals the
    reference's order (FAITHFUL) to rounding -- 1e-14 of R(|f| + |A||x| + |B| |t|) -- and the split is
    taken only above LR_BLK = 4096 unknowns (12^3 has 1331: the column stays an entry list)."""
    import multigridmc_amd as mg
    p = MultigridParameters(nlevel=2)
    lat = mg.Lattice(*shape)
    op = mg.synthetic_posterior(mg.ShiftedLaplaceFDOperator(lat, 25.0), 4, 0.0, True)
    lr = op.get_B()
    fa = O.Oracle.fd(shape, p, 25.0, mode=O.FAITHFUL)
    mc = O.Oracle.fd(shape, p, 25.0, mode=O.MULTICOLOUR)
    fa.set_lowrank(lr)
    mc.set_lowrank(lr)
    rng = np.random.default_rng(7)
    n = fa.ndof(0)
    assert (n > 4096) == split
    x, f = rng.standard_normal(n), rng.standard_normal(n)
    a, b = fa.residual_restrict(0, f, x), mc.residual_restrict(0, f, x)
    # scale of every term: |f| + |A||x| + |B| |Sigma^-1| |B^T| |x|
    import scipy.sparse as sp
    B = sp.csc_matrix((lr.vals, lr.rows, lr.colptr), shape=(n, lr.m))
    A = fa.csr_matrix(0)
    scale = np.abs(f) + abs(A) @ np.abs(x) + abs(B) @ ((abs(B).T @ np.abs(x)) / lr.sigma)
    R = lambda v: fa.restrict(0, v)
    assert np.all(np.abs(a - b) <= 1e-14 * R(scale) + 1e-300)
