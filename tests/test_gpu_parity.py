"""GPU parity tests (-m gpu): the HIP path through the C-ABI against the CPU oracle.

Tiers (DESIGN.md "Parity contract"):
  T2  bitwise: every kernel (operator, restriction, prolongation, fused residual+restriction,
      deterministic and noisy multicolour sweeps, Philox normals) and whole MGMC cycles equal the
      oracle's MULTICOLOUR replay on the same (seed, chain, tag, sample) -- compared with
      np.array_equal (exact, signed zeros equal).  Component kernels are also compared with the
      FAITHFUL oracle's CSR arithmetic (reference expression order): bitwise, except the residual of
      the fold levels (3D reflection-symmetric 27-point stencils, class-folded sum), within 1e-14 of
      R(|f| + |A||x|).
  T3  statistical: the device chain's mean / covariance against the dense exact Q^-1, and the QoI
      variance against the exact (A^-1)_cc -- tolerances stated in each test.
  Size-independent properties at the benchmark sizes (256^3, 512^3): smoother fixed point,
  determinism, chain independence, finiteness.
"""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513


def make(shape, kappa_sq=25.0, chain=0, **kw):
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, kappa_sq), SEED, p, device=0, chain_id=chain)
    return s, p, lat


def oracle_for(sampler, p, lat, kappa_sq=25.0, mode=O.MULTICOLOUR, chain=0):
    """The oracle with its own Galerkin hierarchy (no device stencil fed in)."""
    return O.Oracle.fd_own(lat.shape, p, kappa_sq, mode=mode, seed=SEED, chain=chain)


CONFIGS = {
    "2d64_template_W": ((64, 64), dict(nlevel=4, cycle=2)),
    "2d_aniso_ssor": ((32, 64), dict(nlevel=3, smoother="SSOR", npresmooth=2, npostsmooth=1, ncoarsesmooth=2,
                                     omega=0.8, coarse_scaling=1.1)),
    "3d16": ((16, 16, 16), dict(nlevel=3)),
    "3d_aniso": ((32, 16, 16), dict(nlevel=2, ncoarsesmooth=3)),
    "3d64_4lvl": ((64, 64, 64), dict(nlevel=4, omega=1.2)),
    "2d16_1lvl": ((16, 16), dict(nlevel=1, ncoarsesmooth=2)),
    "3d8_1lvl": ((8, 8, 8), dict(nlevel=1)),
    "2d256_global_coarse": ((256, 256), dict(nlevel=2)),
    "3d32_W_ssor": ((32, 32, 32), dict(nlevel=3, cycle=2, smoother="SSOR")),
    # fused z-marching fine sweep (nx % 128 == 0): ping-pong buffers, prolongation fused into the
    # first post-sweep, odd sweep counts (copy back), both directions, omega != 1
    "3d128_zsweep": ((128, 128, 128), dict(nlevel=3)),
    "3d_aniso_zsweep_ssor": ((256, 128, 64), dict(nlevel=3, smoother="SSOR", npresmooth=2, npostsmooth=1,
                                                  omega=1.1, coarse_scaling=0.9)),
    "3d128_zsweep_odd": ((128, 64, 96), dict(nlevel=2, npresmooth=2, npostsmooth=1, ncoarsesmooth=2)),
    "3d192_zsweep": ((192, 48, 40), dict(nlevel=2)),  # nx multiple of 64 (32-pair tiles), not of 128
    # z-marching residual+restriction (coarse nx >= 128): 7-point fine -> level 1 and 27-point
    # level 1 -> level 2, partial tiles in y and z
    "3d_zres7": ((256, 40, 48), dict(nlevel=2)),
    "3d_zres27": ((512, 16, 24), dict(nlevel=3)),
    # coarse rows / planes ending exactly at a tile / chunk boundary, SSOR pre-sampler
    "3d_zsr_edges": ((128, 34, 18), dict(nlevel=2)),
    # n/2 - 1 = 1 (mod 64): the residual + restriction's last tile runs past the row end (columns
    # clamped onto the zero pad pair since round 3, tests/test_layout.py)
    "3d_zres_lasttile": ((132, 36, 20), dict(nlevel=2)),
    "3d_zsr_ssor_W": ((128, 64, 64), dict(nlevel=3, cycle=2, smoother="SSOR", npresmooth=2, omega=0.9)),
    # j-marching half-sweeps (k_jsweep_half) on a short level 1 of 128-pair rows, SSOR, W-cycle
    "3d_jsweep_ssor_W": ((512, 44, 60), dict(nlevel=3, cycle=2, smoother="SSOR", npresmooth=2, omega=1.1)),
    # a tail (levels 3-4) followed by a 127 x 7 x 7 quad-pass level whose post-sweep reads the Box-Muller pairs
    # the tail launch's spare workgroups drew (plan_post_noise), and a 255 x 15 x 15 j-marching level
    "3d_jsweep_tail": ((512, 32, 32), dict(nlevel=5)),
    # dense Cholesky coarse sampler (CholeskySampler, x = G f + U xi on the coarsest level)
    "2d64_chol_W": ((64, 64), dict(nlevel=4, cycle=2, coarse_solver="Cholesky")),
    "3d32_chol_ssor": ((32, 32, 32), dict(nlevel=3, smoother="SSOR", coarse_solver="Cholesky")),
    "3d128_zsweep_chol": ((128, 128, 128), dict(nlevel=5, coarse_solver="Cholesky")),
    # 2D Galerkin levels' last pre-sweep + residual + restriction in one launch (k_quads_restrict2d):
    # 255^2 (1024-thread workgroups... 128 pairs: 512) and 127^2 levels, one coarse row per workgroup
    "2d512_qrestrict": ((512, 512), dict(nlevel=4)),
    # ... backward last pre-sweep (SSOR), two pre-sweeps, W-cycle, non-square (64-pair rows)
    "2d_qr_aniso_ssor_W": ((256, 128), dict(nlevel=3, cycle=2, smoother="SSOR", npresmooth=2, omega=1.1)),
    # ... 32-pair rows: 5 coarse rows per workgroup, the last workgroup partial (23 coarse rows); the
    # level sits in k_tail unless MGMC_DISABLE=tail (variant below)
    "2d_qr_cj5": ((128, 96), dict(nlevel=3, ncoarsesmooth=2)),
}


def test_normals_bitwise(hip_device):
    s, p, lat = make((16, 16))
    for chain in (0, 7):
        s2 = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, chain_id=chain)
        for pair0, tag, sample in [(0, 0, 0), (12345, 3, 1), (2 ** 31 + 5, 17, 2 ** 33 + 9)]:
            d = s2.normals(pair0, 20000, tag, sample)
            o = O.philox_normals(SEED, chain, pair0, 20000, tag, sample)
            assert np.array_equal(d, o), f"chain {chain} pair0 {pair0}: max diff {np.max(np.abs(d - o))}"
        s2.close()
    s.close()


@pytest.mark.parametrize("name", ["2d64_template_W", "3d16", "3d_aniso", "2d_aniso_ssor", "3d_zres7", "3d_zres27",
                                  "3d_zres_lasttile", "3d128_zsweep"])
def test_component_kernels_bitwise(hip_device, name):
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    faithful = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL, seed=SEED)
    mc = oracle_for(s, p, lat)
    rng = np.random.default_rng(42)
    folds = 0
    for level in range(p.nlevel):
        n = s.level_desc(level)["ndof"]
        assert n == faithful.ndof(level)
        x = rng.standard_normal(n)
        f = rng.standard_normal(n)
        assert np.array_equal(s.operator_apply(level, x), faithful.operator_apply(level, x))
        if level + 1 < p.nlevel:
            nc = s.level_desc(level + 1)["ndof"]
            xc = rng.standard_normal(nc)
            assert np.array_equal(s.restrict(level, f), faithful.restrict(level, f))
            assert np.array_equal(s.prolongate_add(level, 1.3, xc, x), faithful.prolongate_add(level, 1.3, xc, x))
            d = s.residual_restrict(level, f, x)
            if O.fold_level(s.level_desc(level)):
                # fold levels: the class-folded sum (fold27) -- bitwise the MULTICOLOUR oracle, and the
                # reference's CSR order (linear_operator.hh:66-76) to 1e-14 of R(|f| + |A||x|)
                folds += 1
                assert np.array_equal(d, mc.residual_restrict(level, f, x))
                assert O.residual_tolerance_ok(d, faithful.residual_restrict(level, f, x), faithful.csr_matrix(level),
                                               f, x, lambda v: faithful.restrict(level, v))
            else:
                assert np.array_equal(d, faithful.residual_restrict(level, f, x))
    if name in ("3d16", "3d_aniso", "3d128_zsweep"):  # their Galerkin levels are reflection-symmetric
        assert folds == p.nlevel - 2
    s.close()


# (3d_zres27's anisotropic level 1 is not bitwise reflection-symmetric: no fold level there)
@pytest.mark.parametrize("name", ["3d16", "3d128_zsweep", "3d64_4lvl", "3d_zsr_ssor_W", "3d32_W_ssor"])
def test_fold_levels_reference_order_bitwise(hip_device, monkeypatch, name):
    """MGMC_DISABLE=fold: the residual + restriction of every 3D reflection-symmetric 27-point level
    keeps the reference's CSR summation order (A x ascending from 0.0, then f - Ax:
    linear_operator.hh:66-76, multigridmc_sampler.cc:118-120), so it equals the FAITHFUL oracle's CSR
    SpMV + restriction bit for bit on the levels where the default path sums class-folded."""
    monkeypatch.setenv("MGMC_DISABLE", "fold")
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    faithful = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL, seed=SEED)
    rng = np.random.default_rng(43)
    folds = 0
    for level in range(p.nlevel - 1):
        desc = s.level_desc(level)
        x = rng.standard_normal(desc["ndof"])
        f = rng.standard_normal(desc["ndof"])
        folds += O.fold_level(desc)
        assert np.array_equal(s.residual_restrict(level, f, x), faithful.residual_restrict(level, f, x)), level
    assert folds >= 1
    s.close()


@pytest.mark.parametrize("name", ["2d64_template_W", "3d16", "3d_aniso", "2d_aniso_ssor", "3d64_4lvl",
                                  "3d128_zsweep", "3d_aniso_zsweep_ssor"])
def test_multicolour_sweeps_bitwise(hip_device, name):
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    mc = oracle_for(s, p, lat)
    rng = np.random.default_rng(7)
    for level in range(p.nlevel):
        n = s.level_desc(level)["ndof"]
        b = rng.standard_normal(n)
        x = rng.standard_normal(n)
        for direction in (mg.FORWARD, mg.BACKWARD):
            d = s.smoother_apply(level, direction, 2, b, x)
            o = mc.smoother_apply(level, direction, 2, b, x)
            assert np.array_equal(d, o), f"level {level} dir {direction} smoother"
            d = s.sor_sampler_apply(level, direction, 5 + level, 77, b, x)
            o = mc.sor_sampler_apply(level, direction, 5 + level, 77, b, x)
            assert np.array_equal(d, o), f"level {level} dir {direction} sampler"
    s.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_mgmc_cycles_bitwise(hip_device, name):
    """Whole MGMC cycles: Sampler::apply and the device-resident QoI loop equal the oracle's
    multicolour replay exactly."""
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    mc = oracle_for(s, p, lat)
    rng = np.random.default_rng(11)
    f = rng.standard_normal(lat.Nvertex)
    x_dev = np.zeros(lat.Nvertex)
    x_orc = np.zeros(lat.Nvertex)
    for _ in range(2):
        s.apply(f, x_dev)
        mc.apply(f, x_orc)
        assert np.array_equal(x_dev, x_orc)
    # device-resident chain with QoI series (measure_sampling_time)
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    s.fix_rhs(f)
    s.set_state(x_dev)
    mc.set_rhs(f)
    mc.set_state(x_orc)
    z_dev = s.sample(6, qoi)
    z_orc = mc.sample(6, qoi)
    assert np.array_equal(z_dev, z_orc)
    assert np.array_equal(s.get_state(), mc.get_state())
    assert s.get_sample_index() == 8
    n, mean, m2 = s.qoi_moments()
    assert n == 6 and mean == pytest.approx(z_dev.mean(), rel=1e-12, abs=1e-300)
    s.close()


def test_tail_drawn_post_noise_path(hip_device, monkeypatch):
    """The quad-pass levels between a tail and the fine level read their first post-sweep's Box-Muller
    pairs from the tail launch's spare workgroups and their first pre-sweep's from the 27-point residual +
    restriction launch before it (not the j-marching level 1, not the fine level), and the cycle is
    bitwise the same with the sweeps drawing them themselves (MGMC_DISABLE=post_noise)."""
    shape, kw = CONFIGS["3d_jsweep_tail"]
    s, p, lat = make(shape, **kw)
    assert s.level_kernels(1)["sweep"].startswith("k_jsweep_half<128")
    assert s.level_kernels(2)["sweep"] == "k_sweep_quads<3>" and s.level_kernels(2).get("noise") == "restriction+tail"
    assert "noise" not in s.level_kernels(0) and "noise" not in s.level_kernels(1)
    monkeypatch.setenv("MGMC_DISABLE", "post_noise")
    s2, _, _ = make(shape, **kw)
    assert "noise" not in s2.level_kernels(2)
    f = np.random.default_rng(3).standard_normal(lat.Nvertex)
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    out = []
    for h in (s, s2):
        h.fix_rhs(f)
        out.append((h.sample(4, q), h.get_state()))
        h.close()
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


# every MGMC_DISABLE token of mgmc_capi.hip (PathFlag), alone and all together, on configurations
# where the fast path it turns off would run
ALL_PATHS = "tail,fuse_prolong,quads,rb2d,zsweep,pairs,zrestrict,lr_small,lr_merge,jsweep,qrestrict,fold,post_noise"
VARIANTS = [("fuse_prolong", "3d128_zsweep"), ("fuse_prolong", "3d_aniso_zsweep_ssor"),
            ("fuse_prolong", "3d128_zsweep_odd"), ("fuse_prolong", "3d_zres27"), ("fuse_prolong", "3d_jsweep_ssor_W"),
            ("tail", "3d16"), ("tail", "3d64_4lvl"), ("tail", "2d64_template_W"), ("tail", "3d32_W_ssor"),
            ("quads", "3d64_4lvl"), ("quads", "3d_aniso_zsweep_ssor"), ("quads", "3d_zres27"), ("quads", "2d256_global_coarse"),
            ("quads", "2d_aniso_ssor"),
            ("rb2d", "2d64_template_W"), ("rb2d", "2d_aniso_ssor"),
            ("zsweep", "3d128_zsweep"), ("zsweep", "3d_aniso_zsweep_ssor"), ("zsweep", "3d192_zsweep"),
            ("pairs", "3d64_4lvl"), ("pairs", "2d64_template_W"), ("pairs,quads", "3d32_W_ssor"),
            ("zrestrict", "3d_zres7"), ("zrestrict", "3d_zres27"), ("zrestrict", "3d128_zsweep"),
            (ALL_PATHS, "3d128_zsweep"), (ALL_PATHS, "3d_aniso_zsweep_ssor"), (ALL_PATHS, "2d64_template_W"),
            (ALL_PATHS, "2d_aniso_ssor"), (ALL_PATHS, "3d_zres27"),
            ("chol_dense", "2d64_chol_W"), ("chol_dense", "3d32_chol_ssor"), ("chol_dense", "3d128_zsweep_chol"),
            ("jsweep", "3d_zres27"), ("jsweep", "3d_jsweep_ssor_W"),
            ("qrestrict", "2d512_qrestrict"), ("qrestrict", "2d_qr_aniso_ssor_W"), ("tail", "2d_qr_cj5"),
            ("tail,qrestrict", "2d_qr_cj5"), (ALL_PATHS, "2d512_qrestrict"),
            ("prolong_z", "3d128_zsweep"), ("prolong_z", "3d_aniso_zsweep_ssor"), ("prolong_z,fuse_prolong", "3d128_zsweep"),
            ("xzero", "3d_zres27"), ("xzero", "3d_jsweep_ssor_W"), ("xzero", "3d64_4lvl"), ("xzero", "3d32_W_ssor"),
            ("fold", "3d16"), ("fold", "3d64_4lvl"), ("fold", "3d_zres27"), ("fold,tail", "3d64_4lvl"),
            ("fold,zrestrict", "3d32_W_ssor"),
            ("post_noise", "3d64_4lvl"), ("post_noise", "3d32_W_ssor"), ("post_noise", "3d_jsweep_tail"),
            ("jsweep", "3d_jsweep_tail")]


@pytest.mark.parametrize("paths,name", VARIANTS)
def test_variant_cycles_bitwise(hip_device, monkeypatch, paths, name):
    """MGMC_DISABLE=<paths> turns default fast paths off (mgmc_capi.hip PathFlag): tail = the coarsest
    levels as separate launches instead of one k_tail workgroup; fuse_prolong = the separate
    prolongate-add pass instead of the fold into the first post-sweep's plane loads; quads = one
    colour pair per launch; rb2d / zsweep = the 2D / 3D fine level in colour passes; pairs = one
    colour per pass on Galerkin levels; jsweep = colour-pair passes instead of the j-marching half-sweeps
    on 3D Galerkin levels of 64 / 128 pairs per row; zrestrict = the per-point residual + restriction;
    qrestrict = a 2D Galerkin level's last pre-sweep and its residual + restriction as two launches
    instead of one k_quads_restrict2d; prolong_z = the per-point prolongation instead of the z-marching
    one on 3D levels; xzero = the restriction zeroes x_{l+1} and the coarse level's first (j-marching)
    pre-sweep loads it, instead of taking it as zeros; fold = the residuals of reflection-symmetric
    27-point levels in the reference's CSR order instead of fold27's;
    chol_dense = the coarse Cholesky's blocked banded solves on a small coarsest level (the oracle's
    blocked mode); post_noise = every sweep draws its own Box-Muller pairs instead of reading those a
    restriction launch or a tail launch's spare workgroups drew.  Every combination gives the oracle's cycle
    exactly."""
    monkeypatch.setenv("MGMC_DISABLE", paths)
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    O.set_chol_blocked("chol_dense" in paths.split(","))
    O.set_no_fold("fold" in paths.split(","))
    try:
        mc = oracle_for(s, p, lat)
    finally:
        O.set_chol_blocked(False)
        O.set_no_fold(False)
    f = np.random.default_rng(7).standard_normal(lat.Nvertex)
    x_dev, x_orc = np.zeros(lat.Nvertex), np.zeros(lat.Nvertex)
    for _ in range(2):
        s.apply(f, x_dev)
        mc.apply(f, x_orc)
    assert np.array_equal(x_dev, x_orc)
    s.close()


@pytest.mark.parametrize("name,qoi", [("3d128_zsweep", True), ("2d64_template_W", False), ("3d16", True)])
def test_nonfinite_state_fails_loudly(hip_device, name, qoi):
    """A NaN injected into the state (away from the watched vertex) reaches the QoI vertex / lattice
    centre within a few cycles: mgmc_sample returns MGMC_E_NONFINITE with the sample index instead of
    a chain that silently carries NaN; mgmc_set_state clears the guard."""
    from multigridmc_amd import _native
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim) if qoi else -1
    s.sample(3, q)  # finite chain: no error
    x = s.get_state()
    x[1] = np.nan
    s.set_state(x)
    with pytest.raises(mg.MgmcError, match="non-finite chain state") as e:
        s.sample(40, q)
    assert e.value.code == _native.MGMC_E_NONFINITE
    with pytest.raises(mg.MgmcError):  # sticky until a new state
        s.synchronize()
    s.set_state(np.zeros(lat.Nvertex))
    s.sample(2, q)
    f = np.zeros(lat.Nvertex)
    f[lat.Nvertex // 2] = np.inf
    with pytest.raises(mg.MgmcError, match="non-finite"):
        s.apply(f, np.zeros(lat.Nvertex))
    s.close()


@pytest.mark.parametrize("name,level,sweep", [("2d64_template_W", 0, "k_rb2d"), ("3d128_zsweep", 0, "k_zsweep_rb7<"),
                                              ("3d16", 0, "k_sweep_rb<3>"), ("3d_jsweep_ssor_W", 1, "k_jsweep_half<128>"),
                                              ("3d_zres27", 1, "k_jsweep_half<128>"), ("3d128_zsweep", 1, "k_sweep_quads<3>"),
                                              ("3d_aniso_zsweep_ssor", 1, "k_sweep_quads<3>"),
                                              ("3d64_4lvl", 1, "k_sweep_quads<3>")])
def test_level_kernels_labels(hip_device, name, level, sweep):
    """mgmc_level_kernels names the sweep each level really runs (bench.py's roofline labels)."""
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    assert s.level_kernels(level)["sweep"].startswith(sweep)
    s.close()


@pytest.mark.parametrize("name,levels", [("2d512_qrestrict", (1, 2)), ("2d_qr_aniso_ssor_W", (1,))])
def test_qrestrict_labels(hip_device, name, levels):
    """2D Galerkin levels outside k_tail run their last pre-sweep and residual + restriction as one
    k_quads_restrict2d launch (mgmc_qrestrict.hpp); MGMC_DISABLE=qrestrict is covered above."""
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    for level in levels:
        k = s.level_kernels(level)
        assert k["residual_restrict"] == "k_quads_restrict2d" and "post_sweep" not in k
    assert s.level_kernels(0) == {"sweep": "k_rb2d", "residual_restrict": "k_residual_restrict<2,5>"}
    s.close()


def test_unknown_disable_token_rejected(hip_device, monkeypatch):
    monkeypatch.setenv("MGMC_DISABLE", "tail,no_such_path")
    with pytest.raises(mg.MgmcError, match="no_such_path"):
        make((16, 16, 16))


def test_mgmc_seed_chain_independence(hip_device):
    a, p, lat = make((32, 32, 32))
    b, _, _ = make((32, 32, 32))
    c, _, _ = make((32, 32, 32), chain=1)
    q = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    za, zb, zc = a.sample(50, q), b.sample(50, q), c.sample(50, q)
    assert np.array_equal(za, zb)
    assert not np.array_equal(za, zc)
    assert abs(np.corrcoef(za, zc)[0, 1]) < 0.5
    for s in (a, b, c):
        s.close()


def _mean_cov(s, f, nsamples, nwarmup=200):
    n = s.ndof
    s.fix_rhs(f)
    s.set_state(np.zeros(n))
    s.sample(nwarmup)
    ex = np.zeros(n)
    exx = np.zeros((n, n))
    for k in range(nsamples):
        s.sample(1)
        x = s.get_state()
        ex += (x - ex) / (k + 1)
        exx += (np.outer(x, x) - exx) / (k + 1)
    return ex, exx - np.outer(ex, ex)


@pytest.mark.parametrize("shape,kw,nsamples,tol", [
    ((8, 8), dict(nlevel=3, ncoarsesmooth=2), 40000, 0.04),
    ((8, 8), dict(nlevel=3, smoother="SSOR", cycle=2), 40000, 0.04),
    ((8, 8), dict(nlevel=3, smoother="SSOR", coarse_solver="Cholesky"), 40000, 0.04),
    ((8, 8, 8), dict(nlevel=2, ncoarsesmooth=2), 20000, 0.07),
])
def test_mgmc_statistics_vs_exact_covariance(hip_device, shape, kw, nsamples, tol):
    """sampler/test_sampler.hh:113-153 on the device chain: sample mean and covariance against the
    exact Q^-1 f and Q^-1 (infinity norm), relative to max|Q^-1|.  tol ~ 5 sigma of the max over
    all entries: sqrt(2 IACT / n) per entry (IACT ~ 1.5); the CPU oracle in either mode shows
    0.013-0.022 (2D, n = 40000) and 0.03 (3D, n = 20000) on the same cases."""
    s, p, lat = make(shape, kappa_sq=4.0, **kw)
    orc = O.Oracle.fd(lat.shape, p, 4.0, mode=O.FAITHFUL)
    Q = orc.csr_matrix(0).toarray()
    mu = np.random.default_rng(1342517).random(lat.Nvertex)
    ex, cov = _mean_cov(s, Q @ mu, nsamples)
    Qinv = np.linalg.inv(Q)
    scale = np.max(np.abs(Qinv))
    assert np.max(np.abs(ex - mu)) < 2 * tol * scale
    assert np.max(np.abs(cov - Qinv)) < tol * scale
    s.close()


def _iact(z):
    z = z - z.mean()
    var = z.var()
    tau = 1.0
    for t in range(1, len(z) // 10):
        rho = np.dot(z[:-t], z[t:]) / ((len(z) - t) * var)
        if rho < 0.05:
            break
        tau += 2 * rho
    return tau


@pytest.mark.parametrize("shape,nlevel,nsamples", [((64, 64), 4, 20000), ((32, 32, 32), 4, 10000)])
def test_qoi_variance_vs_exact(hip_device, shape, nlevel, nsamples):
    """driver_mgmc.cc:86-104: prior (f = 0): E[z] = 0, Var[z] = (A^-1)_cc.  Tolerance: 5 sigma of the
    Monte Carlo error with the integrated autocorrelation time (Var of a variance estimate ~ 2 var^2)."""
    s, p, lat = make(shape, nlevel=nlevel)
    orc = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL)
    A = orc.csr_matrix(0).tocsc()
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    e = np.zeros(lat.Nvertex)
    e[q] = 1.0
    var_exact = spla.spsolve(A, e)[q]
    s.sample(100, q)
    z = s.sample(nsamples, q)
    tau = _iact(z)
    n_eff = nsamples / tau
    assert abs(z.mean()) < 5 * np.sqrt(var_exact / n_eff)
    assert abs(z.var() - var_exact) < 5 * var_exact * np.sqrt(2.0 / n_eff)
    n, mean, m2 = s.qoi_moments()
    assert n == nsamples + 100
    s.close()


@pytest.mark.parametrize("n", [256, 512])
def test_fine_smoother_fixed_point_at_scale(hip_device, n):
    """smoother/test_smoother.hh:90-101 at the benchmark sizes: a forward+backward deterministic
    sweep leaves the exact solution of A x = b invariant (relative 1e-12)."""
    s, p, lat = make((n, n, n), nlevel=2)
    x_exact = np.random.default_rng(1).standard_normal(lat.Nvertex)
    b = s.operator_apply(0, x_exact)
    x = s.smoother_apply(0, mg.FORWARD, 1, b, x_exact)
    x = s.smoother_apply(0, mg.BACKWARD, 1, b, x)
    assert np.linalg.norm(x - x_exact) / np.linalg.norm(x_exact) < 1e-12
    s.close()


def test_benchmark_hierarchy_cycles_finite_and_deterministic(hip_device):
    """3D 512^3 7-level V-cycle (BASELINE config 4, one chain): cycles stay finite, the state moves,
    and a second handle with the same (seed, chain) reproduces the QoI series bit for bit."""
    shape = (512, 512, 512)
    q = mg.measurement_vector_index(mg.Lattice(*shape), [0.5, 0.5, 0.5])
    a, p, lat = make(shape, nlevel=7)
    za = a.sample(4, q)
    assert np.all(np.isfinite(za)) and np.all(za != 0)
    x = a.get_state()
    assert np.all(np.isfinite(x)) and np.std(x) > 0
    a.close()
    b, _, _ = make(shape, nlevel=7)
    zb = b.sample(4, q)
    assert np.array_equal(za, zb)
    b.close()


def test_invalid_level_and_sizes_raise(hip_device):
    s, p, lat = make((16, 16))
    with pytest.raises(mg.MgmcError):
        s.operator_apply(5, np.zeros(10))
    with pytest.raises(ValueError):
        s.apply(np.zeros(3), np.zeros(3))
    with pytest.raises(mg.MgmcError):
        s.sample(3, lat.Nvertex + 5)
    s.close()
    with pytest.raises(mg.MgmcError, match="bandwidth"):  # coarse Cholesky: rows of at most 4096 above 8192 dofs
        make((8192, 8), nlevel=1, coarse_solver="Cholesky")


def test_cpp_host_side_sample_matches_python_path(hip_device, tmp_path):
    """The C++ host side (include/mgmc_sampler.hh, g++-built client) and the Python host side drive the
    same C-ABI: the 3D 16^3 QoI series at vertex (8,8,8) agree bit for bit."""
    import subprocess
    from tests.cpp_client import build_client
    exe = build_client(tmp_path)
    r = subprocess.run([exe, "sample", "6"], capture_output=True, text=True, check=True)
    zc = np.array([float(v) for v in r.stdout.split()])
    s, p, lat = make((16, 16, 16), nlevel=3)
    zp = s.sample(6, 7 * 15 * 15 + 7 * 15 + 7)
    s.close()
    assert np.array_equal(zc, zp)


@pytest.mark.parametrize("shape,nlevel,batch", [((64, 64), 4, 3), ((32, 32, 32), 3, 4)])
def test_convergence_chains_batched_equal_sequential(hip_device, shape, nlevel, batch):
    """measure_convergence's chains (driver_mgmc.cc:236-254) run `batch` at a time on cloned handles
    with the sequential loop's sample indices: the same QoI series bit for bit."""
    from multigridmc_amd.driver import convergence_series
    lat = mg.Lattice(*shape)
    op = mg.ShiftedLaplaceFDOperator(lat, 25.0)
    p = mg.MultigridParameters(nlevel=nlevel)
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    f = np.random.default_rng(3).standard_normal(lat.Nvertex)
    a = mg.MultigridMCSampler(op, SEED, p)
    b = mg.MultigridMCSampler(op, SEED, p)
    a.fix_rhs(f)
    b.fix_rhs(f)
    za = convergence_series(a, 7, 5, [q], [1.0], batch=1)
    zb = convergence_series(b, 7, 5, [q], [1.0], batch=batch)
    assert np.all(np.isfinite(za)) and np.array_equal(za, zb)
    assert a.get_sample_index() == b.get_sample_index() == 35
    a.close()
    b.close()


@pytest.mark.parametrize("name,unroll", [("2d64_template_W", None), ("3d32_W_ssor", "3"), ("3d16", "1")])
def test_unrolled_sample_loop_bitwise(hip_device, monkeypatch, name, unroll):
    """The sample loop replays `unroll` cycles per graph launch (8 on small lattices by default,
    MGMC_GRAPH_UNROLL): 19 cycles = whole unrolled launches + single-cycle launches, QoI series and
    state equal to the oracle's sequential cycles."""
    if unroll is not None:
        monkeypatch.setenv("MGMC_GRAPH_UNROLL", unroll)
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    mc = oracle_for(s, p, lat)
    f = np.random.default_rng(3).standard_normal(lat.Nvertex)
    qoi = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    s.fix_rhs(f)
    s.set_state(np.zeros(lat.Nvertex))
    mc.set_rhs(f)
    mc.set_state(np.zeros(lat.Nvertex))
    for nsteps in (19, 8, 5):
        assert np.array_equal(s.sample(nsteps, qoi), mc.sample(nsteps, qoi))
    assert np.array_equal(s.get_state(), mc.get_state())
    assert s.get_sample_index() == 32
    s.close()


@pytest.mark.parametrize("name,nsteps,stride,ntimed", [("3d128_zsweep", 4, 1, 4), ("2d64_template_W", 4, 1, 4),
                                                       ("3d128_zsweep", 7, 3, 3), ("2d64_template_W", 6, 4, 3)])
def test_sample_timed_segments(hip_device, name, nsteps, stride, ntimed):
    """mgmc_sample_timed_stride (the bench's timing path): one fine pre-sweep and one fine post-sweep
    per timed cycle in their own event segments (the post segment ends before the QoI record; every
    stride-th cycle and the last are timed, the others replay the plain graph), positive segment
    times inside the total, and the same chain as the plain sample loop bit for bit."""
    shape, kw = CONFIGS[name]
    s, p, lat = make(shape, **kw)
    t = make(shape, **kw)[0]
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    r = s.sample_timed(nsteps, q, stride=stride)
    assert r["npre"] == ntimed * (2 if p.smoother == "SSOR" else 1) and r["npost"] == r["npre"]
    assert 0 < r["pre_ms"] and 0 < r["post_ms"] and r["pre_ms"] + r["post_ms"] < r["total_ms"]
    z = s.get_series(nsteps)
    assert np.array_equal(z, t.sample(nsteps, q))
    assert np.array_equal(s.get_state(), t.get_state())
    s.close()
    t.close()


def test_poison_switch_fills_unwritten_memory_and_leaves_results_alone(hip_device, monkeypatch):
    """MGMC_POISON=1: the QoI series buffer starts as NaN bytes -- entries past
    the recorded samples read NaN (positive control of the allocation poison) -- while the recorded
    series and the state, with NaN-filled LDS before every op of the cycle graph, equal an unpoisoned
    handle's bit for bit (no kernel of the cycle reads memory it did not write)."""
    lat = mg.Lattice(32, 32, 32)
    q = mg.measurement_vector_index(lat, [0.5] * 3)
    p = mg.MultigridParameters(nlevel=4)
    ref = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 7, p, device=0)
    z_ref = ref.sample(5, q)
    x_ref = ref.get_state()
    ref.close()
    monkeypatch.setenv("MGMC_POISON", "1")
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 7, p, device=0)
    z = s.sample(5, q)
    tail = s.get_series(12)[5:]
    assert np.array_equal(z, z_ref) and np.array_equal(s.get_state(), x_ref)
    assert np.all(np.isnan(tail))
    s.close()
