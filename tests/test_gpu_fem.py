"""GPU parity of the FEM prior (-m gpu): ShiftedLaplaceFEMOperator (shiftedlaplace_fem_operator.cc:
9-145) as the fine level.  Its 3^d-point stencil puts the fine level on the Galerkin-level kernels
(2^d colours: colour-pair / quad passes, z-marching 27-point residual + restriction, k_tail).

T2 (bitwise, np.array_equal) against the oracle's MULTICOLOUR replay: the oracle assembles the FEM
matrix cell by cell as the reference does (bitwise the device's fine stencil, test_fem.py) and forms
its own coarse levels by SpGEMM (linear_operator.cc:10-23); no device stencil is fed in.  T3: mean / covariance of the device chain
against the exact Q^-1 of the assembled matrix.
"""
import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513

CONFIGS = {
    "2d64_W": ((64, 64), dict(nlevel=4, cycle=2)),  # fine level in quad passes
    "2d256": ((256, 256), dict(nlevel=3, smoother="SSOR")),  # colour-pair passes
    "3d32_tail": ((32, 32, 32), dict(nlevel=4, ncoarsesmooth=2)),  # quads + k_tail below
    "3d128_zres": ((128, 128, 128), dict(nlevel=3, omega=1.1)),  # pairs, 27-point z-marching zres
    "3d_aniso": ((64, 32, 48), dict(nlevel=3, smoother="SSOR", coarse_scaling=0.9)),
    "3d32_chol": ((32, 32, 32), dict(nlevel=3, coarse_solver="Cholesky")),
    # j-marching half-sweeps on the 27-point fine level (256-pair rows) and level 1 (128-pair rows)
    "3d_jsweep": ((512, 24, 20), dict(nlevel=3, smoother="SSOR")),
}


def make(name, kappa_sq=25.0, chain=0):
    shape, kw = CONFIGS[name]
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFEMOperator(lat, kappa_sq), SEED, p, device=0, chain_id=chain)
    mc = O.Oracle.fem(shape, p, kappa_sq, mode=O.MULTICOLOUR, seed=SEED, chain=chain)
    return s, mc, p, lat


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fem_components_bitwise(hip_device, name):
    s, mc, p, lat = make(name)
    rng = np.random.default_rng(5)
    assert s.level_desc(0)["npoints"] == 3 ** lat.dim
    for level in range(p.nlevel):
        n = s.level_desc(level)["ndof"]
        assert n == mc.ndof(level)
        x = rng.standard_normal(n)
        b = rng.standard_normal(n)
        assert np.array_equal(s.operator_apply(level, x), mc.operator_apply(level, x)), f"level {level} apply"
        for direction in (mg.FORWARD, mg.BACKWARD):
            assert np.array_equal(s.smoother_apply(level, direction, 2, b, x),
                                  mc.smoother_apply(level, direction, 2, b, x)), f"level {level} smoother"
            assert np.array_equal(s.sor_sampler_apply(level, direction, 3 + level, 19, b, x),
                                  mc.sor_sampler_apply(level, direction, 3 + level, 19, b, x)), f"level {level} sampler"
        if level + 1 < p.nlevel:
            assert np.array_equal(s.residual_restrict(level, b, x), mc.residual_restrict(level, b, x))
    s.close()


@pytest.mark.parametrize("name", list(CONFIGS))
def test_fem_cycles_bitwise(hip_device, name):
    s, mc, p, lat = make(name)
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
    assert np.array_equal(s.sample(5, qoi), mc.sample(5, qoi))
    assert np.array_equal(s.get_state(), mc.get_state())
    s.close()


@pytest.mark.parametrize("shape,kw,nsamples,tol", [
    ((8, 8), dict(nlevel=3, ncoarsesmooth=2), 40000, 0.04),
    ((8, 8, 8), dict(nlevel=2, ncoarsesmooth=2), 20000, 0.07),
])
def test_fem_statistics_vs_exact_covariance(hip_device, shape, kw, nsamples, tol):
    """sampler/test_sampler.hh:113-153 for the FEM prior: mean and covariance of the device chain
    against Q^-1 f and Q^-1 of the assembled FEM matrix (same tolerances as the FD case)."""
    p = mg.MultigridParameters(**{"nlevel": 3, "smoother": "SOR", "coarse_solver": "SSOR", **kw})
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFEMOperator(lat, 4.0), SEED, p, device=0)
    Q = O.Oracle.fem(shape, p, 4.0).csr_matrix(0).toarray()
    mu = np.random.default_rng(1342517).random(lat.Nvertex)
    f = Q @ mu
    s.fix_rhs(f)
    s.set_state(np.zeros(lat.Nvertex))
    s.sample(1000)
    ex = np.zeros(lat.Nvertex)
    exx = np.zeros((lat.Nvertex, lat.Nvertex))
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


def test_fem_jsweep_kernel_instances(hip_device):
    """The 27-point fine level of 256-pair rows and its 128-pair level 1 run the j-marching half-sweeps."""
    s, mc, p, lat = make("3d_jsweep")
    assert s.level_kernels(0)["sweep"] == "k_jsweep_half<256>"
    assert s.level_kernels(1)["sweep"] == "k_jsweep_half<128>"
    s.close()
