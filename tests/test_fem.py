"""ShiftedLaplaceFEMOperator (constant kappa^2) on the host side (no GPU): the device hierarchy's
fine stencil (mgmc_describe) against the oracle's restatement of the reference's cell-by-cell
assembly (shiftedlaplace_fem_operator.cc:9-145), the reference's coarsening known answer
(test_intergrid.hh:179-206: R A_h R^T = A_2h to 1e-12), the Galerkin stencils of the device
hierarchy against the oracle's SpGEMM, and the manufactured-solution check of
test_linear_operator.hh:175-210 with constant kappa^2.
"""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import multigridmc_amd as mg
from tests import oracle_lib as O

SHAPES = [(8, 8), (16, 12), (8, 8, 8), (8, 12, 6)]


def _stencil_of(A, shape):
    """Map every CSR entry (row, col) of a lattice operator to its 3^d stencil slot."""
    dim = len(shape)
    n = [s - 1 for s in shape]
    A = A.tocsr()
    rows = np.repeat(np.arange(A.shape[0]), np.diff(A.indptr))
    ri = np.unravel_index(rows, tuple(reversed(n)))
    ci = np.unravel_index(A.indices, tuple(reversed(n)))
    off = [ci[dim - 1 - q] - ri[dim - 1 - q] for q in range(dim)]  # x, y, (z)
    slot = (off[1] + 1) * 3 + (off[0] + 1)
    if dim == 3:
        slot = slot + (off[2] + 1) * 9
    return slot, A.data


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("kappa_sq", [1.0, 25.0])
def test_fem_fine_stencil_equals_reference_assembly(shape, kappa_sq):
    """Every entry of the assembled FEM matrix (cells ascending, basis pairs in cartesian-product
    order, order-1 Gauss-Legendre) equals the device's one-row stencil bit for bit, rows at the
    boundary included (truncated stencil)."""
    lat = mg.Lattice(*shape)
    p = mg.MultigridParameters(nlevel=1)
    d = mg.describe(mg.make_config(mg.ShiftedLaplaceFEMOperator(lat, kappa_sq), p))
    assert d[0]["npoints"] == 3 ** len(shape) and d[0]["ncolours"] == 2 ** len(shape)
    A = O.Oracle.fem(shape, p, kappa_sq).csr_matrix(0)
    # symmetric except in the last bits on lattices with three different extents, where
    # grad phi_a . (h^-2 grad phi_b) and its mirror round differently
    if len(set(shape)) < 3:
        assert (A != A.T).nnz == 0
    assert abs(A - A.T).max() <= 1e-15 * abs(A).max()
    slot, val = _stencil_of(A, shape)
    st = np.asarray(d[0]["stencil"])
    assert np.array_equal(val, st[slot])


@pytest.mark.parametrize("shape", [(8, 8), (8, 8, 8)])
def test_fem_coarsening_gives_coarse_fem_operator(shape):
    """test_intergrid.hh:179-206 (Lambda = 1): coarsening the FEM operator with the linear
    intergrid operator reproduces the FEM operator of the coarse lattice, ||.||_F < 1e-12."""
    p = mg.MultigridParameters(nlevel=2)
    fine = O.Oracle.fem(shape, p, 1.0)
    coarse = O.Oracle.fem(tuple(s // 2 for s in shape), mg.MultigridParameters(nlevel=1), 1.0)
    assert spla.norm(fine.csr_matrix(1) - coarse.csr_matrix(0)) < 1e-12


@pytest.mark.parametrize("shape,nlevel", [((32, 32), 4), ((16, 16, 16), 3), ((32, 16, 8), 3)])
def test_fem_device_galerkin_stencils_match_spgemm(shape, nlevel):
    """The device hierarchy's analytic (R A) R^T stencils against the oracle's SpGEMM of the
    assembled matrices, every row of every level (relative 1e-14)."""
    lat = mg.Lattice(*shape)
    p = mg.MultigridParameters(nlevel=nlevel)
    d = mg.describe(mg.make_config(mg.ShiftedLaplaceFEMOperator(lat, 25.0), p))
    o = O.Oracle.fem(shape, p, 25.0)
    cur = list(shape)
    for lev in range(nlevel):
        A = o.csr_matrix(lev)
        slot, val = _stencil_of(A, tuple(cur))
        st = np.asarray(d[lev]["stencil"])
        assert np.max(np.abs(val - st[slot])) <= 1e-14 * np.max(np.abs(st)), f"level {lev}"
        cur = [c // 2 for c in cur]


@pytest.mark.parametrize("shape,tol", [((512, 512), 2e-4), ((64, 64, 64), 7e-3)])
def test_fem_operator_manufactured_solution(shape, tol):
    """test_linear_operator.hh:175-210 with constant kappa^2 = 25: relative L2 error of A u
    against h^d (-lap u + kappa^2 u) for u = prod sin(k_d pi x_d); 2D 512^2 tol 2e-4, 3D 64^3
    tol 7e-3 (the reference's tolerances)."""
    o = O.Oracle.fem(shape, mg.MultigridParameters(nlevel=1), 25.0)
    dim = len(shape)
    h = 1.0 / shape[0]
    axes = [np.arange(1, n) / n for n in reversed(shape)]
    grids = np.meshgrid(*axes, indexing="ij")
    ks = [1.0, 2.0, 1.0][:dim]
    u = np.ones_like(grids[0])
    for d in range(dim):
        u = u * np.sin(ks[d] * np.pi * grids[dim - 1 - d])
    rhs_exact = (np.pi ** 2 * sum(k * k for k in ks) + 25.0) * u * h ** dim
    rhs = o.operator_apply(0, u.ravel())
    assert np.linalg.norm(rhs - rhs_exact.ravel()) / np.linalg.norm(rhs) < tol


def test_fem_config_field_and_invalid_operator():
    lat = mg.Lattice(16, 16, 16)
    p = mg.MultigridParameters(nlevel=3)
    cfg = mg.make_config(mg.ShiftedLaplaceFEMOperator(lat, 25.0), p)
    assert cfg.fine_operator == 1
    assert mg.make_config(mg.ShiftedLaplaceFDOperator(lat, 25.0), p).fine_operator == 0
    meas = mg.MeasuredOperator(mg.ShiftedLaplaceFEMOperator(lat, 25.0), _meas_params())
    assert mg.make_config(meas, p).fine_operator == 1
    cfg.fine_operator = 7
    with pytest.raises(mg.MgmcError):
        mg.describe(cfg)


def _meas_params():
    from multigridmc_amd.parameters import MeasurementParameters
    mp = MeasurementParameters(radius=0.0, variance_scaling=1e-3, measure_global=False, variance_global=0.02)
    mp.measurement_locations = [[0.3, 0.4, 0.5]]
    mp.variance = [1.0]
    return mp
