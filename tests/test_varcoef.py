"""Matrix-built operators on the host (no GPU): the library's assembly of the reference's fine
operators with the constant and the periodic correlation-length model (mgmc_operator_csr) against
the CPU oracle's independent restatement, bit for bit, and against the constant-stencil hierarchy.

  * ShiftedLaplaceFDOperator   shiftedlaplace_fd_operator.cc:9-57
  * ShiftedLaplaceFEMOperator  shiftedlaplace_fem_operator.cc:9-145 (kappa^2 at the quadrature points)
  * SquaredShiftedLaplaceFDOperator  squared_shiftedlaplace_fd_operator.cc:9-96 (2D, Neumann diagonal)
  * PeriodicCorrelationLengthModel  correlationlength_model.hh:68-112
"""
import math

import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

OPS = {"fd": mg.ShiftedLaplaceFDOperator, "fem": mg.ShiftedLaplaceFEMOperator,
       "squared": mg.SquaredShiftedLaplaceFDOperator}
PDE = {"fd": 0, "fem": 1, "squared": 2}


@pytest.mark.parametrize("pde,shape", [("fd", (8, 8)), ("fd", (16, 12)), ("fd", (8, 6, 10)), ("fem", (8, 8)),
                                       ("fem", (16, 12)), ("fem", (6, 8, 10)), ("squared", (8, 8)),
                                       ("squared", (16, 12)), ("squared", (6, 4))])
@pytest.mark.parametrize("periodic", [False, True])
def test_operator_csr_matches_oracle_bitwise(pde, shape, periodic):
    lat = mg.Lattice(*shape)
    model = mg.PeriodicCorrelationLengthModel(1.2, 2.3) if periodic else mg.ConstantCorrelationLengthModel(0.2)
    op = OPS[pde](lat, model)
    rowptr, col, val = op.get_csr()
    r2, c2, v2 = O.operator_csr(shape, PDE[pde], periodic, Lambda=0.2, Lambda_min=1.2, Lambda_max=2.3)
    assert np.array_equal(rowptr, r2) and np.array_equal(col, c2)
    assert np.array_equal(val, v2)
    A = op.matrix()
    assert A.shape == (lat.Nvertex, lat.Nvertex)
    if pde != "squared" or not periodic:  # the squared operator with periodic kappa^2 is not symmetric
        assert abs(A - A.T).max() <= 1e-12 * abs(A).max()


def test_periodic_model_values():
    """correlationlength_model.hh:90-104: Lambda(x) = L1 + L2 prod cos(pi x_d), kappa^2 = 1/Lambda^2."""
    m = mg.PeriodicCorrelationLengthModel(1.2, 2.3)
    for x in [(0.0, 0.0), (0.5, 0.25), (0.3, 0.7, 0.9)]:
        lam = 0.55
        for v in x:
            lam *= math.cos(math.pi * v)
        lam += 1.75
        assert m.kappa_sq(x) == 1.0 / (lam * lam)
    assert m.kappa_sq((0.0, 0.0)) == 1.0 / (2.3 * 2.3)


@pytest.mark.parametrize("pde,shape", [("fd", (16, 16)), ("fd", (8, 8, 8)), ("fem", (16, 16)), ("fem", (8, 8, 8))])
def test_constant_model_matrix_equals_stencil_hierarchy(pde, shape):
    """With a constant kappa^2 the matrix path and the stencil path describe the same fine operator:
    every interior row of the assembled matrix equals the fine stencil bit for bit."""
    lat = mg.Lattice(*shape)
    op = OPS[pde](lat, 25.0)
    st = mg.describe(mg.make_config(op, mg.MultigridParameters(nlevel=2)))[0]["stencil"]
    A = op.matrix()
    dim = lat.dim
    r = lat.vertexidx_euclidean2linear([shape[d] // 2 for d in range(dim)])
    row = A.getrow(r)
    got = {}
    for c, v in zip(row.indices, row.data):
        idx = lat.vertexidx_linear2euclidean(int(c))
        k = sum((idx[d] - shape[d] // 2 + 1) * 3 ** d for d in range(dim))
        got[k] = v
    for k in range(3 ** dim):
        assert st[k] == got.get(k, 0.0), k


def test_squared_operator_is_2d_only():
    with pytest.raises(ValueError, match="only implemented for d=2"):
        mg.SquaredShiftedLaplaceFDOperator(mg.Lattice(8, 8, 8), 25.0)


def test_invalid_operator_descriptor_rejected():
    op = mg.ShiftedLaplaceFDOperator(mg.Lattice(8, 8), mg.PeriodicCorrelationLengthModel(0.5, 0.2))
    with pytest.raises(mg.MgmcError, match="Lambda_min"):
        op.get_csr()
