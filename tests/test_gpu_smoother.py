"""The Smoother drop-in on the GPU (-m gpu; SURVEY.md section 8(b) row "Smoother API").

* include/reference_adapter/hip_sor_smoother.hh -- HipSORSmoother / HipSSORSmoother : public Smoother,
  obtained through their SmootherFactory (multigrid_preconditioner.cc:18-33) on LinearOperators whose
  get_sparse() is the reference operator's matrix (FD / FEM stencil path, periodic-FD matrix path), with
  and without a MeasuredOperator-like low-rank part: Smoother::apply(b, x) equals the CPU oracle's
  MULTICOLOUR restatement of SORSmoother::apply (sor_smoother.cc:41-78, nsmooth x (nsmooth sweeps, then
  the B_bar fix)) and SSORSmoother::apply (ssor_smoother.cc:9-15) bit for bit, for nsmooth 1 and 2.
* The reference's own smoother tests (smoother/test_smoother.hh:90-114): the smoother leaves the
  exact solution of Q x = b invariant (relative 1e-12), in the fixture's configuration -- 32 x 32 FEM
  with the periodic correlation length Lambda in [1.2, 2.3], omega 0.8, and 10 measurements of radius
  0.05 with Sigma = 1e-6 (1 + 2 u) for the low-rank case (locations drawn with numpy here).
"""
import subprocess
import types

import numpy as np
import pytest

import multigridmc_amd as mg
from multigridmc_amd.measured import MeasurementParameters
from tests import oracle_lib as O
from tests.test_adapter import build_adapter_client

pytestmark = pytest.mark.gpu

SHAPES = {"fd": (16, 16, 16), "fem": (16, 16, 16), "periodic": (32, 32)}


def _oracle(kind, lowrank):
    shape = SHAPES[kind]
    p = mg.MultigridParameters(nlevel=1, smoother="SOR", coarse_solver="SSOR", omega=1.0)
    if kind == "fd":
        orc = O.Oracle.fd(shape, p, 25.0, mode=O.MULTICOLOUR)
    elif kind == "fem":
        orc = O.Oracle.fem(shape, p, 25.0, mode=O.MULTICOLOUR)
    else:
        rowptr, col, val = O.operator_csr(shape, 0, periodic=True, Lambda_min=0.2, Lambda_max=0.4)
        orc = O.Oracle.csr(shape, p, rowptr, col, val, mode=O.MULTICOLOUR)
    n = int(np.prod([v - 1 for v in shape]))
    if lowrank:  # the client's two point measurements (adapter_client.cpp AssembledOperator)
        lr = types.SimpleNamespace(m=2, n=n, colptr=np.array([0, 1, 2], dtype=np.int64),
                                   rows=np.array([n // 3, 2 * n // 3], dtype=np.int64), vals=np.array([1.0, 1.0]),
                                   sigma=np.array([1e-3, 2e-3]))
        orc.set_lowrank(lr)
    return orc, n


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    return build_adapter_client(str(tmp_path_factory.mktemp("smoother_client")))


@pytest.mark.parametrize("lowrank", [False, True], ids=["prior", "lowrank"])
@pytest.mark.parametrize("kind", list(SHAPES))
@pytest.mark.parametrize("variant", [("sor", 1, "fwd"), ("sor", 2, "bwd"), ("sor", 2, "fwd"), ("ssor", 1, None),
                                     ("ssor", 2, None)], ids=lambda v: "-".join(str(t) for t in v if t))
def test_adapter_smoother_matches_oracle(hip_device, client, kind, variant, lowrank):
    smoother, nsmooth, d = variant
    args = [client, "smoother", kind, smoother, str(nsmooth), d or "fwd"] + (["lowrank"] if lowrank else [])
    r = subprocess.run(args, capture_output=True, text=True, check=True)
    vals = np.array([float(v) for v in r.stdout.split()])
    orc, n = _oracle(kind, lowrank)
    assert vals.size == 3 * n
    b, x0, x1 = vals[:n], vals[n:2 * n], vals[2 * n:]
    if smoother == "sor":
        ref = orc.sor_smoother_apply(0, mg.FORWARD if d == "fwd" else mg.BACKWARD, nsmooth, b, x0)
    else:
        ref = orc.ssor_smoother_apply(0, nsmooth, b, x0)
    assert np.all(np.isfinite(x1)) and not np.array_equal(x1, x0)
    assert np.array_equal(x1, ref)


def test_sor_smoother_nesting_is_nsmooth_squared_sweeps(hip_device):
    """Without a low-rank part the reference's nesting is nsmooth^2 plain sweeps
    (sor_smoother.cc:43-45 over :64): SORSmoother(nsmooth = 2) = 4 single sweeps, bit for bit."""
    lat = mg.Lattice(24, 16, 20)
    op = mg.ShiftedLaplaceFDOperator(lat, 25.0)
    rng = np.random.default_rng(5)
    b = rng.standard_normal(lat.Nvertex)
    x = rng.standard_normal(lat.Nvertex)
    sm = mg.SORSmoother(op, 1.0, 2, mg.BACKWARD)
    y = x.copy()
    sm.apply(b, y)
    z = sm._s.smoother_apply(0, mg.BACKWARD, 4, b, x)
    sm.close()
    assert np.array_equal(y, z)


def _fixture_operator(lowrank, seed=1212417):
    """smoother/test_smoother.hh:18-66: 32 x 32 FEM, periodic Lambda in [1.2, 2.3]; the MeasuredOperator
    with 10 measurements of radius 0.05 and Sigma = 1e-6 (1 + 2 u)."""
    lat = mg.Lattice(32, 32)
    prior = mg.ShiftedLaplaceFEMOperator(lat, mg.PeriodicCorrelationLengthModel(1.2, 2.3))
    if not lowrank:
        return prior, lat
    rng = np.random.default_rng(seed)
    mp = MeasurementParameters(radius=0.05, variance_scaling=1.0, measure_global=False, variance_global=0.0)
    mp.measurement_locations = [list(rng.uniform(0.0, 1.0, 2)) for _ in range(10)]
    mp.variance = list(1e-6 * (1.0 + 2.0 * rng.random(10)))
    return mg.MeasuredOperator(prior, mp), lat


@pytest.mark.parametrize("lowrank", [False, True], ids=["TestSSORSmoother", "TestSSORLowRankSmoother"])
@pytest.mark.parametrize("which", ["ssor", "sor_fwd", "sor_bwd"])
def test_smoother_leaves_exact_solution_invariant(hip_device, lowrank, which):
    """smoother/test_smoother.hh:90-114 (SSOR; here also forward / backward SOR): x = x_exact,
    b = Q x_exact, apply(b, x) with omega 0.8 changes x by less than 1e-12 relative."""
    op, lat = _fixture_operator(lowrank)
    x_exact = np.random.default_rng(1212417).standard_normal(lat.Nvertex)
    A = (op.base_operator if lowrank else op).matrix()
    b = A @ x_exact
    if lowrank:
        lr = op.get_B()
        B = np.zeros((lat.Nvertex, lr.m))
        for k in range(lr.m):
            B[lr.rows[lr.colptr[k]:lr.colptr[k + 1]], k] = lr.vals[lr.colptr[k]:lr.colptr[k + 1]]
        b = b + B @ ((B.T @ x_exact) / lr.sigma)
    if which == "ssor":
        sm = mg.SSORSmootherFactory(0.8, 1).get(op)
    else:
        sm = mg.SORSmootherFactory(0.8, 1, mg.FORWARD if which == "sor_fwd" else mg.BACKWARD).get(op)
    x = x_exact.copy()
    sm.apply(b, x)
    sm.close()
    assert np.linalg.norm(x - x_exact) / np.linalg.norm(x_exact) < 1e-12
