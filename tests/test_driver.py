"""Driver-level host logic (CPU): the exact targets of measure_sampling_time / measure_convergence
(LinearOperator::mean and observed_mean_and_variance, linear_operator.hh:119-174) computed the
driver's way (solves with the posterior Q) equal the reference's Woodbury formulas on A."""
import numpy as np
import pytest

import multigridmc_amd as mg
from multigridmc_amd.driver import ExactTargets, _measured_values, main
from multigridmc_amd.parameters import MeasurementParameters
from tests import oracle_lib as O


class _DenseSolveStub:
    """Stands in for the device sampler: solve() with a dense Q."""

    def __init__(self, op, Q):
        self.linear_operator = op
        self.ndof = Q.shape[0]
        self.Q = Q

    def solve(self, b, method="cg", rtol=1e-12, maxiter=200):
        return np.linalg.solve(self.Q, b), 1, 0.0


@pytest.mark.parametrize("radius,glob", [(0.0, False), (0.1, True)])
def test_exact_targets_equal_reference_woodbury_formulas(radius, glob):
    lat = mg.Lattice(16, 16)
    rng = np.random.default_rng(4)
    mp = MeasurementParameters(radius=radius, variance_scaling=1e-3, measure_global=glob, variance_global=0.01,
                               mean_global=0.7)
    mp.measurement_locations = [list(rng.uniform(0.2, 0.8, 2)) for _ in range(3)]
    mp.variance = list(1.0 + rng.random(3))
    mp.mean = list(rng.uniform(1, 2, 3))
    op = mg.MeasuredOperator(mg.ShiftedLaplaceFDOperator(lat, 25.0), mp)
    A = O.Oracle.fd(lat.shape, mg.MultigridParameters(nlevel=1), 25.0).csr_matrix(0).toarray()
    B = op.get_B().dense()
    Sigma = np.diag(op.get_Sigma())
    exact = ExactTargets(_DenseSolveStub(op, A + B @ np.linalg.inv(Sigma) @ B.T))
    y = _measured_values(mp)
    rows, vals = mg.measurement_vector(lat, [0.5, 0.5], radius)
    b = np.zeros(lat.Nvertex)
    b[rows] = vals
    # linear_operator.hh:119-136 / 153-174 with xbar = 0
    Bbar = np.linalg.solve(A, B)
    x_post = Bbar @ np.linalg.solve(Sigma + B.T @ Bbar, y)
    b_bar = np.linalg.solve(A, b)
    Sinv = np.linalg.inv(Sigma + B.T @ Bbar)
    mean_ref = b_bar @ (B @ Sinv @ y)
    var_ref = b @ b_bar - b_bar @ (B @ Sinv @ B.T @ b_bar)
    assert np.allclose(exact.posterior_mean(y), x_post, rtol=1e-10, atol=1e-12)
    mean, var = exact.observed_mean_and_variance(y, rows, vals)
    assert mean == pytest.approx(mean_ref, rel=1e-10)
    assert var == pytest.approx(var_ref, rel=1e-10)


def test_driver_usage_and_loud_failure_without_gpu(tmp_path, capsys):
    assert main([]) == -1
    assert "Usage" in capsys.readouterr().out
    import shutil
    import os
    gold = os.path.join(os.path.dirname(__file__), "golden")
    for f in ("parameters_template.cfg", "measurements_template.cfg"):
        shutil.copy(os.path.join(gold, f), tmp_path / f)
    import ctypes
    n = ctypes.c_int(0)
    if ctypes.CDLL("libamdhip64.so").hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a HIP device is present (the driver run is covered by test_gpu_exact.py)")
    with pytest.raises(mg.MgmcError):  # no HIP device here: the product path fails loudly
        main([str(tmp_path / "parameters_template.cfg")])


@pytest.mark.parametrize("lmin,lmax,msg", [(0.4, 0.2, "upper bound on correlation length"),
                                           (0.0, 0.4, "lower bound on correlation length")])
def test_driver_rejects_invalid_periodic_model(tmp_path, capsys, lmin, lmax, msg):
    """parameters.cc:233-242: Lambda_max >= Lambda_min > 0, else the message and exit(-1) -- before any
    device work (no GPU needed)."""
    import os
    import re
    gold = os.path.join(os.path.dirname(__file__), "golden")
    text = open(os.path.join(gold, "parameters_template.cfg")).read()
    text = re.sub(r'correlationlengthmodel = "constant";', 'correlationlengthmodel = "periodic";', text)
    text = re.sub(r"Lambda_min = 0.2;", f"Lambda_min = {lmin};", text)
    text = re.sub(r"Lambda_max = 0.4;", f"Lambda_max = {lmax};", text)
    (tmp_path / "parameters.cfg").write_text(text)
    (tmp_path / "measurements_template.cfg").write_text(open(os.path.join(gold, "measurements_template.cfg")).read())
    assert main([str(tmp_path / "parameters.cfg")]) == -1
    assert msg in capsys.readouterr().out
