"""Exact-statistics engine (-m gpu): multigrid-preconditioned solvers on the device (mgmc_solve)
and T3 parity of the sampler against exact targets at sizes where the reference's sparse Cholesky
(LinearOperator::mean / observed_mean_and_variance, linear_operator.hh:119-174) is infeasible.

  * solver/test_solver.hh:111-171: b = Q x_exact on a 256^2 lattice, nlevel 5, SSOR smoother,
    LoopSolver with rtol 1e-13 / atol 1e-12 (1e-11 low-rank), error < 1e-10 -- here with the FD
    prior and with a posterior (ball measurements) operator;
  * CG with the same cycle against scipy's sparse direct solve (oracle CSR + B Sigma^-1 B^T);
  * the QoI mean / variance of the device chain at 256^3 (prior) and 128^3 (posterior) against
    e^T Q^-1 e and e^T Q^-1 f from the solver, within 5 sigma of the Monte Carlo error (IACT).
"""
import numpy as np
import pytest
import scipy.sparse.linalg as spla

import multigridmc_amd as mg
from multigridmc_amd.parameters import MeasurementParameters
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513


def _posterior(lat, kappa_sq, radius, nmeas, scale, glob=False, seed=7):
    rng = np.random.default_rng(seed)
    mp = MeasurementParameters(radius=radius, variance_scaling=scale, measure_global=glob, variance_global=0.01)
    mp.measurement_locations = [list(rng.uniform(0.2, 0.8, lat.dim)) for _ in range(nmeas)]
    mp.variance = list(1.0 + 2.0 * rng.random(nmeas))
    return mg.MeasuredOperator(mg.ShiftedLaplaceFDOperator(lat, kappa_sq), mp)


@pytest.mark.parametrize("lowrank", [False, True])
def test_loop_solver_reference_case(hip_device, lowrank):
    """solver/test_solver.hh:111-171 (TestMultigrid / TestMultigridLowRank) with the FD operator."""
    lat = mg.Lattice(256, 256)
    op = _posterior(lat, 25.0, 0.05, 10, 1e-6) if lowrank else mg.ShiftedLaplaceFDOperator(lat, 25.0)
    p = mg.MultigridParameters(nlevel=5, smoother="SSOR", coarse_solver="SSOR", omega=1.0, cycle=1)
    s = mg.MultigridMCSampler(op, SEED, p)
    x_exact = np.random.default_rng(1212417).standard_normal(lat.Nvertex)
    b = s.operator_apply(0, x_exact)
    x, it, rn = s.solve(b, method="loop", rtol=1e-13, atol=1e-11 if lowrank else 1e-12, maxiter=100)
    assert it < 100, f"loop solver did not converge: ||r|| = {rn}"
    assert np.linalg.norm(x - x_exact) / np.linalg.norm(x_exact) < 1e-10
    s.close()


@pytest.mark.parametrize("shape,nlevel,lowrank", [((64, 64), 4, False), ((64, 64), 4, True),
                                                  ((32, 32, 32), 3, False), ((32, 32, 32), 3, True)])
def test_cg_matches_sparse_direct(hip_device, shape, nlevel, lowrank):
    lat = mg.Lattice(*shape)
    op = _posterior(lat, 25.0, 0.1, 4, 1e-3, glob=True) if lowrank else mg.ShiftedLaplaceFDOperator(lat, 25.0)
    p = mg.MultigridParameters(nlevel=nlevel)
    s = mg.MultigridMCSampler(op, SEED, p)
    orc = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL)
    Q = orc.csr_matrix(0)
    if lowrank:
        Q = (Q.toarray() + op.get_B().precision_update())
    b = np.random.default_rng(3).standard_normal(lat.Nvertex)
    x_ref = np.linalg.solve(Q, b) if lowrank else spla.spsolve(Q.tocsc(), b)
    x, it, rn = s.solve(b, method="cg", rtol=1e-13, maxiter=200)
    assert it < 200
    assert np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref) < 1e-10
    # the loop solver reaches the same solution
    x2, it2, _ = s.solve(b, method="loop", rtol=1e-12, maxiter=400)
    assert np.linalg.norm(x2 - x_ref) / np.linalg.norm(x_ref) < 1e-9
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


def _check_moments(z, mean_exact, var_exact):
    n_eff = len(z) / _iact(z)
    print(f"T3: n={len(z)} n_eff={n_eff:.0f} mean={z.mean():.6g} (exact {mean_exact:.6g}) "
          f"var={z.var():.6g} (exact {var_exact:.6g})")
    assert abs(z.mean() - mean_exact) < 5 * np.sqrt(var_exact / n_eff), (z.mean(), mean_exact)
    assert abs(z.var() - var_exact) < 5 * var_exact * np.sqrt(2.0 / n_eff), (z.var(), var_exact)


def test_prior_qoi_variance_at_256_cubed(hip_device):
    """a13 prior target at BASELINE config 3's size: Var z = (A^-1)_cc at the centre vertex of the
    3D 256^3 lattice (6 levels), from the device CG; the chain's QoI variance within 5 sigma."""
    lat = mg.Lattice(256, 256, 256)
    p = mg.MultigridParameters(nlevel=6)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p)
    q = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    e = np.zeros(lat.Nvertex)
    e[q] = 1.0
    x, it, rn = s.solve(e, method="cg", rtol=1e-10, maxiter=100)
    assert it < 100
    var_exact = x[q]
    s.sample(100, q)
    z = s.sample(20000, q)
    _check_moments(z, 0.0, var_exact)
    s.close()


def test_prior_qoi_variance_at_headline_512_cubed(hip_device):
    """T3 at the bench's own configuration (BASELINE config 4: 3D 512^3, 7 levels, V-cycle, SOR,
    SSOR coarse, f = 0) and QoI vertex (the centre, index 66,716,415), as measure_sampling_time does
    on the timed chain (driver_mgmc.cc:86-104): Var z = (A^-1)_cc from the device MG-CG (a13,
    linear_operator.hh:153-174 with m = 0), mean 0; 200 warm-up + 20,000 samples within 5 sigma
    (IACT)."""
    lat = mg.Lattice(512, 512, 512)
    p = mg.MultigridParameters(nlevel=7)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p)
    q = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    assert q == 66716415
    e = np.zeros(lat.Nvertex)
    e[q] = 1.0
    g, it, rn = s.solve(e, method="cg", rtol=1e-10, maxiter=100)
    assert it < 100
    var_exact = g[q]
    del g, e
    s.sample(200, q)
    z = s.sample(20000, q)
    assert np.all(np.isfinite(z))
    _check_moments(z, 0.0, var_exact)
    s.close()


def test_posterior_qoi_mean_and_variance_at_128_cubed(hip_device):
    """a13 posterior targets (observed_mean_and_variance): 8 point measurements, f = B Sigma^-1 y,
    mean z = e^T Q^-1 f and Var z = e^T Q^-1 e at a vertex next to a measurement, from the device
    CG on the posterior operator; the chain's QoI moments within 5 sigma."""
    lat = mg.Lattice(128, 128, 128)
    op = _posterior(lat, 25.0, 0.0, 8, 1e-4)
    p = mg.MultigridParameters(nlevel=5)
    s = mg.MultigridMCSampler(op, SEED, p)
    lr = op.get_B()
    y = np.random.default_rng(5).uniform(1.0, 3.0, lr.m)
    f = lr.dense() @ (y / lr.sigma)
    q = int(lr.rows[lr.colptr[0]])  # the first measured vertex
    e = np.zeros(lat.Nvertex)
    e[q] = 1.0
    mean_field, it1, _ = s.solve(f, method="cg", rtol=1e-11, maxiter=200)
    g, it2, _ = s.solve(e, method="cg", rtol=1e-11, maxiter=200)
    assert it1 < 200 and it2 < 200
    s.fix_rhs(f)
    s.set_state(mean_field)
    s.sample(200, q)
    z = s.sample(20000, q)
    _check_moments(z, mean_field[q], g[q])
    s.close()


@pytest.mark.parametrize("pde,model", [("shiftedlaplace_fd", "constant"), ("shiftedlaplace_fem", "constant"),
                                       ("shiftedlaplace_fd", "periodic"), ("shiftedlaplace_fem", "periodic"),
                                       ("squared_shiftedlaplace_fd", "constant"),
                                       ("squared_shiftedlaplace_fd", "periodic")])
def test_driver_posterior_template_run(hip_device, tmp_path, monkeypatch, pde, model):
    """multigridmc_amd.driver on the reference's parameters_template.cfg / measurements_template.cfg
    (config 1: 2D posterior, 8 measurements, W-cycle), lattice 64^2 and shortened sampling, for every
    prior and correlation length model of driver_mgmc.cc:398-429: the timeseries and convergence files
    are written in the reference's formats, and the sample mean and variance of z agree with the exact
    observed statistics within 5 sigma (IACT)."""
    import os
    import re
    from multigridmc_amd.driver import main
    gold = os.path.join(os.path.dirname(__file__), "golden")
    text = open(os.path.join(gold, "parameters_template.cfg")).read()
    text = re.sub(r"nx = 32;", "nx = 64;", text)
    text = re.sub(r"ny = 32;", "ny = 64;", text)
    text = re.sub(r"nsamples = 10000;", "nsamples = 20000;", text)
    text = re.sub(r"nsamples = 1000;", "nsamples = 200;", text)
    text = re.sub(r'pdemodel = "shiftedlaplace_fd";', f'pdemodel = "{pde}";', text)
    text = re.sub(r'correlationlengthmodel = "constant";', f'correlationlengthmodel = "{model}";', text)
    assert f'pdemodel = "{pde}";' in text and f'correlationlengthmodel = "{model}";' in text
    (tmp_path / "parameters.cfg").write_text(text)
    (tmp_path / "measurements_template.cfg").write_text(open(os.path.join(gold, "measurements_template.cfg")).read())
    monkeypatch.chdir(tmp_path)
    assert main([str(tmp_path / "parameters.cfg")]) == 0
    z = np.loadtxt(tmp_path / "timeseries_multigridmc.txt")
    assert z.shape == (20000,)
    conv = (tmp_path / "convergence_multigridmc.txt").read_text()
    assert "**** q_k = |E[z^k] - E[z]| ****" in conv and "**** q_k = |Var[z^k] - Var[z]| ****" in conv
    assert len([ln for ln in conv.splitlines() if ln.strip().startswith("mean")]) == 17
    # exact targets printed by the driver: recompute them the same way to compare
    from multigridmc_amd.driver import ExactTargets, _measured_values
    from multigridmc_amd.parameters import MeasurementParameters, MultigridParameters, read_config
    cfg = read_config(str(tmp_path / "parameters.cfg"))
    mp = MeasurementParameters.from_config(cfg, str(tmp_path))
    lat = mg.Lattice(64, 64)
    prior_cls = {"shiftedlaplace_fd": mg.ShiftedLaplaceFDOperator, "shiftedlaplace_fem": mg.ShiftedLaplaceFEMOperator,
                 "squared_shiftedlaplace_fd": mg.SquaredShiftedLaplaceFDOperator}[pde]
    cl = mg.ConstantCorrelationLengthModel(0.2) if model == "constant" else mg.PeriodicCorrelationLengthModel(0.2, 0.4)
    op = mg.MeasuredOperator(prior_cls(lat, cl), mp)
    s = mg.MultigridMCSampler(op, SEED, MultigridParameters.from_config(cfg))
    rows, vals = mg.measurement_vector(lat, mp.sample_location, mp.radius)
    mean_exact, var_exact = ExactTargets(s).observed_mean_and_variance(_measured_values(mp), rows, vals)
    _check_moments(z, mean_exact, var_exact)
    s.close()
