"""BASELINE.json's configurations on the device (-m gpu), at their full sizes.

  * config 1 -- T3(ii) of SURVEY §8(c), the north_star's "match the reference CPU sampler's posterior
    mean/variance of the QoI on identical seeds": parameters_template.cfg at 64^2 (posterior, 8
    measurements, W-cycle, SSOR coarse), 1,000 warm-up + 10,000 samples, seed 5418513, in the loop
    of driver_mgmc.cc:40-107 (f = Q mean_x, x0 = 0).  The device chain and the FAITHFUL oracle chain
    (the reference algorithm: lexicographic SOR, mt19937_64, dense lexicographic B_bar) agree within
    5 combined sigma (IACT), and both agree with the exact observed_mean_and_variance
    (linear_operator.hh:153-174);
  * config 2 -- 2D 1024^2 prior, 5 levels, V-cycle: two cycles and a 6-sample QoI series bitwise
    against the MULTICOLOUR oracle;
  * config 5 -- 3D 256^3 posterior, 8 point measurements (with and without the global average), 6
    levels: one cycle bitwise against the MULTICOLOUR oracle, and the QoI mean / variance at the
    lattice centre against the device-CG exact targets within 5 sigma (IACT).
"""
import os

import numpy as np
import pytest

import multigridmc_amd as mg
from multigridmc_amd.driver import ExactTargets, _measured_values
from multigridmc_amd.parameters import MeasurementParameters, MultigridParameters, read_config
from tests import oracle_lib as O
from tests.test_gpu_exact import _check_moments, _iact

pytestmark = pytest.mark.gpu

SEED = 5418513
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _mc_oracle(s, p, lat, lowrank=None):
    o = O.Oracle.fd_own(lat.shape, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=0)
    if lowrank is not None:
        o.set_lowrank(lowrank)
    return o


def test_config2_2d1024_bitwise(hip_device):
    """BASELINE config 2: 2D 1024^2 FD prior, nlevel 5, V-cycle, SOR 1/1, SSOR coarse 1, omega 1."""
    lat = mg.Lattice(1024, 1024)
    p = MultigridParameters(nlevel=5, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                            ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p)
    mc = _mc_oracle(s, p, lat)
    f = np.random.default_rng(11).standard_normal(lat.Nvertex)
    x_dev, x_orc = np.zeros(lat.Nvertex), np.zeros(lat.Nvertex)
    for _ in range(2):
        s.apply(f, x_dev)
        mc.apply(f, x_orc)
    assert np.array_equal(x_dev, x_orc)
    q = mg.measurement_vector_index(lat, [0.5, 0.5])
    s.fix_rhs(f)
    s.set_state(x_dev)
    mc.set_rhs(f)
    mc.set_state(x_orc)
    z_dev = s.sample(6, q)
    z_orc = mc.sample(6, q)
    assert np.array_equal(z_dev, z_orc)
    assert np.array_equal(s.get_state(), mc.get_state())
    s.close()


def _config5(measure_global):
    lat = mg.Lattice(256, 256, 256)
    op = mg.synthetic_posterior(mg.ShiftedLaplaceFDOperator(lat, 25.0), 8, 0.0, measure_global)
    p = MultigridParameters(nlevel=6, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                            ncoarsesmooth=1, omega=1.0, cycle=1, coarse_scaling=1.0)
    return lat, op, p


@pytest.mark.parametrize("measure_global", [False, True])
def test_config5_256_posterior_bitwise(hip_device, measure_global):
    """BASELINE config 5: one 256^3 posterior cycle (8 point measurements [+ global average]) on a
    random rhs, bitwise equal to the MULTICOLOUR oracle (B_bar fix and low-rank noise included)."""
    lat, op, p = _config5(measure_global)
    s = mg.MultigridMCSampler(op, SEED, p)
    mc = _mc_oracle(s, p, lat, op.get_B())
    f = np.random.default_rng(12).standard_normal(lat.Nvertex)
    x_dev, x_orc = np.zeros(lat.Nvertex), np.zeros(lat.Nvertex)
    s.apply(f, x_dev)
    mc.apply(f, x_orc)
    assert np.array_equal(x_dev, x_orc)
    s.close()


@pytest.mark.parametrize("measure_global,nsamples", [(False, 20000), (True, 8000)])
def test_config5_256_posterior_moments(hip_device, measure_global, nsamples):
    """BASELINE config 5 statistics: QoI at the lattice centre (the bench's QoI), f = B Sigma^-1 y with
    y ~ U(1, 3): sample mean and variance against e^T Q^-1 f and e^T Q^-1 e from the device CG on the
    posterior operator, within 5 sigma (IACT)."""
    lat, op, p = _config5(measure_global)
    s = mg.MultigridMCSampler(op, SEED, p)
    lr = op.get_B()
    y = np.random.default_rng(5).uniform(1.0, 3.0, lr.m)
    f = _bsy(lr, y)
    q = mg.measurement_vector_index(lat, [0.5, 0.5, 0.5])
    e = np.zeros(lat.Nvertex)
    e[q] = 1.0
    mean_field, it1, _ = s.solve(f, method="cg", rtol=1e-11, maxiter=200)
    g, it2, _ = s.solve(e, method="cg", rtol=1e-11, maxiter=200)
    assert it1 < 200 and it2 < 200
    s.fix_rhs(f)
    s.set_state(mean_field)
    s.sample(200, q)
    z = s.sample(nsamples, q)
    assert np.all(np.isfinite(z))
    _check_moments(z, mean_field[q], g[q])
    s.close()


def _bsy(lr, y):
    out = np.zeros(lr.n)
    for k in range(lr.m):
        sl = slice(lr.colptr[k], lr.colptr[k + 1])
        out[lr.rows[sl]] += lr.vals[sl] * (y[k] / lr.sigma[k])
    return out


def config1_chains(nwarmup=1000, nsamples=10000):
    """parameters_template.cfg at 64^2 (BASELINE config 1): the device chain and the FAITHFUL oracle
    chain in the loop of driver_mgmc.cc:40-107, plus the exact observed mean and variance."""
    cfg = read_config(os.path.join(GOLDEN, "parameters_template.cfg"))
    p = MultigridParameters.from_config(cfg)
    mp = MeasurementParameters.from_config(cfg, GOLDEN)
    lat = mg.Lattice(64, 64)
    op = mg.MeasuredOperator(mg.ShiftedLaplaceFDOperator(lat, 25.0), mp)  # Lambda 0.2 -> kappa^2 = 25
    s = mg.MultigridMCSampler(op, SEED, p)
    exact = ExactTargets(s)
    y = _measured_values(mp)
    mean_x = exact.posterior_mean(y)
    f = s.operator_apply(0, mean_x)
    q = mg.measurement_vector_index(lat, mp.sample_location)
    mean_exact, var_exact = exact.observed_mean_and_variance(y, [q], [1.0])
    s.fix_rhs(f)
    s.set_state(np.zeros(lat.Nvertex))
    s.sample(nwarmup, q)
    z_dev = s.sample(nsamples, q)
    s.close()
    o = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL, seed=SEED)
    o.set_lowrank(op.get_B())
    o.set_rhs(f)
    o.set_state(np.zeros(lat.Nvertex))
    o.sample(nwarmup)
    z_cpu = o.sample(nsamples, q)
    return z_dev, z_cpu, mean_exact, var_exact


def test_config1_gpu_vs_faithful_oracle_qoi_moments(hip_device):
    """T3(ii): GPU chain vs the reference algorithm's chain (FAITHFUL oracle) on identical seeds and
    inputs: QoI mean and variance within 5 combined sigma of each other (IACT-corrected), and each
    within 5 sigma of the exact observed mean / variance."""
    z_dev, z_cpu, mean_exact, var_exact = config1_chains()
    assert np.all(np.isfinite(z_dev)) and np.all(np.isfinite(z_cpu))
    n_dev = len(z_dev) / _iact(z_dev)
    n_cpu = len(z_cpu) / _iact(z_cpu)
    sig_mean = np.sqrt(var_exact / n_dev + var_exact / n_cpu)
    sig_var = var_exact * np.sqrt(2.0 / n_dev + 2.0 / n_cpu)
    assert abs(z_dev.mean() - z_cpu.mean()) < 5 * sig_mean, (z_dev.mean(), z_cpu.mean(), sig_mean)
    assert abs(z_dev.var() - z_cpu.var()) < 5 * sig_var, (z_dev.var(), z_cpu.var(), sig_var)
    _check_moments(z_dev, mean_exact, var_exact)
    _check_moments(z_cpu, mean_exact, var_exact)
