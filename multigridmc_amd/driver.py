"""driver_mgmc for the device sampler: `python -m multigridmc_amd.driver parameters.cfg`.

Mirrors the Multigrid MC part of the reference's driver (src/driver_mgmc.cc):
  * main: read the parameters file, build the lattice, the FD prior, the posterior
    (MeasuredOperator, always built) and the MGMC sampler with seed 5418513 ........ :319-535
  * measure_sampling_time: fix f = Q mean_x, nwarmup + nsamples cycles, QoI z = b^T x per
    sample, "time per sample", timeseries_multigridmc.txt, mean / variance against the exact
    observed mean and variance ......................................................... :40-107
  * measure_convergence: nsamplesconvergence chains from x = 0, nstepsconvergence cycles
    each; |E[z^k] - E[z]| and |Var[z^k] - Var[z]| with error bars to
    convergence_multigridmc.txt ........................................................ :188-314
The exact targets (LinearOperator::mean, observed_mean_and_variance, linear_operator.hh:119-174)
come from the device multigrid-preconditioned CG on the posterior operator (mgmc_solve) instead of
a sparse Cholesky factorisation.  As in the reference, the "exact" observed statistics always
refer to the measured (posterior) operator built on top of the chosen operator.

Out of scope (not the device hot path): the Cholesky and SSOR samplers of the whole lattice
(do_cholesky / do_ssor are reported and skipped) and the VTK output of posterior_statistics.
Every prior of the reference is on the device path (driver_mgmc.cc:398-429): pdemodel =
"shiftedlaplace_fd", "shiftedlaplace_fem" and "squared_shiftedlaplace_fd" (2D), with the
"constant" or the "periodic" correlation length model; operators with per-vertex coefficients go to
the device as matrices (mgmc_create_csr).
"""
from __future__ import annotations

import datetime
import os
import sys
import time

import numpy as np

from . import _native as mg_native
from .measured import MeasuredOperator, measurement_vector
from .parameters import (ConfigError, ConstantCorrelationLengthModelParameters, GeneralParameters,
                         LatticeParameters, MeasurementFileError, MeasurementParameters, MultigridParameters,
                         PeriodicCorrelationLengthModelParameters, PriorParameters, SamplingParameters, read_config)
from .sampler import (ConstantCorrelationLengthModel, Lattice, MultigridMCSampler, PeriodicCorrelationLengthModel,
                      ShiftedLaplaceFDOperator, ShiftedLaplaceFEMOperator, SquaredShiftedLaplaceFDOperator)

SEED = 5418513  # driver_mgmc.cc:448


def _measured_values(mp: MeasurementParameters) -> np.ndarray:
    y = list(mp.mean[:len(mp.measurement_locations)])
    if mp.measure_global:
        y.append(mp.mean_global)
    return np.asarray(y, dtype=np.float64)


class ExactTargets:
    """LinearOperator::mean / observed_mean_and_variance (linear_operator.hh:119-174) with xbar = 0,
    from device CG solves with the posterior precision Q = A + B Sigma^-1 B^T:
    x_post = Q^-1 B Sigma^-1 y,  mean z = b^T x_post,  Var z = b^T Q^-1 b."""

    def __init__(self, posterior_sampler: MultigridMCSampler, rtol: float = 1e-12, maxiter: int = 200):
        self.s = posterior_sampler
        self.rtol = rtol
        self.maxiter = maxiter

    def solve(self, b):
        x, it, rn = self.s.solve(b, method="cg", rtol=self.rtol, maxiter=self.maxiter)
        if it >= self.maxiter:
            raise RuntimeError(f"exact-statistics solve did not converge (||r|| = {rn})")
        return x

    def posterior_mean(self, y) -> np.ndarray:
        lr = self.s.linear_operator.get_B()
        g = np.zeros(lr.n)
        for k in range(lr.m):
            sl = slice(lr.colptr[k], lr.colptr[k + 1])
            g[lr.rows[sl]] += lr.vals[sl] * (y[k] / lr.sigma[k])
        return self.solve(g)

    def observed_mean_and_variance(self, y, rows, vals):
        b = np.zeros(self.s.ndof)
        b[rows] = vals
        bbar = self.solve(b)
        x_post = self.posterior_mean(y)
        return float(np.dot(b, x_post)), float(np.dot(b, bbar))


def _qoi_series(sampler: MultigridMCSampler, nsteps: int, rows, vals) -> np.ndarray:
    """z = b^T x after every cycle (driver_mgmc.cc:76), recorded on the device inside the cycle graph:
    radius 0 reads the vertex, radius > 0 the dot with the installed vector (mgmc_set_qoi_vector,
    blocked order) -- the state never leaves HBM."""
    if len(rows) == 1 and vals[0] == 1.0:
        return sampler.sample(nsteps, int(rows[0]))
    if getattr(sampler, "_qv", None) is None or not (np.array_equal(sampler._qv[0], rows)
                                                      and np.array_equal(sampler._qv[1], vals)):
        sampler.set_qoi_vector(rows, vals)
    return sampler.sample(nsteps, mg_native.QOI_VECTOR)


def measure_sampling_time(sampler, exact: ExactTargets, sampling_params: SamplingParameters,
                          measurement_params: MeasurementParameters, label: str, filename: str):
    """driver_mgmc.cc:40-107."""
    op = sampler.get_linear_operator()
    y = _measured_values(measurement_params)
    mean_x_exact = exact.posterior_mean(y) if op.get_m_lowrank() > 0 else np.zeros(op.get_ndof())
    rows, vals = measurement_vector(op.get_lattice(), measurement_params.sample_location, measurement_params.radius)
    f = sampler.operator_apply(0, mean_x_exact)
    sampler.fix_rhs(f)
    sampler.set_state(np.zeros(op.get_ndof()))
    _qoi_series(sampler, sampling_params.nwarmup, rows, vals)
    t0 = time.perf_counter()
    data = _qoi_series(sampler, sampling_params.nsamples, rows, vals)
    t_elapsed = (time.perf_counter() - t0) * 1e3 / sampling_params.nsamples
    print(f"  {label:>12s} time per sample = {t_elapsed:12.4f} ms")
    with open(filename, "w") as out:
        for v in data:
            out.write(f"{v:g}\n")
    x_avg = 0.0
    xsq_avg = 0.0
    for k, d in enumerate(data):
        x_avg += (d - x_avg) / (k + 1.0)
        xsq_avg += (d * d - xsq_avg) / (k + 1.0)
    variance = xsq_avg - x_avg * x_avg
    x_error = np.sqrt(variance / sampling_params.nsamples)
    mean_exact, variance_exact = exact.observed_mean_and_variance(y, rows, vals)
    print(f"  {label:>12s} mean     = {x_avg:12.4e} +/- {x_error:12.4e} [ignoring IACT]")
    print(f"  {'exact':>12s} mean     = {mean_exact:12.4e}")
    print(f"  {label:>12s} variance = {variance:12.4e}")
    print(f"  {'exact':>12s} variance = {variance_exact:12.4e}\n")
    return data, (mean_exact, variance_exact)


def convergence_series(sampler, nsamples: int, nsteps: int, rows, vals, batch: int = 1) -> np.ndarray:
    """QoI series z[k, j] of nsamples chains from x = 0, nsteps cycles each (driver_mgmc.cc:236-254).
    Chain k draws sample indices s0 + k nsteps .. s0 + (k+1) nsteps - 1, exactly as one handle running
    the chains one after the other.  batch > 1 runs that many chains at a time on
    clones of the handle, each on its own HIP stream, with those sample indices: the same draws, so
    the same series bit for bit, with the small lattices' idle GPU filled by the concurrent chains.
    A radius > 0 QoI is the device-side dot with the measurement vector on every handle."""
    x0 = np.zeros(sampler.ndof)
    z = np.empty((nsamples, nsteps))
    if batch <= 1:
        for k in range(nsamples):
            sampler.set_state(x0)
            z[k] = _qoi_series(sampler, nsteps, rows, vals)
        return z
    s0 = sampler.get_sample_index()
    handles = [sampler] + [sampler.clone() for _ in range(min(batch, nsamples) - 1)]
    vertex = len(rows) == 1 and vals[0] == 1.0
    if not vertex:  # radius > 0: every handle records the dot with the measurement vector
        for h in handles:
            h.set_qoi_vector(rows, vals)
    q = int(rows[0]) if vertex else mg_native.QOI_VECTOR
    try:
        for k0 in range(0, nsamples, len(handles)):
            ks = list(range(k0, min(k0 + len(handles), nsamples)))
            for h, k in zip(handles, ks):
                h.set_sample_index(s0 + k * nsteps)
                h.set_state(x0)
                h.sample_async(nsteps, q)
            for h, k in zip(handles, ks):
                z[k] = h.get_series(nsteps)
        sampler.set_sample_index(s0 + nsamples * nsteps)
    finally:
        for h in handles[1:]:
            h.close()
    return z


def measure_convergence(sampler, exact: ExactTargets, sampling_params: SamplingParameters,
                        measurement_params: MeasurementParameters, filename: str, batch: int = 1):
    """driver_mgmc.cc:188-314: nsamplesconvergence independent chains from x = 0 (batch: chains run
    concurrently, convergence_series)."""
    op = sampler.get_linear_operator()
    y = _measured_values(measurement_params)
    mean_x_exact = exact.posterior_mean(y) if op.get_m_lowrank() > 0 else np.zeros(op.get_ndof())
    rows, vals = measurement_vector(op.get_lattice(), measurement_params.sample_location, measurement_params.radius)
    sampler.fix_rhs(sampler.operator_apply(0, mean_x_exact))
    nsteps = sampling_params.nstepsconvergence
    nsamples = sampling_params.nsamplesconvergence
    avg = np.zeros((4, nsteps + 1))
    zs = convergence_series(sampler, nsamples, nsteps, rows, vals, batch)
    for k in range(nsamples):
        z = zs[k]
        for j in range(1, nsteps + 1):
            for a in range(4):
                avg[a, j] += (z[j - 1] ** (a + 1) - avg[a, j]) / (k + 1.0)
    mean_exact, variance_exact = exact.observed_mean_and_variance(y, rows, vals)
    x1, x2, x3, x4 = avg
    diff_mean = np.abs(x1 - mean_exact)
    diff_variance = np.abs(x2 - x1 * x1 - variance_exact)
    sigma_sq = nsamples / (nsamples - 1.0) * (x2 - x1 * x1)
    mu4 = x4 - 4 * x1 * x3 + 6 * x1 ** 2 * x2 - 3 * x1 ** 4
    error_mean = np.sqrt(sigma_sq / nsamples)
    error_variance = np.sqrt(np.maximum(mu4 - (nsamples - 3.0) / (nsamples - 1.0) * sigma_sq * sigma_sq, 0.0) / nsamples)
    with open(filename, "w") as out:
        for q, (label, diff, err) in enumerate([("mean", diff_mean, error_mean),
                                                ("variance", diff_variance, error_variance)]):
            out.write("**** q_k = |E[z^k] - E[z]| **** \n" if q == 0 else "**** q_k = |Var[z^k] - Var[z]| **** \n")
            out.write(f"  {'':>12s}   {'k':>3s} : {'q_k':>12s} {'q_k/q_0':>35s} {'q_k/q_{k-1}':>35s}\n")
            for j in range(nsteps + 1):
                out.write(f"  {label:>12s}   {j:3d} : {diff[j]:12.8f} +/- {err[j]:12.8f}       "
                          f"{diff[j] / diff[0]:12.8f} +/- {err[j] / diff[0]:12.8f}      ")
                if j > 0:
                    rel = diff[j] / diff[j - 1] * np.sqrt((err[j] / diff[j]) ** 2 + (err[j - 1] / diff[j - 1]) ** 2)
                    out.write(f" {diff[j] / diff[j - 1]:12.8f} +/- {rel:12.8f} \n")
                else:
                    out.write(f" {'---':>12s}\n")
            out.write("\n")
    return diff_mean, diff_variance


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    batch = 1
    if len(argv) == 3 and argv[0] == "--convergence-batch":  # concurrent measure_convergence chains
        batch = int(argv[1])
        argv = argv[2:]
    if len(argv) != 1:
        print(f"Usage: {sys.argv[0]} [--convergence-batch N] CONFIGURATIONFILE")
        return -1
    t_start = time.time()
    print("\n+--------------------------------+")
    print("! Multigrid Monte Carlo sampling !")
    print("+--------------------------------+\n")
    print(f"Starting run at {datetime.datetime.now().ctime()}\n")
    filename = argv[0]
    print(f"Reading parameters from file '{filename}'")
    cfg = read_config(filename)
    base = os.path.dirname(os.path.abspath(filename))
    general = GeneralParameters.from_config(cfg)
    lattice_params = LatticeParameters.from_config(cfg)
    mg_params = MultigridParameters.from_config(cfg)
    sampling_params = SamplingParameters.from_config(cfg)
    prior_params = PriorParameters.from_config(cfg)
    try:
        measurement_params = MeasurementParameters.from_config(cfg, base)
    except MeasurementFileError as e:  # parameters.cc:273-276: message on stderr, exit(-1)
        print(str(e), file=sys.stderr)
        return -1
    if measurement_params.dim != general.dim:
        print("ERROR: dimension of measurement locations differs from problem dimension")
        return -1
    if general.dim == 2:
        lattice = Lattice(lattice_params.nx, lattice_params.ny)
    elif general.dim == 3:
        lattice = Lattice(lattice_params.nx, lattice_params.ny, lattice_params.nz)
    else:
        print(f"ERROR: Invalid dimension : {general.dim}")
        return -1
    # driver_mgmc.cc:398-429
    try:
        if prior_params.correlationlength_model == "constant":
            model = ConstantCorrelationLengthModel(ConstantCorrelationLengthModelParameters.from_config(cfg).Lambda)
        elif prior_params.correlationlength_model == "periodic":
            pp = PeriodicCorrelationLengthModelParameters.from_config(cfg)
            model = PeriodicCorrelationLengthModel(pp.Lambda_min, pp.Lambda_max)
        else:
            print(f"Error: invalid correlationlengthmodel '{prior_params.correlationlength_model}'")
            return -1
    except ConfigError as e:
        print(str(e))
        return -1
    prior_classes = {"shiftedlaplace_fd": ShiftedLaplaceFDOperator, "shiftedlaplace_fem": ShiftedLaplaceFEMOperator,
                     "squared_shiftedlaplace_fd": SquaredShiftedLaplaceFDOperator}
    if prior_params.pde_model not in prior_classes:
        print(f"Error: invalid prior '{prior_params.pde_model}'")
        return -1
    try:
        prior = prior_classes[prior_params.pde_model](lattice, model)
    except ValueError as e:  # squared_shiftedlaplace_fd in 3D (squared_shiftedlaplace_fd_operator.cc:15-19)
        print(f"ERROR: {e}")
        return -1
    posterior = MeasuredOperator(prior, measurement_params)
    if general.operator_name == "prior":
        linear_operator = prior
    elif general.operator_name == "posterior":
        linear_operator = posterior
    else:
        print(f"ERROR: invalid operator : {general.operator_name}")
        return -1
    sampler = MultigridMCSampler(linear_operator, SEED, mg_params)
    # the exact observed statistics always refer to the measured operator (driver_mgmc.cc:58-60)
    solver_sampler = sampler if linear_operator is posterior else MultigridMCSampler(posterior, SEED, mg_params)
    exact = ExactTargets(solver_sampler)
    print()
    for flag, name in ((general.do_cholesky, "Cholesky"), (general.do_ssor, "SSOR")):
        if flag:
            print(f"**** {name} **** skipped: the whole-lattice {name} sampler is not on the device path\n")
    if general.do_multigridmc:
        print("**** Multigrid MC ****")
        measure_sampling_time(sampler, exact, sampling_params, measurement_params, "MGMC",
                              "timeseries_multigridmc.txt")
        measure_convergence(sampler, exact, sampling_params, measurement_params, "convergence_multigridmc.txt",
                            batch)
        if general.save_posterior_statistics:
            print("  posterior_statistics (VTK output) is not on the device path: skipped")
        print()
    secs = int(time.time() - t_start)
    print(f"Completed run at {datetime.datetime.now().ctime()}")
    print(f"Total elapsed time = {secs // 3600:3d} h {(secs // 60) % 60:2d} m {secs % 60:2d} s\n")
    if solver_sampler is not sampler:
        solver_sampler.close()
    sampler.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
