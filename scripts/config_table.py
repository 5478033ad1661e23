"""BASELINE.md §4 numbers on the GPU box (test infrastructure: it imports the CPU oracle for the CPU
columns).  One JSON object per line into the file given as argv[1]:

  config 1  parameters_template.cfg at 64^2 (posterior, 8 measurements, W-cycle, SSOR coarse): the
            device chain and the FAITHFUL oracle chain (the reference algorithm) on identical seeds
            and inputs, 1,000 warm-up + 10,000 samples each (driver_mgmc.cc:40-107), timed; QoI
            mean / variance of both and the exact observed mean / variance
            (linear_operator.hh:153-174);
  configs 2, 3, 5 (and 4 with --with-512): bench.py lines, CPU baselines included.

  python scripts/config_table.py out.jsonl [--with-512]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def config1():
    import numpy as np
    import multigridmc_amd as mg
    from multigridmc_amd.driver import ExactTargets, _measured_values
    from multigridmc_amd.parameters import MeasurementParameters, MultigridParameters, read_config
    from tests import oracle_lib as O
    from tests.test_gpu_exact import _iact
    golden = os.path.join(ROOT, "tests", "golden")
    cfg = read_config(os.path.join(golden, "parameters_template.cfg"))
    p = MultigridParameters.from_config(cfg)
    mp_ = MeasurementParameters.from_config(cfg, golden)
    lat = mg.Lattice(64, 64)
    op = mg.MeasuredOperator(mg.ShiftedLaplaceFDOperator(lat, 25.0), mp_)
    s = mg.MultigridMCSampler(op, 5418513, p)
    exact = ExactTargets(s)
    y = _measured_values(mp_)
    f = s.operator_apply(0, exact.posterior_mean(y))
    q = mg.measurement_vector_index(lat, mp_.sample_location)
    mean_exact, var_exact = exact.observed_mean_and_variance(y, [q], [1.0])
    s.fix_rhs(f)
    s.set_state(np.zeros(lat.Nvertex))
    s.sample(1000, q)
    s.synchronize()
    t0 = time.perf_counter()
    z_dev = s.sample(10000, q)
    t_dev = time.perf_counter() - t0
    s.close()
    o = O.Oracle.fd(lat.shape, p, 25.0, mode=O.FAITHFUL, seed=5418513)
    o.set_lowrank(op.get_B())
    o.set_rhs(f)
    o.set_state(np.zeros(lat.Nvertex))
    o.sample(1000)
    t0 = time.perf_counter()
    z_cpu = o.sample(10000, q)
    t_cpu = time.perf_counter() - t0

    def err(z):
        return float(np.sqrt(np.var(z) * _iact(z) / len(z)))
    return {"config": 1, "gpu_samples_per_s": 10000 / t_dev, "cpu_1core_samples_per_s": 10000 / t_cpu,
            "qoi_gpu": {"mean": float(z_dev.mean()), "mean_err": err(z_dev), "var": float(z_dev.var()),
                        "iact": float(_iact(z_dev))},
            "qoi_cpu": {"mean": float(z_cpu.mean()), "mean_err": err(z_cpu), "var": float(z_cpu.var()),
                        "iact": float(_iact(z_cpu))},
            "qoi_exact": {"mean": float(mean_exact), "var": float(var_exact)},
            "note": "parameters_template.cfg at 64^2, W-cycle, 8 measurements; 1,000 warm-up + 10,000 samples; "
                    "the GPU time includes one host round trip per sample (the QoI series read-back)"}


def bench(config, args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=1800)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-1000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    line["table_config"] = config
    line["table_args"] = args
    return line


def main():
    out = open(sys.argv[1], "w")

    def emit(d):
        out.write(json.dumps(d) + "\n")
        out.flush()
        print(json.dumps(d)[:300], flush=True)
    emit(config1())
    emit(bench(2, ["--dim", "2", "--n", "1024", "--nlevel", "5", "--steps", "2000", "--warmup", "50",
                   "--cpu-samples", "100", "--cpu-warmup", "10"]))
    emit(bench(3, ["--n", "256", "--nlevel", "6", "--steps", "500", "--warmup", "20",
                   "--cpu-samples", "20", "--cpu-warmup", "3"]))
    emit(bench(5, ["--posterior", "8", "--steps", "500", "--warmup", "20", "--cpu-samples", "3", "--cpu-warmup", "1"]))
    emit(bench(5.1, ["--posterior", "8", "--measure-global", "--steps", "200", "--warmup", "10", "--no-cpu-baseline"]))
    if "--with-512" in sys.argv:
        emit(bench(4, ["--steps", "100", "--warmup", "10"]))


if __name__ == "__main__":
    main()
