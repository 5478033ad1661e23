"""The reference-side adapter on the GPU (-m gpu): include/reference_adapter/hip_multigridmc_sampler.hh
driven like driver_mgmc.cc drives a Sampler (fix_rhs, then apply(f, x) per sample,
driver_mgmc.cc:66-78), on LinearOperators whose get_sparse() is the reference operator's matrix.
The FD / FEM priors with a constant correlation length take the stencil fast path, the periodic one
the matrix path; each QoI series equals the Python host side's (ShiftedLaplaceFDOperator /
ShiftedLaplaceFEMOperator with the same seed) bit for bit."""
import subprocess

import numpy as np
import pytest

import multigridmc_amd as mg
from tests.test_adapter import build_adapter_client

pytestmark = pytest.mark.gpu

OPS = {
    "fd": ((16, 16, 16), mg.ShiftedLaplaceFDOperator, mg.ConstantCorrelationLengthModel(0.2), "stencil"),
    "fem": ((16, 16, 16), mg.ShiftedLaplaceFEMOperator, mg.ConstantCorrelationLengthModel(0.2), "stencil"),
    "periodic": ((32, 32), mg.ShiftedLaplaceFDOperator, mg.PeriodicCorrelationLengthModel(0.2, 0.4), "matrix"),
}


@pytest.mark.parametrize("kind", list(OPS))
def test_reference_adapter_series_matches_python_host_side(hip_device, tmp_path, kind):
    exe = build_adapter_client(str(tmp_path))
    r = subprocess.run([exe, "sample", "5", kind], capture_output=True, text=True, check=True)
    lines = r.stdout.split()
    assert lines[0] == "seed" and lines[2] == "path"
    seed, path = int(lines[1]), lines[3]
    z_adapter = np.array([float(v) for v in lines[4:]])
    shape, cls, model, expect_path = OPS[kind]
    assert path == expect_path
    lat = mg.Lattice(*shape)
    s = mg.MultigridMCSampler(cls(lat, model), seed, mg.MultigridParameters(nlevel=3), device=0, chain_id=0)
    s.fix_rhs(np.zeros(lat.Nvertex))
    z = s.sample(5, lat.Nvertex // 2)
    s.close()
    assert len(z_adapter) == 5 and np.all(np.isfinite(z_adapter))
    assert np.array_equal(z_adapter, z)


def test_adapter_ownership_releases_device_handles(hip_device, tmp_path):
    """Samplers and smoothers owned through std::make_shared<Derived> as shared_ptr<Base> (the
    reference's ownership, driver_mgmc.cc:450-457, multigrid_preconditioner.cc:18-33; the base classes
    have no virtual destructor) release every device handle when the base pointers go: after each round
    mgmc_live_handles() is back to 0."""
    exe = build_adapter_client(str(tmp_path))
    r = subprocess.run([exe, "ownership", "4"], capture_output=True, text=True, check=True)
    lines = r.stdout.splitlines()
    assert lines[0] == "live 0"
    rounds = [line.split() for line in lines[1:]]
    assert len(rounds) == 4
    for w in rounds:
        assert w[0] == "round" and w[2] == "held" and int(w[3]) == 3, w
        assert w[4] == "live" and int(w[5]) == 0 and w[6] == "x" and w[7] == "1", w
