"""Device-side QoI for radius > 0 (-m gpu): the measurement vector b of
MeasuredOperator::measurement_vector (measured_operator.cc:92-171) dotted with every sample inside the
cycle graph (mgmc_set_qoi_vector + qoi_index = MGMC_QOI_VECTOR), as driver_mgmc.cc:58-59, :76 do.

The dot has a fixed order (4096-entry blocks, lane-strided sums, xor butterflies -- the low-rank dots'
order); the oracle computes the same sequence (refcpu blocked_dot) on its multicolour chain's state,
so the series are compared bit for bit.  Against the reference's Eigen dense dot the values agree to
rounding (tested to 1e-13 relative): its summation order is Eigen's packet reduction."""
import numpy as np
import pytest

import multigridmc_amd as mg
from tests import oracle_lib as O

pytestmark = pytest.mark.gpu

SEED = 5418513


def _pair(shape, nlevel, nchains=1, chain=0):
    lat = mg.Lattice(*shape)
    p = mg.MultigridParameters(nlevel=nlevel)
    s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, device=0, chain_id=chain,
                              nchains=nchains)
    o = O.Oracle.fd_own(lat.shape, p, 25.0, mode=O.MULTICOLOUR, seed=SEED, chain=chain)
    return s, o, lat


@pytest.mark.parametrize("shape,nlevel,radius", [((64, 64), 4, 0.1), ((32, 32, 32), 3, 0.2),
                                                  ((128, 128, 128), 4, 0.15)])
def test_qoi_vector_series_bitwise(hip_device, shape, nlevel, radius):
    s, o, lat = _pair(shape, nlevel)
    rows, vals = mg.measurement_vector(lat, [0.5] * lat.dim, radius)
    assert len(rows) > 1
    if lat.dim == 3 and shape[0] == 128:
        assert len(rows) > 4096  # several blocks
    f = np.random.default_rng(4).standard_normal(lat.Nvertex)
    s.fix_rhs(f)
    o.set_rhs(f)
    s.set_qoi_vector(rows, vals)
    z_dev = s.sample(5, mg.QOI_VECTOR)
    z_orc = []
    for _ in range(5):
        o.sample(1)
        z_orc.append(O.blocked_dot(rows, vals, o.get_state()))
    assert np.array_equal(z_dev, np.array(z_orc))
    x = s.get_state()
    assert abs(z_dev[-1] - np.dot(vals, x[rows])) <= 1e-13 * np.sum(np.abs(vals * x[rows]))
    n, mean, m2 = s.qoi_moments()
    assert n == 5 and mean == pytest.approx(np.mean(z_dev), rel=1e-12)
    # vertex QoI still works on the same graph, and removing the vector restores the plain record
    q = mg.measurement_vector_index(lat, [0.5] * lat.dim)
    z1 = s.sample(2, q)
    for k in range(2):
        o.sample(1)
        assert z1[k] == o.get_state()[q]
    s.set_qoi_vector([], [])
    with pytest.raises(mg.MgmcError, match="no QoI vector"):
        s.sample(1, mg.QOI_VECTOR)
    s.close()


def test_qoi_vector_batched_chains_equal_single(hip_device):
    shape, radius = (32, 32, 32), 0.2
    lat = mg.Lattice(*shape)
    rows, vals = mg.measurement_vector(lat, [0.5] * 3, radius)
    p = mg.MultigridParameters(nlevel=3)
    b = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, chain_id=4, nchains=3)
    b.set_qoi_vector(rows, vals)
    zb = b.sample(4, mg.QOI_VECTOR, chain=None)
    for c in range(3):
        s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), SEED, p, chain_id=4 + c)
        s.set_qoi_vector(rows, vals)
        assert np.array_equal(s.sample(4, mg.QOI_VECTOR), zb[c])
        s.close()
    b.close()


def test_driver_template_radius_runs_on_device(hip_device, tmp_path, monkeypatch):
    """The driver on the template (config 1: 2D posterior) with radius 0.05 records the QoI on the
    device: the sampling loops never download the state per sample (get_state is not called)."""
    import os
    import re
    from multigridmc_amd import driver
    gold = os.path.join(os.path.dirname(__file__), "golden")
    text = open(os.path.join(gold, "parameters_template.cfg")).read()
    text = re.sub(r"radius = 0.0;", "radius = 0.05;", text)
    text = re.sub(r"nsamples = 10000;", "nsamples = 2000;", text)
    text = re.sub(r"nsamples = 1000;", "nsamples = 40;", text)
    assert "radius = 0.05;" in text and "nsamples = 2000;" in text
    (tmp_path / "parameters.cfg").write_text(text)
    (tmp_path / "measurements_template.cfg").write_text(open(os.path.join(gold, "measurements_template.cfg")).read())
    monkeypatch.chdir(tmp_path)
    calls = {"n": 0}
    orig = mg.MultigridMCSampler.get_state

    def counting(self, chain=0):
        calls["n"] += 1
        return orig(self, chain)
    monkeypatch.setattr(mg.MultigridMCSampler, "get_state", counting)
    assert driver.main([str(tmp_path / "parameters.cfg")]) == 0
    assert calls["n"] < 20  # no per-sample downloads (2000 + convergence samples)
    z = np.loadtxt(tmp_path / "timeseries_multigridmc.txt")
    assert z.shape == (2000,) and np.all(np.isfinite(z)) and np.std(z) > 0
