"""Host-side logic and the C-ABI boundary without a GPU: library loads and exports every symbol of
include/mgmc.h, configuration validation, Galerkin stencils vs the oracle's SpGEMM, the
libconfig-subset parser, QoI indexing, and the rank-order moment merge (gloo, world_size 2)."""
import ctypes
import os
import sys
import re

import numpy as np
import pytest

import multigridmc_amd as mg
from multigridmc_amd import _native
from multigridmc_amd.distributed import merge_moments, moments_of
from tests import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def header_symbols():
    text = open(os.path.join(ROOT, "include", "mgmc.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mgmc_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    lib = mg.load_library()
    syms = header_symbols()
    assert len(syms) >= 25
    bound = {name for name, _, _ in _native.SIGNATURES}
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/mgmc.h but not exported"
        assert s in bound, f"{s} not bound in multigridmc_amd/_native.py"
    assert lib.mgmc_abi_version() == _native.ABI_VERSION == 5


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def _cfg(shape=(16, 16, 16), **kw):
    p = mg.MultigridParameters(**{"nlevel": 3, **kw})
    return mg.make_config(mg.ShiftedLaplaceFDOperator(mg.Lattice(*shape), 25.0), p)


@pytest.mark.parametrize("shape,nlevel,msg", [
    ((15, 16, 16), 2, "one of the extents is odd"),
    ((8, 8, 8), 4, "no interior vertices"),
    ((6, 6), 2, None),
])
def test_describe_validation(shape, nlevel, msg):
    lib = mg.load_library()
    c = _cfg(shape, nlevel=nlevel)
    rc = lib.mgmc_describe(ctypes.byref(c), None, 0)
    if msg is None:
        assert rc == nlevel
    else:
        assert rc == _native.MGMC_E_INVALID
        assert msg in _native.last_error()


def test_invalid_parameters_rejected():
    lib = mg.load_library()
    for field, value in [("omega", 2.5), ("cycle", 0), ("smoother", 7), ("dim", 4)]:
        c = _cfg()
        setattr(c, field, value)
        assert lib.mgmc_describe(ctypes.byref(c), None, 0) == _native.MGMC_E_INVALID
    with pytest.raises(ValueError):
        mg.make_config(mg.ShiftedLaplaceFDOperator(mg.Lattice(8, 8), 1.0), mg.MultigridParameters(smoother="Jacobi"))


def test_create_without_gpu_fails_loudly():
    """On a host without a HIP device the product path must raise, never fall back to the CPU."""
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(0)
    if hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        pytest.skip("a HIP device is present (covered by the gpu tests)")
    lat = mg.Lattice3d(8, 8, 8)
    with pytest.raises(mg.MgmcError):
        mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=2))


def test_unknown_disable_token_rejected_before_any_device_call(monkeypatch):
    """MGMC_DISABLE (the kernel-path switches, mgmc_capi.hip PathFlag) is parsed before the device is
    touched; an unknown token is MGMC_E_INVALID with its name, on any host."""
    monkeypatch.setenv("MGMC_DISABLE", "tail,bogus_path")
    lat = mg.Lattice3d(8, 8, 8)
    with pytest.raises(mg.MgmcError, match="bogus_path") as e:
        mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=2))
    assert e.value.code == _native.MGMC_E_INVALID


def test_product_reads_only_documented_switches():
    """The only environment the library reads: MGMC_DISABLE (kernel-path switches, each covered by
    tests/test_gpu_parity.py VARIANTS / test_gpu_lowrank.py), MGMC_GRAPH_UNROLL
    (test_unrolled_sample_loop_bitwise) and MGMC_POISON (debug: NaN-filled scratch and LDS,
    scripts/profile_round.sh RUN_POISON=1 runs the headline determinism test with it)."""
    src = ""
    csrc = os.path.join(ROOT, "multigridmc_amd", "csrc")
    for fn in os.listdir(csrc):
        if fn.endswith((".hip", ".hpp", ".cpp", ".h")):
            src += open(os.path.join(csrc, fn)).read()
    assert sorted(set(re.findall(r'getenv\("([A-Z_0-9]+)"\)', src))) == ["MGMC_DISABLE", "MGMC_GRAPH_UNROLL", "MGMC_POISON"]
    tokens = re.findall(r'\{"([a-z_0-9]+)", PATH_NO_', src)
    assert len(tokens) == 17
    tested = open(os.path.join(ROOT, "tests", "test_gpu_parity.py")).read() + \
        open(os.path.join(ROOT, "tests", "test_gpu_lowrank.py")).read()
    for t in tokens:
        assert re.search(rf'["(,]{t}[",)]', tested), f"MGMC_DISABLE token {t} has no variant test"


@pytest.mark.parametrize("shape", [(16, 16), (64, 32), (16, 16, 16), (32, 16, 16), (64, 64, 64)])
def test_stencils_match_oracle_spgemm_bitwise(shape):
    nlevel = 3
    c = _cfg(shape, nlevel=nlevel)
    levels = mg.describe(c)
    o = O.Oracle.fd(shape, mg.MultigridParameters(nlevel=nlevel), 25.0, galerkin=0 if np.prod(shape) < 70000 else 1)
    for lev, d in enumerate(levels):
        A = o.csr_matrix(lev)
        lat = mg.Lattice(*d["shape"])
        assert A.shape[0] == d["ndof"] == lat.Nvertex
        assert d["npoints"] == (2 * lat.dim + 1 if lev == 0 else 3 ** lat.dim)
        assert d["ncolours"] == (2 if lev == 0 else 2 ** lat.dim)
        # interior row (2,2[,2]) of the oracle matrix vs the device stencil
        r = lat.vertexidx_euclidean2linear([2] * lat.dim)
        row = A.getrow(r)
        got = {}
        for col, v in zip(row.indices, row.data):
            idx = lat.vertexidx_linear2euclidean(int(col))
            k = sum((idx[dd] - 2 + 1) * 3 ** dd for dd in range(lat.dim))
            got[k] = v
        for k in range(3 ** lat.dim):
            assert d["stencil"][k] == got.get(k, 0.0), f"level {lev} offset {k}"


@pytest.mark.parametrize("shape,nlevel", [
    ((512, 512, 512), 7),   # BASELINE config 4 (bench.py's hierarchy)
    ((256, 256, 256), 6),   # configs 3 and 5 (the prior part of the posterior operator)
    ((1024, 1024), 5),      # config 2
    ((64, 64), 4),          # config 1's lattice size with the template's nlevel
    ((128, 128, 128), 5),
])
def test_full_size_hierarchy_stencils_match_oracle_rap(shape, nlevel):
    """Every level of BASELINE's hierarchies, at their real h: the device's stencil-algebra RAP
    (mgmc_hierarchy.cpp galerkin_stencil) equals the oracle's own R*A*R^T (linear_operator.cc:10-23),
    formed by SpGEMM from the oracle's FD row (shiftedlaplace_fd_operator.cc:9-57), bit for bit.
    No device stencil is fed to the oracle."""
    levels = mg.describe(_cfg(shape, nlevel=nlevel))
    ref = O.fd_level_stencils(shape, mg.MultigridParameters(nlevel=nlevel), 25.0)
    assert len(levels) == nlevel
    for lev, d in enumerate(levels):
        assert np.array_equal(d["stencil"], ref[lev]), f"level {lev}: {d['stencil']} != {ref[lev]}"


def test_oracle_level_stencils_equal_its_assembled_hierarchy():
    """orc_fd_level_stencils (no level assembled) equals the interior rows of the oracle's full
    SpGEMM hierarchy (galerkin=0), so it is the same RAP the small-size tests pin."""
    shape, nlevel = (32, 32, 32), 4
    p = mg.MultigridParameters(nlevel=nlevel)
    ref = O.fd_level_stencils(shape, p, 25.0)
    o = O.Oracle.fd(shape, p, 25.0, galerkin=0)
    for lev in range(nlevel):
        n = shape[0] >> lev
        lat = mg.Lattice(n, n, n)
        r = lat.vertexidx_euclidean2linear([2, 2, 2])
        cols, vals = o.csr_row(lev, r)
        got = np.zeros(27)
        for c, v in zip(cols, vals):
            i = lat.vertexidx_linear2euclidean(int(c))
            got[sum((i[dd] - 2 + 1) * 3 ** dd for dd in range(3))] = v
        assert np.array_equal(got, ref[lev]), f"level {lev}"


def test_parameters_template_parses():
    from multigridmc_amd.parameters import (ConstantCorrelationLengthModelParameters, GeneralParameters,
                                            LatticeParameters, MeasurementParameters, MultigridParameters,
                                            SamplingParameters, read_config)
    cfg = read_config(os.path.join(GOLDEN, "parameters_template.cfg"))
    g = GeneralParameters.from_config(cfg)
    assert g.dim == 2 and g.operator_name == "posterior" and g.do_multigridmc
    lat = LatticeParameters.from_config(cfg)
    assert (lat.nx, lat.ny, lat.nz) == (32, 32, 32)
    m = MultigridParameters.from_config(cfg)
    assert (m.smoother, m.coarse_solver, m.nlevel, m.cycle, m.omega) == ("SOR", "SSOR", 4, 2, 1.0)
    s = SamplingParameters.from_config(cfg)
    assert (s.nsamples, s.nwarmup, s.nstepsconvergence, s.nsamplesconvergence) == (10000, 1000, 16, 1000)
    assert ConstantCorrelationLengthModelParameters.from_config(cfg).kappa_sq == pytest.approx(25.0)
    meas = MeasurementParameters.from_config(cfg, base_dir=GOLDEN)
    assert meas.dim == 2 and meas.n == 8 and len(meas.measurement_locations) == 8
    assert meas.measurement_locations[0] == [0.29024507839949776, 0.4429559665392171]
    assert meas.variance[7] == 1.864273250664901e-06


def test_missing_measurements_file_fails_like_the_reference(tmp_path, monkeypatch, capsys):
    """parameters.cc:268-276: a measurements file that cannot be opened is an error (message, exit -1),
    never a posterior with zero measurements.  The name is tried relative to the working directory
    first (the reference's readFile), then next to the configuration file."""
    from multigridmc_amd import driver
    from multigridmc_amd.parameters import MeasurementFileError, MeasurementParameters, read_config
    text = open(os.path.join(GOLDEN, "parameters_template.cfg")).read()
    cfg_path = tmp_path / "p.cfg"
    cfg_path.write_text(text.replace('"measurements_template.cfg"', '"no_such_measurements.cfg"'))
    cfg = read_config(str(cfg_path))
    with pytest.raises(MeasurementFileError, match="ERROR opening configuration file with measurements"):
        MeasurementParameters.from_config(cfg, base_dir=str(tmp_path))
    monkeypatch.chdir(tmp_path)
    assert driver.main([str(cfg_path)]) == -1
    assert "no_such_measurements.cfg" in capsys.readouterr().err
    # working directory first: a file of that name in the cwd wins over the config directory
    sub = tmp_path / "cfgdir"
    sub.mkdir()
    (sub / "p.cfg").write_text(text)
    other = open(os.path.join(GOLDEN, "measurements_template.cfg")).read().replace("n =  8;", "n =  7;")
    (tmp_path / "measurements_template.cfg").write_text(other)
    meas = MeasurementParameters.from_config(read_config(str(sub / "p.cfg")), base_dir=str(sub))
    assert meas.n == 7
    (tmp_path / "measurements_template.cfg").unlink()
    (sub / "measurements_template.cfg").write_text(open(os.path.join(GOLDEN, "measurements_template.cfg")).read())
    meas = MeasurementParameters.from_config(read_config(str(sub / "p.cfg")), base_dir=str(sub))
    assert meas.n == 8


def test_measurement_vector_index():
    """radius-0 QoI (measured_operator.cc:74-91): 2D 64^2 [0.5,0.5] -> (32,32); 3D 512^3 -> (256,256,256)."""
    lat = mg.Lattice2d(64, 64)
    assert lat.vertexidx_linear2euclidean(mg.measurement_vector_index(lat, [0.5, 0.5])) == (32, 32)
    lat3 = mg.Lattice3d(512, 512, 512)
    assert lat3.vertexidx_linear2euclidean(mg.measurement_vector_index(lat3, [0.5, 0.5, 0.5])) == (256, 256, 256)
    # brute force on a small lattice, reference loop semantics (first strict minimum)
    lat = mg.Lattice2d(8, 6)
    x0 = (0.37, 0.61)
    best, dmin = 0, 2.0
    for ell in range(lat.Nvertex):
        c = lat.vertex_coordinates(ell)
        dist = np.sqrt(sum((c[d] - x0[d]) ** 2 for d in range(2)))
        if dist < dmin:
            best, dmin = ell, dist
    assert mg.measurement_vector_index(lat, x0) == best


def test_merge_moments_matches_pooled():
    rng = np.random.default_rng(3)
    chunks = [rng.standard_normal(n) + k for k, n in enumerate([10, 1, 57, 0, 300])]
    parts = [moments_of(c) for c in chunks]
    n, mean, m2 = merge_moments(parts)
    allv = np.concatenate(chunks)
    assert n == allv.size
    assert mean == pytest.approx(allv.mean(), rel=1e-13)
    assert m2 / n == pytest.approx(allv.var(), rel=1e-12)


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from multigridmc_amd.distributed import moments_of, pooled_statistics
    series = np.random.default_rng(100 + rank).standard_normal(1000 + 10 * rank) * (1 + rank)
    stats = pooled_statistics(moments_of(series))
    q.put((rank, stats))
    dist.barrier()
    dist.destroy_process_group()


def test_pooled_statistics_gloo_world2():
    import socket

    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    allv = np.concatenate([np.random.default_rng(100 + r).standard_normal(1000 + 10 * r) * (1 + r) for r in range(2)])
    for r in range(2):
        assert res[r]["chains"] == 2
        assert res[r]["n"] == allv.size
        assert res[r]["mean"] == pytest.approx(allv.mean(), rel=1e-12)
        assert res[r]["variance"] == pytest.approx(allv.var(), rel=1e-12)


@pytest.mark.parametrize("asan", [False, True])
def test_cpp_host_side_describe_and_loud_failure(tmp_path, asan):
    """include/mgmc_sampler.hh compiles with g++ against the C-ABI library (also with AddressSanitizer
    and UBSan on the client); the host-only path matches mgmc_describe through ctypes, and on a host
    without a GPU constructing the sampler prints the library error and exits with -1 (the
    reference's error convention, multigridmc_sampler.cc:47-49)."""
    import subprocess
    from tests.cpp_client import build_client
    exe = build_client(tmp_path, asan=asan)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    out = subprocess.run([exe, "describe"], capture_output=True, text=True, check=True, env=env).stdout.split("\n")
    assert out[0] == "abi 5"
    cfg_levels = mg.describe(mg.make_config(mg.ShiftedLaplaceFDOperator(mg.Lattice3d(64, 64, 64), 25.0),
                                            mg.MultigridParameters(nlevel=4)))
    for level, line in enumerate(out[1:5]):
        tok = line.split()
        assert int(tok[5]) == cfg_levels[level]["ndof"]
        assert float(tok[11]) == cfg_levels[level]["stencil"][13]
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(0)
    if hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0:
        return
    r = subprocess.run([exe, "sample", "2"], capture_output=True, text=True, env=env)
    assert r.returncode == 255 and "ERROR: mgmc_create failed" in r.stderr


class _FakeChain:
    """Stands in for a device sampler in bench.Collectives.  mode: "rehearsal" / "shared" = both ranks
    report one PCI bus id (with / without MGMC_BENCH_DEVICE); "init_fails" = distinct devices, the
    communicator cannot be created; "short" = it is created but spans one rank; "ok" = it works (its
    collectives are simulated over the gloo group, like RCCL would compute them)."""

    def __init__(self, rank, mode):
        self.rank, self.mode, self.comm = rank, mode, False

    def comm_info(self):
        shared = self.mode in ("rehearsal", "shared")
        n = {"ok": 2, "short": 1}.get(self.mode, 0) if self.comm else 0
        return {"rccl_ranks": n, "rccl_rank": self.rank if self.comm else -1,
                "pci_bus_id": 7 if shared else 7 + self.rank}

    def comm_init(self, world, rank, uid):
        assert len(uid) == 128
        if self.mode == "init_fails":
            raise mg.MgmcError(-2, "RCCL error invalid usage (test)")
        self.comm = True

    def synchronize(self):
        pass

    nchains = 2

    def qoi_moments(self, chain=0):
        return np.array([10.0 + self.rank + chain, 0.5 * self.rank, 2.0])

    def comm_barrier(self):
        import torch.distributed as dist
        dist.barrier()

    def comm_allreduce_max(self, v):
        import torch.distributed as dist
        out = [None, None]
        dist.all_gather_object(out, v)
        return max(out)

    def comm_allgather_moments(self, world):
        import torch.distributed as dist
        out = [None] * world
        dist.all_gather_object(out, [list(self.qoi_moments(c)) for c in range(self.nchains)])
        return np.array(out).reshape(-1, 3)


def _bench_coll_worker(rank, world, port, mode, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if mode == "rehearsal":
        os.environ["MGMC_BENCH_DEVICE"] = "0"
    import torch.distributed as dist
    import bench
    bench.mg.comm_unique_id = lambda: bytes(128)
    try:
        c = bench.Collectives(_FakeChain(rank, mode), rank, world)
    except (bench.CommError, mg.MgmcError) as e:
        q.put((rank, type(e).__name__, str(e), None, None, None))
        dist.barrier()
        dist.destroy_process_group()
        return
    c.barrier()
    q.put((rank, c.kind, c.rccl_ranks, c.max(1.0 + rank), c.allgather_moments().tolist(), None))
    c.dist.barrier()
    c.dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["rehearsal", "ok", "shared", "init_fails", "short"])
def test_bench_collectives_world2(mode):
    """bench.py's N > 1 collectives (barrier, max time, per-chain moments, world_size 2 on gloo):
    RCCL on distinct devices reports collectives "rccl" and the communicator's rank count; ranks
    sharing a device run gloo collectives only as an explicit rehearsal (MGMC_BENCH_DEVICE); a
    shared device without it, a communicator that fails, or one that spans fewer ranks is an error
    on every rank (bench.main exits non-zero), never a silent gloo fallback."""
    import socket

    import torch.multiprocessing as tmp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_coll_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        if mode in ("rehearsal", "ok"):
            kind, nranks, tmax, parts, _ = res[r]
            assert kind == ("gloo" if mode == "rehearsal" else "rccl")
            assert nranks == (0 if mode == "rehearsal" else 2)
            assert tmax == 2.0
            # every chain of every rank, rank-major (2 chains per rank)
            assert parts == [[10.0, 0.0, 2.0], [11.0, 0.0, 2.0], [11.0, 0.5, 2.0], [12.0, 0.5, 2.0]]
        else:
            err, msg = res[r][0], res[r][1]
            assert err == ("MgmcError" if mode == "init_fails" else "CommError"), (err, msg)
            if mode == "shared":
                assert "share GPUs" in msg
            if mode == "short":
                assert "spans 1 ranks" in msg


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("mode", ["shared", "rehearsal", "distinct"])
def test_bench_world2_through_torchrun(mode):
    """the driver's N > 1 launch line itself --
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1
    --master-port P bench.py --gpus 2 --steps K --warmup W -- end to end through bench.main() on two
    gloo ranks (tests/bench_rehearsal.py stands in only for the device sampler).  Ranks sharing one
    device without MGMC_BENCH_DEVICE exit 2 ("share GPUs"); with it they rehearse on gloo collectives
    and the line says so; on distinct devices the line reports the RCCL communicator's 2 ranks.  The
    JSON line's value is the whole job's rate (2 chains x K / max-over-ranks time)."""
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("MGMC_BENCH_DEVICE", None)
    env["MGMC_FAKE_MODE"] = "distinct" if mode == "distinct" else "shared"
    if mode == "rehearsal":
        env["MGMC_BENCH_DEVICE"] = "0"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "bench_rehearsal.py"),
           "--gpus", "2", "--steps", "6", "--warmup", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, cwd=ROOT, timeout=240)
    if mode == "shared":
        assert r.returncode != 0
        assert "share GPUs" in r.stderr and "(exitcode: 2)" in r.stderr  # bench.main's sys.exit(2)
        return
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 6 and line["warmup"] == 2 and line["scaling"] == "weak"
    assert line["config"]["chains"] == 2
    assert line["config"]["collectives"] == ("gloo" if mode == "rehearsal" else "rccl")
    assert line["config"]["rccl_ranks"] == (0 if mode == "rehearsal" else 2)
    assert line["n_devices"] == (1 if mode == "rehearsal" else 2)
    assert line["qoi"]["chains"] == 2 and line["qoi"]["samples"] == 12
    assert line["value"] == pytest.approx(12 / (6 * line["ms_per_step"] / 1e3), rel=1e-3)
    assert line["cpu_baseline"] is None  # rank 0 at N = 1 only
