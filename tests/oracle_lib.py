"""ctypes wrapper of the CPU oracle (oracle/refcpu.cpp -> oracle/build/liboracle.so).

TEST INFRASTRUCTURE: used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker / CPU baseline -- never by the product path."""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")

FAITHFUL = 0
MULTICOLOUR = 1


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("dim", c_int), ("nx", c_int), ("ny", c_int), ("nz", c_int),
        ("nlevel", c_int), ("cycle", c_int), ("npresmooth", c_int), ("npostsmooth", c_int),
        ("ncoarsesmooth", c_int), ("smoother", c_int), ("coarse_solver", c_int), ("galerkin", c_int),
        ("omega", c_double), ("coarse_scaling", c_double), ("kappa_sq", c_double),
    ]


_DP = POINTER(c_double)
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
        L = ctypes.CDLL(LIB)
        sigs = {
            "orc_create_fd": (c_void_p, [POINTER(OrcParams), c_int, c_uint64, c_uint64, _DP]),
            "orc_fd_level_stencils": (c_int, [POINTER(OrcParams), _DP]),
            "orc_create_fem": (c_void_p, [POINTER(OrcParams), c_int, c_uint64, c_uint64, _DP]),
            "orc_create_csr": (c_void_p, [POINTER(OrcParams), c_int, c_uint64, c_int64, POINTER(c_int64),
                                          POINTER(c_int32), _DP]),
            "orc_destroy": (None, [c_void_p]),
            "orc_set_threads": (None, [c_int]),
            "orc_set_chol_blocked": (None, [c_int]),
            "orc_set_no_fold": (None, [c_int]),
            "orc_get_threads": (c_int, []),
            "orc_ndof": (c_int64, [c_void_p, c_int]),
            "orc_nlevel": (c_int, [c_void_p]),
            "orc_nnz": (c_int64, [c_void_p, c_int]),
            "orc_get_csr": (None, [c_void_p, c_int, POINTER(c_int64), POINTER(c_int32), _DP]),
            "orc_get_row": (c_int64, [c_void_p, c_int, c_int64, POINTER(c_int32), _DP]),
            "orc_set_rhs": (None, [c_void_p, _DP]),
            "orc_set_state": (None, [c_void_p, _DP]),
            "orc_get_state": (None, [c_void_p, _DP]),
            "orc_set_sample_index": (None, [c_void_p, c_uint64]),
            "orc_sor_smoother_apply": (None, [c_void_p, c_int, c_int, c_int, _DP, _DP]),
            "orc_ssor_smoother_apply": (None, [c_void_p, c_int, c_int, _DP, _DP]),
            "orc_reseed": (None, [c_void_p, c_uint64, c_uint64]),
            "orc_operator_nnz": (c_int64, [c_int, POINTER(c_int), c_int, c_int, c_double, c_double, c_double]),
            "orc_operator_csr": (None, [c_int, POINTER(c_int), c_int, c_int, c_double, c_double, c_double,
                                        POINTER(c_int64), POINTER(c_int32), _DP]),
            "orc_apply": (None, [c_void_p, _DP, _DP]),
            "orc_sample": (None, [c_void_p, c_int, c_int64, _DP]),
            "orc_time_samples": (c_double, [c_void_p, c_int]),
            "orc_operator_apply": (None, [c_void_p, c_int, _DP, _DP]),
            "orc_mean_cov": (None, [c_void_p, _DP, c_int, c_int64, _DP, _DP]),
            "orc_smoother_apply": (None, [c_void_p, c_int, c_int, c_int, _DP, _DP]),
            "orc_sor_sampler_apply": (None, [c_void_p, c_int, c_int, c_uint32, c_uint64, _DP, _DP]),
            "orc_restrict": (None, [c_void_p, c_int, _DP, _DP]),
            "orc_prolongate_add": (None, [c_void_p, c_int, c_double, _DP, _DP]),
            "orc_residual_restrict": (None, [c_void_p, c_int, _DP, _DP, _DP]),
            "orc_set_lowrank": (None, [c_void_p, c_int, POINTER(c_int64), POINTER(c_int64), _DP, _DP]),
            "orc_lowrank_nnz": (c_int64, [c_void_p, c_int]),
            "orc_get_lowrank": (None, [c_void_p, c_int, POINTER(c_int64), POINTER(c_int64), _DP]),
            "orc_philox_normals": (None, [c_uint64, c_uint64, c_uint64, c_int64, c_uint32, c_uint64, _DP]),
            "orc_blocked_dot": (c_double, [c_int64, POINTER(c_int64), _DP, _DP]),
            "orc_philox_raw": (None, [POINTER(c_uint32), c_uint32, c_uint32, POINTER(c_uint32)]),
            "orc_ln_unit": (c_double, [c_double]),
            "orc_cos_sin_2pi": (None, [c_double, _DP, _DP]),
            "orc_mt_normals": (None, [c_uint64, c_int64, _DP]),
            "orc_lattice_fine_vertex_idx": (c_int64, [c_int, POINTER(c_int), c_int64]),
            "orc_lattice_lin2euc": (None, [c_int, POINTER(c_int), c_int64, POINTER(c_int)]),
            "orc_lattice_euc2lin": (c_int64, [c_int, POINTER(c_int), POINTER(c_int)]),
            "orc_lattice_shift": (c_int64, [c_int, POINTER(c_int), c_int64, POINTER(c_int)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_DP)


def ivec(v):
    arr = (c_int * len(v))(*v)
    return arr


def params_struct(shape, mg, kappa_sq: float, galerkin: int = 0) -> OrcParams:
    p = OrcParams()
    p.dim = len(shape)
    p.nx = shape[0]
    p.ny = shape[1] if len(shape) > 1 else 0
    p.nz = shape[2] if len(shape) > 2 else 0
    p.nlevel = mg.nlevel
    p.cycle = mg.cycle
    p.npresmooth = mg.npresmooth
    p.npostsmooth = mg.npostsmooth
    p.ncoarsesmooth = mg.ncoarsesmooth
    p.smoother = {"SOR": 0, "SSOR": 1}[mg.smoother]
    p.coarse_solver = {"SSOR": 0, "Cholesky": 1}[mg.coarse_solver]
    p.galerkin = galerkin
    p.omega = mg.omega
    p.coarse_scaling = mg.coarse_scaling
    p.kappa_sq = kappa_sq
    return p


class Oracle:
    """One oracle MGMC chain (FAITHFUL = reference algorithm, MULTICOLOUR = device replay)."""

    def __init__(self, handle, params):
        self.h = handle
        self.params = params
        self.L = lib()

    @classmethod
    def fd(cls, shape, mg, kappa_sq, mode=FAITHFUL, seed=5418513, chain=0, galerkin=0, override_stencils=None):
        p = params_struct(shape, mg, kappa_sq, galerkin)
        st = None
        if override_stencils is not None:
            override_stencils = np.ascontiguousarray(override_stencils, dtype=np.float64)
            st = dp(override_stencils)
        h = lib().orc_create_fd(ctypes.byref(p), mode, seed, chain, st)
        return cls(h, p)

    @classmethod
    def fd_own(cls, shape, mg, kappa_sq, mode=MULTICOLOUR, seed=5418513, chain=0):
        """FD hierarchy with the oracle's OWN Galerkin levels (no device stencil fed in): the full
        SpGEMM R*A*R^T (linear_operator.cc:10-23) up to 2^18 fine unknowns, above that the
        stencil-mode RAP (galerkin=1: SpGEMM on an 8^d lattice from the full-size FD row), which
        tests/test_oracle.py pins to the full SpGEMM and tests/test_host.py to every level of
        BASELINE's hierarchies."""
        big = int(np.prod([n - 1 for n in shape])) > (1 << 18)
        return cls.fd(shape, mg, kappa_sq, mode=mode, seed=seed, chain=chain, galerkin=1 if big else 0)

    @classmethod
    def fem(cls, shape, mg, kappa_sq, mode=FAITHFUL, seed=5418513, chain=0, override_stencils=None):
        """ShiftedLaplaceFEMOperator prior (constant kappa^2); override_stencils replaces the
        Galerkin stencils of levels >= 1 (multicolour replay of a device hierarchy)."""
        p = params_struct(shape, mg, kappa_sq, 0)
        st = None
        if override_stencils is not None:
            override_stencils = np.ascontiguousarray(override_stencils, dtype=np.float64)
            st = dp(override_stencils)
        h = lib().orc_create_fem(ctypes.byref(p), mode, seed, chain, st)
        o = cls(h, p)
        o._st = override_stencils  # keep the buffer alive
        return o

    @classmethod
    def csr(cls, shape, mg, rowptr, col, val, mode=FAITHFUL, seed=0):
        p = params_struct(shape, mg, 0.0)
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        val = np.ascontiguousarray(val, dtype=np.float64)
        h = lib().orc_create_csr(ctypes.byref(p), mode, seed, len(rowptr) - 1,
                                 rowptr.ctypes.data_as(POINTER(c_int64)), col.ctypes.data_as(POINTER(c_int32)),
                                 dp(val))
        if not h:
            raise ValueError("the multicolour order needs a 2D / 3D lattice")
        return cls(h, p)

    def __del__(self):
        try:
            if self.h:
                self.L.orc_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def ndof(self, level=0):
        return int(self.L.orc_ndof(self.h, level))

    def csr_matrix(self, level=0):
        import scipy.sparse as sp
        n = self.ndof(level)
        nnz = int(self.L.orc_nnz(self.h, level))
        rowptr = np.empty(n + 1, dtype=np.int64)
        col = np.empty(nnz, dtype=np.int32)
        val = np.empty(nnz)
        self.L.orc_get_csr(self.h, level, rowptr.ctypes.data_as(POINTER(c_int64)),
                           col.ctypes.data_as(POINTER(c_int32)), dp(val))
        return sp.csr_matrix((val, col, rowptr), shape=(n, n))

    def csr_row(self, level, row):
        """(columns, values) of one row of a level's CSR, without copying the matrix."""
        col = np.empty(27, dtype=np.int32)
        val = np.empty(27)
        k = int(self.L.orc_get_row(self.h, level, row, col.ctypes.data_as(POINTER(c_int32)), dp(val)))
        return col[:k].copy(), val[:k].copy()

    def apply(self, f, x):
        f = np.ascontiguousarray(f, dtype=np.float64)
        self.L.orc_apply(self.h, dp(f), dp(x))

    def set_rhs(self, f):
        f = np.ascontiguousarray(f, dtype=np.float64)
        self.L.orc_set_rhs(self.h, dp(f))

    def set_state(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        self.L.orc_set_state(self.h, dp(x))

    def set_sample_index(self, index):
        self.L.orc_set_sample_index(self.h, int(index))

    def get_state(self):
        x = np.empty(self.ndof())
        self.L.orc_get_state(self.h, dp(x))
        return x

    def sample(self, nsteps, qoi=-1):
        out = np.empty(max(nsteps, 0))
        self.L.orc_sample(self.h, nsteps, qoi, dp(out) if qoi >= 0 else None)
        return out

    def time_samples(self, nsteps):
        return float(self.L.orc_time_samples(self.h, nsteps))

    def mean_cov(self, f, nwarmup, nsamples):
        f = np.ascontiguousarray(f, dtype=np.float64)
        n = self.ndof()
        ex = np.empty(n)
        exx = np.empty((n, n))
        self.L.orc_mean_cov(self.h, dp(f), nwarmup, nsamples, dp(ex), dp(exx))
        return ex, exx - np.outer(ex, ex)

    def operator_apply(self, level, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.empty(self.ndof(level))
        self.L.orc_operator_apply(self.h, level, dp(x), dp(y))
        return y

    def smoother_apply(self, level, direction, nsweeps, b, x):
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self.L.orc_smoother_apply(self.h, level, direction, nsweeps, dp(b), dp(out))
        return out

    def sor_smoother_apply(self, level, direction, nsmooth, b, x):
        """SORSmoother::apply with the reference's nesting: nsmooth x (nsmooth sweeps, low-rank fix)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self.L.orc_sor_smoother_apply(self.h, level, direction, nsmooth, dp(b), dp(out))
        return out

    def ssor_smoother_apply(self, level, nsmooth, b, x):
        """SSORSmoother::apply: nsmooth x (forward + fix, backward + fix)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self.L.orc_ssor_smoother_apply(self.h, level, nsmooth, dp(b), dp(out))
        return out

    def sor_sampler_apply(self, level, direction, tag, sample, f, x):
        f = np.ascontiguousarray(f, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self.L.orc_sor_sampler_apply(self.h, level, direction, tag, sample, dp(f), dp(out))
        return out

    def restrict(self, level, r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        out = np.empty(self.ndof(level + 1))
        self.L.orc_restrict(self.h, level, dp(r), dp(out))
        return out

    def prolongate_add(self, level, alpha, xc, x):
        xc = np.ascontiguousarray(xc, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self.L.orc_prolongate_add(self.h, level, alpha, dp(xc), dp(out))
        return out

    def set_lowrank(self, lr):
        """lr: multigridmc_amd.measured.LowRankUpdate (B as CSC, Sigma)."""
        self._lr = lr  # keep the arrays alive for the call
        P = POINTER(c_int64)
        self.L.orc_set_lowrank(self.h, lr.m, lr.colptr.ctypes.data_as(P), lr.rows.ctypes.data_as(P),
                               dp(lr.vals), dp(lr.sigma))

    def lowrank(self, level):
        """(colptr, rows, vals) of B on a level (B_c = R B on coarse levels)."""
        m = len(self._lr.sigma)
        nnz = int(self.L.orc_lowrank_nnz(self.h, level))
        colptr = np.empty(m + 1, dtype=np.int64)
        rows = np.empty(nnz, dtype=np.int64)
        vals = np.empty(nnz)
        P = POINTER(c_int64)
        self.L.orc_get_lowrank(self.h, level, colptr.ctypes.data_as(P), rows.ctypes.data_as(P), dp(vals))
        return colptr, rows, vals

    def residual_restrict(self, level, f, x):
        f = np.ascontiguousarray(f, dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=np.float64)
        out = np.empty(self.ndof(level + 1))
        self.L.orc_residual_restrict(self.h, level, dp(f), dp(x), dp(out))
        return out


def fold_level(desc) -> bool:
    """A level whose residual the device (and the MULTICOLOUR oracle) sums class-folded (fold27,
    mgmc_kernels.hpp): 3D, 27-point, bitwise reflection-symmetric stencil (desc = level_desc(l))."""
    st = np.ascontiguousarray(desc["stencil"], dtype=np.float64)
    if len(desc["shape"]) != 3 or desc["npoints"] != 27:
        return False
    b = st.view(np.uint64).reshape(3, 3, 3)
    return bool(np.array_equal(b, b[::-1]) and np.array_equal(b, b[:, ::-1]) and np.array_equal(b, b[:, :, ::-1]))


def residual_tolerance_ok(got, faithful, A, f, x, R, rtol=1e-14):
    """|got - faithful| <= rtol * R (|f| + |A| |x|) elementwise: the fold levels' residual (a different
    summation order from the reference's CSR SpMV) agrees with it to rounding.  R: the restriction as a
    function of a fine vector (the FAITHFUL oracle's restrict)."""
    scale = R(np.abs(f) + abs(A) @ np.abs(x))
    return bool(np.all(np.abs(got - faithful) <= rtol * scale))


def fd_level_stencils(shape, mg, kappa_sq) -> np.ndarray:
    """The oracle's own (nlevel, 27) stencils of an FD hierarchy: the reference FD row at full size,
    then R*A*R^T by SpGEMM per level (the galerkin=1 construction), without assembling any level."""
    p = params_struct(shape, mg, kappa_sq, 1)
    out = np.empty((mg.nlevel, 27))
    if lib().orc_fd_level_stencils(ctypes.byref(p), dp(out)) != 0:
        raise ValueError(f"lattice {shape} too small")
    return out


def operator_csr(shape, pde, periodic=False, Lambda=0.2, Lambda_min=0.2, Lambda_max=0.4):
    """The oracle's own assembly of the reference's fine operators (pde 0 FD, 1 FEM, 2 squared FD)
    with the constant (Lambda) or periodic (Lambda_min, Lambda_max) correlation-length model."""
    n = (c_int * 3)(*(list(shape) + [0] * (3 - len(shape))))
    args = (len(shape), n, int(pde), 1 if periodic else 0, float(Lambda), float(Lambda_min), float(Lambda_max))
    nnz = lib().orc_operator_nnz(*args)
    nrow = int(np.prod([v - 1 for v in shape]))
    rowptr = np.empty(nrow + 1, dtype=np.int64)
    col = np.empty(nnz, dtype=np.int32)
    val = np.empty(nnz, dtype=np.float64)
    lib().orc_operator_csr(*args, rowptr.ctypes.data_as(POINTER(c_int64)), col.ctypes.data_as(POINTER(c_int32)),
                           dp(val))
    return rowptr, col, val


def set_threads(n: int) -> None:
    """Worker threads of the oracle's row-parallel loops (bitwise the same results; default 1)."""
    lib().orc_set_threads(int(n))


def set_chol_blocked(on: bool) -> None:
    """Coarse Cholesky: the blocked banded solves at any size (the device's MGMC_DISABLE=chol_dense);
    read when an oracle is built."""
    lib().orc_set_chol_blocked(1 if on else 0)


def set_no_fold(on: bool) -> None:
    """No fold levels: residuals of reflection-symmetric 27-point levels in the reference's CSR order
    (the device's MGMC_DISABLE=fold); read when an oracle is built."""
    lib().orc_set_no_fold(1 if on else 0)


def cpu_share() -> int:
    """Cores this process may use (affinity mask, capped by OMP_NUM_THREADS on the GPU box)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def philox_normals(seed, chain, pair0, n, tag, sample):
    out = np.empty(n)
    lib().orc_philox_normals(seed, chain, pair0, n, tag, sample, dp(out))
    return out


def blocked_dot(rows, vals, x):
    """sum_e vals[e] x[rows[e]] in the device's blocked order (refcpu blocked_dot = lr_dot's order)."""
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    x = np.ascontiguousarray(x, dtype=np.float64)
    return float(lib().orc_blocked_dot(len(rows), rows.ctypes.data_as(POINTER(c_int64)), dp(vals), dp(x)))


def philox_raw(ctr, key):
    c = (c_uint32 * 4)(*ctr)
    o = (c_uint32 * 4)()
    lib().orc_philox_raw(c, key[0], key[1], o)
    return list(o)


def mt_normals(seed, n):
    out = np.empty(n)
    lib().orc_mt_normals(seed, n, dp(out))
    return out
