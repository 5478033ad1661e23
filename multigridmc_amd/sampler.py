"""Host-side mirror of the reference's Sampler / Smoother / LinearOperator interfaces, backed by
the HIP C-ABI (include/mgmc.h).

Reference interface shapes (nilsfriess/MultigridMC, src/):
  Lattice2d / Lattice3d ............ lattice/lattice2d.hh, lattice/lattice3d.hh
  ShiftedLaplaceFDOperator ......... linear_operator/shiftedlaplace_fd_operator.{hh,cc}
  MeasuredOperator.measurement_vector (radius 0) .. linear_operator/measured_operator.cc:69-91
  MultigridMCSampler(op, rng, params).apply(f, x) .. sampler/multigridmc_sampler.{hh,cc}
  SORSampler.apply(f, x) ........... sampler/sor_sampler.cc:37-59
  SORSmoother.apply(b, x) .......... smoother/sor_smoother.cc:41-78
  LinearOperator.apply(x, y) ....... linear_operator/linear_operator.hh:66-76

Differences, by design: the reference passes a `std::mt19937_64&`; the device samplers take an
integer seed and a chain id instead (the counter-based noise stream, DESIGN.md "Noise").  Vectors
are numpy float64 arrays in the reference's lexicographic interior-vertex order.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._native import FORWARD, BACKWARD, MgmcConfig, MgmcLevelDesc, check, load_library
from .parameters import MultigridParameters


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _as_f64(a, n: int, name: str) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.shape != (n,):
        raise ValueError(f"{name} must have shape ({n},), got {a.shape}")
    return a


class Lattice:
    """Structured lattice with n cells per direction and (n-1)^d interior vertices."""

    def __init__(self, *n: int):
        if len(n) not in (2, 3):
            raise ValueError("only 2D and 3D lattices are on the device path")
        self.shape = tuple(int(v) for v in n)
        self.dim = len(n)
        self.Nvertex = int(np.prod([v - 1 for v in self.shape]))

    def vertexidx_euclidean2linear(self, idx) -> int:
        ell = 0
        for d in reversed(range(self.dim)):
            if not (0 < idx[d] < self.shape[d]):
                raise IndexError("vertex is not interior")
            ell = ell * (self.shape[d] - 1) + (idx[d] - 1)
        return ell

    def vertexidx_linear2euclidean(self, ell: int):
        out = []
        for d in range(self.dim):
            out.append(ell % (self.shape[d] - 1) + 1)
            ell //= self.shape[d] - 1
        return tuple(out)

    def vertex_coordinates(self, ell: int):
        idx = self.vertexidx_linear2euclidean(ell)
        return tuple(float(idx[d]) * (1.0 / float(self.shape[d])) for d in range(self.dim))

    def get_coarse_lattice(self) -> "Lattice":
        if any(v % 2 for v in self.shape):
            raise ValueError(f"cannot coarsen lattice of size {self.shape} [one of the extents is odd]")
        if any(v // 2 <= 1 for v in self.shape):
            raise ValueError(f"cannot coarsen lattice of size {self.shape} "
                             "[resulting lattice would have no interior vertices]")
        return Lattice(*[v // 2 for v in self.shape])

    def get_info(self) -> str:
        return f"{self.dim}d lattice, {' x '.join(str(v) for v in self.shape)} points, {self.Nvertex} unknowns"


def Lattice2d(nx: int, ny: int) -> Lattice:
    return Lattice(nx, ny)


def Lattice3d(nx: int, ny: int, nz: int) -> Lattice:
    return Lattice(nx, ny, nz)


class ConstantCorrelationLengthModel:
    """kappa^2 = 1 / Lambda^2 everywhere (correlationlength_model.hh:45-66)."""

    kind = _native.KAPPA_CONSTANT

    def __init__(self, Lambda: float):
        self.Lambda = float(Lambda)

    def kappa_sq(self, x=None) -> float:
        import math
        return 1.0 / math.pow(self.Lambda, 2)


class PeriodicCorrelationLengthModel:
    """Lambda(x) = Lambda_1 + Lambda_2 prod_d cos(pi x_d), Lambda_1,2 = (Lambda_max +/- Lambda_min) / 2,
    kappa^2 = 1 / Lambda^2 (correlationlength_model.hh:68-112).  Its operators have per-vertex
    coefficients: they go to the device as matrices (mgmc_create_csr)."""

    kind = _native.KAPPA_PERIODIC

    def __init__(self, Lambda_min: float, Lambda_max: float):
        self.Lambda_min, self.Lambda_max = float(Lambda_min), float(Lambda_max)

    def kappa_sq(self, x) -> float:
        import math
        lam = 0.5 * (self.Lambda_max - self.Lambda_min)
        for v in x:
            lam *= math.cos(math.pi * float(v))
        lam += 0.5 * (self.Lambda_max + self.Lambda_min)
        return 1.0 / (lam * lam)


class ShiftedLaplaceFDOperator:
    """Fine-level precision operator: FD shifted Laplacian (shiftedlaplace_fd_operator.cc:9-57).

    With a constant kappa^2 (a number, or ConstantCorrelationLengthModel) the device consumes the
    operator's data as a constant stencil per level (the reference's LinearOperator::apply is not
    virtual, linear_operator.hh:66); with PeriodicCorrelationLengthModel it consumes the assembled
    matrix (get_csr(), the reference's A_sparse) and builds the Galerkin levels from it."""

    fine_operator = _native.OPERATOR_FD

    def __init__(self, lattice: Lattice, kappa_sq=None, correlation_model=None):
        self.lattice = lattice
        if isinstance(kappa_sq, (ConstantCorrelationLengthModel, PeriodicCorrelationLengthModel)):
            correlation_model, kappa_sq = kappa_sq, None
        if correlation_model is None:
            if kappa_sq is None:
                raise ValueError("need kappa_sq or a correlation-length model")
            self.correlation_model = None
            self.kappa_sq = float(kappa_sq)
        else:
            self.correlation_model = correlation_model
            self.kappa_sq = correlation_model.kappa_sq() if correlation_model.kind == _native.KAPPA_CONSTANT else 0.0
        self._csr = None

    def get_lattice(self) -> Lattice:
        return self.lattice

    def get_ndof(self) -> int:
        return self.lattice.Nvertex

    def get_m_lowrank(self) -> int:
        return 0

    @property
    def variable_coefficients(self) -> bool:
        """True if the device gets the matrix (per-vertex coefficients) instead of a stencil."""
        return self.correlation_model is not None and self.correlation_model.kind != _native.KAPPA_CONSTANT

    def operator_desc(self) -> "_native.MgmcOperatorDesc":
        d = _native.MgmcOperatorDesc()
        lat = self.lattice
        d.dim = lat.dim
        d.nx, d.ny = lat.shape[0], lat.shape[1]
        d.nz = lat.shape[2] if lat.dim == 3 else 0
        d.pde = self.fine_operator
        m = self.correlation_model
        if m is None:
            d.kappa_model = _native.KAPPA_GIVEN
            d.kappa_sq = self.kappa_sq
        elif m.kind == _native.KAPPA_CONSTANT:
            d.kappa_model = _native.KAPPA_CONSTANT
            d.Lambda = m.Lambda
        else:
            d.kappa_model = _native.KAPPA_PERIODIC
            d.Lambda_min, d.Lambda_max = m.Lambda_min, m.Lambda_max
        return d

    def get_csr(self):
        """A_sparse as (rowptr int64, col int32, val float64), assembled by the library's host code
        in the reference's arithmetic (mgmc_operator_csr); cached."""
        if self._csr is None:
            lib = load_library()
            d = self.operator_desc()
            nrow, nnz = ctypes.c_int64(), ctypes.c_int64()
            check(lib.mgmc_operator_csr_size(ctypes.byref(d), ctypes.byref(nrow), ctypes.byref(nnz)))
            rowptr = np.empty(nrow.value + 1, dtype=np.int64)
            col = np.empty(nnz.value, dtype=np.int32)
            val = np.empty(nnz.value, dtype=np.float64)
            check(lib.mgmc_operator_csr(ctypes.byref(d), rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                        col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _dp(val)))
            self._csr = (rowptr, col, val)
        return self._csr

    def matrix(self):
        """A_sparse as a scipy CSR matrix (host)."""
        import scipy.sparse as sp
        rowptr, col, val = self.get_csr()
        n = self.get_ndof()
        return sp.csr_matrix((val, col, rowptr), shape=(n, n))


class ShiftedLaplaceFEMOperator(ShiftedLaplaceFDOperator):
    """Fine-level precision operator: Q1 finite elements for -div grad + kappa^2
    (shiftedlaplace_fem_operator.cc:9-145).  With a constant kappa^2 its interior stencil has 3^d
    points, so the fine level is swept in 2^d colours like the Galerkin levels; R A_h R^T of it is
    the FEM operator of the coarse lattice (test_intergrid.hh:179-206).  With the periodic model the
    matrix goes to the device (kappa^2 at the quadrature points of every cell)."""

    fine_operator = _native.OPERATOR_FEM


class SquaredShiftedLaplaceFDOperator(ShiftedLaplaceFDOperator):
    """(kappa^2 - Laplace)^2 by finite differences, 2D only (squared_shiftedlaplace_fd_operator.cc:9-96):
    a 13-point diamond with homogeneous Neumann corrections on the diagonal.  Always a matrix on the
    device (couplings two vertices apart: the Galerkin levels are 25-point, swept in 3^d colours).
    With a periodic kappa^2 the reference's matrix is not symmetric (the x / y neighbour entries use
    the row vertex's kappa^2); the device sweeps with its rows."""

    fine_operator = _native.OPERATOR_SQUARED_FD

    def __init__(self, lattice: Lattice, kappa_sq=None, correlation_model=None):
        if lattice.dim != 2:
            raise ValueError("SquaredShiftedLaplaceFDOperator only implemented for d=2")
        super().__init__(lattice, kappa_sq, correlation_model)

    @property
    def variable_coefficients(self) -> bool:
        return True


class SparseMatrixOperator(ShiftedLaplaceFDOperator):
    """Any LinearOperator given by its matrix A_sparse (linear_operator.hh:187) on a lattice: CSR with
    interior vertices as rows (x fastest), columns strictly ascending, a positive diagonal and
    couplings at most two vertices apart.  The device takes the matrix path (mgmc_create_csr): the
    Galerkin levels R A R^T are formed on the host, the colouring follows the couplings
    (csr_colour_scheme).  This is what the reference-side adapter feeds from get_sparse()
    (INTEGRATION.md)."""

    def __init__(self, lattice: Lattice, A):
        import scipy.sparse as sp
        A = sp.csr_matrix(A)
        A.sort_indices()
        n = lattice.Nvertex
        if A.shape != (n, n):
            raise ValueError(f"matrix is {A.shape}, the lattice has {n} interior vertices")
        self.lattice = lattice
        self.correlation_model = None
        self.kappa_sq = 0.0
        self._csr = (A.indptr.astype(np.int64), A.indices.astype(np.int32), A.data.astype(np.float64))

    @property
    def variable_coefficients(self) -> bool:
        return True

    def get_csr(self):
        return self._csr

    def constant_stencil(self, config):
        """The 3^d stencil every row of the matrix truncates (mgmc_stencil_of_csr), or None: the
        sampler then builds the stencil hierarchy (mgmc_create_stencil_batch) instead of the matrix
        path -- the fast path for constant-coefficient operators handed over as matrices."""
        lib = load_library()
        rowptr, col, val = self._csr
        st = np.zeros(27)
        rc = lib.mgmc_stencil_of_csr(ctypes.byref(config), len(rowptr) - 1,
                                     rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                     col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _dp(val), _dp(st))
        if rc == _native.MGMC_E_UNSUPPORTED:
            return None
        check(rc)
        return st


def sampler_csr_matrix(rowptr, col, val, n: int):
    """(rowptr, col, val) as a scipy CSR matrix of shape (n, n)."""
    import scipy.sparse as sp
    return sp.csr_matrix((val, col, rowptr), shape=(n, n))


def csr_colour_scheme(lattice: Lattice, rowptr, col, level: int = 0) -> int:
    """Colour classes the device sweeps a matrix level with (mgmc_csr_colour_scheme, host only):
    2 (red-black: all couplings axis neighbours, fine level only), 2^d (coordinate parities) or
    3^d (coordinates mod 3: couplings two vertices apart)."""
    lib = load_library()
    c = MgmcConfig()
    c.dim = lattice.dim
    c.nx, c.ny = lattice.shape[0], lattice.shape[1]
    c.nz = lattice.shape[2] if lattice.dim == 3 else 0
    c.nlevel, c.cycle, c.npresmooth, c.npostsmooth, c.ncoarsesmooth = 1, 1, 1, 1, 1
    c.omega, c.coarse_scaling = 1.0, 1.0
    rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    out = ctypes.c_int()
    check(lib.mgmc_csr_colour_scheme(ctypes.byref(c), int(level), len(rowptr) - 1,
                                     rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                     col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.byref(out)))
    return out.value


def measurement_vector_index(lattice: Lattice, x0, radius: float = 0.0) -> int:
    """Index of the radius-0 measurement vector (measured_operator.cc:74-91): the interior vertex
    nearest to x0.  The distance is separable, so the nearest vertex is found per direction;
    ties go to the lower index, as the reference's strict '<' keeps the first minimum."""
    if radius >= 1e-12:
        raise NotImplementedError("measurement radius > 0 (quadrature) is not on the device path")
    idx = []
    for d in range(lattice.dim):
        n = lattice.shape[d]
        coords = np.arange(1, n, dtype=np.float64) * (1.0 / float(n))
        idx.append(int(np.argmin(np.abs(coords - float(x0[d])))) + 1)
    return lattice.vertexidx_euclidean2linear(idx)


def make_config(linear_operator: ShiftedLaplaceFDOperator, params: MultigridParameters) -> MgmcConfig:
    lat = linear_operator.get_lattice()
    smoother = {"SOR": _native.SMOOTHER_SOR, "SSOR": _native.SMOOTHER_SSOR}.get(params.smoother)
    if smoother is None:
        raise ValueError(f"ERROR: invalid sampler '{params.smoother}'")
    coarse = {"SSOR": _native.COARSE_SSOR, "Cholesky": _native.COARSE_CHOLESKY}.get(params.coarse_solver)
    if coarse is None:
        raise ValueError(f"ERROR: multigrid coarse sampler '{params.coarse_solver}'")
    c = MgmcConfig()
    c.dim = lat.dim
    c.nx, c.ny = lat.shape[0], lat.shape[1]
    c.nz = lat.shape[2] if lat.dim == 3 else 0
    c.nlevel = params.nlevel
    c.cycle = params.cycle
    c.npresmooth = params.npresmooth
    c.npostsmooth = params.npostsmooth
    c.ncoarsesmooth = params.ncoarsesmooth
    c.smoother = smoother
    c.coarse_solver = coarse
    c.verbose = params.verbose
    c.omega = params.omega
    c.coarse_scaling = params.coarse_scaling
    c.kappa_sq = linear_operator.kappa_sq
    base = getattr(linear_operator, "base_operator", linear_operator)
    c.fine_operator = getattr(base, "fine_operator", _native.OPERATOR_FD)
    return c


def describe(config: MgmcConfig) -> list:
    """Host-only: level hierarchy and Galerkin stencils (no GPU touched)."""
    lib = load_library()
    n = check(lib.mgmc_describe(ctypes.byref(config), None, 0))
    out = (MgmcLevelDesc * n)()
    check(lib.mgmc_describe(ctypes.byref(config), out, n))
    levels = []
    for d in out:
        levels.append({
            "shape": (d.nx, d.ny) if config.dim == 2 else (d.nx, d.ny, d.nz),
            "npoints": d.npoints, "ncolours": d.ncolours, "ndof": int(d.ndof),
            "stencil": np.array(d.stencil[:], dtype=np.float64),
        })
    return levels


class MultigridMCSampler:
    """Device MGMC sampler with the reference's Sampler interface (sampler/sampler.hh:23-72).

    apply(f, x) performs one MGMC cycle (multigridmc_sampler.cc:133-138) with x in/out.  The chain
    state and the right hand side stay resident in HBM between calls; apply() moves both across
    PCIe (like the reference's by-reference vectors), sample() runs the device-resident loop."""

    def __init__(self, linear_operator, seed: int, params: MultigridParameters,
                 device: int = 0, chain_id: int = 0, nchains: int = 1):
        """nchains > 1: a batch of independent chains chain_id, chain_id + 1, ... in one handle
        (mgmc_create_batch): every kernel of a cycle covers all of them, chain c draws exactly what a
        one-chain sampler with chain_id + c draws.  set_state / fix_rhs set every chain, get_state,
        sample and qoi_moments take a `chain` argument (default 0; chain=None in sample and get_state
        returns all chains)."""
        self.linear_operator = linear_operator
        self.params = params
        self.seed, self.device, self.chain_id = int(seed), int(device), int(chain_id)
        self.nchains = int(nchains)
        self.config = make_config(linear_operator, params)
        self.lib = load_library()
        h = ctypes.c_void_p()
        base = getattr(linear_operator, "base_operator", linear_operator)
        st = base.constant_stencil(self.config) if isinstance(base, SparseMatrixOperator) else None
        if st is not None:
            # a matrix that is one constant stencil (mgmc_stencil_of_csr): the stencil hierarchy
            check(self.lib.mgmc_create_stencil_batch(ctypes.byref(self.config), _dp(st), int(device),
                                                     int(seed) & (2**64 - 1), int(chain_id) & (2**64 - 1),
                                                     self.nchains, ctypes.byref(h)))
        elif getattr(base, "variable_coefficients", False):
            # per-vertex coefficients: the assembled matrix (A_sparse) and a Galerkin hierarchy of matrices
            rowptr, col, val = base.get_csr()
            check(self.lib.mgmc_create_csr_batch(ctypes.byref(self.config), len(rowptr) - 1,
                                                 rowptr.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                 col.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), _dp(val),
                                                 int(device), int(seed) & (2**64 - 1), int(chain_id) & (2**64 - 1),
                                                 self.nchains, ctypes.byref(h)))
        elif self.nchains == 1:
            check(self.lib.mgmc_create(ctypes.byref(self.config), int(device), int(seed) & (2**64 - 1),
                                       int(chain_id) & (2**64 - 1), ctypes.byref(h)))
        else:
            check(self.lib.mgmc_create_batch(ctypes.byref(self.config), int(device), int(seed) & (2**64 - 1),
                                             int(chain_id) & (2**64 - 1), self.nchains, ctypes.byref(h)))
        self.handle = h
        self.ndof = linear_operator.get_ndof()
        self.nlevel = params.nlevel
        self._fixed_rhs = None   # rhs promised by fix_rhs (apply then skips the upload)
        self._device_rhs = None  # the rhs the device holds (fix_rhs or the last apply); clones copy it
        if linear_operator.get_m_lowrank() > 0:  # MeasuredOperator (measured.py): Q = A + B Sigma^-1 B^T
            self.set_lowrank(linear_operator.get_B())

    def set_lowrank(self, lr):
        """Low-rank part B, Sigma (a measured.LowRankUpdate, or None to drop it); sets up B_bar of
        every level's smoothers (sor_smoother.cc:17-37)."""
        P = ctypes.POINTER(ctypes.c_int64)
        if lr is None or lr.m == 0:
            self._chk(self.lib.mgmc_set_lowrank(self.handle, 0, None, None, None, None))
            self._lowrank = None
            return
        if lr.n != self.ndof:
            raise ValueError(f"B has {lr.n} rows, the operator {self.ndof}")
        self._lowrank = lr  # arrays stay alive for the call
        self._chk(self.lib.mgmc_set_lowrank(self.handle, lr.m, lr.colptr.ctypes.data_as(P), lr.rows.ctypes.data_as(P),
                                            _dp(lr.vals), _dp(lr.sigma)))

    def solve(self, b, method: str = "cg", rtol: float = 1e-12, atol: float = 1e300, maxiter: int = 100):
        """x = Q^{-1} b with the hierarchy as multigrid preconditioner (MultigridPreconditioner,
        preconditioner/multigrid_preconditioner.cc:74-109) in LoopSolver (method="loop",
        solver/loop_solver.cc:9-53) or CG (method="cg").  Returns (x, iterations, ||r||)."""
        m = {"loop": _native.SOLVER_LOOP, "cg": _native.SOLVER_CG}.get(method)
        if m is None:
            raise ValueError(f"unknown solver method '{method}'")
        b = _as_f64(b, self.ndof, "b")
        x = np.empty(self.ndof)
        it = ctypes.c_int()
        rn = ctypes.c_double()
        self._chk(self.lib.mgmc_solve(self.handle, m, _dp(b), _dp(x), float(rtol), float(atol), int(maxiter),
                                      ctypes.byref(it), ctypes.byref(rn)))
        return x, it.value, rn.value

    def lowrank_info(self, level: int, direction: int):
        """(m, rows stored for B_bar of this level and sweep direction)"""
        m = ctypes.c_int()
        n = ctypes.c_int64()
        self._chk(self.lib.mgmc_lowrank_info(self.handle, int(level), int(direction), ctypes.byref(m), ctypes.byref(n)))
        return m.value, n.value

    # -- lifetime --
    def close(self):
        if getattr(self, "handle", None):
            self.lib.mgmc_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, code):
        return check(code, self.handle)

    # -- Sampler interface --
    def get_linear_operator(self):
        return self.linear_operator

    def fix_rhs(self, f):
        """Upload f once and keep it resident: later apply() calls use it and do not upload their
        f argument (the promise of Sampler::fix_rhs, sampler.hh:49-56, as CholeskySampler::apply
        keeps g_rhs; include/mgmc_sampler.hh behaves the same)."""
        f = _as_f64(f, self.ndof, "f").copy()
        self._chk(self.lib.mgmc_set_rhs(self.handle, _dp(f), self.ndof))
        self._fixed_rhs = f
        self._device_rhs = f

    def unfix_rhs(self):
        """apply() uploads its f argument again (the device keeps the last rhs until then)."""
        self._fixed_rhs = None

    def apply(self, f, x: np.ndarray):
        """Draw a new sample x (in/out), one MGMC cycle (MultigridMCSampler::apply,
        multigridmc_sampler.cc:132-138).  Without a fixed rhs f is uploaded and used.  After fix_rhs,
        f = None or a vector equal to the fixed one skips the upload; any other f is used, as the
        reference uses the f it is given (MultigridMCSampler keeps Sampler::fix_rhs a no-op), and
        becomes the resident fixed rhs."""
        if not (isinstance(x, np.ndarray) and x.dtype == np.float64 and x.flags.c_contiguous and x.shape == (self.ndof,)):
            raise ValueError("x must be a contiguous float64 array of length ndof")
        if self._fixed_rhs is not None and f is not None and not np.array_equal(_as_f64(f, self.ndof, "f"),
                                                                                 self._fixed_rhs):
            self.fix_rhs(f)
        if self._fixed_rhs is not None:
            self._chk(self.lib.mgmc_set_state(self.handle, _dp(x), self.ndof))
            self._chk(self.lib.mgmc_sample(self.handle, 1, -1, None))
            self._chk(self.lib.mgmc_get_state(self.handle, _dp(x), self.ndof))
            return
        f = _as_f64(f, self.ndof, "f").copy()
        self._chk(self.lib.mgmc_apply(self.handle, _dp(f), _dp(x), self.ndof))
        self._device_rhs = f

    # -- device-resident chain (driver_mgmc.cc:66-94) --
    def set_state(self, x, chain=None):
        """every chain (chain=None) or one chain of a batch"""
        x = _as_f64(x, self.ndof, "x")
        if chain is None:
            self._chk(self.lib.mgmc_set_state(self.handle, _dp(x), self.ndof))
        else:
            self._chk(self.lib.mgmc_set_state_chain(self.handle, int(chain), _dp(x), self.ndof))

    def get_state(self, chain=0) -> np.ndarray:
        """one chain's state; chain=None: an (nchains, ndof) array"""
        if chain is None:
            return np.stack([self.get_state(c) for c in range(self.nchains)])
        x = np.empty(self.ndof)
        self._chk(self.lib.mgmc_get_state_chain(self.handle, int(chain), _dp(x), self.ndof))
        return x

    def sample(self, nsteps: int, qoi_index: int = -1, chain=0) -> np.ndarray:
        """nsteps cycles of every chain; the QoI series of one chain (chain=None: (nchains, nsteps)).
        qoi_index: a vertex, -1 (none) or QOI_VECTOR (the dot with set_qoi_vector's vector)."""
        records = qoi_index >= 0 or qoi_index == _native.QOI_VECTOR
        if chain == 0 or not records:
            out = np.empty(max(nsteps, 0))
            self._chk(self.lib.mgmc_sample(self.handle, int(nsteps), int(qoi_index), _dp(out) if records else None))
            return out
        self._chk(self.lib.mgmc_sample(self.handle, int(nsteps), int(qoi_index), None))
        if chain is None:
            return np.stack([self.get_series(nsteps, c) for c in range(self.nchains)])
        return self.get_series(nsteps, chain)

    def set_qoi_vector(self, rows, vals):
        """The QoI vector b (MeasuredOperator::measurement_vector, radius > 0: measured_operator.cc:92-171)
        for sample(..., QOI_VECTOR): z = b^T x recorded on the device after every cycle (blocked dot
        order).  rows strictly ascending; empty rows remove it."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.float64)
        if rows.shape != vals.shape:
            raise ValueError("rows and vals differ in length")
        self._qv = (rows, vals)
        self._chk(self.lib.mgmc_set_qoi_vector(self.handle, len(rows),
                                               rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)) if len(rows) else None,
                                               _dp(vals) if len(rows) else None))

    def sample_async(self, nsteps: int, qoi_index: int = -1):
        self._chk(self.lib.mgmc_sample_async(self.handle, int(nsteps), int(qoi_index)))

    def synchronize(self):
        self._chk(self.lib.mgmc_synchronize(self.handle))

    def sample_timed(self, nsteps: int, qoi_index: int = -1, stride: int = 1) -> dict:
        """nsteps cycles replayed as [fine pre-sampler | coarse correction | fine post-sampler | QoI]
        graph segments with HIP events on the handle's stream (mgmc_sample_timed_stride: the segments
        of every stride-th cycle and the last are timed, the others replay the plain graph)."""
        tot, pre, post = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        npre, npost = ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.mgmc_sample_timed_stride(self.handle, int(nsteps), int(stride), int(qoi_index),
                                                    ctypes.byref(tot), ctypes.byref(pre), ctypes.byref(npre),
                                                    ctypes.byref(post), ctypes.byref(npost)))
        # the timed cycles: every stride-th and the last (mgmc_sample_timed_stride's selection)
        ncyc = sum(1 for s in range(int(nsteps)) if s % int(stride) == 0 or s == int(nsteps) - 1)
        return {"total_ms": tot.value, "pre_ms": pre.value, "npre": npre.value, "post_ms": post.value,
                "npost": npost.value, "ncycles_timed": ncyc}

    def qoi_moments(self, chain: int = 0):
        out = np.zeros(3)
        self._chk(self.lib.mgmc_qoi_moments_chain(self.handle, int(chain), _dp(out)))
        return out

    def reset_moments(self):
        self._chk(self.lib.mgmc_reset_moments(self.handle))

    def get_series(self, n: int, chain: int = 0) -> np.ndarray:
        """The QoI series of the last sample / sample_async call (waits for this handle's stream)."""
        out = np.empty(max(int(n), 0))
        self._chk(self.lib.mgmc_get_series_chain(self.handle, int(chain), _dp(out), out.size))
        return out

    def clone(self) -> "MultigridMCSampler":
        """A second handle of the same chain: same operator, parameters, device and Philox key
        (seed, chain_id), its own state, right hand side and HIP stream.  With disjoint sample
        indices it reproduces the draws this handle would make there (batched chains)."""
        c = MultigridMCSampler(self.linear_operator, self.seed, self.params, self.device, self.chain_id,
                               self.nchains)
        if self._device_rhs is not None:  # the same right hand side as this handle's device copy
            c.fix_rhs(self._device_rhs)
            if self._fixed_rhs is None:
                c.unfix_rhs()
        return c

    def set_sample_index(self, index: int):
        self._chk(self.lib.mgmc_set_sample_index(self.handle, int(index)))

    def get_sample_index(self) -> int:
        v = ctypes.c_uint64()
        self._chk(self.lib.mgmc_get_sample_index(self.handle, ctypes.byref(v)))
        return v.value

    def level_desc(self, level: int) -> dict:
        d = MgmcLevelDesc()
        self._chk(self.lib.mgmc_level_desc_get(self.handle, int(level), ctypes.byref(d)))
        return {"shape": (d.nx, d.ny, d.nz)[: self.config.dim], "npoints": d.npoints, "ncolours": d.ncolours,
                "ndof": int(d.ndof), "stencil": np.array(d.stencil[:]), "varcoef": bool(d.varcoef)}

    # -- component operations (reference layout host vectors) --
    def level_kernels(self, level: int) -> dict:
        """The kernels the handle runs on a level (mgmc_level_kernels): {"sweep": ..., "post_sweep": ...,
        "residual_restrict": ..., "lowrank": ..., "noise": ...} ("lowrank" on posterior levels: "small",
        "rows", "dense" or "dense,rhs_inplace"; "noise": "restriction", "tail" or "restriction+tail" when sweeps
        of the level read Box-Muller pairs drawn by the restriction launch before them / a tail launch)"""
        buf = ctypes.create_string_buffer(512)
        self._chk(self.lib.mgmc_level_kernels(self.handle, int(level), buf, 512))
        return dict(kv.split("=", 1) for kv in buf.value.decode().split(";"))

    def operator_apply(self, level: int, x) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        x = _as_f64(x, n, "x")
        y = np.empty(n)
        self._chk(self.lib.mgmc_operator_apply(self.handle, level, _dp(x), _dp(y)))
        return y

    def smoother_apply(self, level: int, direction: int, nsweeps: int, b, x) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        b = _as_f64(b, n, "b")
        out = _as_f64(x, n, "x").copy()
        self._chk(self.lib.mgmc_smoother_apply(self.handle, level, direction, nsweeps, _dp(b), _dp(out)))
        return out

    def sor_smoother_apply(self, level: int, direction: int, nsmooth: int, b, x) -> np.ndarray:
        """SORSmoother::apply (sor_smoother.cc:41-53 over apply_sparse :56-78): nsmooth x (nsmooth
        noise-free multicolour sweeps, then the B_bar fix once)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self._chk(self.lib.mgmc_sor_smoother_apply(self.handle, level, direction, nsmooth, _dp(b), _dp(out)))
        return out

    def ssor_smoother_apply(self, level: int, nsmooth: int, b, x) -> np.ndarray:
        """SSORSmoother::apply (ssor_smoother.cc:9-15): nsmooth x (forward sweep + fix, backward + fix)."""
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = np.ascontiguousarray(x, dtype=np.float64).copy()
        self._chk(self.lib.mgmc_ssor_smoother_apply(self.handle, level, nsmooth, _dp(b), _dp(out)))
        return out

    def sor_sampler_apply(self, level: int, direction: int, tag: int, sample_index: int, f, x) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        f = _as_f64(f, n, "f")
        out = _as_f64(x, n, "x").copy()
        self._chk(self.lib.mgmc_sor_sampler_apply(self.handle, level, direction, tag, sample_index, _dp(f), _dp(out)))
        return out

    def restrict(self, level: int, r) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        nc = self.level_desc(level + 1)["ndof"]
        r = _as_f64(r, n, "r")
        out = np.empty(nc)
        self._chk(self.lib.mgmc_restrict(self.handle, level, _dp(r), _dp(out)))
        return out

    def prolongate_add(self, level: int, alpha: float, xc, x) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        nc = self.level_desc(level + 1)["ndof"]
        xc = _as_f64(xc, nc, "xc")
        out = _as_f64(x, n, "x").copy()
        self._chk(self.lib.mgmc_prolongate_add(self.handle, level, float(alpha), _dp(xc), _dp(out)))
        return out

    def residual_restrict(self, level: int, f, x) -> np.ndarray:
        n = self.level_desc(level)["ndof"]
        nc = self.level_desc(level + 1)["ndof"]
        f = _as_f64(f, n, "f")
        x = _as_f64(x, n, "x")
        out = np.empty(nc)
        self._chk(self.lib.mgmc_residual_restrict(self.handle, level, _dp(f), _dp(x), _dp(out)))
        return out

    def normals(self, pair0: int, n: int, tag: int, sample_index: int) -> np.ndarray:
        out = np.empty(n)
        self._chk(self.lib.mgmc_normals(self.handle, int(pair0), int(n), int(tag), int(sample_index), _dp(out)))
        return out

    # -- multi-GPU chains: RCCL communicator owned by the handle --
    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        if len(unique_id) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self._chk(self.lib.mgmc_comm_init(self.handle, int(nranks), int(rank), unique_id))

    def comm_allgather_moments(self, nranks: int) -> np.ndarray:
        """(count, mean, M2) of every chain of every rank: rows rank-major, nranks * nchains of them"""
        out = np.zeros(3 * max(nranks, 1) * self.nchains)
        self._chk(self.lib.mgmc_comm_allgather_moments(self.handle, _dp(out)))
        return out.reshape(-1, 3)

    def comm_allreduce_max(self, value: float) -> float:
        v = ctypes.c_double(value)
        self._chk(self.lib.mgmc_comm_allreduce_max(self.handle, ctypes.byref(v)))
        return v.value

    def comm_barrier(self):
        self._chk(self.lib.mgmc_comm_barrier(self.handle))

    def comm_info(self) -> dict:
        """{'rccl_ranks': ncclCommCount (0 without a communicator), 'rccl_rank', 'pci_bus_id'}"""
        n, r, bus = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._chk(self.lib.mgmc_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r), ctypes.byref(bus)))
        return {"rccl_ranks": n.value, "rccl_rank": r.value, "pci_bus_id": bus.value}

    def comm_destroy(self):
        self._chk(self.lib.mgmc_comm_destroy(self.handle))

    def time_fine_sweeps(self, nsweeps: int) -> float:
        ms = ctypes.c_float()
        self._chk(self.lib.mgmc_time_fine_sweeps(self.handle, int(nsweeps), ctypes.byref(ms)))
        return ms.value


def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0), to be shipped to the other ranks over any host channel."""
    buf = ctypes.create_string_buffer(128)
    check(load_library().mgmc_comm_unique_id(buf))
    return buf.raw


class HipMulticolourSORSmoother:
    """Smoother interface (smoother/smoother.hh:15-34): deterministic multicolour SOR sweep on a
    level of a device hierarchy (the level-0 operator for a one-level sampler)."""

    def __init__(self, sampler: MultigridMCSampler, level: int, direction: int, nsmooth: int = 1):
        self.sampler = sampler
        self.level = level
        self.direction = direction
        self.nsmooth = nsmooth

    def apply(self, b, x: np.ndarray):
        x[:] = self.sampler.smoother_apply(self.level, self.direction, self.nsmooth, b, x)


class _OneLevelSmoother:
    """A Smoother (smoother/smoother.hh:15-34) on its own device handle: the operator as a one-level
    hierarchy (MultigridMCSampler with nlevel 1; a MeasuredOperator's B / Sigma installed, so the
    B_bar fix of sor_smoother.cc:17-51 runs), the state uploaded per apply (host vectors, like the
    reference's Eigen vectors)."""

    def __init__(self, linear_operator, omega: float, device: int):
        self.linear_operator = linear_operator
        self.omega = float(omega)
        p = MultigridParameters(nlevel=1, smoother="SOR", coarse_solver="SSOR", npresmooth=1, npostsmooth=1,
                                ncoarsesmooth=1, omega=self.omega, cycle=1, coarse_scaling=1.0)
        self._s = MultigridMCSampler(linear_operator, 0, p, device=device)

    def close(self):
        self._s.close()

    def _check(self, b, x):
        n = self.linear_operator.get_ndof()
        if len(b) != n or len(x) != n:
            raise ValueError(f"vector sizes {len(b)} / {len(x)}, operator {n}")


class SORSmoother(_OneLevelSmoother):
    """SORSmoother(linear_operator, omega, nsmooth, direction) (smoother/sor_smoother.hh:53-60):
    apply(b, x) is the reference's SORSmoother::apply -- nsmooth x (nsmooth sweeps, then the
    low-rank fix), sor_smoother.cc:41-78 -- with multicolour sweeps."""

    def __init__(self, linear_operator, omega: float, nsmooth: int, direction: int, device: int = 0):
        if direction not in (FORWARD, BACKWARD):
            raise ValueError("direction must be FORWARD (1) or BACKWARD (2)")
        super().__init__(linear_operator, omega, device)
        self.nsmooth, self.direction = int(nsmooth), int(direction)

    def apply(self, b, x: np.ndarray):
        self._check(b, x)
        x[:] = self._s.sor_smoother_apply(0, self.direction, self.nsmooth, b, x)


class SSORSmoother(_OneLevelSmoother):
    """SSORSmoother(linear_operator, omega, nsmooth) (smoother/ssor_smoother.hh:31-48): nsmooth x
    (forward SOR sweep + fix, backward SOR sweep + fix), ssor_smoother.cc:9-15."""

    def __init__(self, linear_operator, omega: float, nsmooth: int, device: int = 0):
        super().__init__(linear_operator, omega, device)
        self.nsmooth = int(nsmooth)

    def apply(self, b, x: np.ndarray):
        self._check(b, x)
        x[:] = self._s.ssor_smoother_apply(0, self.nsmooth, b, x)


class SORSmootherFactory:
    """SmootherFactory (smoother/smoother.hh:39-44) of SORSmoother (sor_smoother.hh:91-125)."""

    def __init__(self, omega: float, nsmooth: int, direction: int, device: int = 0):
        self.omega, self.nsmooth, self.direction, self.device = omega, nsmooth, direction, device

    def get(self, linear_operator) -> SORSmoother:
        return SORSmoother(linear_operator, self.omega, self.nsmooth, self.direction, self.device)


class SSORSmootherFactory:
    """SmootherFactory of SSORSmoother (ssor_smoother.hh:70-100)."""

    def __init__(self, omega: float, nsmooth: int, device: int = 0):
        self.omega, self.nsmooth, self.device = omega, nsmooth, device

    def get(self, linear_operator) -> SSORSmoother:
        return SSORSmoother(linear_operator, self.omega, self.nsmooth, self.device)


__all__ = [
    "Lattice", "Lattice2d", "Lattice3d", "ShiftedLaplaceFDOperator", "MultigridMCSampler",
    "HipMulticolourSORSmoother", "SORSmoother", "SSORSmoother", "SORSmootherFactory", "SSORSmootherFactory", "measurement_vector_index", "ConstantCorrelationLengthModel",
    "PeriodicCorrelationLengthModel", "SquaredShiftedLaplaceFDOperator", "comm_unique_id", "make_config", "describe", "FORWARD", "BACKWARD",
]
