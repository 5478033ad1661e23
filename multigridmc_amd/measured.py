"""Posterior (measured) operator: the low-rank part B, Sigma of Q = A + B Sigma^{-1} B^T.

Host-side mirror of MeasuredOperator (nilsfriess/MultigridMC, src/linear_operator/measured_operator.cc):
  * constructor: one column of B per measurement location (measurement_vector), plus a dense column
    of cell volumes when measure_global is set; Sigma = variance_scaling * variance
    (+ variance_global) ............................................. measured_operator.cc:9-49
  * measurement_vector(x0, radius): radius 0 -> indicator of the nearest interior vertex
    (:74-91); radius > 0 -> the integral of the normalised indicator of the ball |x - x0| < radius
    against each multilinear basis function, by the order-1 Gauss-Legendre rule on every cell the
    ball touches (:92-170, quadrature.cc)
  * V_sphere ......................................................... measured_operator.cc:52-67

B is built once on the host (it is O(N m) setup work, not the path) and handed to the device
through mgmc_set_lowrank as CSC columns with ascending row indices -- the layout of the reference's
Eigen sparse matrix.  Floating-point expressions keep the reference's operand order.
"""
from __future__ import annotations

import math

import numpy as np

from .parameters import MeasurementParameters
from .sampler import Lattice, ShiftedLaplaceFDOperator, measurement_vector_index


def V_sphere(radius: float, dim: int) -> float:
    """Volume of the radius-R ball in d dimensions (measured_operator.cc:52-67)."""
    if dim == 0:
        return 1.0
    if dim == 1:
        return 2.0 * radius
    return 2.0 * math.pi / float(dim) * radius * radius * V_sphere(radius, dim - 2)


def _cartesian_product(v, n):
    """common.hh:29-53: the last coordinate varies fastest."""
    if n == 1:
        return [[a] for a in v]
    return [s + [a] for s in _cartesian_product(v, n - 1) for a in v]


def gauss_legendre_order1(dim: int):
    """GaussLegendreQuadrature(dim, 1) on [0, 1]^dim (quadrature.cc): points (p + 1) / 2 for
    p = -+1/sqrt(3), weights prod 0.5 * 1.0."""
    p1 = [-1.0 / math.sqrt(3.0), +1.0 / math.sqrt(3.0)]
    w1 = [1.0, 1.0]
    weights = []
    for wp in _cartesian_product(w1, dim):
        w = 1.0
        for s in wp:
            w *= 0.5 * s
        weights.append(w)
    points = [[0.5 * (c + 1.0) for c in pp] for pp in _cartesian_product(p1, dim)]
    return points, weights


def measurement_vector(lattice: Lattice, x0, radius: float):
    """Sparse measurement vector: (rows ascending, values) (measured_operator.cc:69-171)."""
    dim = lattice.dim
    x0 = [float(v) for v in x0]
    if len(x0) != dim:
        raise ValueError(f"measurement location has dimension {len(x0)}, lattice has {dim}")
    if radius < 1.0e-12:
        return np.array([measurement_vector_index(lattice, x0, 0.0)], dtype=np.int64), np.array([1.0])
    shape = lattice.shape
    h = [1.0 / float(shape[d]) for d in range(dim)]
    cell_volume = 1.0
    for d in range(dim):
        cell_volume /= shape[d]
    normalisation = 1.0 / V_sphere(radius, dim)
    qpts, qw = gauss_legendre_order1(dim)
    corners = _cartesian_product([0, 1], dim)
    # Only cells whose bounding box meets [x0 - r, x0 + r] can overlap the ball (a corner inside the
    # ball or x0 inside the cell both imply it); visit them in the reference's linear cell order.
    lo = [max(0, int(math.floor((x0[d] - radius) / h[d])) - 1) for d in range(dim)]
    hi = [min(shape[d] - 1, int(math.floor((x0[d] + radius) / h[d])) + 1) for d in range(dim)]
    acc = {}
    ranges = [range(lo[d], hi[d] + 1) for d in range(dim)]
    cells = [[c] for c in ranges[0]]
    for d in range(1, dim):
        cells = [c + [q] for q in ranges[d] for c in cells]  # dimension 0 fastest
    for cell in cells:
        overlap = False
        cmin = [2.0] * dim
        cmax = [-1.0] * dim
        for om in corners:
            xc = [h[d] * float(cell[d] + om[d]) for d in range(dim)]
            cmin = [min(cmin[d], xc[d]) for d in range(dim)]
            cmax = [max(cmax[d], xc[d]) for d in range(dim)]
            overlap = overlap or (math.sqrt(sum((xc[d] - x0[d]) ** 2 for d in range(dim))) < radius)
        inside = all(cmin[d] <= x0[d] <= cmax[d] for d in range(dim))
        if not (overlap or inside):
            continue
        for alpha in corners:
            v = [cell[d] + alpha[d] for d in range(dim)]
            if not all(0 < v[d] < shape[d] for d in range(dim)):
                continue
            ell = lattice.vertexidx_euclidean2linear(v)
            local = 0.0
            for xhat, w in zip(qpts, qw):
                x = [h[d] * (xhat[d] + float(cell[d])) for d in range(dim)]
                ss = 0.0
                for d in range(dim):
                    ss += (x[d] - x0[d]) * (x[d] - x0[d])
                xi = math.sqrt(ss) / radius
                if xi < 1.0:
                    phihat = 1.0  # f_meas(xi) = 1 (measured_operator.hh:65)
                    for d in range(dim):
                        phihat *= (1.0 - xhat[d]) if alpha[d] == 0 else xhat[d]
                    local += phihat * w * cell_volume * normalisation
            acc[ell] = acc.get(ell, 0.0) + local
    rows = np.array(sorted(acc), dtype=np.int64)
    vals = np.array([acc[r] for r in rows], dtype=np.float64)
    keep = vals != 0.0
    return rows[keep], vals[keep]


class LowRankUpdate:
    """B (N x m) as CSC arrays and the diagonal of Sigma."""

    def __init__(self, n: int, colptr, rows, vals, sigma):
        self.n = int(n)
        self.colptr = np.ascontiguousarray(colptr, dtype=np.int64)
        self.rows = np.ascontiguousarray(rows, dtype=np.int64)
        self.vals = np.ascontiguousarray(vals, dtype=np.float64)
        self.sigma = np.ascontiguousarray(sigma, dtype=np.float64)
        self.m = len(self.sigma)
        if len(self.colptr) != self.m + 1 or self.colptr[0] != 0 or self.colptr[-1] != len(self.rows):
            raise ValueError("inconsistent CSC column pointers")
        if len(self.vals) != len(self.rows):
            raise ValueError("rows and values differ in length")
        for k in range(self.m):
            r = self.rows[self.colptr[k]:self.colptr[k + 1]]
            if len(r) and (r[0] < 0 or r[-1] >= self.n or np.any(np.diff(r) <= 0)):
                raise ValueError(f"column {k}: row indices must be ascending in [0, {self.n})")
        if np.any(self.sigma <= 0.0):
            raise ValueError("Sigma must be positive")

    @classmethod
    def from_columns(cls, n: int, columns, sigma):
        """columns: list of (rows, values)."""
        colptr = [0]
        for r, _ in columns:
            colptr.append(colptr[-1] + len(r))
        rows = np.concatenate([np.asarray(r, dtype=np.int64) for r, _ in columns]) if columns else np.zeros(0, np.int64)
        vals = np.concatenate([np.asarray(v, dtype=np.float64) for _, v in columns]) if columns else np.zeros(0)
        return cls(n, colptr, rows, vals, sigma)

    def dense(self) -> np.ndarray:
        B = np.zeros((self.n, self.m))
        for k in range(self.m):
            s = slice(self.colptr[k], self.colptr[k + 1])
            B[self.rows[s], k] = self.vals[s]
        return B

    def precision_update(self) -> np.ndarray:
        """B Sigma^{-1} B^T (dense; small cases only)."""
        B = self.dense()
        return B @ np.diag(1.0 / self.sigma) @ B.T


class MeasuredOperator:
    """Q = A + B Sigma^{-1} B^T for a FD prior (measured_operator.hh / measured_operator.cc:9-49)."""

    def __init__(self, base_operator: ShiftedLaplaceFDOperator, params: MeasurementParameters):
        self.base_operator = base_operator
        self.lattice = base_operator.get_lattice()
        self.params = params
        lat = self.lattice
        nmeas = len(params.measurement_locations)
        if len(params.variance) < nmeas:
            raise ValueError("one variance per measurement location is required")
        cols = [measurement_vector(lat, x0, params.radius) for x0 in params.measurement_locations]
        sigma = [params.variance_scaling * float(params.variance[k]) for k in range(nmeas)]
        if params.measure_global:
            cell_volume = 1.0
            for d in range(lat.dim):
                cell_volume /= float(lat.shape[d])
            cols.append((np.arange(lat.Nvertex, dtype=np.int64), np.full(lat.Nvertex, cell_volume)))
            sigma.append(float(params.variance_global))
        self.lowrank = LowRankUpdate.from_columns(lat.Nvertex, cols, sigma)

    @property
    def kappa_sq(self) -> float:
        return self.base_operator.kappa_sq

    def get_lattice(self) -> Lattice:
        return self.lattice

    def get_ndof(self) -> int:
        return self.lattice.Nvertex

    def get_m_lowrank(self) -> int:
        return self.lowrank.m

    def get_B(self) -> LowRankUpdate:
        return self.lowrank

    def get_Sigma(self) -> np.ndarray:
        return self.lowrank.sigma.copy()

    def measurement_vector(self, x0, radius: float):
        return measurement_vector(self.lattice, x0, radius)


__all__ = ["V_sphere", "gauss_legendre_order1", "measurement_vector", "LowRankUpdate", "MeasuredOperator"]


def synthetic_posterior(prior, m: int, radius: float = 0.0, measure_global: bool = False,
                        seed: int = 20250219) -> MeasuredOperator:
    """BASELINE config 5's synthetic posterior: m measurements at fixed pseudo-random interior
    locations (uniform in [0.1, 0.9]^d, numpy PCG64 seeded with `seed`) with variances on the scale of
    measurements_template.cfg (1e-6 (1 + U)), optionally the global average (variance_global 0.01 as
    in parameters_template.cfg).  The measured values stay 0 (f = 0 in the bench); bench.py and the
    CPU baseline build the same operator from these arguments."""
    rng = np.random.default_rng(seed)
    dim = prior.get_lattice().dim
    mp = MeasurementParameters(radius=radius, variance_scaling=1.0, measure_global=measure_global,
                               variance_global=0.01)
    mp.dim = dim
    mp.measurement_locations = [list(rng.uniform(0.1, 0.9, dim)) for _ in range(m)]
    mp.variance = list(1e-6 * (1.0 + rng.random(m)))
    mp.n = m
    return MeasuredOperator(prior, mp)
