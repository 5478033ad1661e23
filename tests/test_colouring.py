"""Colour-conflict checker (race detection): a multicolour Gibbs sweep updates every
vertex of one colour at once, which equals the reference's lexicographic SOR sweep only in
distribution, and is a valid Gibbs sweep at all only if no two vertices of one colour are coupled by
the level's operator.  These host-only tests check that for every level the library builds:

  * stencil levels (mgmc_describe: the library's own npoints / ncolours per level): red-black
    (i + j + k) & 1 for the fine 5 / 7-point level, coordinate parities for the 9 / 27-point Galerkin
    levels (colour_of in mgmc_kernels.hpp);
  * matrix levels (the periodic correlation-length model and the squared FD operator, mgmc_field.hpp):
    the fine CSR from the library (mgmc_operator_csr) and Galerkin levels R A R^T with the reference's
    restriction pattern (intergrid_operator.hh:74-88; positive weights, so the pattern is a superset of
    the true one), coloured by make_field's rule (mgmc_capi.hip): red-black for a fine level of at most
    2d+1 entries per row and reach 1, coordinates mod 3 for reach 2, parities otherwise.
"""
import itertools

import numpy as np
import pytest
import scipy.sparse as sp

import multigridmc_amd as mg


def _offsets(dim, stencil):
    """Nonzero off-centre offsets of a constant stencil, index (dz+1)*9 + (dy+1)*3 + (dx+1)."""
    out = []
    for k in range(3 ** dim):
        if stencil[k] == 0.0:
            continue
        o = tuple(k // 3 ** d % 3 - 1 for d in range(dim))
        if any(o):
            out.append(o)
    return out


def _stencil_colour(npoints, idx):
    if npoints in (5, 7):
        return sum(idx) & 1
    return sum((v & 1) << d for d, v in enumerate(idx))


@pytest.mark.parametrize("op,shape,nlevel", [
    (mg.ShiftedLaplaceFDOperator, (64, 64), 5), (mg.ShiftedLaplaceFDOperator, (32, 32, 32), 4),
    (mg.ShiftedLaplaceFDOperator, (64, 32, 16), 3), (mg.ShiftedLaplaceFEMOperator, (64, 64), 5),
    (mg.ShiftedLaplaceFEMOperator, (16, 16, 16), 3)])
def test_stencil_levels_have_no_same_colour_coupling(op, shape, nlevel):
    lat = mg.Lattice(*shape)
    levels = mg.describe(mg.make_config(op(lat, 25.0), mg.MultigridParameters(nlevel=nlevel)))
    assert len(levels) == nlevel
    dim = lat.dim
    for lv in levels:
        npts, nc = lv["npoints"], lv["ncolours"]
        assert nc == (2 if npts in (5, 7) else 2 ** dim), lv
        offs = _offsets(dim, lv["stencil"])
        assert offs, "a level without couplings"
        # the colouring is periodic with period 2 in every coordinate: every residue class
        seen = set()
        for base in itertools.product(range(2), repeat=dim):
            c = _stencil_colour(npts, base)
            seen.add(c)
            for o in offs:
                nb = tuple(b + d for b, d in zip(base, o))
                assert _stencil_colour(npts, nb) != c, (lv["shape"], base, o)
        assert seen == set(range(nc))


def _restriction(dim, n):
    """Pattern of the reference's restriction (full weighting) from an n^dim lattice to (n/2)^dim,
    rows / columns interior vertices in the lattice order (x fastest)."""
    nc = [v // 2 for v in n]
    fi = [v - 1 for v in n]
    ci = [v - 1 for v in nc]
    rows, cols, vals = [], [], []
    for I in itertools.product(*[range(1, v) for v in reversed(nc)]):
        I = tuple(reversed(I))
        r = sum((I[d] - 1) * int(np.prod(ci[:d])) for d in range(dim))
        for s in itertools.product((-1, 0, 1), repeat=dim):
            f = [2 * I[d] + s[d] for d in range(dim)]
            rows.append(r)
            cols.append(sum((f[d] - 1) * int(np.prod(fi[:d])) for d in range(dim)))
            vals.append(0.5 ** sum(abs(v) for v in s))
    return sp.csr_matrix((vals, (rows, cols)), shape=(int(np.prod(ci)), int(np.prod(fi))))


def _coords(n, dim):
    fi = [v - 1 for v in n]
    e = np.arange(int(np.prod(fi)))
    out = []
    for d in range(dim):
        out.append(e % fi[d] + 1)
        e = e // fi[d]
    return np.stack(out)


def _field_colour(scheme, xyz):
    if scheme == 2:
        return xyz.sum(axis=0) & 1
    if scheme in (4, 8):
        return sum((xyz[d] & 1) << d for d in range(xyz.shape[0]))
    return sum((xyz[d] % 3) * 3 ** d for d in range(xyz.shape[0]))


@pytest.mark.parametrize("op,shape,nlevel", [
    (mg.ShiftedLaplaceFDOperator, (32, 32), 4), (mg.ShiftedLaplaceFDOperator, (16, 16, 16), 3),
    (mg.ShiftedLaplaceFEMOperator, (32, 32), 4), (mg.ShiftedLaplaceFEMOperator, (16, 8, 16), 3),
    (mg.SquaredShiftedLaplaceFDOperator, (32, 32), 4), (mg.SquaredShiftedLaplaceFDOperator, (16, 24), 3)])
def test_matrix_levels_have_no_same_colour_coupling(op, shape, nlevel):
    lat = mg.Lattice(*shape)
    A = abs(op(lat, mg.PeriodicCorrelationLengthModel(1.2, 2.3)).matrix()).tocsr()
    dim, n = lat.dim, list(shape)
    schemes = []
    for level in range(nlevel):
        xyz = _coords(n, dim)
        C = A.tocoo()
        off = C.row != C.col
        d = np.abs(xyz[:, C.col] - xyz[:, C.row]).max(axis=0)
        reach = int(d.max())
        A.sort_indices()
        scheme = mg.csr_colour_scheme(mg.Lattice(*n), A.indptr, A.indices, level)  # make_field's rule
        assert scheme == ((27 if dim == 3 else 9) if reach >= 2 else (2 if level == 0 and dim * 2 + 1 >= int(
            np.diff(A.indptr).max()) else 2 ** dim))
        schemes.append(scheme)
        col = _field_colour(scheme, xyz)
        clash = off & (col[C.row] == col[C.col])
        assert not clash.any(), (level, n, scheme, int(clash.sum()))
        assert set(np.unique(col)) == set(range(scheme)) or min(n) < 6
        if level + 1 < nlevel:
            R = _restriction(dim, n)
            A = (R @ A @ R.T).tocsr()
            n = [v // 2 for v in n]
    if op is mg.SquaredShiftedLaplaceFDOperator:
        assert schemes[0] == 9 and all(s == 9 for s in schemes)  # reach-2 diamond on every level
    else:
        assert schemes[0] == (2 if op is mg.ShiftedLaplaceFDOperator else 2 ** dim)
        assert all(s == 2 ** dim for s in schemes[1:])


def test_checker_catches_a_conflict():
    """The checker itself: red-black colouring of a 9-point (diagonal) stencil must be flagged."""
    offs = _offsets(2, np.ones(9))
    assert any(_stencil_colour(5, o) == _stencil_colour(5, (0, 0)) for o in offs)


def _offset_csr(dim, shape, offsets, diag=10.0, off=-1.0):
    """CSR on an interior-vertex lattice coupling every vertex to the given offsets (plus itself)."""
    xyz = _coords(list(shape), dim)
    n = xyz.shape[1]
    fi = [v - 1 for v in shape]
    rows, cols, vals = [], [], []
    for o in [(0,) * dim] + list(offsets):
        nb = xyz + np.array(o)[:, None]
        ok = np.all((nb >= 1) & (nb <= np.array(fi)[:, None]), axis=0)
        lin = sum((nb[d] - 1) * int(np.prod(fi[:d])) for d in range(dim))
        rows.append(np.arange(n)[ok])
        cols.append(lin[ok])
        vals.append(np.full(int(ok.sum()), diag if not any(o) else off))
    A = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    A.sort_indices()
    return A


@pytest.mark.parametrize("dim,shape,offsets,expect", [
    (2, (16, 16), [(1, 1), (-1, -1), (1, -1), (-1, 1)], 4),                          # 5 entries, all diagonal
    (3, (8, 8, 8), [(1, 1, 0), (-1, -1, 0), (0, 0, 1), (0, 0, -1), (1, 0, 0), (-1, 0, 0)], 8),  # 7 entries, 2 edge
    (2, (16, 16), [(1, 0), (-1, 0), (0, 1), (0, -1)], 2),                            # the 5-point FD pattern
    (3, (8, 8, 8), [(1, 0, 0), (-1, 0, 0), (0, 0, 2), (0, 0, -2)], 27),              # reach 2
])
def test_user_csr_colouring_has_no_same_colour_coupling(dim, shape, offsets, expect):
    """A user matrix of at most 2d+1 entries per row is swept red-black only when every coupling is
    an axis neighbour (diagonal couplings put coupled vertices in one red-black
    colour).  The library's choice (mgmc_csr_colour_scheme = make_field's rule) has no clash."""
    lat = mg.Lattice(*shape)
    A = _offset_csr(dim, shape, offsets)
    scheme = mg.csr_colour_scheme(lat, A.indptr, A.indices)
    assert scheme == expect
    xyz = _coords(list(shape), dim)
    C = A.tocoo()
    col = _field_colour(scheme, xyz)
    assert not ((C.row != C.col) & (col[C.row] == col[C.col])).any()
    # the same matrix on a coarse level never gets red-black
    if expect == 2:
        assert mg.csr_colour_scheme(lat, A.indptr, A.indices, level=1) == 2 ** dim


def test_csr_shape_checked_before_reading_entries():
    """mgmc_create_csr / mgmc_csr_colour_scheme validate nrow against the lattice and the row
    pointer's monotonicity before reading rowptr[nrow] or copying entries."""
    lat = mg.Lattice(8, 8)
    A = _offset_csr(2, (8, 8), [(1, 0), (-1, 0), (0, 1), (0, -1)])
    with pytest.raises(mg.MgmcError, match="interior vertices"):
        mg.csr_colour_scheme(mg.Lattice(16, 8), A.indptr, A.indices)
    bad = A.indptr.copy()
    bad[5] = bad[4] - 1  # decreasing
    with pytest.raises(mg.MgmcError, match="entries"):
        mg.csr_colour_scheme(lat, bad, A.indices)
    # mgmc_create_csr with a lattice of 105 interior vertices and a 49-row matrix: refused on the host
    import ctypes
    from multigridmc_amd import _native
    lib = mg.load_library()
    cfg = mg.make_config(mg.ShiftedLaplaceFDOperator(mg.Lattice(16, 8), 25.0), mg.MultigridParameters(nlevel=1))
    h = ctypes.c_void_p()
    rp = A.indptr.astype(np.int64)
    ci = A.indices.astype(np.int32)
    va = A.data.astype(np.float64)
    rc = lib.mgmc_create_csr(ctypes.byref(cfg), len(rp) - 1, rp.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                             ci.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                             va.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 0, 1, 0, ctypes.byref(h))
    assert rc == _native.MGMC_E_INVALID and b"mgmc_create_csr: nrow 49" in lib.mgmc_last_error(None)
