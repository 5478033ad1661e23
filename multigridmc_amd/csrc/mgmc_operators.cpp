// mgmc_operators.cpp -- see mgmc_operators.hpp.
#include "mgmc_operators.hpp"

#include <math.h>

#include <algorithm>
#include <sstream>

namespace mgmc {

namespace {

struct Lat {
    int dim;
    int n[3];  // cells per direction (n[2] = 1 in 2D: one layer of cells, no k index)
    int64_t ni[3];
    int64_t nvertex() const { return ni[0] * ni[1] * (dim == 3 ? ni[2] : 1); }
    int64_t ncell() const { return (int64_t)n[0] * n[1] * (dim == 3 ? n[2] : 1); }
    explicit Lat(int d, const int* nn) : dim(d) {
        n[0] = nn[0];
        n[1] = nn[1];
        n[2] = d == 3 ? nn[2] : 1;
        for (int q = 0; q < 3; ++q) ni[q] = n[q] - 1;
    }
    // interior vertex ell <-> (i, j, k), 1 <= i <= n-1, x fastest (lattice2d.hh / lattice3d.hh)
    void lin2euc(int64_t ell, int* idx) const {
        idx[0] = (int)(ell % ni[0]) + 1;
        idx[1] = (int)((ell / ni[0]) % ni[1]) + 1;
        idx[2] = dim == 3 ? (int)(ell / (ni[0] * ni[1])) + 1 : 0;
    }
    bool interior(const int* idx) const {
        for (int d = 0; d < dim; ++d)
            if (idx[d] < 1 || idx[d] > n[d] - 1) return false;
        return true;
    }
    int64_t euc2lin(const int* idx) const {
        int64_t e = idx[0] - 1 + ni[0] * (int64_t)(idx[1] - 1);
        if (dim == 3) e += ni[0] * ni[1] * (int64_t)(idx[2] - 1);
        return e;
    }
};

// rows of (col, value) triplets as setFromTriplets sums them (the first value of a column stored,
// duplicates added in order), emitted with columns ascending
struct RowBuilder {
    std::vector<std::pair<int32_t, double>> e;
    void add(int64_t c, double v) {
        for (auto& p : e)
            if (p.first == (int32_t)c) {
                p.second += v;
                return;
            }
        e.push_back({(int32_t)c, v});
    }
    void flush(CsrHost& A) {
        std::sort(e.begin(), e.end(), [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
            return a.first < b.first;
        });
        for (auto& p : e) {
            A.col.push_back(p.first);
            A.val.push_back(p.second);
        }
        A.rowptr.push_back((int64_t)A.col.size());
        e.clear();
    }
};

void spacing(const Lat& L, double* h, double* hinv2, double* cell_volume) {
    *cell_volume = 1.0;
    for (int d = 0; d < L.dim; ++d) {
        h[d] = 1. / double(L.n[d]);
        hinv2[d] = 1. / (h[d] * h[d]);
        *cell_volume *= h[d];
    }
}

// vertex coordinates (lattice2d.hh:188-195): (index + 1.0) * h with the 0-based index
void vertex_coordinates(const Lat& L, int64_t ell, const double* h, double* x) {
    x[0] = (double)(ell % L.ni[0] + 1) * h[0];
    x[1] = (double)((ell / L.ni[0]) % L.ni[1] + 1) * h[1];
    if (L.dim == 3) x[2] = (double)(ell / (L.ni[0] * L.ni[1]) + 1) * h[2];
}

// ShiftedLaplaceFDOperator (shiftedlaplace_fd_operator.cc:9-57)
CsrHost assemble_fd(const mgmc_operator_desc& d, const Lat& L) {
    double h[3], hinv2[3], cv;
    spacing(L, h, hinv2, &cv);
    CsrHost A;
    A.nrow = L.nvertex();
    A.rowptr.push_back(0);
    RowBuilder rb;
    for (int64_t ell = 0; ell < A.nrow; ++ell) {
        double x[3];
        vertex_coordinates(L, ell, h, x);
        double diagonal = cv * kappa_sq_at(d, x);
        int idx[3];
        L.lin2euc(ell, idx);
        for (int dd = 0; dd < L.dim; ++dd) {
            for (int j = 0; j < 2; ++j) {
                int s[3] = {idx[0], idx[1], idx[2]};
                s[dd] += 2 * j - 1;
                if (L.interior(s)) rb.add(L.euc2lin(s), -cv * hinv2[dd]);
            }
            diagonal += 2. * cv * hinv2[dd];
        }
        rb.add(ell, diagonal);
        rb.flush(A);
    }
    return A;
}

// Q1 shape functions on the reference cell (shiftedlaplace_fem_operator.cc:148-187)
double phi(int dim, const int* a, const double* xh) {
    double v = 1.0;
    for (int j = 0; j < dim; ++j) v *= (a[j] == 0) ? (1.0 - xh[j]) : xh[j];
    return v;
}
void grad_phi(int dim, const int* a, const double* xh, double* g) {
    for (int k = 0; k < dim; ++k) {
        double v = 1.0;
        for (int j = 0; j < dim; ++j) {
            if (j == k)
                v *= (a[j] == 0) ? -1.0 : +1.0;
            else
                v *= (a[j] == 0) ? (1.0 - xh[j]) : xh[j];
        }
        g[k] = v;
    }
}

// ShiftedLaplaceFEMOperator (shiftedlaplace_fem_operator.cc:9-145): cells ascending (x fastest),
// basis pairs in cartesian-product order (last dimension fastest), order-1 Gauss-Legendre points
// (quadrature.cc:11-55, 2 per direction, last dimension fastest); every entry starts at 0.0 and
// receives local * cell_volume per cell, local = sum_q (kappa^2(x_q) phi_a phi_b + grad phi_a .
// (h^-2 grad phi_b)) w_q with x_q = h (xhat_q + cell)
CsrHost assemble_fem(const mgmc_operator_desc& d, const Lat& L) {
    const int dim = L.dim;
    double h[3], hinv2[3], cv;
    spacing(L, h, hinv2, &cv);
    const double p1[2] = {-1.0 / sqrt(3.0), +1.0 / sqrt(3.0)};
    const int nq = 1 << dim, nb = 1 << dim;
    double qp[8][3], qw[8];
    for (int q = 0; q < nq; ++q) {
        double w = 1.0;
        for (int j = 0; j < dim; ++j) {
            const int b = (q >> (dim - 1 - j)) & 1;
            w *= 0.5 * 1.0;
            qp[q][j] = 0.5 * (p1[b] + 1.0);
        }
        qw[q] = w;
    }
    int basis[8][3];
    for (int a = 0; a < nb; ++a)
        for (int j = 0; j < dim; ++j) basis[a][j] = (a >> (dim - 1 - j)) & 1;
    // phi_a phi_b and grad phi_a . (h^-2 grad phi_b) per (alpha, beta, q) -- Eigen dot ((t0 + t1) + t2)
    std::vector<double> pp((size_t)nb * nb * nq), gg((size_t)nb * nb * nq);
    for (int a = 0; a < nb; ++a)
        for (int b = 0; b < nb; ++b)
            for (int q = 0; q < nq; ++q) {
                const size_t c = ((size_t)a * nb + b) * nq + q;
                pp[c] = phi(dim, basis[a], qp[q]) * phi(dim, basis[b], qp[q]);
                double ga[3] = {0, 0, 0}, gb[3] = {0, 0, 0};
                grad_phi(dim, basis[a], qp[q], ga);
                grad_phi(dim, basis[b], qp[q], gb);
                double s = ga[0] * (hinv2[0] * gb[0]);
                for (int k = 1; k < dim; ++k) s = s + ga[k] * (hinv2[k] * gb[k]);
                gg[c] = s;
            }
    // accumulate per row in cell order: entry (row, col) collects its cells ascending
    const int64_t nrow = L.nvertex();
    std::vector<std::vector<std::pair<int32_t, double>>> rows((size_t)nrow);
    const int64_t ncell = L.ncell();
    for (int64_t cell = 0; cell < ncell; ++cell) {
        const int cc[3] = {(int)(cell % L.n[0]), (int)((cell / L.n[0]) % L.n[1]),
                           dim == 3 ? (int)(cell / ((int64_t)L.n[0] * L.n[1])) : 0};
        double kq[8];
        for (int q = 0; q < nq; ++q) {
            double x[3];
            for (int j = 0; j < dim; ++j) x[j] = h[j] * (qp[q][j] + (double)cc[j]);
            kq[q] = kappa_sq_at(d, x);
        }
        for (int a = 0; a < nb; ++a) {
            int va[3] = {0, 0, 0};
            for (int j = 0; j < dim; ++j) va[j] = cc[j] + basis[a][j];
            if (!L.interior(va)) continue;
            const int64_t r = L.euc2lin(va);
            for (int b = 0; b < nb; ++b) {
                int vb[3] = {0, 0, 0};
                for (int j = 0; j < dim; ++j) vb[j] = cc[j] + basis[b][j];
                if (!L.interior(vb)) continue;
                const int32_t c = (int32_t)L.euc2lin(vb);
                double local = 0.0;
                for (int q = 0; q < nq; ++q) {
                    const size_t t = ((size_t)a * nb + b) * nq + q;
                    local += (kq[q] * pp[t] + gg[t]) * qw[q];
                }
                auto& row = rows[(size_t)r];
                bool found = false;
                for (auto& p : row)
                    if (p.first == c) {
                        p.second += local * cv;
                        found = true;
                        break;
                    }
                if (!found) row.push_back({c, 0.0 + local * cv});
            }
        }
    }
    CsrHost A;
    A.nrow = nrow;
    A.rowptr.push_back(0);
    for (auto& row : rows) {
        std::sort(row.begin(), row.end(), [](const std::pair<int32_t, double>& x, const std::pair<int32_t, double>& y) {
            return x.first < y.first;
        });
        for (auto& p : row) {
            A.col.push_back(p.first);
            A.val.push_back(p.second);
        }
        A.rowptr.push_back((int64_t)A.col.size());
    }
    return A;
}

// SquaredShiftedLaplaceFDOperator, 2D (squared_shiftedlaplace_fd_operator.cc:9-96): the row of
// (kappa^2 - Laplace)^2 at a vertex is the 13-point diamond of the squared 5-point Laplacian (weights
// `bilap` by |offset|) plus -2 kappa^2 times the Laplacian on the 4 axis neighbours; an axis neighbour
// outside the domain folds the point mirrored two steps beyond it back onto the centre (homogeneous
// Neumann).  Entries in the assembly order of the reference (x offset outer, y inner, ascending),
// each with its expression order, so the CSR is bit for bit the reference's (tests/test_varcoef.py).
struct DiamondPoint {
    int dx, dy;
    bool axis;     // |dx| + |dy| == 1
    double bilap;  // squared-Laplacian weight of the offset
    double lap;    // Laplacian weight (axis neighbours)
    double fold;   // Neumann fold-back weight onto the centre (axis neighbours)
};

CsrHost assemble_squared_fd(const mgmc_operator_desc& d, const Lat& L) {
    double h[3], hinv2[3], cv;
    spacing(L, h, hinv2, &cv);
    const double gx = hinv2[0], gy = hinv2[1];
    // squared-Laplacian weights by (|dx|, |dy|) and the Laplacian's centre
    auto bilap = [&](int ax, int ay) -> double {
        if (ax == 0 && ay == 0) return 6 * (gx * gx + gy * gy) + 8 * gx * gy;
        if (ax == 1 && ay == 0) return -4 * gx * (gx + gy);
        if (ax == 0 && ay == 1) return -4 * gy * (gx + gy);
        if (ax == 2 && ay == 0) return gx * gx;
        if (ax == 0 && ay == 2) return gy * gy;
        if (ax == 1 && ay == 1) return 2 * gx * gy;
        return 0.0;
    };
    const double lap_centre = -2 * (gx + gy);
    std::vector<DiamondPoint> pts;
    for (int dx = -2; dx <= 2; ++dx)
        for (int dy = -2; dy <= 2; ++dy) {
            const int ax = abs(dx), ay = abs(dy);
            if (ax + ay > 2 || ax + ay == 0) continue;
            DiamondPoint q{dx, dy, ax + ay == 1, bilap(ax, ay), 0.0, 0.0};
            if (q.axis) {
                q.lap = ax ? gx : gy;
                q.fold = bilap(2 * ax, 2 * ay);
            }
            pts.push_back(q);
        }
    CsrHost A;
    A.nrow = L.nvertex();
    A.rowptr.push_back(0);
    RowBuilder rb;
    for (int64_t ell = 0; ell < A.nrow; ++ell) {
        double x[3];
        vertex_coordinates(L, ell, h, x);
        const double k2 = kappa_sq_at(d, x);
        double centre = (k2 * k2 - 2. * k2 * lap_centre + bilap(0, 0)) * cv;
        int idx[3];
        L.lin2euc(ell, idx);
        for (const DiamondPoint& q : pts) {
            const int nb[3] = {idx[0] + q.dx, idx[1] + q.dy, 0};
            if (L.interior(nb)) {
                double w = q.bilap;
                if (q.axis) w += -2. * k2 * q.lap;
                rb.add(L.euc2lin(nb), w * cv);
            } else if (q.axis) {
                centre += q.fold * cv;
            }
        }
        rb.add(ell, centre);
        rb.flush(A);
    }
    return A;
}

// C = A B, Gustavson: row r of C collects a_rk b_kc over the entries k of A's row in order, the
// first term of each column assigned, later ones added; columns sorted
CsrHost spgemm(const CsrHost& A, const CsrHost& B, int64_t ncol) {
    CsrHost C;
    C.nrow = A.nrow;
    C.rowptr.assign(A.nrow + 1, 0);
    std::vector<double> acc(ncol, 0.0);
    std::vector<char> used(ncol, 0);
    std::vector<int32_t> cols;
    for (int64_t r = 0; r < A.nrow; ++r) {
        cols.clear();
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            const int32_t k = A.col[q];
            const double a = A.val[q];
            for (int64_t t = B.rowptr[k]; t < B.rowptr[k + 1]; ++t) {
                const int32_t c = B.col[t];
                if (!used[c]) {
                    used[c] = 1;
                    acc[c] = a * B.val[t];
                    cols.push_back(c);
                } else {
                    acc[c] += a * B.val[t];
                }
            }
        }
        std::sort(cols.begin(), cols.end());
        for (int32_t c : cols) {
            C.col.push_back(c);
            C.val.push_back(acc[c]);
            used[c] = 0;
        }
        C.rowptr[r + 1] = (int64_t)C.col.size();
    }
    return C;
}

CsrHost transpose(const CsrHost& A, int64_t ncol) {
    CsrHost T;
    T.nrow = ncol;
    T.rowptr.assign(ncol + 1, 0);
    for (int32_t c : A.col) ++T.rowptr[c + 1];
    for (int64_t r = 0; r < ncol; ++r) T.rowptr[r + 1] += T.rowptr[r];
    T.col.resize(A.col.size());
    T.val.resize(A.val.size());
    std::vector<int64_t> pos(T.rowptr.begin(), T.rowptr.end() - 1);
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            const int64_t p = pos[A.col[q]]++;
            T.col[p] = (int32_t)r;
            T.val[p] = A.val[q];
        }
    return T;
}

// restriction R (coarse rows): coarse vertex I takes the fine vertices 2I + s, s in {-1,0,1}^d, with
// weights prod_d (1/2, 1, 1/2)[s_d] (intergrid_operator_linear.cc:13-29; unnormalised), columns sorted
CsrHost restriction(const Lat& F, const Lat& C) {
    const int dim = F.dim;
    const int ns = dim == 3 ? 27 : 9;
    const double w1d[3] = {0.5, 1.0, 0.5};
    CsrHost R;
    R.nrow = C.nvertex();
    R.rowptr.push_back(0);
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t ec = 0; ec < R.nrow; ++ec) {
        int idx[3];
        C.lin2euc(ec, idx);
        row.clear();
        for (int j = 0; j < ns; ++j) {
            double m = 1.0;
            int f[3] = {0, 0, 0};
            int mu = j;
            for (int dd = 0; dd < dim; ++dd) {
                m *= w1d[mu % 3];
                f[dd] = 2 * idx[dd] + (mu % 3) - 1;
                mu /= 3;
            }
            row.push_back({(int32_t)F.euc2lin(f), m});
        }
        std::sort(row.begin(), row.end(), [](const std::pair<int32_t, double>& a, const std::pair<int32_t, double>& b) {
            return a.first < b.first;
        });
        for (auto& p : row) {
            R.col.push_back(p.first);
            R.val.push_back(p.second);
        }
        R.rowptr.push_back((int64_t)R.col.size());
    }
    return R;
}

}  // namespace

std::string validate_operator(const mgmc_operator_desc& d) {
    std::ostringstream err;
    if (d.dim != 2 && d.dim != 3) {
        err << "invalid dimension : " << d.dim;
        return err.str();
    }
    const int n[3] = {d.nx, d.ny, d.dim == 3 ? d.nz : 2};
    double nv = 1.0;
    for (int q = 0; q < d.dim; ++q) {
        if (n[q] < 2) return "every lattice extent must be >= 2";
        nv *= (n[q] - 1);
    }
    if (nv > 2.0e9) return "lattice too large for a CSR operator (more than 2e9 unknowns)";
    if (d.pde != MGMC_OPERATOR_FD && d.pde != MGMC_OPERATOR_FEM && d.pde != MGMC_OPERATOR_SQUARED_FD) {
        err << "Error: invalid prior '" << d.pde << "'";  // driver_mgmc.cc:426-429
        return err.str();
    }
    if (d.pde == MGMC_OPERATOR_SQUARED_FD && d.dim != 2)
        return "SquaredShiftedLaplaceFDOperator only implemented for d=2";  // squared_..._operator.cc:17-21
    if (d.kappa_model == MGMC_KAPPA_CONSTANT) {
        if (!(d.Lambda > 0.0)) return "Lambda must be > 0";
    } else if (d.kappa_model == MGMC_KAPPA_PERIODIC) {
        if (!(d.Lambda_min > 0.0 && d.Lambda_max >= d.Lambda_min)) return "need 0 < Lambda_min <= Lambda_max";
    } else if (d.kappa_model == MGMC_KAPPA_GIVEN) {
        if (!(d.kappa_sq >= 0.0)) return "kappa_sq must be >= 0";
    } else {
        err << "Error: invalid correlation length model '" << d.kappa_model << "'";
        return err.str();
    }
    return "";
}

double kappa_sq_at(const mgmc_operator_desc& d, const double* x) {
    if (d.kappa_model == MGMC_KAPPA_CONSTANT) return 1. / pow(d.Lambda, 2);  // correlationlength_model.hh:52
    if (d.kappa_model == MGMC_KAPPA_GIVEN) return d.kappa_sq;
    // PeriodicCorrelationLengthModel (correlationlength_model.hh:90-104): the correlation length
    // oscillates around the middle of [Lambda_min, Lambda_max] with half its width as amplitude,
    // ell(x) = mid + amp prod_d cos(pi x_d), and kappa^2 = ell^-2 (the reference's operation order)
    const double mid = 0.5 * (d.Lambda_max + d.Lambda_min);
    const double amp = 0.5 * (d.Lambda_max - d.Lambda_min);
    double ell = amp;
    for (int axis = 0; axis < d.dim; ++axis) ell *= cos(M_PI * x[axis]);
    ell += mid;
    return 1. / (ell * ell);
}

CsrHost assemble_operator(const mgmc_operator_desc& d) {
    const int n[3] = {d.nx, d.ny, d.nz};
    const Lat L(d.dim, n);
    if (d.pde == MGMC_OPERATOR_FEM) return assemble_fem(d, L);
    if (d.pde == MGMC_OPERATOR_SQUARED_FD) return assemble_squared_fd(d, L);
    return assemble_fd(d, L);
}

CsrHost galerkin_csr(const CsrHost& A, int dim, const int* nfine) {
    const Lat F(dim, nfine);
    const int nc[3] = {nfine[0] / 2, nfine[1] / 2, dim == 3 ? nfine[2] / 2 : 1};
    const Lat C(dim, nc);
    const CsrHost R = restriction(F, C);
    const CsrHost P = transpose(R, F.nvertex());
    const CsrHost RA = spgemm(R, A, F.nvertex());
    return spgemm(RA, P, C.nvertex());
}

int csr_reach(int dim, const int* n, const CsrHost& A) {
    const Lat L(dim, n);
    int reach = 0;
    for (int64_t r = 0; r < A.nrow; ++r) {
        int a[3], b[3];
        L.lin2euc(r, a);
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            L.lin2euc(A.col[q], b);
            for (int d = 0; d < dim; ++d) reach = std::max(reach, abs(a[d] - b[d]));
        }
    }
    return reach;
}

std::string check_lattice_csr(int dim, const int* n, const CsrHost& A) {
    const Lat L(dim, n);
    if (A.nrow != L.nvertex()) return "CSR rows differ from the lattice's interior vertices";
    if ((int64_t)A.rowptr.size() != A.nrow + 1 || A.rowptr[0] != 0) return "invalid CSR row pointer";
    for (int64_t r = 0; r < A.nrow; ++r) {
        if (A.rowptr[r + 1] < A.rowptr[r]) return "invalid CSR row pointer";
        bool diag = false;
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            const int32_t c = A.col[q];
            if (c < 0 || c >= A.nrow) return "CSR column out of range";
            if (q > A.rowptr[r] && c <= A.col[q - 1]) return "CSR columns must be strictly ascending within a row";
            if (c == r) {
                if (!(A.val[q] > 0.0)) return "non-positive diagonal entry";
                diag = true;
            }
        }
        if (!diag) return "missing diagonal entry";
    }
    if (csr_reach(dim, n, A) > 2) return "couplings more than 2 vertices apart (the multicolour sweeps need reach <= 2)";
    return "";
}

}  // namespace mgmc
