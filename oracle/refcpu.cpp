// oracle/refcpu.cpp -- CPU restatement of the reference MGMC hot path (TEST INFRASTRUCTURE).
//
// This file is the parity oracle and the CPU baseline.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it; the product (multigridmc_amd) never does.
//
// It restates nilsfriess/MultigridMC (citations relative to the reference's src/) with plain
// std:: containers instead of Eigen (absent in this image, so the reference itself cannot be
// compiled here -- see DESIGN.md "Oracle"):
//   Lattice index maps ............ lattice/lattice{1,2,3}d.hh
//   FD shifted-Laplace assembly ... linear_operator/shiftedlaplace_fd_operator.cc:9-57
//   intergrid colidx / weights .... intergrid/intergrid_operator.cc:8-20, intergrid_operator_linear.cc:8-30
//   restrict / prolongate_add ..... intergrid/intergrid_operator.hh:74-120, to_sparse :123-144
//   Galerkin coarsening ........... linear_operator/linear_operator.cc:10-23 (R*A*R^T, SpGEMM)
//   LinearOperator::apply ......... linear_operator/linear_operator.hh:66-76
//   SORSmoother::apply_sparse ..... smoother/sor_smoother.cc:56-78
//   SORSampler / SSORSampler ...... sampler/sor_sampler.cc:9-59, sampler/ssor_sampler.cc:9-15
//   DenseCholeskySampler .......... sampler/cholesky_sampler.{hh,cc} (LLT, no permutation; banded storage)
//   MultigridMCSampler ............ sampler/multigridmc_sampler.cc:8-138
//   RNG plumbing .................. one shared std::mt19937_64, one std::normal_distribution<double>
//                                   per sampler object (sampler/sampler.hh:31-34, :69-71)
//
// Two modes:
//   FAITHFUL (0): the reference algorithm -- lexicographic forward / reverse sweeps, libstdc++
//                 mt19937_64 + normal_distribution (Marsaglia polar) in the reference's
//                 construction and call order.  Tier T1 of the parity contract.
//   MULTICOLOUR (1): the Gibbs updates visit the vertices colour by colour (red-black on the fine
//                 FD level, 2^d colours on Galerkin levels), the noise is the counter-based
//                 Philox4x32-10 / Box-Muller stream keyed by (seed, chain, pair, sweep tag,
//                 sample), and the SOR update is evaluated in the device's fused form
//                 (c = fma(sd, xi, f), x = fma(omega/diag, c - S, x), S an fma chain in ascending
//                 column order; restriction / prolongation / residual keep the reference
//                 arithmetic).  This replays the device chain bit for bit; it is written
//                 independently of multigridmc_amd/csrc.  Tier T2.
//
// Build: oracle/Makefile (g++ -O3 -ffp-contract=off -fopenmp, shared library; threads default to 1).
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "log_table_oracle.h"

namespace orc {

// Worker threads of the oracle's row-parallel loops (orc_set_threads; default 1 = serial, and the
// CPU baseline never changes it).  Only loops whose iterations are independent are split -- rows of
// an SpMV, vertices of one colour class, coarse points of a restriction, fine planes of a
// prolongation -- and every element is produced by the same operation sequence whatever the thread
// count, so a threaded oracle gives bitwise the serial oracle's results.  This is what makes the
// headline 512^3 hierarchy checkable in a GPU test (tests/test_gpu_headline.py).
static int g_threads = 1;
template <class F>
static void par_for(int64_t n, F&& f) {
    if (g_threads <= 1 || n < 8192) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
#pragma omp parallel for num_threads(g_threads) schedule(static)
    for (int64_t i = 0; i < n; ++i) f(i);
}
template <class F>
static int64_t par_max(int64_t n, F&& f) {
    int64_t m = 0;
    if (g_threads <= 1 || n < 8192) {
        for (int64_t i = 0; i < n; ++i) m = std::max(m, (int64_t)f(i));
        return m;
    }
#pragma omp parallel for num_threads(g_threads) schedule(static) reduction(max : m)
    for (int64_t i = 0; i < n; ++i) m = std::max(m, (int64_t)f(i));
    return m;
}

// =============================================================================================
// Lattice (lattice/lattice1d.hh, lattice2d.hh, lattice3d.hh): n cells -> (n-1)^d interior
// vertices, vertex 0 at Euclidean (1,1,1), lexicographic with x fastest.
// =============================================================================================
struct Lattice {
    int dim = 0;
    int n[3] = {0, 0, 0};
    int64_t nvertex() const {
        int64_t v = 1;
        for (int d = 0; d < dim; ++d) v *= (n[d] - 1);
        return v;
    }
    void lin2euc(int64_t ell, int idx[3]) const {
        idx[0] = idx[1] = idx[2] = 0;
        const int64_t a = n[0] - 1;
        if (dim == 1) {
            idx[0] = (int)ell + 1;
        } else if (dim == 2) {
            idx[0] = (int)(ell % a) + 1;
            idx[1] = (int)(ell / a) + 1;
        } else {
            const int64_t b = n[1] - 1;
            idx[0] = (int)((ell % (a * b)) % a) + 1;
            idx[1] = (int)((ell % (a * b)) / a) + 1;
            idx[2] = (int)(ell / (a * b)) + 1;
        }
    }
    int64_t euc2lin(const int idx[3]) const {
        if (dim == 1) return idx[0] - 1;
        if (dim == 2) return (int64_t)(idx[1] - 1) * (n[0] - 1) + (idx[0] - 1);
        return ((int64_t)(idx[2] - 1) * (n[1] - 1) + (idx[1] - 1)) * (n[0] - 1) + (idx[0] - 1);
    }
    bool interior(const int idx[3]) const {
        for (int d = 0; d < dim; ++d)
            if (idx[d] <= 0 || idx[d] >= n[d]) return false;
        return true;
    }
    // shifted_vertex_is_internal_vertex
    bool shifted(int64_t ell, const int s[3], int64_t& out) const {
        int idx[3];
        lin2euc(ell, idx);
        for (int d = 0; d < dim; ++d) idx[d] += s[d];
        if (!interior(idx)) return false;
        out = euc2lin(idx);
        return true;
    }
    // lattice3d.hh:227-234 etc: index on the next-finer lattice (2n cells)
    int64_t fine_vertex_idx(int64_t ell) const {
        int idx[3];
        lin2euc(ell, idx);
        Lattice f = *this;
        for (int d = 0; d < dim; ++d) {
            f.n[d] = 2 * n[d];
            idx[d] *= 2;
        }
        return f.euc2lin(idx);
    }
    Lattice coarse() const {
        Lattice c = *this;
        for (int d = 0; d < dim; ++d) c.n[d] = n[d] / 2;
        return c;
    }
};

// =============================================================================================
// CSR matrix (rows sorted by column, as Eigen's compressed storage after setFromTriplets)
// =============================================================================================
struct CSR {
    int64_t nrow = 0, ncol = 0;
    std::vector<int64_t> rowptr;
    std::vector<int32_t> col;
    std::vector<double> val;
    double diag(int64_t r) const {
        for (int64_t q = rowptr[r]; q < rowptr[r + 1]; ++q)
            if (col[q] == r) return val[q];
        return 0.0;
    }
};

// y = A x with Eigen's ColMajor accumulation order: y_i = ((0 + a_i,j1 x_j1) + a_i,j2 x_j2) ...
// with j ascending (A symmetric, so the row-wise ascending sum is the same sequence)
static void spmv(const CSR& A, const double* x, double* y) {
    par_for(A.nrow, [&](int64_t r) {
        double s = 0.0;
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) s += A.val[q] * x[A.col[q]];
        y[r] = s;
    });
}

// CSR from a per-row builder row(ell, cols, vals) -> count (entries sorted by column, at most 27):
// counts first, then every row written at its offset (row-parallel, same entries as a serial build)
template <class RowFn>
static CSR csr_from_rows(int64_t nrow, RowFn&& row) {
    CSR A;
    A.nrow = A.ncol = nrow;
    A.rowptr.assign(nrow + 1, 0);
    par_for(nrow, [&](int64_t ell) {
        int32_t c[27];
        double v[27];
        A.rowptr[ell + 1] = row(ell, c, v);
    });
    for (int64_t r = 0; r < nrow; ++r) A.rowptr[r + 1] += A.rowptr[r];
    A.col.resize((size_t)A.rowptr[nrow]);
    A.val.resize((size_t)A.rowptr[nrow]);
    par_for(nrow, [&](int64_t ell) { row(ell, A.col.data() + A.rowptr[ell], A.val.data() + A.rowptr[ell]); });
    return A;
}

// C = A * B (Gustavson, dense accumulator, sorted output)
static CSR spgemm(const CSR& A, const CSR& B) {
    CSR C;
    C.nrow = A.nrow;
    C.ncol = B.ncol;
    C.rowptr.assign(A.nrow + 1, 0);
    std::vector<double> acc(B.ncol, 0.0);
    std::vector<char> used(B.ncol, 0);
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

static CSR transpose(const CSR& A) {
    CSR T;
    T.nrow = A.ncol;
    T.ncol = A.nrow;
    T.rowptr.assign(A.ncol + 1, 0);
    for (int32_t c : A.col) T.rowptr[c + 1]++;
    for (int64_t r = 0; r < T.nrow; ++r) T.rowptr[r + 1] += T.rowptr[r];
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

// =============================================================================================
// Correlation-length models (correlationlength_model.hh:45-112): kappa^2 at a point
// =============================================================================================
struct KappaModel {
    int periodic = 0;
    double kappa_sq_const = 0.0;       // constant model: 1 / Lambda^2
    double Lambda_1 = 0.0, Lambda_2 = 0.0;  // periodic: (Lambda_max +/- Lambda_min) / 2
    double operator()(const double* x, int dim) const {
        if (!periodic) return kappa_sq_const;
        double L = Lambda_2;
        for (int d = 0; d < dim; ++d) L *= cos(M_PI * x[d]);
        L += Lambda_1;
        return 1. / (L * L);
    }
    static KappaModel constant(double kappa_sq) {
        KappaModel k;
        k.kappa_sq_const = kappa_sq;
        return k;
    }
};

// Lattice::vertex_coordinates (lattice2d.hh:188-195, lattice3d.hh): (0-based index + 1.0) * h
static void vertex_coords(const Lattice& lat, int64_t ell, double* x) {
    int idx[3];
    lat.lin2euc(ell, idx);
    for (int d = 0; d < lat.dim; ++d) x[d] = ((double)(idx[d] - 1) + 1.0) * (1. / double(lat.n[d]));
}

// =============================================================================================
// Fine operator: ShiftedLaplaceFDOperator (shiftedlaplace_fd_operator.cc:9-57)
// =============================================================================================
// One row of the FD operator: triplets (shifts in (d, -/+) order, then the diagonal), sorted by
// column as setFromTriplets leaves them (columns are distinct)
static int64_t fd_row(const Lattice& lat, const KappaModel& kappa, int64_t ell, int32_t* cols, double* vals) {
    const int dim = lat.dim;
    double hinv2[3] = {0, 0, 0};
    double cell_volume = 1.0;
    for (int d = 0; d < dim; ++d) {
        const double h = 1. / double(lat.n[d]);
        hinv2[d] = 1. / (h * h);
        cell_volume *= h;
    }
    std::pair<int64_t, double> r[7];
    int cnt = 0;
    double xv[3] = {0, 0, 0};
    vertex_coords(lat, ell, xv);
    double diagonal = cell_volume * kappa(xv, dim);
    for (int d = 0; d < dim; ++d) {
        for (int j = 0; j < 2; ++j) {
            int s[3] = {0, 0, 0};
            s[d] = 2 * j - 1;
            int64_t e;
            if (lat.shifted(ell, s, e)) r[cnt++] = {e, -cell_volume * hinv2[d]};
        }
        diagonal += 2. * cell_volume * hinv2[d];
    }
    r[cnt++] = {ell, diagonal};
    std::sort(r, r + cnt, [](const std::pair<int64_t, double>& a, const std::pair<int64_t, double>& b) {
        return a.first < b.first;
    });
    for (int q = 0; q < cnt; ++q) {
        cols[q] = (int32_t)r[q].first;
        vals[q] = r[q].second;
    }
    return cnt;
}

static CSR fd_operator(const Lattice& lat, const KappaModel& kappa) {
    return csr_from_rows(lat.nvertex(),
                         [&](int64_t ell, int32_t* cols, double* vals) { return fd_row(lat, kappa, ell, cols, vals); });
}

// ShiftedLaplaceFEMOperator with constant kappa^2 (shiftedlaplace_fem_operator.cc:9-145): sparsity
// of every valid 3^d shift (STEP 1, entries 0.0), then the cell loop (STEP 2): cells ascending (x
// fastest), basis pairs (alpha, beta) in cartesian_product order (common.hh:29-50: last dimension
// fastest), each entry += local * cell_volume with local = sum_q (kappa^2 phi_a phi_b + grad phi_a .
// (h^-2 grad phi_b)) w_q over GaussLegendreQuadrature(dim, 1) (quadrature.cc:11-55).
static CSR fem_operator(const Lattice& lat, const KappaModel& kappa) {
    const int dim = lat.dim;
    double h[3] = {1, 1, 1}, hinv2[3] = {0, 0, 0};
    double cell_volume = 1.0;
    for (int d = 0; d < dim; ++d) {
        h[d] = 1. / double(lat.n[d]);
        hinv2[d] = 1. / (h[d] * h[d]);
        cell_volume *= h[d];
    }
    const int nb = 1 << dim;  // basis functions / quadrature points per cell
    // cartesian products, last dimension fastest
    auto bits = [&](int q, int* b) {
        for (int j = 0; j < dim; ++j) b[j] = (q >> (dim - 1 - j)) & 1;
    };
    const double p1[2] = {-1.0 / sqrt(3.0), +1.0 / sqrt(3.0)};
    std::vector<double> qw(nb), qp((size_t)nb * 3, 0.0);
    for (int q = 0; q < nb; ++q) {
        int b[3];
        bits(q, b);
        double w = 1.0;
        for (int j = 0; j < dim; ++j) {
            w *= 0.5 * 1.0;
            qp[(size_t)q * 3 + j] = 0.5 * (p1[b[j]] + 1.0);
        }
        qw[q] = w;
    }
    auto phi = [&](const int* a, const double* x) {
        double v = 1.0;
        for (int j = 0; j < dim; ++j) v *= (a[j] == 0) ? (1.0 - x[j]) : x[j];
        return v;
    };
    auto grad = [&](const int* a, const double* x, double* g) {
        for (int k = 0; k < dim; ++k) {
            double v = 1.0;
            for (int j = 0; j < dim; ++j) v *= (j == k) ? ((a[j] == 0) ? -1.0 : +1.0) : ((a[j] == 0) ? (1.0 - x[j]) : x[j]);
            g[k] = v;
        }
    };
    // phi_phi / gradphi_gradphi tables in the reference's (alpha, beta, q) order
    std::vector<double> pp, gg;
    for (int ia = 0; ia < nb; ++ia)
        for (int ib = 0; ib < nb; ++ib)
            for (int q = 0; q < nb; ++q) {
                int a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
                bits(ia, a);
                bits(ib, b);
                const double* x = &qp[(size_t)q * 3];
                pp.push_back(phi(a, x) * phi(b, x));
                double ga[3] = {0, 0, 0}, gb[3] = {0, 0, 0};
                grad(a, x, ga);
                grad(b, x, gb);
                double t = ga[0] * (hinv2[0] * gb[0]);
                for (int k = 1; k < dim; ++k) t = t + ga[k] * (hinv2[k] * gb[k]);
                gg.push_back(t);
            }
    // STEP 1: sparsity, columns ascending
    CSR A;
    const int64_t nrow = lat.nvertex();
    A.nrow = A.ncol = nrow;
    A.rowptr.assign(nrow + 1, 0);
    const int zr = dim == 3 ? 1 : 0;
    for (int64_t ell = 0; ell < nrow; ++ell) {
        for (int sz = -zr; sz <= zr; ++sz)
            for (int sy = (dim >= 2 ? -1 : 0); sy <= (dim >= 2 ? 1 : 0); ++sy)
                for (int sx = -1; sx <= 1; ++sx) {
                    const int sh[3] = {sx, sy, sz};
                    int64_t e;
                    if (lat.shifted(ell, sh, e)) {
                        A.col.push_back((int32_t)e);
                        A.val.push_back(0.0);
                    }
                }
        A.rowptr[ell + 1] = (int64_t)A.col.size();
    }
    auto entry = [&](int64_t r, int64_t c) -> double& {
        for (int64_t k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k)
            if (A.col[k] == c) return A.val[k];
        fprintf(stderr, "fem_operator: missing entry\n");
        abort();
    };
    // STEP 2: cells ascending, cell coordinate x fastest (lattice3d.hh:83-91)
    int64_t ncell = 1;
    for (int d = 0; d < dim; ++d) ncell *= lat.n[d];
    for (int64_t cell = 0; cell < ncell; ++cell) {
        int cc[3] = {0, 0, 0};
        int64_t r = cell;
        for (int d = 0; d < dim; ++d) {
            cc[d] = (int)(r % lat.n[d]);
            r /= lat.n[d];
        }
        int count = 0;
        for (int ia = 0; ia < nb; ++ia)
            for (int ib = 0; ib < nb; ++ib) {
                int a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
                bits(ia, a);
                bits(ib, b);
                int va[3] = {0, 0, 0}, vb[3] = {0, 0, 0};
                for (int d = 0; d < dim; ++d) {
                    va[d] = cc[d] + a[d];
                    vb[d] = cc[d] + b[d];
                }
                if (lat.interior(va) && lat.interior(vb)) {
                    double local = 0.0;
                    for (int q = 0; q < nb; ++q) {
                        // x = h (xhat_q + cell), shiftedlaplace_fem_operator.cc:118-126
                        double xq[3] = {0, 0, 0};
                        for (int d = 0; d < dim; ++d) xq[d] = h[d] * (qp[(size_t)q * 3 + d] + (double)cc[d]);
                        local += (kappa(xq, dim) * pp[count] + gg[count]) * qw[q];
                        count++;
                    }
                    entry(lat.euc2lin(va), lat.euc2lin(vb)) += local * cell_volume;
                } else {
                    count += nb;
                }
            }
    }
    return A;
}

// SquaredShiftedLaplaceFDOperator, 2D only (squared_shiftedlaplace_fd_operator.cc:9-96): the 13-point
// diamond; an offset (+-1, 0) / (0, +-1) whose vertex is on the boundary adds the (+-2, 0) / (0, +-2)
// entry to the diagonal (homogeneous Neumann)
static CSR squared_fd_operator(const Lattice& lat, const KappaModel& kappa) {
    double h0 = 1. / double(lat.n[0]), h1 = 1. / double(lat.n[1]);
    const double hinv2[2] = {1. / (h0 * h0), 1. / (h1 * h1)};
    const double cell_volume = h0 * h1;
    double lap[2][2] = {{0, 0}, {0, 0}}, sq[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    lap[0][0] = -2 * (hinv2[0] + hinv2[1]);
    lap[1][0] = hinv2[0];
    lap[0][1] = hinv2[1];
    sq[0][0] = 6 * (hinv2[0] * hinv2[0] + hinv2[1] * hinv2[1]) + 8 * hinv2[0] * hinv2[1];
    sq[1][0] = -4 * hinv2[0] * (hinv2[0] + hinv2[1]);
    sq[0][1] = -4 * hinv2[1] * (hinv2[0] + hinv2[1]);
    sq[2][0] = hinv2[0] * hinv2[0];
    sq[0][2] = hinv2[1] * hinv2[1];
    sq[1][1] = 2 * hinv2[0] * hinv2[1];
    CSR A;
    const int64_t nrow = lat.nvertex();
    A.nrow = A.ncol = nrow;
    A.rowptr.assign(nrow + 1, 0);
    std::vector<std::pair<int64_t, double>> row;
    for (int64_t ell = 0; ell < nrow; ++ell) {
        row.clear();
        double xv[3] = {0, 0, 0};
        vertex_coords(lat, ell, xv);
        const double ab = kappa(xv, 2);
        double diagonal = (ab * ab - 2. * ab * lap[0][0] + sq[0][0]) * cell_volume;
        for (int j = -2; j <= 2; ++j)
            for (int k = -2; k <= 2; ++k) {
                const int aj = j < 0 ? -j : j, ak = k < 0 ? -k : k;
                if (aj + ak > 2 || (j == 0 && k == 0)) continue;
                const int sh[3] = {j, k, 0};
                int64_t e;
                if (lat.shifted(ell, sh, e)) {
                    double v = sq[aj][ak];
                    if (aj + ak == 1) v += -2. * ab * lap[aj][ak];
                    row.push_back({e, v * cell_volume});
                } else if (aj + ak == 1) {
                    diagonal += sq[2 * aj][2 * ak] * cell_volume;
                }
            }
        row.push_back({ell, diagonal});
        std::sort(row.begin(), row.end(), [](const std::pair<int64_t, double>& a, const std::pair<int64_t, double>& b) {
            return a.first < b.first;
        });
        for (auto& e : row) {
            A.col.push_back((int32_t)e.first);
            A.val.push_back(e.second);
        }
        A.rowptr[ell + 1] = (int64_t)A.col.size();
    }
    return A;
}

// =============================================================================================
// IntergridOperatorLinear
// =============================================================================================
struct Intergrid {
    Lattice fine, coarse;
    int stencil_size = 0;
    std::vector<double> matrix;
    std::vector<int64_t> colidx;
    std::vector<int> shift_last;  // shift of stencil entry k in the last dimension
    explicit Intergrid(const Lattice& lat) : fine(lat), coarse(lat.coarse()) {
        const int dim = lat.dim;
        stencil_size = (int)lround(pow(3, dim));
        const double stencil1d[3] = {0.5, 1.0, 0.5};
        const int shift1d[3] = {-1, 0, +1};
        std::vector<std::array<int, 3>> shift;
        for (int j = 0; j < stencil_size; ++j) {
            double m = 1.0;
            std::array<int, 3> s = {0, 0, 0};
            int mu = j;
            for (int d = 0; d < dim; ++d) {
                m *= stencil1d[mu % 3];
                s[d] = shift1d[mu % 3];
                mu /= 3;
            }
            matrix.push_back(m);
            shift.push_back(s);
            shift_last.push_back(s[dim - 1]);
        }
        const int64_t nc = coarse.nvertex();
        colidx.resize((size_t)nc * stencil_size);
        par_for(nc, [&](int64_t ec) {
            int idx[3];
            coarse.lin2euc(ec, idx);
            for (int d = 0; d < dim; ++d) idx[d] *= 2;
            const int64_t ell = fine.euc2lin(idx);
            for (int j = 0; j < stencil_size; ++j) {
                int64_t e = -1;
                if (!fine.shifted(ell, shift[j].data(), e)) {
                    fprintf(stderr, "oracle: intergrid shift left the lattice\n");
                    abort();
                }
                colidx[(size_t)ec * stencil_size + j] = e;
            }
        });
    }
    void restrict_(const double* x, double* xc) const {
        par_for(coarse.nvertex(), [&](int64_t ec) {
            double result = 0;
            for (int k = 0; k < stencil_size; ++k) result += matrix[k] * x[colidx[(size_t)ec * stencil_size + k]];
            xc[ec] = result;
        });
    }
    // The reference's scatter (coarse index ascending, then k).  Split by the fine vertices' last
    // coordinate p: the targets on fine plane (2D: row) p come from the coarse planes kc with
    // 2 kc + s = p, visited in ascending kc, each in ascending ec, taking the k whose last shift is
    // s.  Each fine vertex therefore receives its terms in the serial order (one per (ec, k)).
    void prolongate_add(double alpha, const double* xc, double* x) const {
        const int dim = fine.dim;
        const int64_t nc = coarse.nvertex();
        const int ncl = coarse.n[dim - 1];       // coarse planes 1 .. ncl-1
        const int64_t cplane = nc / (ncl - 1);  // coarse points per plane
        auto plane = [&](int64_t pi) {
            const int p = (int)pi + 1;  // fine plane 1 .. nfl-1
            for (int kc = (p - 1) / 2; kc <= (p + 1) / 2; ++kc) {
                if (kc < 1 || kc > ncl - 1) continue;
                const int s = p - 2 * kc;
                if (s < -1 || s > 1) continue;
                for (int64_t ec = (int64_t)(kc - 1) * cplane; ec < (int64_t)kc * cplane; ++ec) {
                    const double v = xc[ec];
                    for (int k = 0; k < stencil_size; ++k)
                        if (shift_last[k] == s) x[colidx[(size_t)ec * stencil_size + k]] += alpha * matrix[k] * v;
                }
            }
        };
        if (g_threads <= 1) {  // the reference's loop as written
            for (int64_t ec = 0; ec < nc; ++ec) {
                const double v = xc[ec];
                for (int k = 0; k < stencil_size; ++k) x[colidx[(size_t)ec * stencil_size + k]] += alpha * matrix[k] * v;
            }
            return;
        }
        const int nfl = fine.n[dim - 1];
        if (nfl - 1 < 64) {
            for (int64_t pi = 0; pi < nfl - 1; ++pi) plane(pi);
            return;
        }
#pragma omp parallel for num_threads(g_threads) schedule(static, 1)
        for (int64_t pi = 0; pi < nfl - 1; ++pi) plane(pi);
    }
    CSR to_sparse() const {
        CSR R;
        R.nrow = coarse.nvertex();
        R.ncol = fine.nvertex();
        R.rowptr.assign(R.nrow + 1, 0);
        std::vector<std::pair<int64_t, double>> row;
        for (int64_t ec = 0; ec < R.nrow; ++ec) {
            row.clear();
            for (int k = 0; k < stencil_size; ++k) row.push_back({colidx[(size_t)ec * stencil_size + k], matrix[k]});
            std::sort(row.begin(), row.end(),
                      [](const std::pair<int64_t, double>& a, const std::pair<int64_t, double>& b) { return a.first < b.first; });
            for (auto& e : row) {
                R.col.push_back((int32_t)e.first);
                R.val.push_back(e.second);
            }
            R.rowptr[ec + 1] = (int64_t)R.col.size();
        }
        return R;
    }
};

static CSR galerkin_spgemm(const CSR& A, const Intergrid& ig) {
    const CSR R = ig.to_sparse();
    const CSR P = transpose(R);
    const CSR RA = spgemm(R, A);
    return spgemm(RA, P);
}

// Galerkin coarse operator built row-by-row from the interior row of an R*A*R^T product
// evaluated on a small lattice (8 cells per direction).  Because the fine operator has constant
// coefficients and every row of the product is formed from the same terms in the same order,
// that row equals every row of the full product (Dirichlet truncation only drops entries);
// this is what makes the 512^3 hierarchy buildable on a CPU in seconds.
static CSR stencil_csr(const Lattice& lat, const double st[27]);
static void stencil_of_interior_row(const CSR& A, const Lattice& lat, double st[27]);

static CSR galerkin_stencil_mode(const CSR& A_small_src, const Lattice& small, const Lattice& coarse_big,
                                 double st_out[27]) {
    Intergrid ig(small);
    const CSR Ac = galerkin_spgemm(A_small_src, ig);
    stencil_of_interior_row(Ac, ig.coarse, st_out);
    return stencil_csr(coarse_big, st_out);
}

static inline int sidx(int dim, int dx, int dy, int dz) {
    if (dim == 3) return (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1);
    if (dim == 2) return (dy + 1) * 3 + (dx + 1);
    return dx + 1;
}

static CSR stencil_csr(const Lattice& lat, const double st[27]) {
    const int dim = lat.dim;
    const int zr = dim == 3 ? 1 : 0, yr = dim >= 2 ? 1 : 0;
    return csr_from_rows(lat.nvertex(), [&](int64_t ell, int32_t* cols, double* vals) -> int64_t {
        int64_t cnt = 0;
        for (int dz = -zr; dz <= zr; ++dz)
            for (int dy = -yr; dy <= yr; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const double v = st[sidx(dim, dx, dy, dz)];
                    if (v == 0.0) continue;
                    int s[3] = {dx, dy, dz};
                    int64_t e;
                    if (lat.shifted(ell, s, e)) {
                        cols[cnt] = (int32_t)e;
                        vals[cnt++] = v;
                    }
                }
        return cnt;
    });
}

static void stencil_of_interior_row(const CSR& A, const Lattice& lat, double st[27]) {
    for (int k = 0; k < 27; ++k) st[k] = 0.0;
    int idx[3] = {2, 2, 2};
    const int64_t r = lat.euc2lin(idx);
    int ci[3];
    for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
        lat.lin2euc(A.col[q], ci);
        const int dx = ci[0] - idx[0];
        const int dy = lat.dim >= 2 ? ci[1] - idx[1] : 0;
        const int dz = lat.dim == 3 ? ci[2] - idx[2] : 0;
        st[sidx(lat.dim, dx, dy, dz)] = A.val[q];
    }
}

// =============================================================================================
// Philox4x32-10 + Box-Muller (multicolour mode); same definition as the device path
// (DESIGN.md "Noise"), written independently.
// =============================================================================================
static inline void philox10(uint32_t ctr[4], uint32_t key0, uint32_t key1) {
    for (int round = 0; round < 10; ++round) {
        const uint64_t prod0 = (uint64_t)0xD2511F53u * (uint64_t)ctr[0];
        const uint64_t prod1 = (uint64_t)0xCD9E8D57u * (uint64_t)ctr[2];
        const uint32_t out0 = (uint32_t)(prod1 >> 32) ^ ctr[1] ^ key0;
        const uint32_t out2 = (uint32_t)(prod0 >> 32) ^ ctr[3] ^ key1;
        ctr[0] = out0;
        ctr[1] = (uint32_t)prod1;
        ctr[2] = out2;
        ctr[3] = (uint32_t)prod0;
        key0 += 0x9E3779B9u;
        key1 += 0xBB67AE85u;
    }
}

static inline double bits_to_double(uint64_t b) {
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static inline uint64_t double_to_bits(double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    return b;
}

// log(u), u in [2^-52, 1]: u = 2^e m, r = fma(m, rc_i, -1) with the literal 64-entry table
// (log_table_oracle.h, i = top 6 mantissa bits), log1p(r) to degree 8, plus -log(rc_i) = hi + lo
static double ln_unit(double u) {
    const uint64_t b = double_to_bits(u);
    const int e = (int)((b >> 52) & 0x7ff) - 1023;
    const uint64_t mant = b & 0x000fffffffffffffull;
    const int idx = (int)(mant >> 46);
    const double m = bits_to_double(mant | 0x3ff0000000000000ull);
    const double r = fma(m, LOGTAB_RC[idx], -1.0);
    static const double coef[7] = {-1.0 / 8.0, 1.0 / 7.0, -1.0 / 6.0, 1.0 / 5.0, -1.0 / 4.0, 1.0 / 3.0, -0.5};
    double q = coef[0];
    for (int k = 1; k < 7; ++k) q = fma(q, r, coef[k]);
    const double p = fma(r * r, q, r);
    const double de = (double)e;
    return fma(de, 6.93147180369123816490e-01, LOGTAB_HI[idx]) + (fma(de, 1.90821492927058770002e-10, LOGTAB_LO[idx]) + p);
}

// (cos 2 pi t, sin 2 pi t): k = round(64 t), exact remainder r = t - k/64, theta = 2 pi r, sin theta
// to degree 9, cos theta - 1 to degree 8, addition theorem with the literal table SINCOS_TAB
// (log_table_oracle.h: cos, sin of 2 pi k/64)
static void cos_sin_2pi(double t, double& c, double& s) {
    const int k = (int)fma(t, 64.0, 0.5);
    const double r = fma((double)(-k), 0.015625, t);
    const double th = r * 6.28318530717958647692;
    const double t2 = th * th;
    static const double sc[4] = {1.0 / 362880.0, -1.0 / 5040.0, 1.0 / 120.0, -1.0 / 6.0};
    double ps = sc[0];
    for (int q = 1; q < 4; ++q) ps = fma(ps, t2, sc[q]);
    const double sn = fma(th * t2, ps, th);
    static const double cc[4] = {1.0 / 40320.0, -1.0 / 720.0, 1.0 / 24.0, -0.5};
    double pc = cc[0];
    for (int q = 1; q < 4; ++q) pc = fma(pc, t2, cc[q]);
    const double w = pc * t2;
    const double C = SINCOS_TAB[2 * k], S = SINCOS_TAB[2 * k + 1];
    c = fma(C, w, fma(-S, sn, C));
    s = fma(S, w, fma(C, sn, S));
}

static void philox_normals(uint64_t seed, uint64_t chain, uint32_t pair, uint32_t tag, uint64_t sample, double& z0,
                           double& z1) {
    uint32_t ctr[4] = {pair, tag, (uint32_t)sample, (uint32_t)(sample >> 32)};
    philox10(ctr, (uint32_t)seed, (uint32_t)chain ^ (uint32_t)(seed >> 32));
    // exact 52-bit uniforms: v = 1.m in [1,2), u1 = 2 - v in (0,1], u2 = v - 1 in [0,1)
    const uint64_t m1 = ((uint64_t)ctr[0] << 20) | (uint64_t)(ctr[1] >> 12);
    const uint64_t m2 = ((uint64_t)ctr[2] << 20) | (uint64_t)(ctr[3] >> 12);
    const double u1 = 2.0 - bits_to_double(0x3ff0000000000000ull | m1);
    const double u2 = bits_to_double(0x3ff0000000000000ull | m2) - 1.0;
    const double rr = -2.0 * ln_unit(u1);
    const double rad = sqrt(rr > 0.0 ? rr : 0.0);
    double c, s;
    cos_sin_2pi(u2, c, s);
    z0 = rad * c;
    z1 = rad * s;
}

// =============================================================================================
// Samplers
// =============================================================================================
enum Mode { FAITHFUL = 0, MULTICOLOUR = 1 };
static const uint32_t LR_PAIR0 = 0xFFFFF000u;  // Philox pair ids of the low-rank noise (above any lattice pair)
enum Direction { FORWARD = 1, BACKWARD = 2 };

// Low-rank measurement part of a posterior operator (measured_operator.cc:9-49,
// linear_operator.hh:187-197): B (N x m, sparse columns, rows ascending), Sigma (diagonal).  Coarse
// levels carry B_c = R B (linear_operator.cc:15-19), Sigma_c = Sigma.  A column that covers every
// vertex (the global average measurement and its restrictions) is "dense".
struct LowRank {
    int m = 0;
    std::vector<std::vector<std::pair<int64_t, double>>> cols;
    std::vector<char> dense;
    std::vector<double> sigma;
    int split = -1;  // MULTICOLOUR patch order: the split column (lr_patch_mc), -1 none
};

struct Level {
    Lattice lat;
    CSR A;
    bool fold = false;  // multicolour: residual by folded_row_sum (a 3D 27-point reflection-symmetric stencil level)
    int ncolours = 2;  // multicolour scheme: 2 (FD level) or 2^d (Galerkin level)
    std::vector<int> colour;  // per row
    std::vector<uint32_t> pair;
    std::vector<char> cos_branch;
    LowRank lr;
};

struct Ctx {
    Mode mode = FAITHFUL;
    std::mt19937_64 rng;
    uint64_t seed = 0, chain = 0;
    uint64_t sample = 0;  // multicolour: sample index of the current cycle
    uint32_t tag = 0;     // multicolour: running sweep tag within the current cycle
};

// largest coordinate distance between coupled vertices (1 for 3^d-point operators, 2 for the
// squared FD operator and its Galerkin levels)
static int coupling_reach(const Level& L) {
    return (int)par_max(L.A.nrow, [&](int64_t r) {
        int reach = 0, a[3], b[3];
        L.lat.lin2euc(r, a);
        for (int64_t q = L.A.rowptr[r]; q < L.A.rowptr[r + 1]; ++q) {
            L.lat.lin2euc(L.A.col[q], b);
            for (int d = 0; d < L.lat.dim; ++d) reach = std::max(reach, std::abs(a[d] - b[d]));
        }
        return reach;
    });
}

// 1 if some row couples two vertices that are not axis neighbours (|dx| + |dy| + |dz| > 1)
static bool off_axis_coupling(const Level& L) {
    return par_max(L.A.nrow, [&](int64_t r) {
               int a[3], b[3];
               L.lat.lin2euc(r, a);
               for (int64_t q = L.A.rowptr[r]; q < L.A.rowptr[r + 1]; ++q) {
                   L.lat.lin2euc(L.A.col[q], b);
                   int taxi = 0;
                   for (int d = 0; d < L.lat.dim; ++d) taxi += std::abs(a[d] - b[d]);
                   if (taxi > 1) return 1;
               }
               return 0;
           }) != 0;
}

// colour classes of the multicolour sweeps: red-black for a fine level whose couplings are all axis
// neighbours (the 5/7-point FD pattern), coordinate parities (2^d colours) for other reach-1
// levels, coordinates mod 3 (3^d colours) for reach-2 levels
static void init_colouring(Level& L, bool fine_level) {
    const int64_t n = L.lat.nvertex();
    L.colour.resize(n);
    L.pair.resize(n);
    L.cos_branch.resize(n);
    const int dim = L.lat.dim;
    const bool mod3 = coupling_reach(L) >= 2;
    bool fd_level = fine_level && !mod3 && !off_axis_coupling(L);
    L.ncolours = fd_level ? 2 : (mod3 ? (dim == 3 ? 27 : 9) : (1 << dim));
    par_for(n, [&](int64_t e) {
        int idx[3];
        L.lat.lin2euc(e, idx);
        if (fd_level)
            L.colour[e] = (idx[0] + idx[1] + idx[2]) & 1;
        else if (mod3)
            L.colour[e] = (idx[0] % 3) + 3 * (idx[1] % 3) + (dim == 3 ? 9 * (idx[2] % 3) : 0);
        else
            L.colour[e] = (idx[0] & 1) | ((idx[1] & 1) << 1) | ((idx[2] & 1) << 2);
        uint64_t row = 0;
        if (dim == 2) row = (uint64_t)(idx[1] - 1);
        if (dim == 3) row = (uint64_t)(idx[2] - 1) * (uint64_t)(L.lat.n[1] - 1) + (uint64_t)(idx[1] - 1);
        L.pair[e] = (uint32_t)(row * (uint64_t)(L.lat.n[0] / 2) + (uint64_t)((idx[0] - 1) >> 1));
        L.cos_branch[e] = (idx[0] & 1) ? 1 : 0;
    });
}

// one SOR update of row ell (sor_smoother.cc:70-75), reference arithmetic
static inline void sor_row(const CSR& A, const double* diag, double omega, const double* b, double* x, int64_t ell) {
    double residual = 0.0;
    for (int64_t k = A.rowptr[ell]; k < A.rowptr[ell + 1]; ++k) residual += A.val[k] * x[A.col[k]];
    x[ell] += omega * (b[ell] - residual) / diag[ell];
}

// the same update in the device's fused form (MULTICOLOUR mode): S = fma chain over the row in
// ascending column order, x = fma(omega/diag, b - S, x)
static inline void sor_row_fused(const CSR& A, const double* wd, const double* b, double* x, int64_t ell) {
    int64_t k = A.rowptr[ell];
    double s = A.val[k] * x[A.col[k]];
    for (++k; k < A.rowptr[ell + 1]; ++k) s = fma(A.val[k], x[A.col[k]], s);
    x[ell] = fma(wd[ell], b[ell] - s, x[ell]);
}

// ---- low-rank helpers ----
// sum_i (sc B_ik) v_i.  FAITHFUL: sequential over the column's entries (the reference's sparse
// products).  MULTICOLOUR (= device order, mgmc_lowrank.hpp): the column's entry list (rows
// ascending; a dense column lists every row) is cut into blocks of LR_BLK entries; in each block
// lane l of 64 sums entries l, l+64, ... from 0.0 and the lanes combine by the xor butterfly
// (32, 16, 8, 4, 2, 1); the block partials are combined the same way (lane-strided + butterfly).
static const int LR_BLK = 4096;
static double butterfly64(double* v) {
    for (int off = 32; off >= 1; off >>= 1) {
        double t[64];
        for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
        std::copy(t, t + 64, v);
    }
    return v[0];
}
static double blocked_dot(const std::vector<std::pair<int64_t, double>>& col, double sc, const double* v);
static double lr_dot(const Level& L, int k, double sc, const double* v, Mode mode) {
    const auto& col = L.lr.cols[k];
    if (mode == FAITHFUL) {
        double s = 0.0;
        for (const auto& e : col) s += (sc * e.second) * v[e.first];
        return s;
    }
    return blocked_dot(col, sc, v);
}
// the device's fixed dot order (4096-entry blocks, lane-strided sums, xor butterflies)
static double blocked_dot(const std::vector<std::pair<int64_t, double>>& col, double sc, const double* v) {
    const int64_t n = (int64_t)col.size();
    const int64_t nblk = (n + LR_BLK - 1) / LR_BLK;
    std::vector<double> part(nblk);
    double acc[64];
    for (int64_t b = 0; b < nblk; ++b) {
        const int64_t end = std::min(n, (b + 1) * LR_BLK);
        for (int l = 0; l < 64; ++l) {
            acc[l] = 0.0;
            for (int64_t e = b * LR_BLK + l; e < end; e += 64) acc[l] = acc[l] + (sc * col[e].second) * v[col[e].first];
        }
        part[b] = butterfly64(acc);
    }
    for (int l = 0; l < 64; ++l) {
        acc[l] = 0.0;
        for (int64_t b = l; b < nblk; b += 64) acc[l] = acc[l] + part[b];
    }
    return butterfly64(acc);
}
// e = B s (e_i accumulates its columns in ascending k; Eigen's sparse-times-dense order)
static void lr_expand(const Level& L, const double* s, double* e) {
    std::fill(e, e + L.A.nrow, 0.0);
    for (int k = 0; k < L.lr.m; ++k)
        for (const auto& en : L.lr.cols[k]) e[en.first] += en.second * s[k];
}
// out = f +/- B s in the device's order (mgmc_lowrank.hpp lr_row_patch, MULTICOLOUR): f_i +/- e_i,
// e_i = 0.0 + sum_k B_ik s_k in ascending k -- or, on a level with a split column g (lr.split), the
// column added last on its own: (f_i +/- e_loc,i) +/- e_g,i, e_loc summed over k != g and applied on
// the rows with such a k, e_g,i = 0.0 + B_ig s_g.  The same sum in another order as the reference's
// c += B xi (sor_sampler.cc:48-56) and its residual (FAITHFUL keeps the reference's).
static void lr_patch_mc(const Level& L, const double* s, const double* f, double* out, bool minus) {
    const int64_t n = L.A.nrow;
    const int g = L.lr.split;
    std::vector<double> e(n, 0.0);
    std::vector<char> any(n, 0);
    for (int k = 0; k < L.lr.m; ++k) {
        if (k == g) continue;
        for (const auto& en : L.lr.cols[k]) {
            e[en.first] += en.second * s[k];
            any[en.first] = 1;
        }
    }
    for (int64_t i = 0; i < n; ++i) {
        if (g < 0) {
            out[i] = minus ? f[i] - e[i] : f[i] + e[i];
            continue;
        }
        double t = f[i];
        if (any[i]) t = minus ? t - e[i] : t + e[i];
        const double eg = 0.0 + L.lr.cols[g][i].second * s[g];  // (a dense column lists every row)
        out[i] = minus ? t - eg : t + eg;
    }
}

// y = A x + B (Sigma^{-1} B^T x)  (linear_operator.hh:66-76); t_k in lr_dot order with the
// Sigma^{-1}-scaled column values of Sigma_inv_BT (measured_operator.cc:48)
static void posterior_apply(const Level& L, const double* x, double* y, Mode mode) {
    spmv(L.A, x, y);
    if (L.lr.m == 0) return;
    std::vector<double> t(L.lr.m), g(L.A.nrow);
    for (int k = 0; k < L.lr.m; ++k) t[k] = lr_dot(L, k, 1.0 / L.lr.sigma[k], x, mode);
    lr_expand(L, t.data(), g.data());
    for (int64_t i = 0; i < L.A.nrow; ++i) y[i] += g[i];
}

// ---- the device's class-folded residual sum (mgmc_kernels.hpp fold27, restated) ----
// A level folds when its stencil is 27-point and bitwise reflection-symmetric (each of dx, dy, dz ->
// -d leaves every coefficient's bits unchanged): every Galerkin level of the cubic FD hierarchies.
static bool fold_stencil(const Lattice& lat, const CSR& A) {
    if (lat.dim != 3) return false;
    for (int d = 0; d < 3; ++d)
        if (lat.n[d] < 4) return false;  // no interior row (2,2,2): nothing to fold
    int idx[3] = {2, 2, 2};
    const int64_t r = lat.euc2lin(idx);
    if (A.rowptr[r + 1] - A.rowptr[r] != 27) return false;
    double st[27];
    stencil_of_interior_row(A, lat, st);
    for (int dz = 0; dz < 3; ++dz)
        for (int dy = 0; dy < 3; ++dy)
            for (int dx = 0; dx < 3; ++dx) {
                const double a = st[dz * 9 + dy * 3 + dx], b = st[(2 - dz) * 9 + dy * 3 + dx];
                const double c = st[dz * 9 + (2 - dy) * 3 + dx], e = st[dz * 9 + dy * 3 + (2 - dx)];
                if (memcmp(&a, &b, 8) || memcmp(&a, &c, 8) || memcmp(&a, &e, 8)) return false;
            }
    return true;
}
// sum_k a_k x_k of row r by coefficient class: the neighbours with equal (|dx|, |dy|, |dz|) share one
// coefficient; class c = [dx == 0] + 2 [dy == 0] + 4 [dz == 0] sums its present entries in CSR
// (= ascending offset) order, then y = a_7 s_7, fma(a_c, s_c, y) for c = 6 .. 0 over the present
// classes.  Truncated entries are zeros on the device (adding them changes no bits but a zero's sign).
static double folded_row_sum(const Level& L, int64_t r, const double* x) {
    double s[8], a[8];
    bool has[8] = {false, false, false, false, false, false, false, false};
    int rc[3], cc[3];
    L.lat.lin2euc(r, rc);
    for (int64_t q = L.A.rowptr[r]; q < L.A.rowptr[r + 1]; ++q) {
        L.lat.lin2euc(L.A.col[q], cc);
        const int c = (cc[0] == rc[0] ? 1 : 0) + (cc[1] == rc[1] ? 2 : 0) + (cc[2] == rc[2] ? 4 : 0);
        if (!has[c]) {
            s[c] = x[L.A.col[q]];
            a[c] = L.A.val[q];
            has[c] = true;
        } else {
            s[c] = s[c] + x[L.A.col[q]];
        }
    }
    double y = 0.0;
    bool started = false;
    for (int c = 7; c >= 0; --c) {
        if (!has[c]) continue;
        y = started ? fma(a[c], s[c], y) : a[c] * s[c];
        started = true;
    }
    return y;
}
static void spmv_level(const Level& L, const double* x, double* y, Mode mode) {
    if (mode == MULTICOLOUR && L.fold)
        par_for(L.A.nrow, [&](int64_t r) { y[r] = folded_row_sum(L, r, x); });
    else
        spmv(L.A, x, y);
}

// r = f - (A x + B Sigma^{-1} B^T x).  FAITHFUL: the reference's apply then subtract.  MULTICOLOUR
// (device order): the low-rank term is folded into f first (lr_patch_mc), r = (f - g) - A x, so the
// device's residual kernels run unchanged on a patched f.
// MULTICOLOUR on a fold level: A x by folded_row_sum (the device's residual kernels).
static void posterior_residual(const Level& L, const double* f, const double* x, double* r, Mode mode) {
    const int64_t n = L.A.nrow;
    if (mode == FAITHFUL || L.lr.m == 0) {
        if (mode == MULTICOLOUR && L.fold && L.lr.m == 0)
            spmv_level(L, x, r, mode);
        else
            posterior_apply(L, x, r, mode);
        par_for(n, [&](int64_t q) { r[q] = f[q] - r[q]; });
        return;
    }
    std::vector<double> t(L.lr.m), fp(n);
    for (int k = 0; k < L.lr.m; ++k) t[k] = lr_dot(L, k, 1.0 / L.lr.sigma[k], x, mode);
    lr_patch_mc(L, t.data(), f, fp.data(), true);
    spmv_level(L, x, r, mode);
    for (int64_t q = 0; q < n; ++q) r[q] = fp[q] - r[q];
}

// inverse of a small dense matrix (row-major m x m): Gauss-Jordan with partial pivoting
static std::vector<double> small_inverse(std::vector<double> M, int m) {
    std::vector<double> I((size_t)m * m, 0.0);
    for (int i = 0; i < m; ++i) I[(size_t)i * m + i] = 1.0;
    for (int c = 0; c < m; ++c) {
        int piv = c;
        for (int r = c + 1; r < m; ++r)
            if (fabs(M[(size_t)r * m + c]) > fabs(M[(size_t)piv * m + c])) piv = r;
        if (piv != c)
            for (int q = 0; q < m; ++q) {
                std::swap(M[(size_t)c * m + q], M[(size_t)piv * m + q]);
                std::swap(I[(size_t)c * m + q], I[(size_t)piv * m + q]);
            }
        const double d = M[(size_t)c * m + c];
        for (int q = 0; q < m; ++q) {
            M[(size_t)c * m + q] /= d;
            I[(size_t)c * m + q] /= d;
        }
        for (int r = 0; r < m; ++r) {
            if (r == c) continue;
            const double f = M[(size_t)r * m + c];
            for (int q = 0; q < m; ++q) {
                M[(size_t)r * m + q] -= f * M[(size_t)c * m + q];
                I[(size_t)r * m + q] -= f * I[(size_t)c * m + q];
            }
        }
    }
    return I;
}

struct SORSmoother {
    const Level* L;
    double omega;
    Direction direction;
    std::vector<double> diag, wd;
    mutable std::vector<double> bbar;  // N x m row-major; built on first use (low-rank operators)
    mutable Mode bbar_mode = FAITHFUL;
    SORSmoother(const Level* L_, double omega_, Direction d) : L(L_), omega(omega_), direction(d) {
        diag.resize(L->A.nrow);
        wd.resize(L->A.nrow);
        par_for(L->A.nrow, [&](int64_t r) {
            diag[r] = L->A.diag(r);
            wd[r] = omega / diag[r];
        });
    }
    // bar(B) = (L + D/omega)^{-1} B (Sigma + B^T (L + D/omega)^{-1} B)^{-1} (forward; L^T backward),
    // sor_smoother.cc:17-37.  The triangular solves: FAITHFUL = lexicographic substitution (the
    // reference's split), MULTICOLOUR = one noise-free multicolour sweep from zero in this
    // smoother's colour order (the split of the multicolour sweep; the device computes the same).
    void build_bbar(Mode mode) const {
        const int m = L->lr.m;
        const int64_t n = L->A.nrow;
        std::vector<double> Y((size_t)n * m), b(n), y(n);
        for (int l = 0; l < m; ++l) {
            std::fill(b.begin(), b.end(), 0.0);
            for (const auto& e : L->lr.cols[l]) b[e.first] = e.second;
            std::fill(y.begin(), y.end(), 0.0);
            if (mode == FAITHFUL) {
                const CSR& A = L->A;
                for (int64_t e_ = 0; e_ < n; ++e_) {
                    const int64_t i = direction == FORWARD ? e_ : n - 1 - e_;
                    double s = b[i];
                    for (int64_t q = A.rowptr[i]; q < A.rowptr[i + 1]; ++q) {
                        const int64_t j = A.col[q];
                        if (direction == FORWARD ? j < i : j > i) s -= A.val[q] * y[j];
                    }
                    y[i] = s / (diag[i] + (1. - omega) / omega * diag[i]);
                }
            } else {
                sweep(MULTICOLOUR, b.data(), y.data());
            }
            for (int64_t i = 0; i < n; ++i) Y[(size_t)i * m + l] = y[i];
        }
        std::vector<double> M((size_t)m * m), col(n);
        for (int l = 0; l < m; ++l) {
            for (int64_t i = 0; i < n; ++i) col[i] = Y[(size_t)i * m + l];
            for (int k = 0; k < m; ++k) M[(size_t)k * m + l] = (k == l ? L->lr.sigma[k] : 0.0) + lr_dot(*L, k, 1.0, col.data(), mode);
        }
        const std::vector<double> Minv = small_inverse(M, m);
        bbar.assign((size_t)n * m, 0.0);
        for (int64_t i = 0; i < n; ++i)
            for (int k = 0; k < m; ++k) {
                double u = 0.0;
                for (int l = 0; l < m; ++l)
                    u = mode == FAITHFUL ? u + Y[(size_t)i * m + l] * Minv[(size_t)l * m + k]
                                         : fma(Y[(size_t)i * m + l], Minv[(size_t)l * m + k], u);
                bbar[(size_t)i * m + k] = u;
            }
        bbar_mode = mode;
    }
    // SORSmoother::apply (sor_smoother.cc:41-53) with nsmooth = 1: sweep, then x -= bar(B) (B^T x)
    void apply(Mode mode, const double* b, double* x) const {
        sweep(mode, b, x);
        fix(mode, x);
    }
    // the low-rank update after apply_sparse (sor_smoother.cc:46-51): x -= bar(B) (B^T x)
    void fix(Mode mode, double* x) const {
        const int m = L->lr.m;
        if (m == 0) return;
        if (bbar.empty() || bbar_mode != mode) build_bbar(mode);
        std::vector<double> w(m);
        for (int k = 0; k < m; ++k) w[k] = lr_dot(*L, k, 1.0, x, mode);
        for (int64_t i = 0; i < L->A.nrow; ++i) {
            double u = 0.0;
            for (int k = 0; k < m; ++k) u = mode == FAITHFUL ? u + bbar[(size_t)i * m + k] * w[k] : fma(bbar[(size_t)i * m + k], w[k], u);
            x[i] = x[i] - u;
        }
    }
    void sweep(Mode mode, const double* b, double* x) const {
        const int64_t nrow = L->A.nrow;
        if (mode == FAITHFUL) {
            for (int64_t e_ = 0; e_ < nrow; ++e_) {
                const int64_t ell = (direction == FORWARD) ? e_ : nrow - 1 - e_;
                sor_row(L->A, diag.data(), omega, b, x, ell);
            }
        } else {
            const int nc = L->ncolours;
            for (int cc = 0; cc < nc; ++cc) {
                const int colour = (direction == FORWARD) ? cc : nc - 1 - cc;
                // a colour class reads only other colours: its rows are independent
                par_for(nrow, [&](int64_t ell) {
                    if (L->colour[ell] == colour) sor_row_fused(L->A, wd.data(), b, x, ell);
                });
            }
        }
    }
};

struct Sampler {
    Ctx* ctx;
    mutable std::normal_distribution<double> normal_dist{0.0, 1.0};
    explicit Sampler(Ctx* c) : ctx(c) {}
    virtual ~Sampler() {}
    virtual void apply(const double* f, double* x) = 0;
};

struct SORSampler : Sampler {
    const Level* L;
    double omega;
    Direction direction;
    unsigned nsmooth;
    std::vector<double> c_rhs;
    std::vector<double> sqrt_precision_diag;
    SORSmoother smoother;
    SORSampler(Ctx* c, const Level* L_, double omega_, unsigned nsmooth_, Direction d)
        : Sampler(c), L(L_), omega(omega_), direction(d), nsmooth(nsmooth_), smoother(L_, omega_, d) {
        const int64_t nrow = L->A.nrow;
        c_rhs.resize(nrow);
        sqrt_precision_diag.resize(nrow);
        par_for(nrow, [&](int64_t ell) { sqrt_precision_diag[ell] = sqrt(smoother.diag[ell] * (2. - omega) / omega); });
    }
    void apply(const double* f, double* x) override {
        const int64_t n = (int64_t)c_rhs.size();
        for (unsigned k = 0; k < nsmooth; ++k) {
            if (ctx->mode == FAITHFUL) {
                for (int64_t ell = 0; ell < n; ++ell) {
                    const double tmp = sqrt_precision_diag[ell];
                    c_rhs[ell] = tmp * normal_dist(ctx->rng) + f[ell];
                }
                if (L->lr.m > 0) {  // c += (B Sigma^{-1/2}) xi' (sor_sampler.cc:48-56)
                    std::vector<double> xi(L->lr.m), e(n, 0.0);
                    for (int k = 0; k < L->lr.m; ++k) xi[k] = normal_dist(ctx->rng);
                    for (int k = 0; k < L->lr.m; ++k) {
                        const double s = sqrt(1.0 / L->lr.sigma[k]);
                        for (const auto& en : L->lr.cols[k]) e[en.first] += (en.second * s) * xi[k];
                    }
                    for (int64_t ell = 0; ell < n; ++ell) c_rhs[ell] += e[ell];
                }
            } else {
                const uint32_t tag = ctx->tag++;
                // low-rank noise first: f_eff = f + B Sigma^{-1/2} xi', xi'_k from Philox pair
                // LR_PAIR0 + k/2 (cos for even k) of this sweep's tag; c = fma(sd, xi, f_eff)
                std::vector<double> feff;
                const double* fe = f;
                if (L->lr.m > 0) {
                    feff.resize(n);
                    std::vector<double> sv(L->lr.m);
                    for (int k = 0; k < L->lr.m; ++k) {
                        double z0, z1;
                        philox_normals(ctx->seed, ctx->chain, LR_PAIR0 + (uint32_t)(k >> 1), tag, ctx->sample, z0, z1);
                        sv[k] = sqrt(1.0 / L->lr.sigma[k]) * ((k & 1) ? z1 : z0);
                    }
                    lr_patch_mc(*L, sv.data(), f, feff.data(), false);
                    fe = feff.data();
                }
                const uint64_t sample = ctx->sample;
                par_for(n, [&](int64_t ell) {
                    double z0, z1;
                    philox_normals(ctx->seed, ctx->chain, L->pair[ell], tag, sample, z0, z1);
                    const double xi = L->cos_branch[ell] ? z0 : z1;
                    c_rhs[ell] = fma(sqrt_precision_diag[ell], xi, fe[ell]);
                });
            }
            smoother.apply(ctx->mode, c_rhs.data(), x);
        }
    }
};

struct SSORSampler : Sampler {
    unsigned nsmooth;
    SORSampler fwd, bwd;
    SSORSampler(Ctx* c, const Level* L, double omega, unsigned nsmooth_)
        : Sampler(c), nsmooth(nsmooth_), fwd(c, L, omega, 1, FORWARD), bwd(c, L, omega, 1, BACKWARD) {}
    void apply(const double* f, double* x) override {
        for (unsigned k = 0; k < nsmooth; ++k) {
            fwd.apply(f, x);
            bwd.apply(f, x);
        }
    }
};

// DenseCholeskySampler (cholesky_sampler.hh:50-66, EigenDenseLLT): A = L L^T,
// x = L^{-T}(xi + L^{-1} f)
// U = L^{-T} (upper triangular) and G = U U^T = Q^{-1} from the lower Cholesky factor L (row-major):
// L^{-1} by forward substitution column by column, G_ij = sum_{k >= max(i,j)} U_ik U_jk ascending k.
// The device's host setup (mgmc_capi.hip) runs the same loops.
static void dense_factor_inverses(const std::vector<double>& L, int64_t n, std::vector<double>& U,
                                  std::vector<double>& G) {
    std::vector<double> Li((size_t)n * n, 0.0);  // L^{-1}, lower
    for (int64_t c = 0; c < n; ++c)
        for (int64_t i = c; i < n; ++i) {
            double s = i == c ? 1.0 : 0.0;
            for (int64_t k = c; k < i; ++k) s -= L[(size_t)i * n + k] * Li[(size_t)k * n + c];
            Li[(size_t)i * n + c] = s / L[(size_t)i * n + i];
        }
    U.assign((size_t)n * n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = i; j < n; ++j) U[(size_t)i * n + j] = Li[(size_t)j * n + i];
    G.assign((size_t)n * n, 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j < n; ++j) {
            double s = 0.0;
            for (int64_t k = std::max(i, j); k < n; ++k) s += U[(size_t)i * n + k] * U[(size_t)j * n + k];
            G[(size_t)i * n + j] = s;
        }
}

// Coarsest levels above 8192 unknowns (or g_chol_blocked, the device's MGMC_DISABLE=chol_dense) use
// the blocked banded solves of the device (mgmc_cholesky.hpp k_coarse_chol_blocked): Q is banded
// in lexicographic order, so is L; with B >= bw rows per block L is block lower bidiagonal
// (diagonal blocks L_kk, coupling blocks C_k) and the two triangular solves become
//   t = f_k - C_k y_{k-1}, y_k = L_kk^{-1} t;   y' = y + xi;   t = y'_k - C_{k+1}^T x_{k+1}, x_k = L_kk^{-T} t
// with every row an fma chain in ascending column order.
static int g_chol_blocked = 0;
// g_no_fold: hierarchies built while it is set take no fold levels (the device's MGMC_DISABLE=fold: the
// residuals of the reflection-symmetric 27-point levels in the reference's CSR order)
static int g_no_fold = 0;
static const int64_t kCholDenseMax = 8192;

struct DenseCholeskySampler : Sampler {
    int64_t n, bw = 0;
    std::vector<double> band;  // lower factor, row i holds columns i - bw .. i
    std::vector<double> xi, g;
    double Lat(int64_t i, int64_t k) const {
        return (k <= i && i - k <= bw) ? band[(size_t)(i * (bw + 1) + (k - i + bw))] : 0.0;
    }
    DenseCholeskySampler(Ctx* c, const Level* L) : Sampler(c) {
        lev = L;
        n = L->A.nrow;
        const int m = L->lr.m;
        // bandwidth: the widest nonzero coupling of the matrix and the row span of each low-rank column
        for (int64_t r = 0; r < n; ++r)
            for (int64_t q = L->A.rowptr[r]; q < L->A.rowptr[r + 1]; ++q)
                if (L->A.val[q] != 0.0) bw = std::max(bw, std::abs(r - (int64_t)L->A.col[q]));
        for (int k = 0; k < m; ++k) {
            int64_t lo = n, hi = -1;
            for (const auto& e : L->lr.cols[k])
                if (e.second != 0.0) {
                    lo = std::min(lo, (int64_t)e.first);
                    hi = std::max(hi, (int64_t)e.first);
                }
            if (hi > lo) bw = std::max(bw, hi - lo);
        }
        const int64_t W = bw + 1;
        band.assign((size_t)(n * W), 0.0);
        for (int64_t r = 0; r < n; ++r)
            for (int64_t q = L->A.rowptr[r]; q < L->A.rowptr[r + 1]; ++q) {
                const int64_t col = L->A.col[q];
                if (col <= r && r - col <= bw) band[(size_t)(r * W + (col - r + bw))] = L->A.val[q];
            }
        if (m > 0) {  // A += B Sigma^{-1} B^T (cholesky_sampler.cc:30-36); lower triangle, zero outside the band
            std::vector<double> Bd((size_t)n * m, 0.0);
            for (int k = 0; k < m; ++k)
                for (const auto& e : L->lr.cols[k]) Bd[(size_t)e.first * m + k] = e.second;
            for (int64_t i = 0; i < n; ++i)
                for (int64_t j = std::max<int64_t>(0, i - bw); j <= i; ++j) {
                    double s = 0.0;
                    for (int k = 0; k < m; ++k) s += Bd[(size_t)i * m + k] / L->lr.sigma[k] * Bd[(size_t)j * m + k];
                    band[(size_t)(i * W + (j - i + bw))] += s;
                }
        }
        // the dense LLT loop (column j: diagonal, then the rows below), its skipped products being zeros
        for (int64_t j = 0; j < n; ++j) {
            double& djj = band[(size_t)(j * W + bw)];
            double d = djj;
            for (int64_t k = std::max<int64_t>(0, j - bw); k < j; ++k) d -= Lat(j, k) * Lat(j, k);
            d = sqrt(d);
            djj = d;
            for (int64_t i = j + 1; i <= std::min(n - 1, j + bw); ++i) {
                double& lij = band[(size_t)(i * W + (j - i + bw))];
                double s = lij;
                for (int64_t k = std::max<int64_t>(0, i - bw); k < j; ++k) s -= Lat(i, k) * Lat(j, k);
                lij = s / d;
            }
        }
        blocked = n > kCholDenseMax || g_chol_blocked;
        xi.resize(n);
        g.resize(n);
    }
    // cholesky_sampler.hh:50-66: xi ~ N(0, I), x = L^{-T} (xi + L^{-1} f).  MULTICOLOUR (device order):
    // xi from the Philox pair / branch of each vertex under the op's sweep tag, as a Gibbs sweep of
    // this level would draw it; up to 8192 unknowns the two triangular solves are replaced by products
    // with the precomputed U = L^{-T} and G = Q^{-1} = U U^T (dense_factor_inverses): x = G f + U xi,
    // each row an fma chain in ascending column order -- every row independent, as the device
    // computes it; above, the blocked solves (blocked_solve).
    const Level* lev = nullptr;
    bool blocked = false;
    std::vector<double> U, G;  // row-major n x n (MULTICOLOUR, dense)
    int64_t B = 0, nb = 0;
    std::vector<double> Cb, Db;  // blocked: C_k(r, j) at Cb[k B^2 + r B + j], L_kk^{-1}(r, j) at Db[...]
    void make_blocks() {
        B = std::max<int64_t>(64, (std::max<int64_t>(bw, 1) + 63) / 64 * 64);
        nb = (n + B - 1) / B;
        const size_t BB = (size_t)(B * B);
        Cb.assign(nb * BB, 0.0);
        Db.assign(nb * BB, 0.0);
        for (int64_t k = 0; k < nb; ++k) {
            const int64_t base = k * B, Bk = std::min(B, n - base);
            if (k > 0)
                for (int64_t r = 0; r < Bk; ++r)
                    for (int64_t j = 0; j < B; ++j) Cb[k * BB + r * B + j] = Lat(base + r, base - B + j);
            double* D = &Db[k * BB];
            for (int64_t c = 0; c < Bk; ++c)  // L_kk^{-1} column by column (dense_factor_inverses' loop)
                for (int64_t r = c; r < Bk; ++r) {
                    double s = r == c ? 1.0 : 0.0;
                    for (int64_t q = c; q < r; ++q) s -= Lat(base + r, base + q) * D[q * B + c];
                    D[r * B + c] = s / Lat(base + r, base + r);
                }
        }
    }
    void blocked_solve(const double* f, double* x, bool noise) {
        if (Db.empty()) make_blocks();
        const size_t BB = (size_t)(B * B);
        std::vector<double> t(B), y(n);
        for (int64_t k = 0; k < nb; ++k) {
            const int64_t base = k * B, Bk = std::min(B, n - base);
            for (int64_t r = 0; r < Bk; ++r) {
                double s = 0.0;
                if (k > 0)
                    for (int64_t j = 0; j < B; ++j) s = fma(Cb[k * BB + r * B + j], y[base - B + j], s);
                t[r] = f[base + r] - s;
            }
            for (int64_t r = 0; r < Bk; ++r) {
                double a = 0.0;
                for (int64_t j = 0; j <= r; ++j) a = fma(Db[k * BB + r * B + j], t[j], a);
                y[base + r] = a;
                x[base + r] = noise ? a + xi[base + r] : a;
            }
        }
        for (int64_t k = nb - 1; k >= 0; --k) {
            const int64_t base = k * B, Bk = std::min(B, n - base);
            for (int64_t r = 0; r < Bk; ++r) {
                double s = 0.0;
                if (k + 1 < nb)
                    for (int64_t j = 0; j < std::min(B, n - base - B); ++j)
                        s = fma(Cb[(k + 1) * BB + j * B + r], x[base + B + j], s);
                t[r] = x[base + r] - s;
            }
            for (int64_t r = 0; r < Bk; ++r) {
                double a = 0.0;
                for (int64_t j = r; j < Bk; ++j) a = fma(Db[k * BB + j * B + r], t[j], a);
                x[base + r] = a;
            }
        }
    }
    void apply(const double* f, double* x) override { solve(f, x, true); }
    void solve(const double* f, double* x, bool noise) {
        if (noise) {
            if (ctx->mode == FAITHFUL) {
                for (int64_t ell = 0; ell < n; ++ell) xi[ell] = normal_dist(ctx->rng);
            } else {
                const uint32_t tag = ctx->tag++;
                for (int64_t ell = 0; ell < n; ++ell) {
                    double z0, z1;
                    philox_normals(ctx->seed, ctx->chain, lev->pair[ell], tag, ctx->sample, z0, z1);
                    xi[ell] = lev->cos_branch[ell] ? z0 : z1;
                }
            }
        }
        if (ctx->mode == MULTICOLOUR && blocked) {
            blocked_solve(f, x, noise);
            return;
        }
        if (ctx->mode == MULTICOLOUR) {
            if (U.empty()) {
                std::vector<double> Lmat((size_t)n * n, 0.0);
                for (int64_t i = 0; i < n; ++i)
                    for (int64_t k = std::max<int64_t>(0, i - bw); k <= i; ++k) Lmat[(size_t)i * n + k] = Lat(i, k);
                dense_factor_inverses(Lmat, n, U, G);
            }
            for (int64_t i = 0; i < n; ++i) {
                double a = 0.0;
                for (int64_t j = 0; j < n; ++j) a = fma(G[(size_t)i * n + j], f[j], a);
                double b = 0.0;
                if (noise)
                    for (int64_t j = i; j < n; ++j) b = fma(U[(size_t)i * n + j], xi[j], b);
                x[i] = a + b;
            }
            return;
        }
        for (int64_t i = 0; i < n; ++i) {  // L g = f (banded forward substitution)
            double s = f[i];
            for (int64_t k = std::max<int64_t>(0, i - bw); k < i; ++k) s -= Lat(i, k) * g[k];
            g[i] = s / Lat(i, i);
        }
        for (int64_t i = n - 1; i >= 0; --i) {  // L^T x = xi + g
            double s = noise ? xi[i] + g[i] : g[i];
            for (int64_t k = i + 1; k <= std::min(n - 1, i + bw); ++k) s -= Lat(k, i) * x[k];
            x[i] = s / Lat(i, i);
        }
    }
};

struct Params {
    int dim, nx, ny, nz;
    int nlevel, cycle, npresmooth, npostsmooth, ncoarsesmooth;
    int smoother;       // 0 SOR, 1 SSOR
    int coarse_solver;  // 0 SSOR, 1 Cholesky (dense)
    int galerkin;       // 0 = full SpGEMM, 1 = stencil rows from a small SpGEMM
    double omega, coarse_scaling, kappa_sq;
};

struct MGMC : Sampler {
    Params p;
    std::vector<std::unique_ptr<Level>> levels;
    std::vector<std::unique_ptr<Sampler>> pre, post;
    std::vector<std::unique_ptr<Intergrid>> ig;
    std::unique_ptr<Sampler> coarse;
    std::vector<std::vector<double>> x_ell, f_ell, r_ell;

    // stencil_hierarchy: the device builds this hierarchy as constant stencils (mgmc_create*: FD / FEM),
    // so its fold levels take the folded residual; false for a matrix given as CSR (the device's field path)
    MGMC(Ctx* c, const Params& p_, const Lattice& lat, CSR A0, const double* override_st /* nlevel*27 or null */,
         bool stencil_hierarchy = true)
        : Sampler(c), p(p_) {
        Lattice lattice = lat;
        CSR A = std::move(A0);
        double fine_st[27];
        bool have_small_src = false;
        CSR small_src;
        Lattice small;
        for (int level = 0; level < p.nlevel; ++level) {
            std::unique_ptr<Level> L(new Level());
            L->lat = lattice;
            L->A = std::move(A);  // every branch below assigns A before the next level
            L->fold = stencil_hierarchy && !g_no_fold && fold_stencil(L->lat, L->A);
            // 2 colours for a 5/7-point fine level (FD), 2^d for 3^d-point levels (FEM, Galerkin)
            if (lattice.dim >= 2) init_colouring(*L, level == 0);
            x_ell.emplace_back(L->A.nrow, 0.0);
            f_ell.emplace_back(L->A.nrow, 0.0);
            r_ell.emplace_back(L->A.nrow, 0.0);
            Level* Lp = L.get();
            levels.push_back(std::move(L));
            // samplers in the reference's construction order (multigridmc_sampler.cc:86-89)
            if (p.smoother == 0) {
                pre.emplace_back(new SORSampler(c, Lp, p.omega, p.npresmooth, FORWARD));
                post.emplace_back(new SORSampler(c, Lp, p.omega, p.npostsmooth, BACKWARD));
            } else {
                pre.emplace_back(new SSORSampler(c, Lp, p.omega, p.npresmooth));
                post.emplace_back(new SSORSampler(c, Lp, p.omega, p.npostsmooth));
            }
            if (level < p.nlevel - 1) {
                ig.emplace_back(new Intergrid(lattice));
                const Lattice cl = lattice.coarse();
                if (override_st) {
                    A = stencil_csr(cl, override_st + 27 * (level + 1));
                } else if (p.galerkin == 1 && lattice.dim >= 2) {
                    // stencil mode: level stencil -> small lattice -> SpGEMM -> interior row
                    if (!have_small_src) {
                        // the level's own (constant) stencil, placed on an 8^d lattice
                        small = lattice;
                        for (int d = 0; d < lattice.dim; ++d) small.n[d] = 8;
                        stencil_of_interior_row(Lp->A, lattice, fine_st);
                        small_src = stencil_csr(small, fine_st);
                        have_small_src = true;
                    }
                    A = galerkin_stencil_mode(small_src, small, cl, fine_st);
                    small_src = stencil_csr(small, fine_st);
                } else {
                    A = galerkin_spgemm(Lp->A, *ig.back());
                }
                lattice = cl;
            }
        }
        if (p.coarse_solver == 1)
            coarse.reset(new DenseCholeskySampler(c, levels.back().get()));
        else
            coarse.reset(new SSORSampler(c, levels.back().get(), p.omega, p.ncoarsesmooth));
    }

    void sample(int level) {
        if (level == p.nlevel - 1) {
            coarse->apply(f_ell[level].data(), x_ell[level].data());
            return;
        }
        const int cycle_ = (level > 0) ? p.cycle : 1;
        for (int j = 0; j < cycle_; ++j) {
            pre[level]->apply(f_ell[level].data(), x_ell[level].data());
            posterior_residual(*levels[level], f_ell[level].data(), x_ell[level].data(), r_ell[level].data(), ctx->mode);
            ig[level]->restrict_(r_ell[level].data(), f_ell[level + 1].data());
            std::fill(x_ell[level + 1].begin(), x_ell[level + 1].end(), 0.0);
            sample(level + 1);
            ig[level]->prolongate_add(p.coarse_scaling, x_ell[level + 1].data(), x_ell[level].data());
            post[level]->apply(f_ell[level].data(), x_ell[level].data());
        }
    }

    void apply(const double* f, double* x) override {
        std::copy(f, f + f_ell[0].size(), f_ell[0].begin());
        std::copy(x, x + x_ell[0].size(), x_ell[0].begin());
        ctx->tag = 0;
        sample(0);
        ctx->sample++;
        std::copy(x_ell[0].begin(), x_ell[0].end(), x);
    }
};

}  // namespace orc

// =============================================================================================
// C API for the tests (ctypes) and the CPU baseline
// =============================================================================================
using namespace orc;

struct orc_handle {
    Ctx ctx;
    std::unique_ptr<MGMC> mg;
    std::vector<double> f, x;  // fixed rhs and chain state (measure_sampling_time)
};

extern "C" {

typedef struct orc_params {
    int dim, nx, ny, nz;
    int nlevel, cycle, npresmooth, npostsmooth, ncoarsesmooth;
    int smoother, coarse_solver, galerkin;
    double omega, coarse_scaling, kappa_sq;
} orc_params;

static Params to_params(const orc_params* q) {
    Params p;
    p.dim = q->dim; p.nx = q->nx; p.ny = q->ny; p.nz = q->nz;
    p.nlevel = q->nlevel; p.cycle = q->cycle; p.npresmooth = q->npresmooth; p.npostsmooth = q->npostsmooth;
    p.ncoarsesmooth = q->ncoarsesmooth; p.smoother = q->smoother; p.coarse_solver = q->coarse_solver;
    p.galerkin = q->galerkin; p.omega = q->omega; p.coarse_scaling = q->coarse_scaling; p.kappa_sq = q->kappa_sq;
    return p;
}

static Lattice make_lattice(const orc_params* q) {
    Lattice lat;
    lat.dim = q->dim;
    lat.n[0] = q->nx;
    lat.n[1] = q->dim >= 2 ? q->ny : 0;
    lat.n[2] = q->dim == 3 ? q->nz : 0;
    return lat;
}

// FD shifted-Laplace prior on a 2D/3D lattice; override_st (nlevel*27) replaces the Galerkin
// stencils of levels >= 1 (multicolour replay of a device hierarchy), may be NULL.
orc_handle* orc_create_fd(const orc_params* q, int mode, uint64_t seed, uint64_t chain, const double* override_st) {
    orc_handle* h = new orc_handle();
    h->ctx.mode = (Mode)mode;
    h->ctx.rng.seed(seed);
    h->ctx.seed = seed;
    h->ctx.chain = chain;
    const Lattice lat = make_lattice(q);
    CSR A = fd_operator(lat, KappaModel::constant(q->kappa_sq));
    h->mg.reset(new MGMC(&h->ctx, to_params(q), lat, std::move(A), override_st));
    h->f.assign(h->mg->x_ell[0].size(), 0.0);
    h->x.assign(h->mg->x_ell[0].size(), 0.0);
    return h;
}

// The oracle's own stencil of every level of an FD hierarchy (out: nlevel*27, sidx order) without
// assembling any level: the fine row is the FD assembly's interior row (2,2[,2]) of the full-size
// lattice (fd_row, the reference's expression), each coarse stencil the interior row of R*A*R^T
// evaluated by SpGEMM on an 8^d lattice -- the galerkin == 1 construction of MGMC above, which
// tests/test_oracle.py pins to the full SpGEMM.  Returns 0, or -1 if the fine lattice has
// no interior row (2,2[,2]).
int orc_fd_level_stencils(const orc_params* q, double* out) {
    Lattice lat = make_lattice(q);
    for (int d = 0; d < lat.dim; ++d)
        if (lat.n[d] < 4) return -1;
    const KappaModel kappa = KappaModel::constant(q->kappa_sq);
    int idx[3] = {2, 2, 2};
    int32_t cols[7];
    double vals[7];
    const int64_t r = lat.euc2lin(idx);
    const int64_t cnt = fd_row(lat, kappa, r, cols, vals);
    double st[27];
    for (int k = 0; k < 27; ++k) st[k] = 0.0;
    for (int64_t e = 0; e < cnt; ++e) {
        int ci[3] = {0, 0, 0};
        lat.lin2euc(cols[e], ci);
        st[sidx(lat.dim, ci[0] - 2, lat.dim >= 2 ? ci[1] - 2 : 0, lat.dim == 3 ? ci[2] - 2 : 0)] = vals[e];
    }
    Lattice small = lat;
    for (int d = 0; d < lat.dim; ++d) small.n[d] = 8;
    for (int level = 0; level < q->nlevel; ++level) {
        for (int k = 0; k < 27; ++k) out[27 * level + k] = st[k];
        if (level + 1 == q->nlevel) break;
        const CSR small_src = stencil_csr(small, st);
        Intergrid ig(small);
        const CSR Ac = galerkin_spgemm(small_src, ig);
        stencil_of_interior_row(Ac, ig.coarse, st);
    }
    return 0;
}

// FEM shifted-Laplace prior (constant kappa^2); override_st as for orc_create_fd
orc_handle* orc_create_fem(const orc_params* q, int mode, uint64_t seed, uint64_t chain, const double* override_st) {
    orc_handle* h = new orc_handle();
    h->ctx.mode = (Mode)mode;
    h->ctx.rng.seed(seed);
    h->ctx.seed = seed;
    h->ctx.chain = chain;
    const Lattice lat = make_lattice(q);
    CSR A = fem_operator(lat, KappaModel::constant(q->kappa_sq));
    Params p = to_params(q);
    p.galerkin = 0;
    h->mg.reset(new MGMC(&h->ctx, p, lat, std::move(A), override_st));
    h->f.assign(h->mg->x_ell[0].size(), 0.0);
    h->x.assign(h->mg->x_ell[0].size(), 0.0);
    return h;
}

// Generic fine operator given as CSR on a 1D/2D/3D lattice (e.g. test_sampler.hh TestOperator1d)
orc_handle* orc_create_csr(const orc_params* q, int mode, uint64_t seed, int64_t nrow, const int64_t* rowptr,
                           const int32_t* col, const double* val) {
    if (mode == MULTICOLOUR && q->dim < 2) return nullptr;  // colour / pair maps exist for 2D / 3D only
    orc_handle* h = new orc_handle();
    h->ctx.mode = (Mode)mode;
    h->ctx.rng.seed(seed);
    h->ctx.seed = seed;
    CSR A;
    A.nrow = A.ncol = nrow;
    A.rowptr.assign(rowptr, rowptr + nrow + 1);
    A.col.assign(col, col + rowptr[nrow]);
    A.val.assign(val, val + rowptr[nrow]);
    Params p = to_params(q);
    p.galerkin = 0;
    h->mg.reset(new MGMC(&h->ctx, p, make_lattice(q), std::move(A), nullptr, /*stencil_hierarchy=*/false));
    h->f.assign(nrow, 0.0);
    h->x.assign(nrow, 0.0);
    return h;
}

void orc_destroy(orc_handle* h) { delete h; }

// worker threads of the row-parallel loops (see g_threads); results do not depend on it
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
// coarse Cholesky: the blocked banded solves at any size (read when a sampler is built)
void orc_set_chol_blocked(int on) { g_chol_blocked = on ? 1 : 0; }
void orc_set_no_fold(int on) { g_no_fold = on ? 1 : 0; }
int orc_get_threads(void) { return g_threads; }

// the reference's fine operators (any correlation-length model) as CSR: pde 0 FD, 1 FEM, 2 squared
// FD (2D); kmodel 0 constant (kappa^2 = 1 / pow(Lambda, 2)), 1 periodic (Lambda_min, Lambda_max)
static CSR model_operator(int dim, const int* n, int pde, int kmodel, double Lambda, double Lmin, double Lmax) {
    Lattice lat;
    lat.dim = dim;
    lat.n[0] = n[0];
    lat.n[1] = dim >= 2 ? n[1] : 1;
    lat.n[2] = dim == 3 ? n[2] : 1;
    KappaModel k;
    if (kmodel == 1) {
        k.periodic = 1;
        k.Lambda_1 = 0.5 * (Lmax + Lmin);
        k.Lambda_2 = 0.5 * (Lmax - Lmin);
    } else {
        k.kappa_sq_const = 1. / pow(Lambda, 2);
    }
    if (pde == 1) return fem_operator(lat, k);
    if (pde == 2) return squared_fd_operator(lat, k);
    return fd_operator(lat, k);
}

int64_t orc_operator_nnz(int dim, const int* n, int pde, int kmodel, double Lambda, double Lmin, double Lmax) {
    return (int64_t)model_operator(dim, n, pde, kmodel, Lambda, Lmin, Lmax).col.size();
}

void orc_operator_csr(int dim, const int* n, int pde, int kmodel, double Lambda, double Lmin, double Lmax,
                      int64_t* rowptr, int32_t* col, double* val) {
    const CSR A = model_operator(dim, n, pde, kmodel, Lambda, Lmin, Lmax);
    std::copy(A.rowptr.begin(), A.rowptr.end(), rowptr);
    std::copy(A.col.begin(), A.col.end(), col);
    std::copy(A.val.begin(), A.val.end(), val);
}

int64_t orc_ndof(orc_handle* h, int level) { return h->mg->levels[level]->A.nrow; }
int orc_nlevel(orc_handle* h) { return (int)h->mg->levels.size(); }
int64_t orc_nnz(orc_handle* h, int level) { return (int64_t)h->mg->levels[level]->A.col.size(); }

void orc_get_csr(orc_handle* h, int level, int64_t* rowptr, int32_t* col, double* val) {
    const CSR& A = h->mg->levels[level]->A;
    memcpy(rowptr, A.rowptr.data(), (A.nrow + 1) * sizeof(int64_t));
    memcpy(col, A.col.data(), A.col.size() * sizeof(int32_t));
    memcpy(val, A.val.data(), A.val.size() * sizeof(double));
}

// one row of a level's CSR (columns ascending): returns the entry count (<= 27 copied)
int64_t orc_get_row(orc_handle* h, int level, int64_t row, int32_t* col, double* val) {
    const CSR& A = h->mg->levels[level]->A;
    const int64_t b = A.rowptr[row], e = A.rowptr[row + 1];
    for (int64_t q = b; q < e && q - b < 27; ++q) {
        col[q - b] = A.col[q];
        val[q - b] = A.val[q];
    }
    return e - b;
}

void orc_set_rhs(orc_handle* h, const double* f) { std::copy(f, f + h->f.size(), h->f.begin()); }
void orc_set_state(orc_handle* h, const double* x) { std::copy(x, x + h->x.size(), h->x.begin()); }
void orc_get_state(orc_handle* h, double* x) { std::copy(h->x.begin(), h->x.end(), x); }
void orc_set_sample_index(orc_handle* h, uint64_t s) { h->ctx.sample = s; }
// independent chains of one hierarchy (the CPU all-cores baseline forks one process per chain after
// the setup): FAITHFUL re-seeds the shared mt19937_64 (seed + chain), MULTICOLOUR changes the Philox key
void orc_reseed(orc_handle* h, uint64_t seed, uint64_t chain) {
    h->ctx.rng.seed(seed + chain);
    h->ctx.seed = seed;
    h->ctx.chain = chain;
}

// Sampler::apply(f, x)
void orc_apply(orc_handle* h, const double* f, double* x) { h->mg->apply(f, x); }

// measure_sampling_time loop (driver_mgmc.cc:66-78): nsteps applications on the fixed rhs,
// qoi_out[k] = x[qoi] after step k (qoi < 0 / qoi_out == NULL: no recording)
void orc_sample(orc_handle* h, int nsteps, int64_t qoi, double* qoi_out) {
    for (int k = 0; k < nsteps; ++k) {
        h->mg->apply(h->f.data(), h->x.data());
        if (qoi_out && qoi >= 0) qoi_out[k] = h->x[qoi];
    }
}

// wall-clock of nsteps applications (std::chrono::steady_clock), seconds
double orc_time_samples(orc_handle* h, int nsteps) {
    const auto t0 = std::chrono::steady_clock::now();
    orc_sample(h, nsteps, -1, nullptr);
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// sampler/test_sampler.hh:113-153 mean_covariance_error loop: nwarmup applications, then running
// estimators Ex += (x - Ex)/(k+1), Exx += (x x^T - Exx)/(k+1) over nsamples applications (x starts at 0)
void orc_mean_cov(orc_handle* h, const double* f, int nwarmup, int64_t nsamples, double* Ex, double* Exx) {
    const int64_t n = (int64_t)h->x.size();
    std::vector<double> x(n, 0.0);
    for (int k = 0; k < nwarmup; ++k) h->mg->apply(f, x.data());
    for (int64_t q = 0; q < n; ++q) Ex[q] = 0.0;
    for (int64_t q = 0; q < n * n; ++q) Exx[q] = 0.0;
    for (int64_t k = 0; k < nsamples; ++k) {
        h->mg->apply(f, x.data());
        const double w = 1. / (k + 1);
        for (int64_t i = 0; i < n; ++i) {
            Ex[i] += w * (x[i] - Ex[i]);
            for (int64_t j = 0; j < n; ++j) Exx[i * n + j] += w * (x[i] * x[j] - Exx[i * n + j]);
        }
    }
}

void orc_operator_apply(orc_handle* h, int level, const double* x, double* y) {
    posterior_apply(*h->mg->levels[level], x, y, h->ctx.mode);
}

// Low-rank measurement part of the fine operator (MeasuredOperator): m columns of B as CSC
// (colptr[m+1], rows ascending in [0, N), values) and Sigma[m].  Coarse levels get B_c = R B
// (linear_operator.cc:17) -- columns restricted as dense vectors; a column covering every vertex
// stays dense, others keep their nonzeros -- and Sigma_c = Sigma.  The coarse Cholesky sampler, if
// used, is rebuilt on the posterior precision.
void orc_set_lowrank(orc_handle* h, int m, const int64_t* colptr, const int64_t* rows, const double* vals,
                     const double* sigma) {
    MGMC& mg = *h->mg;
    for (size_t level = 0; level < mg.levels.size(); ++level) {
        Level& L = *mg.levels[level];
        L.lr = LowRank();
        L.lr.m = m;
        L.lr.sigma.assign(sigma, sigma + m);
        L.lr.cols.resize(m);
        L.lr.dense.resize(m);
        const int64_t n = L.A.nrow;
        if (level == 0) {
            for (int k = 0; k < m; ++k) {
                for (int64_t q = colptr[k]; q < colptr[k + 1]; ++q) L.lr.cols[k].push_back({rows[q], vals[q]});
                L.lr.dense[k] = (colptr[k + 1] - colptr[k]) == n;
            }
        } else {
            const Level& F = *mg.levels[level - 1];
            std::vector<double> fine(F.A.nrow), coarse(n);
            for (int k = 0; k < m; ++k) {
                std::fill(fine.begin(), fine.end(), 0.0);
                for (const auto& e : F.lr.cols[k]) fine[e.first] = e.second;
                mg.ig[level - 1]->restrict_(fine.data(), coarse.data());
                L.lr.dense[k] = F.lr.dense[k];
                for (int64_t i = 0; i < n; ++i)
                    if (L.lr.dense[k] || coarse[i] != 0.0) L.lr.cols[k].push_back({i, coarse[i]});
            }
        }
        // the split column of the MULTICOLOUR patch (lr_patch_mc; the device's LowRankDev::split_g):
        // the level's only dense column over more than LR_BLK rows, when its values are one number
        int ndense = 0, g = -1;
        for (int k = 0; k < m; ++k)
            if (L.lr.dense[k] && n > LR_BLK) {
                ++ndense;
                g = k;
            }
        if (ndense == 1 && !L.lr.cols[g].empty()) {
            bool same = true;
            for (const auto& e : L.lr.cols[g]) same = same && memcmp(&e.second, &L.lr.cols[g][0].second, 8) == 0;
            if (same) L.lr.split = g;
        }
    }
    if (mg.p.coarse_solver == 1) mg.coarse.reset(new DenseCholeskySampler(&h->ctx, mg.levels.back().get()));
}

// the low-rank columns of a level (CSC, reference layout) -- for host cross-checks
int64_t orc_lowrank_nnz(orc_handle* h, int level) {
    int64_t s = 0;
    for (const auto& c : h->mg->levels[level]->lr.cols) s += (int64_t)c.size();
    return s;
}
void orc_get_lowrank(orc_handle* h, int level, int64_t* colptr, int64_t* rows, double* vals) {
    const LowRank& lr = h->mg->levels[level]->lr;
    colptr[0] = 0;
    int64_t q = 0;
    for (int k = 0; k < lr.m; ++k) {
        for (const auto& e : lr.cols[k]) {
            rows[q] = e.first;
            vals[q] = e.second;
            ++q;
        }
        colptr[k + 1] = q;
    }
}

void orc_smoother_apply(orc_handle* h, int level, int direction, int nsweeps, const double* b, double* x) {
    SORSmoother s(h->mg->levels[level].get(), h->mg->p.omega, (Direction)direction);
    for (int k = 0; k < nsweeps; ++k) s.apply(h->ctx.mode, b, x);
}

// SORSmoother::apply as the reference nests it (sor_smoother.cc:41-53 loops nsmooth times over
// apply_sparse, which loops nsmooth times over the sweep itself, :64): nsmooth x (nsmooth sweeps, then
// the low-rank fix once)
void orc_sor_smoother_apply(orc_handle* h, int level, int direction, int nsmooth, const double* b, double* x) {
    SORSmoother s(h->mg->levels[level].get(), h->mg->p.omega, (Direction)direction);
    for (int k = 0; k < nsmooth; ++k) {
        for (int j = 0; j < nsmooth; ++j) s.sweep(h->ctx.mode, b, x);
        s.fix(h->ctx.mode, x);
    }
}

// SSORSmoother::apply (ssor_smoother.cc:9-15; smoothers built with nsmooth 1, ssor_smoother.hh:47-48):
// nsmooth x (forward sweep + fix, backward sweep + fix)
void orc_ssor_smoother_apply(orc_handle* h, int level, int nsmooth, const double* b, double* x) {
    SORSmoother fw(h->mg->levels[level].get(), h->mg->p.omega, FORWARD);
    SORSmoother bw(h->mg->levels[level].get(), h->mg->p.omega, BACKWARD);
    for (int k = 0; k < nsmooth; ++k) {
        fw.apply(h->ctx.mode, b, x);
        bw.apply(h->ctx.mode, b, x);
    }
}

// one noisy sweep with explicit (tag, sample) in multicolour mode (SORSampler, nsmooth = 1)
void orc_sor_sampler_apply(orc_handle* h, int level, int direction, uint32_t tag, uint64_t sample, const double* f,
                           double* x) {
    SORSampler s(&h->ctx, h->mg->levels[level].get(), h->mg->p.omega, 1, (Direction)direction);
    const uint32_t save_tag = h->ctx.tag;
    const uint64_t save_sample = h->ctx.sample;
    h->ctx.tag = tag;
    h->ctx.sample = sample;
    s.apply(f, x);
    h->ctx.tag = save_tag;
    h->ctx.sample = save_sample;
}

void orc_restrict(orc_handle* h, int level, const double* r, double* rc) { h->mg->ig[level]->restrict_(r, rc); }
void orc_prolongate_add(orc_handle* h, int level, double alpha, const double* xc, double* x) {
    h->mg->ig[level]->prolongate_add(alpha, xc, x);
}
// R (f - A x), multigridmc_sampler.cc:118-120
void orc_residual_restrict(orc_handle* h, int level, const double* f, const double* x, double* fc) {
    const CSR& A = h->mg->levels[level]->A;
    std::vector<double> r(A.nrow);
    posterior_residual(*h->mg->levels[level], f, x, r.data(), h->ctx.mode);
    h->mg->ig[level]->restrict_(r.data(), fc);
}

// sum_e vals[e] x[rows[e]] in the device's blocked order (the low-rank dots' order; the QoI vector
// record of mgmc_set_qoi_vector)
double orc_blocked_dot(int64_t n, const int64_t* rows, const double* vals, const double* x) {
    std::vector<std::pair<int64_t, double>> col((size_t)n);
    for (int64_t e = 0; e < n; ++e) col[(size_t)e] = {rows[e], vals[e]};
    return blocked_dot(col, 1.0, x);
}

void orc_philox_normals(uint64_t seed, uint64_t chain, uint64_t pair0, int64_t n, uint32_t tag, uint64_t sample,
                        double* out) {
    for (int64_t q = 0; q < n / 2; ++q) philox_normals(seed, chain, (uint32_t)(pair0 + q), tag, sample, out[2 * q], out[2 * q + 1]);
}

void orc_philox_raw(const uint32_t ctr_in[4], uint32_t k0, uint32_t k1, uint32_t out[4]) {
    uint32_t c[4] = {ctr_in[0], ctr_in[1], ctr_in[2], ctr_in[3]};
    philox10(c, k0, k1);
    memcpy(out, c, sizeof(c));
}

double orc_ln_unit(double u) { return ln_unit(u); }
void orc_cos_sin_2pi(double t, double* c, double* s) { cos_sin_2pi(t, *c, *s); }

// first n values of std::normal_distribution<double>(0,1) on std::mt19937_64(seed)
void orc_mt_normals(uint64_t seed, int64_t n, double* out) {
    std::mt19937_64 rng(seed);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (int64_t q = 0; q < n; ++q) out[q] = nd(rng);
}

// ---- lattice known answers (lattice/test_lattice.hh) ----
static Lattice lat_of(int dim, const int* n) {
    Lattice l;
    l.dim = dim;
    for (int d = 0; d < dim; ++d) l.n[d] = n[d];
    return l;
}
int64_t orc_lattice_fine_vertex_idx(int dim, const int* n, int64_t ell) { return lat_of(dim, n).fine_vertex_idx(ell); }
void orc_lattice_lin2euc(int dim, const int* n, int64_t ell, int* idx) { lat_of(dim, n).lin2euc(ell, idx); }
int64_t orc_lattice_euc2lin(int dim, const int* n, const int* idx) {
    int i3[3] = {idx[0], dim >= 2 ? idx[1] : 0, dim == 3 ? idx[2] : 0};
    return lat_of(dim, n).euc2lin(i3);
}
int64_t orc_lattice_shift(int dim, const int* n, int64_t ell, const int* shift) {
    int s[3] = {shift[0], dim >= 2 ? shift[1] : 0, dim == 3 ? shift[2] : 0};
    // shift_vertexidx (lattice*d.hh) does not range-check (asserts only): plain index arithmetic
    const Lattice l = lat_of(dim, n);
    int idx[3];
    l.lin2euc(ell, idx);
    for (int d = 0; d < dim; ++d) idx[d] += s[d];
    return l.euc2lin(idx);
}

}  // extern "C"
