// mgmc_hierarchy.cpp -- see mgmc_hierarchy.hpp.
#include "mgmc_hierarchy.hpp"

#include <math.h>
#include <string.h>

#include <cstdlib>

#include <sstream>

namespace mgmc {

namespace {

// linear-interpolation weight of a 1d offset in {-1,0,1} (intergrid_operator_linear.cc:13-17)
inline double w1(int o) { return o == 0 ? 1.0 : 0.5; }

inline int sidx(int dim, int dx, int dy, int dz) {
    return dim == 3 ? (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1) : (dy + 1) * 3 + (dx + 1);
}

// Q1 shape functions on the reference cell (shiftedlaplace_fem_operator.cc:148-187): a[j] = 0 is the
// factor (1 - xhat_j), a[j] = 1 is xhat_j; products from 1.0 in dimension order
double fem_phi(int dim, const int* a, const double* xh) {
    double v = 1.0;
    for (int j = 0; j < dim; ++j) v *= (a[j] == 0) ? (1.0 - xh[j]) : xh[j];
    return v;
}
void fem_grad_phi(int dim, const int* a, const double* xh, double* g) {
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

// Interior stencil of ShiftedLaplaceFEMOperator with constant kappa^2 (shiftedlaplace_fem_operator.cc
// :9-145).  The reference assembles cell by cell (cells ascending, x fastest; basis pairs (alpha,
// beta) in cartesian-product order, last dimension fastest), each entry starting from 0.0 and adding
// local(alpha, beta) * cell_volume, local = sum_q (kappa^2 phi_a phi_b + grad phi_a . (h^-2 grad
// phi_b)) w_q over the order-1 Gauss-Legendre points (quadrature.cc:11-55).  With constant kappa^2
// every interior row receives the same terms in the same order, so one row (entry v -> v + s, the
// cells c in {v-1, v}^d containing v + s, ascending) gives every row bit for bit; rows next to the
// boundary are this stencil truncated (the columns of boundary vertices are never created).
void fem_stencil(int dim, const int* n, double kappa_sq, double* st) {
    double h[3] = {1, 1, 1}, hinv2[3] = {0, 0, 0};
    double cell_volume = 1.0;
    for (int d = 0; d < dim; ++d) {
        h[d] = 1. / double(n[d]);
        hinv2[d] = 1. / (h[d] * h[d]);
        cell_volume *= h[d];
    }
    // quadrature: 2 points per dimension, cartesian product with the last dimension fastest
    const double p1[2] = {-1.0 / sqrt(3.0), +1.0 / sqrt(3.0)};
    const int nq = 1 << dim;
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
    auto local = [&](const int* a, const int* b) {
        double v = 0.0;
        for (int q = 0; q < nq; ++q) {
            const double pp = fem_phi(dim, a, qp[q]) * fem_phi(dim, b, qp[q]);
            double ga[3] = {0, 0, 0}, gb[3] = {0, 0, 0};
            fem_grad_phi(dim, a, qp[q], ga);
            fem_grad_phi(dim, b, qp[q], gb);
            double gg = ga[0] * (hinv2[0] * gb[0]);  // Eigen dot: ((t0 + t1) + t2)
            for (int k = 1; k < dim; ++k) gg = gg + ga[k] * (hinv2[k] * gb[k]);
            v += (kappa_sq * pp + gg) * qw[q];
        }
        return v;
    };
    for (int k = 0; k < 27; ++k) st[k] = 0.0;
    const int zr = dim == 3 ? 1 : 0;
    for (int sz = -zr; sz <= zr; ++sz)
        for (int sy = -1; sy <= 1; ++sy)
            for (int sx = -1; sx <= 1; ++sx) {
                const int s[3] = {sx, sy, sz};
                double acc = 0.0;
                // cells c = v - alpha, alpha in {0,1}^d, ascending cell index (x fastest)
                for (int cz = zr; cz >= 0; --cz)
                    for (int cy = 1; cy >= 0; --cy)
                        for (int cx = 1; cx >= 0; --cx) {
                            const int alpha[3] = {cx, cy, cz};  // v - c
                            int beta[3] = {0, 0, 0};
                            bool ok = true;
                            for (int d = 0; d < dim; ++d) {
                                beta[d] = alpha[d] + s[d];
                                ok = ok && beta[d] >= 0 && beta[d] <= 1;
                            }
                            if (!ok) continue;
                            acc += local(alpha, beta) * cell_volume;
                        }
                st[sidx(dim, sx, sy, sz)] = acc;
            }
}

}  // namespace

std::string validate_config(const mgmc_config& c) {
    std::ostringstream err;
    if (c.dim != 2 && c.dim != 3) {
        err << "invalid dimension : " << c.dim;
        return err.str();
    }
    if (c.nlevel < 1 || c.nlevel > 24) {
        err << "invalid number of levels : " << c.nlevel;
        return err.str();
    }
    if (c.cycle < 1) return "cycle must be >= 1";
    if (c.npresmooth < 0 || c.npostsmooth < 0 || c.ncoarsesmooth < 0) return "negative number of smoothing steps";
    if (c.smoother != MGMC_SMOOTHER_SOR && c.smoother != MGMC_SMOOTHER_SSOR) {
        err << "ERROR: invalid sampler '" << c.smoother << "'";  // multigridmc_sampler.cc:47
        return err.str();
    }
    if (c.coarse_solver != MGMC_COARSE_SSOR && c.coarse_solver != MGMC_COARSE_CHOLESKY) {
        err << "ERROR: multigrid coarse sampler '" << c.coarse_solver << "'";  // :70-72
        return err.str();
    }
    if (!(c.omega > 0.0 && c.omega < 2.0)) return "omega must lie in (0,2)";
    if (!(c.kappa_sq >= 0.0)) return "kappa_sq must be >= 0";
    if (c.fine_operator != MGMC_OPERATOR_FD && c.fine_operator != MGMC_OPERATOR_FEM) {
        err << "Error: invalid prior '" << c.fine_operator << "'";  // driver_mgmc.cc:426-429
        return err.str();
    }
    int n[3] = {c.nx, c.ny, c.dim == 3 ? c.nz : 2};
    for (int d = 0; d < c.dim; ++d)
        if (n[d] < 2) return "every lattice extent must be >= 2";
    // interior unknown count must fit the reference's unsigned Nvertex and our 32-bit pair ids
    double ndof = 1.0;
    for (int d = 0; d < c.dim; ++d) ndof *= (n[d] - 1);
    if (ndof > 4.0e9) return "lattice too large (more than 4e9 unknowns)";
    for (int level = 0; level < c.nlevel - 1; ++level) {
        // lattice3d.hh:241-257
        bool even = true, big = true;
        for (int d = 0; d < c.dim; ++d) {
            even = even && (n[d] % 2 == 0);
            big = big && (n[d] / 2 > 1);
        }
        if (!even) {
            err << "ERROR: cannot coarsen lattice of size " << n[0] << " x " << n[1];
            if (c.dim == 3) err << " x " << n[2];
            err << " [one of the extents is odd]";
            return err.str();
        }
        if (!big) {
            err << "ERROR: cannot coarsen lattice of size " << n[0] << " x " << n[1];
            if (c.dim == 3) err << " x " << n[2];
            err << " [resulting lattice would have no interior vertices]";
            return err.str();
        }
        for (int d = 0; d < c.dim; ++d) n[d] /= 2;
    }
    return "";
}

void galerkin_stencil(int dim, const double* fine, double* coarse) {
    // Two-step product mirroring (R A) R^T: t(mu) = sum_alpha w(alpha) A(mu - alpha) for fine
    // offsets mu in [-2,2]^d relative to 2i, then A_c(delta) = sum_mu t(mu) w(mu - 2 delta).
    const int zr = (dim == 3) ? 1 : 0;
    double t[5][5][5];
    memset(t, 0, sizeof(t));
    for (int mz = -2 * zr; mz <= 2 * zr; ++mz)
        for (int my = -2; my <= 2; ++my)
            for (int mx = -2; mx <= 2; ++mx) {
                double acc = 0.0;
                for (int az = -zr; az <= zr; ++az)
                    for (int ay = -1; ay <= 1; ++ay)
                        for (int ax = -1; ax <= 1; ++ax) {
                            const int bx = mx - ax, by = my - ay, bz = mz - az;
                            if (bx < -1 || bx > 1 || by < -1 || by > 1 || bz < -zr || bz > zr) continue;
                            const double w = (dim == 3 ? w1(ax) * w1(ay) * w1(az) : w1(ax) * w1(ay));
                            acc += w * fine[sidx(dim, bx, by, bz)];
                        }
                t[mz + 2][my + 2][mx + 2] = acc;
            }
    for (int k = 0; k < 27; ++k) coarse[k] = 0.0;
    for (int dz = -zr; dz <= zr; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                double acc = 0.0;
                for (int mz = -2 * zr; mz <= 2 * zr; ++mz)
                    for (int my = -2; my <= 2; ++my)
                        for (int mx = -2; mx <= 2; ++mx) {
                            const int gx = mx - 2 * dx, gy = my - 2 * dy, gz = mz - 2 * dz;
                            if (gx < -1 || gx > 1 || gy < -1 || gy > 1 || gz < -zr || gz > zr) continue;
                            const double w = (dim == 3 ? w1(gx) * w1(gy) * w1(gz) : w1(gx) * w1(gy));
                            acc += t[mz + 2][my + 2][mx + 2] * w;
                        }
                coarse[sidx(dim, dx, dy, dz)] = acc;
            }
}

bool stencil_axis_only(int dim, const double* st) {
    const int zr = dim == 3 ? 1 : 0;
    for (int dz = -zr; dz <= zr; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx)
                if (std::abs(dx) + std::abs(dy) + std::abs(dz) > 1 && st[sidx(dim, dx, dy, dz)] != 0.0) return false;
    return true;
}

std::vector<LevelSpec> build_hierarchy(const mgmc_config& c, const double* fine_st) {
    std::vector<LevelSpec> levels;
    LevelSpec L;
    memset(&L, 0, sizeof(L));
    L.dim = c.dim;
    L.n[0] = c.nx;
    L.n[1] = c.ny;
    L.n[2] = (c.dim == 3) ? c.nz : 0;
    // fine FD operator, shiftedlaplace_fd_operator.cc:18-56 (same expression order)
    double hinv2[3] = {0, 0, 0};
    double cell_volume = 1.0;
    for (int d = 0; d < c.dim; ++d) {
        const double h = 1. / double(L.n[d]);
        hinv2[d] = 1. / (h * h);
        cell_volume *= h;
    }
    double diagonal = cell_volume * c.kappa_sq;
    for (int d = 0; d < c.dim; ++d) {
        const double off = -cell_volume * hinv2[d];
        int o[3] = {0, 0, 0};
        o[d] = -1;
        L.st[sidx(c.dim, o[0], o[1], o[2])] = off;
        o[d] = +1;
        L.st[sidx(c.dim, o[0], o[1], o[2])] = off;
        diagonal += 2. * cell_volume * hinv2[d];
    }
    L.st[sidx(c.dim, 0, 0, 0)] = diagonal;
    L.npoints = 2 * c.dim + 1;
    L.ncolours = 2;
    if (c.fine_operator == MGMC_OPERATOR_FEM) {
        memset(L.st, 0, sizeof(L.st));
        fem_stencil(c.dim, L.n, c.kappa_sq, L.st);
        L.npoints = (c.dim == 3) ? 27 : 9;
        L.ncolours = 1 << c.dim;
    }
    if (fine_st) {  // a given constant stencil (mgmc_create_stencil)
        memset(L.st, 0, sizeof(L.st));
        for (int k = 0; k < (c.dim == 3 ? 27 : 9); ++k) L.st[k] = fine_st[k];
        const bool axis = stencil_axis_only(c.dim, L.st);
        L.npoints = axis ? 2 * c.dim + 1 : (c.dim == 3 ? 27 : 9);
        L.ncolours = axis ? 2 : 1 << c.dim;
    }
    for (int level = 0; level < c.nlevel; ++level) {
        L.ndof = 1;
        for (int d = 0; d < c.dim; ++d) L.ndof *= (uint64_t)(L.n[d] - 1);
        levels.push_back(L);
        if (level == c.nlevel - 1) break;
        LevelSpec C;
        memset(&C, 0, sizeof(C));
        C.dim = c.dim;
        for (int d = 0; d < c.dim; ++d) C.n[d] = L.n[d] / 2;
        galerkin_stencil(c.dim, L.st, C.st);
        C.npoints = (c.dim == 3) ? 27 : 9;
        C.ncolours = 1 << c.dim;
        L = C;
    }
    return levels;
}

}  // namespace mgmc
