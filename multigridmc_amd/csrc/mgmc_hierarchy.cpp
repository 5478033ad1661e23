// mgmc_hierarchy.cpp -- see mgmc_hierarchy.hpp.
#include "mgmc_hierarchy.hpp"

#include <math.h>
#include <string.h>

#include <sstream>

namespace mgmc {

namespace {

// linear-interpolation weight of a 1d offset in {-1,0,1} (intergrid_operator_linear.cc:13-17)
inline double w1(int o) { return o == 0 ? 1.0 : 0.5; }

inline int sidx(int dim, int dx, int dy, int dz) {
    return dim == 3 ? (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1) : (dy + 1) * 3 + (dx + 1);
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

std::vector<LevelSpec> build_hierarchy(const mgmc_config& c) {
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
