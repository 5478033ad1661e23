// mgmc_field.hpp -- levels with per-vertex coefficients (operators built from a matrix:
// mgmc_create_csr; the periodic correlation-length model, the squared FD operator).
//
// A level's operator is stored as a coefficient field: for every interior vertex (reference order, x
// fastest) its row's np coefficients at the level's np offsets, the union of the row patterns in
// ascending column order (a row's entries missing from the union pattern are zeros).  Arithmetic is
// that of the constant-stencil kernels (mgmc_kernels.hpp) with the row read from the field:
//   * Gibbs / SOR update: S = fma chain over the row in ascending column order, c = fma(sd, xi, f),
//     x = fma(omega / a_cc, c - S, x), sd = sqrt(a_cc (2 - omega) / omega) per vertex
//     (sor_sampler.cc:22-27, sor_smoother.cc:62-76);
//   * residual r = f - A x with A x = ((0 + a_1 x_1) + a_2 x_2) ... (linear_operator.hh:66-76);
// so the CPU oracle's CSR replay (which sums only stored entries) gives the same bits: a zero of the
// field adds an exact +-0.
// Colourings: 2 colours (red-black, (i + j + k) & 1) for a 5/7-point fine level, 2^d (coordinate
// parities) for reach-1 levels, 3^d (coordinates mod 3) for reach-2 levels; colours in ascending
// order forward, descending backward, as the oracle's multicolour mode.
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

constexpr int FIELD_MAXNP = 125;  // 5^3: the reach-2 box

struct FieldArg {
    const double* coef;   // [ndof][np]
    int np;               // points per row
    int diag;             // index of the centre point
    int nxi, nyi;         // interior extents (row index of a vertex)
    int scheme;           // colour count: 2 (red-black), 4 / 8 (parities), 9 / 27 (mod 3)
    int pad_;
    double omega;
    int off[FIELD_MAXNP];  // padded-layout offsets of the points, ascending
};

template <int DIM>
__device__ __forceinline__ long long field_row(const FieldArg& F, int i, int j, int k) {
    return ((long long)(DIM == 3 ? k - 1 : 0) * F.nyi + (j - 1)) * F.nxi + (i - 1);
}

// vertex (i, j, k) of colour c for thread (tx, ty, tz) of a colour pass; false past the lattice
template <int DIM>
__device__ __forceinline__ bool field_vertex(const Layout& L, const FieldArg& F, int c, int tx, int ty, int tz, int& i,
                                             int& j, int& k) {
    if (F.scheme == 2) {
        j = ty + 1;
        k = DIM == 3 ? tz + 1 : 0;
        i = 1 + (((1 + j + k) ^ c) & 1) + 2 * tx;
    } else if (F.scheme == 4 || F.scheme == 8) {
        i = 2 - (c & 1) + 2 * tx;
        j = 2 - ((c >> 1) & 1) + 2 * ty;
        k = DIM == 3 ? 2 - ((c >> 2) & 1) + 2 * tz : 0;
    } else {
        const int ci = c % 3, cj = (c / 3) % 3, ck = c / 9;
        i = (ci ? ci : 3) + 3 * tx;
        j = (cj ? cj : 3) + 3 * ty;
        k = DIM == 3 ? (ck ? ck : 3) + 3 * tz : 0;
    }
    return i <= L.nx - 1 && j <= L.ny - 1 && (DIM != 3 || k <= L.nz - 1);
}

// one colour pass of a Gibbs (NOISE) or SOR sweep
template <int DIM, bool NOISE>
__global__ void __launch_bounds__(256) k_fsweep(Layout L, double* __restrict__ x, const double* __restrict__ f,
                                                FieldArg F, GibbsArg G) {
    int i, j, k;
    if (!field_vertex<DIM>(L, F, G.colour, blockIdx.x * blockDim.x + threadIdx.x,
                           blockIdx.y * blockDim.y + threadIdx.y, blockIdx.z, i, j, k))
        return;
    const long long p = L.at(i, j, k);
    const double* a = F.coef + field_row<DIM>(F, i, j, k) * F.np;
    double s = a[0] * x[p + F.off[0]];
    for (int q = 1; q < F.np; ++q) s = fma(a[q], x[p + F.off[q]], s);
    const double d = a[F.diag];
    double c = f[p];
    if (NOISE) {
        const double xi = point_normal(G.key, pair_id<DIM>(L, i, j, k), (i & 1) != 0, G.tag, *G.sample);
        c = fma(sqrt_rad(d * (2. - F.omega) / F.omega), xi, f[p]);
    }
    x[p] = fma(F.omega / d, c - s, x[p]);
}

// r = f - A x (ZERO_F: r = -A x, i.e. y = A x with the sign folded in by the caller)
template <int DIM>
__global__ void __launch_bounds__(256) k_fresidual(Layout L, const double* __restrict__ x,
                                                   const double* __restrict__ f, FieldArg F, double* __restrict__ r) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = DIM == 3 ? (int)blockIdx.z + 1 : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    const long long p = L.at(i, j, k);
    const double* a = F.coef + field_row<DIM>(F, i, j, k) * F.np;
    double y = 0.0;
    for (int q = 0; q < F.np; ++q) y += a[q] * x[p + F.off[q]];
    r[p] = f[p] - y;
}

// y = A x (LinearOperator::apply, Eigen SpMV order)
template <int DIM>
__global__ void __launch_bounds__(256) k_fapply(Layout L, const double* __restrict__ x, FieldArg F,
                                                double* __restrict__ y) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = DIM == 3 ? (int)blockIdx.z + 1 : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    const long long p = L.at(i, j, k);
    const double* a = F.coef + field_row<DIM>(F, i, j, k) * F.np;
    double s = 0.0;
    for (int q = 0; q < F.np; ++q) s += a[q] * x[p + F.off[q]];
    y[p] = s;
}

}  // namespace mgmc
