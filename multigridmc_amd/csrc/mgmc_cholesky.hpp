// mgmc_cholesky.hpp -- dense Cholesky coarse sampler / coarse solve on the coarsest level.
//
// Reference: DenseCholeskySampler (sampler/cholesky_sampler.cc:26-41, cholesky_sampler.hh:50-66):
// Q = L L^T, xi ~ N(0, I), x = L^{-T} (xi + L^{-1} f); the multigrid preconditioner's coarse solve
// (preconditioner/multigrid_preconditioner.cc:76-80) is the same without xi.  Two triangular
// solves are n sequential steps; on the device both become dense products with factors computed
// once on the host: x = G f + U xi with G = Q^{-1} = U U^T and U = L^{-T}.  Every row is
// independent (one thread, an fma chain in ascending column order -- replayed by the oracle's
// MULTICOLOUR mode), so the coarsest level costs one launch and O(n^2 / threads) work.
// xi_j is the Philox normal of vertex j under the op's sweep tag -- the draw a Gibbs sweep of this
// level would make.  Factors are stored so that a warp's loads at column j are coalesced:
// G (symmetric) and Li = L^{-1} (row j of L^{-1} = column j of U).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "mgmc_kernels.hpp"

namespace mgmc {

constexpr int CHOL_MAX_N = 8192;  // 2 n doubles of LDS per workgroup, 2 n^2 doubles of factors

struct CholArgs {
    Layout L;
    int n;
    const double* G;   // n x n, G[j * n + i] = (Q^{-1})_ij
    const double* Li;  // n x n, Li[j * n + i] = (L^{-1})_ji = U_ij
    const double* f;   // padded
    double* x;         // padded
    int noise;
    RngKey key;
    uint32_t tag;
    const uint64_t* sample;
    long long cs;               // batched chains (blockIdx.z): doubles between chains of f and x
    uint32_t chain0, seed_hi;   // chain c's Philox key: (key.k0, lo32(chain0 + c) ^ seed_hi)
};

template <int DIM>
__device__ __forceinline__ long long chol_vertex(const Layout& L, int e, int* i, int* j, int* k) {
    const int nxi = L.nx - 1, nyi = L.ny - 1;
    *i = e % nxi + 1;
    *j = (e / nxi) % nyi + 1;
    *k = DIM == 3 ? e / (nxi * nyi) + 1 : 0;
    return L.at(*i, *j, *k);
}

template <int DIM>
__global__ void __launch_bounds__(256) k_coarse_chol(CholArgs a) {
    {
        const int ch = (int)blockIdx.z;
        a.f += ch * a.cs;
        a.x += ch * a.cs;
        if (ch) a.key.k1 = (a.chain0 + (uint32_t)ch) ^ a.seed_hi;
    }
    extern __shared__ double sh[];
    double* fl = sh;
    double* xi = sh + a.n;
    const uint64_t sample = a.noise ? *a.sample : 0;
    for (int e = threadIdx.x; e < a.n; e += blockDim.x) {
        int i, j, k;
        const long long p = chol_vertex<DIM>(a.L, e, &i, &j, &k);
        fl[e] = a.f[p];
        if (a.noise) xi[e] = point_normal(a.key, pair_id<DIM>(a.L, i, j, k), (i & 1) != 0, a.tag, sample);
    }
    __syncthreads();
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.n) return;
    double s = 0.0;
    for (int c = 0; c < a.n; ++c) s = fma(a.G[(long long)c * a.n + r], fl[c], s);
    double t = 0.0;
    if (a.noise)
        for (int c = r; c < a.n; ++c) t = fma(a.Li[(long long)c * a.n + r], xi[c], t);
    int i, j, k;
    a.x[chol_vertex<DIM>(a.L, r, &i, &j, &k)] = s + t;
}

// ---- host: dense factor and inverses (the oracle's DenseCholeskySampler / dense_factor_inverses
// loops, operation for operation) ----
// Q (row-major, in place) -> lower Cholesky factor; false if not positive definite
inline bool chol_factor_host(std::vector<double>& Lm, long long n) {
    for (long long j = 0; j < n; ++j) {
        double d = Lm[(size_t)j * n + j];
        for (long long k = 0; k < j; ++k) d -= Lm[(size_t)j * n + k] * Lm[(size_t)j * n + k];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        Lm[(size_t)j * n + j] = d;
        for (long long i = j + 1; i < n; ++i) {
            double s = Lm[(size_t)i * n + j];
            for (long long k = 0; k < j; ++k) s -= Lm[(size_t)i * n + k] * Lm[(size_t)j * n + k];
            Lm[(size_t)i * n + j] = s / d;
        }
        for (long long k = j + 1; k < n; ++k) Lm[(size_t)j * n + k] = 0.0;
    }
    return true;
}

// Li = L^{-1} (row-major), G = U U^T with U = Li^T
inline void chol_inverses_host(const std::vector<double>& L, long long n, std::vector<double>& Li,
                               std::vector<double>& G) {
    Li.assign((size_t)n * n, 0.0);
    for (long long c = 0; c < n; ++c)
        for (long long i = c; i < n; ++i) {
            double s = i == c ? 1.0 : 0.0;
            for (long long k = c; k < i; ++k) s -= L[(size_t)i * n + k] * Li[(size_t)k * n + c];
            Li[(size_t)i * n + c] = s / L[(size_t)i * n + i];
        }
    G.assign((size_t)n * n, 0.0);
    for (long long i = 0; i < n; ++i)
        for (long long j = 0; j < n; ++j) {
            double s = 0.0;
            for (long long k = std::max(i, j); k < n; ++k) s += Li[(size_t)k * n + i] * Li[(size_t)k * n + j];
            G[(size_t)i * n + j] = s;
        }
}

}  // namespace mgmc
