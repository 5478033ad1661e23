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

// ---- blocked banded variant (coarsest levels above CHOL_MAX_N unknowns) ----
// Q is banded (lexicographic order, bandwidth bw = the widest coupling); its Cholesky factor keeps
// the band.  With blocks of B >= bw rows, L is block lower bidiagonal: diagonal blocks L_kk and
// coupling blocks C_k = L(block k, block k-1).  The two triangular solves run block by block in
// one workgroup per chain:
//   forward   t = f_k - C_k y_{k-1},            y_k = D_k t        (D_k = L_kk^{-1}, host)
//   noise     y'_k = y_k + xi_k
//   backward  t = y'_k - C_{k+1}^T x_{k+1},     x_k = D_k^T t
// every row an fma chain in ascending column order (the oracle's blocked mode replays it).  Four
// copies of the blocks are stored so that the threads' loads at a fixed column are coalesced:
//   Cf[k][j][r] = C_k(r, j)   Cb[k][j][r] = C_k(j, r)   Df[k][j][r] = D_k(r, j)   Db[k][j][r] = D_k(j, r)
// Work per solve O(n B) sequential in B-row steps: latency-bound, as the reference's two solves.
constexpr int CHOL_BLOCK_MAX = 4096;  // 2 B doubles of LDS (64 KB), <= 4 rows per thread
constexpr double CHOL_HOST_WORK_MAX = 1e11;  // n bw^2 of the banded host factor (about a minute)

struct CholBlockArgs {
    Layout L;
    int n, B, nb;
    const double* Cf;  // nb x B x B each
    const double* Cb;
    const double* Df;
    const double* Db;
    const double* f;
    double* x;
    int noise;
    RngKey key;
    uint32_t tag;
    const uint64_t* sample;
    long long cs;
    uint32_t chain0, seed_hi;
};

template <int DIM>
__global__ void __launch_bounds__(1024) k_coarse_chol_blocked(CholBlockArgs a) {
    {
        const int ch = (int)blockIdx.z;
        a.f += ch * a.cs;
        a.x += ch * a.cs;
        if (ch) a.key.k1 = (a.chain0 + (uint32_t)ch) ^ a.seed_hi;
    }
    extern __shared__ double sh[];
    double* v = sh;       // y_{k-1} (forward) / x_{k+1} (backward)
    double* t = sh + a.B; // right-hand side of the block
    const int B = a.B;
    const size_t BB = (size_t)B * B;
    const uint64_t sample = a.noise ? *a.sample : 0;
    for (int k = 0; k < a.nb; ++k) {
        const int base = k * B, Bk = min(B, a.n - base);
        for (int r = threadIdx.x; r < Bk; r += blockDim.x) {
            double s = 0.0;
            if (k > 0) {
                const double* C = a.Cf + k * BB + r;
                for (int j = 0; j < B; ++j) s = fma(C[(size_t)j * B], v[j], s);
            }
            int i, jj, kk;
            t[r] = a.f[chol_vertex<DIM>(a.L, base + r, &i, &jj, &kk)] - s;
        }
        __syncthreads();
        for (int r = threadIdx.x; r < Bk; r += blockDim.x) {
            const double* D = a.Df + k * BB + r;
            double y = 0.0;
            for (int j = 0; j <= r; ++j) y = fma(D[(size_t)j * B], t[j], y);
            v[r] = y;
            int i, jj, kk;
            const long long p = chol_vertex<DIM>(a.L, base + r, &i, &jj, &kk);
            if (a.noise) y = y + point_normal(a.key, pair_id<DIM>(a.L, i, jj, kk), (i & 1) != 0, a.tag, sample);
            a.x[p] = y;  // y' (read back by the same thread in the backward pass)
        }
        __syncthreads();
    }
    for (int k = a.nb - 1; k >= 0; --k) {
        const int base = k * B, Bk = min(B, a.n - base);
        for (int r = threadIdx.x; r < Bk; r += blockDim.x) {
            double s = 0.0;
            if (k + 1 < a.nb) {
                const int Bn = min(B, a.n - base - B);
                const double* C = a.Cb + (k + 1) * BB + r;
                for (int j = 0; j < Bn; ++j) s = fma(C[(size_t)j * B], v[j], s);
            }
            int i, jj, kk;
            t[r] = a.x[chol_vertex<DIM>(a.L, base + r, &i, &jj, &kk)] - s;
        }
        __syncthreads();
        for (int r = threadIdx.x; r < Bk; r += blockDim.x) {
            const double* D = a.Db + k * BB + r;
            double y = 0.0;
            for (int j = r; j < Bk; ++j) y = fma(D[(size_t)j * B], t[j], y);
            v[r] = y;
            int i, jj, kk;
            a.x[chol_vertex<DIM>(a.L, base + r, &i, &jj, &kk)] = y;
        }
        __syncthreads();
    }
}

// ---- host: banded factor -- bitwise the dense column-by-column Cholesky loop (the oracle's
// DenseCholeskySampler) restricted to the band: the products it skips are exact zeros ----
// band: row i holds columns i - bw .. i at band[i * (bw + 1) + (c - i + bw)]; in place Q -> L
inline bool chol_band_factor(std::vector<double>& band, long long n, long long bw) {
    const long long W = bw + 1;
    auto at = [&](long long i, long long c) -> double& { return band[(size_t)(i * W + (c - i + bw))]; };
    for (long long j = 0; j < n; ++j) {
        double d = at(j, j);
        for (long long k = std::max(0LL, j - bw); k < j; ++k) d -= at(j, k) * at(j, k);
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        at(j, j) = d;
        const long long iend = std::min(n - 1, j + bw);
        for (long long i = j + 1; i <= iend; ++i) {
            double s = at(i, j);
            for (long long k = std::max(0LL, i - bw); k < j; ++k) s -= at(i, k) * at(j, k);
            at(i, j) = s / d;
        }
    }
    return true;
}

inline long long chol_block_size(long long bw) {
    const long long b = std::max(bw, 1LL);
    return std::max(64LL, (b + 63) / 64 * 64);
}

// the four block copies of a banded factor (layout above); D_k by the dense inverse loop
// restricted to the diagonal block
inline void chol_blocks_host(const std::vector<double>& band, long long n, long long bw, long long B,
                             std::vector<double>& Cf, std::vector<double>& Cb, std::vector<double>& Df,
                             std::vector<double>& Db) {
    const long long W = bw + 1, nb = (n + B - 1) / B;
    auto L = [&](long long i, long long c) -> double {
        return (c <= i && i - c <= bw) ? band[(size_t)(i * W + (c - i + bw))] : 0.0;
    };
    const size_t BB = (size_t)B * B;
    Cf.assign(nb * BB, 0.0);
    Cb.assign(nb * BB, 0.0);
    Df.assign(nb * BB, 0.0);
    Db.assign(nb * BB, 0.0);
    std::vector<double> D(BB);
    for (long long k = 0; k < nb; ++k) {
        const long long base = k * B, Bk = std::min(B, n - base);
        if (k > 0)
            for (long long r = 0; r < Bk; ++r)
                for (long long j = 0; j < B; ++j) {
                    const double c = L(base + r, base - B + j);
                    Cf[k * BB + j * B + r] = c;
                    Cb[k * BB + r * B + j] = c;
                }
        std::fill(D.begin(), D.end(), 0.0);
        for (long long c = 0; c < Bk; ++c)
            for (long long r = c; r < Bk; ++r) {
                double s = r == c ? 1.0 : 0.0;
                for (long long m = c; m < r; ++m) s -= L(base + r, base + m) * D[m * B + c];
                D[r * B + c] = s / L(base + r, base + r);
            }
        for (long long r = 0; r < Bk; ++r)
            for (long long j = 0; j <= r; ++j) {
                Df[k * BB + j * B + r] = D[r * B + j];
                Db[k * BB + r * B + j] = D[r * B + j];
            }
    }
}

// ---- host: dense inverses (the oracle's dense_factor_inverses loops, operation for operation) ----
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
