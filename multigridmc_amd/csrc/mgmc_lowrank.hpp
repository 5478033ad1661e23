// mgmc_lowrank.hpp -- low-rank posterior part of a level: Q = A + B Sigma^{-1} B^T.
//
// Reference (nilsfriess/MultigridMC, src/):
//   * SORSmoother::apply: after every sweep  x -= B_bar (B^T x)          smoother/sor_smoother.cc:41-53
//     B_bar = (L + D/omega)^{-1} B (Sigma + B^T (L + D/omega)^{-1} B)^{-1}  (forward; L^T backward),
//     set up once per smoother                                          smoother/sor_smoother.cc:17-37
//   * SORSampler::apply: c += B Sigma^{-1/2} xi'  (m extra normals per sweep) sampler/sor_sampler.cc:48-56
//   * LinearOperator::apply: y = A x + B (Sigma^{-1} B^T x)              linear_operator.hh:66-76
//   * coarse levels: B_c = R B, Sigma_c = Sigma                          linear_operator.cc:10-23
//
// Why the multicolour splitting makes this cheap.  The reference's B_bar is a dense N x m matrix:
// the lexicographic triangular solve (L + D/omega)^{-1} spreads every column of B over all later
// vertices, so each sweep reads N*m doubles (1.07 GB at 256^3, m = 8).  Under the multicolour
// splitting the same solve is one noise-free multicolour sweep from zero: colour c only reads
// colours < c at distance one, so the fill of a column stays within a few vertices of its
// support.  B_bar keeps that row support (B_bar = Y M^{-1} mixes columns, not rows), and the
// device stores only those rows: a point measurement costs a few dozen rows instead of N.  A dense
// column of B (the global average measurement) makes B_bar dense again, as in the reference.
//
// Device arithmetic order (replayed by the oracle's MULTICOLOUR mode, oracle/refcpu.cpp):
//   * B^T-type dots  sum_e (sc_k B_ek) v_e  over a column's entry list (rows ascending; a dense
//     column lists every row): blocks of LR_BLK entries, lane l of a 64-wide wavefront sums
//     entries l, l+64, ... from 0.0, lanes combine by the xor butterfly 32, 16, ..., 1; the block
//     partials are combined the same way.  sc_k = 1 for the smoother fix, 1/Sigma_k for the
//     residual's Sigma^{-1} B^T x.
//   * e = B s: e_i = sum over the columns of row i in ascending k of B_ik s_k (plain mul + add);
//     sampler noise  f_eff = f + e, s_k = sqrt(1/Sigma_k) xi'_k with xi' from Philox pair
//     LR_PAIR0 + k/2 (cos branch for even k) of the sweep's tag;
//   * smoother fix  u_i = fma chain over k of B_bar_ik w_k,  x_i = x_i - u_i;
//   * posterior residual  r = (f - B t) - A x,  t = Sigma^{-1} B^T x: f is patched on the rows of
//     B, the residual kernels run unchanged, f is restored.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "mgmc_kernels.hpp"
#include "mgmc_tuning.hpp"

namespace mgmc {

constexpr int LR_BLK = 4096;            // entries per dot-product block
constexpr uint32_t LR_PAIR0 = 0xFFFFF000u;  // Philox pair ids of the low-rank noise (above any lattice pair)
constexpr int LR_MAX_M = 64;

struct LRColMeta {
    long long n;     // entries in the column's list
    long long ent0;  // first entry in the sparse entry arrays (sparse columns)
    int dense;       // index of the column's padded value array, or -1
    int blk0, nblk;  // dot-product blocks
    int cflag;       // dense column whose every value is cval (bit for bit): no value array is read
    double cval;     // (the global average on the fine level: the cell volume, measured_operator.cc:31-45)
};

// Everything a dot-product block needs in one load (the kernels used to chase blk_col -> meta -> sc,
// three dependent round trips before the first entry load; built by lr_setup_level)
struct LRBlock {
    long long e0;    // first entry of the block in its column
    long long ent0;  // entry-list columns: the block's first entry in ent_off / ent_val
    int k;           // column
    int cnt;         // entries (<= LR_BLK)
    int dense;       // value array of a dense column, or -1
    int cflag;       // dense column whose every value is cval
    double cval;
    double sc[2];    // the column's dot scales: 1 (B^T x), 1/Sigma_k (Sigma^{-1} B^T x)
};

// padded offset of interior vertex e (reference order, x fastest) of a level: e = (k-1) nyi nxi +
// (j-1) nxi + (i-1) by floating-point reciprocals with one correction step (exact for e < 2^51)
__device__ __forceinline__ long long lr_entry_pos(const Layout& L, long long e, double rnx, double rny) {
    const int nxi = L.nx - 1, nyi = L.ny - 1;
    long long r = (long long)((double)e * rnx);
    long long i = e - r * nxi;
    if (i < 0) {
        --r;
        i += nxi;
    } else if (i >= nxi) {
        ++r;
        i -= nxi;
    }
    long long kk = (long long)((double)r * rny);
    long long j = r - kk * nyi;
    if (j < 0) {
        --kk;
        j += nyi;
    } else if (j >= nyi) {
        ++kk;
        j -= nyi;
    }
    return L.at((int)i + 1, (int)j + 1, L.dim == 3 ? (int)kk + 1 : 0);
}

// ---- dot products, stage 1: one wavefront per block of LR_BLK entries ----
// A dense column lists every vertex in reference order: lane l's entries e, e + 64, ... are walked
// with incremental (i, j, k) (no 64-bit division per entry).  The lane's sum runs in entry order;
// the entries are taken LRP_U at a time with their loads issued together (the coarse levels' dots
// are a handful of wavefronts, each a chain of up to 64 dependent global round trips otherwise).
// Batched chains: blockIdx.y = a group of LRP_CH chains; the column value of an entry is loaded
// once for the group (v cs apart, the partials nblk apart per chain).
constexpr int LRP_U = tune::LR_PART_U, LRP_CH = tune::LR_PART_CH;
static __global__ void __launch_bounds__(64) k_lr_partials(Layout L, const LRBlock* __restrict__ blk, int sel,
                                                     const long long* __restrict__ ent_off,
                                                     const double* __restrict__ ent_val,
                                                     const double* __restrict__ dense_val,
                                                     const double* __restrict__ v,
                                                     double* __restrict__ part, long long cs, int nblk, int nch) {
    const int b = blockIdx.x;
    const int ch0 = blockIdx.y * LRP_CH;
    const int nc = min(LRP_CH, nch - ch0);
    const int lane = threadIdx.x;
    const LRBlock c = blk[b];
    const double s = sel ? c.sc[1] : c.sc[0];  // (a static index: no private-memory copy of c)
    const double* vc = v + ch0 * cs;
    const long long e1 = c.e0 + lane;
    const int cnt = lane < c.cnt ? (c.cnt - lane + 63) / 64 : 0;  // entries of this lane
    double acc[LRP_CH];
#pragma unroll
    for (int q = 0; q < LRP_CH; ++q) acc[q] = 0.0;
    if (c.dense >= 0) {
        const double* dv = dense_val + (long long)c.dense * L.nstore;
        const int nxi = L.nx - 1, nyi = L.ny - 1;
        const long long r = e1 / nxi;
        int i = (int)(e1 - r * nxi) + 1;
        int j = (int)(r % nyi) + 1;
        int kk = L.dim == 3 ? (int)(r / nyi) + 1 : 0;
        for (int base = 0; base < cnt; base += LRP_U) {
            long long p[LRP_U];
            double a[LRP_U], x[LRP_CH][LRP_U];
#pragma unroll
            for (int u = 0; u < LRP_U; ++u) {
                p[u] = L.at(i, j, kk);
                i += 64;  // advance by 64 entries (nxi may be < 64: carry repeatedly)
                while (i > nxi) {
                    i -= nxi;
                    if (++j > nyi) {
                        j = 1;
                        ++kk;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < LRP_U; ++u)
                if (base + u < cnt) {
                    a[u] = c.cflag ? c.cval : dv[p[u]];
#pragma unroll
                    for (int q = 0; q < LRP_CH; ++q)
                        if (q < nc) x[q][u] = vc[q * cs + p[u]];
                }
#pragma unroll
            for (int q = 0; q < LRP_CH; ++q)
#pragma unroll
                for (int u = 0; u < LRP_U; ++u)
                    if (q < nc && base + u < cnt) acc[q] = acc[q] + (s * a[u]) * x[q][u];
        }
    } else {
        const long long q0 = c.ent0 + lane;
        for (int base = 0; base < cnt; base += LRP_U) {
            double a[LRP_U], x[LRP_CH][LRP_U];
#pragma unroll
            for (int u = 0; u < LRP_U; ++u)
                if (base + u < cnt) {
                    const long long q = q0 + 64ll * (base + u);
                    a[u] = ent_val[q];
                    const long long o = ent_off[q];
#pragma unroll
                    for (int w = 0; w < LRP_CH; ++w)
                        if (w < nc) x[w][u] = vc[w * cs + o];
                }
#pragma unroll
            for (int w = 0; w < LRP_CH; ++w)
#pragma unroll
                for (int u = 0; u < LRP_U; ++u)
                    if (w < nc && base + u < cnt) acc[w] = acc[w] + (s * a[u]) * x[w][u];
        }
    }
#pragma unroll
    for (int q = 0; q < LRP_CH; ++q) {
        double t = acc[q];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) t = t + __shfl_xor(t, off, 64);
        if (lane == 0 && q < nc) part[(long long)(ch0 + q) * nblk + b] = t;
    }
}

// ---- dot products, stage 1 on small levels: the same partials, the loads spread over a workgroup ----
// A level with few blocks runs only a handful of wavefronts whose lanes each chase 64 dependent
// round trips.  Here 256 threads form the block's 4096 products (s B_e) v_e at once into LDS, then
// lane l of the first wavefront adds its entries l, l+64, ... in entry order and the butterfly
// follows: the single-wavefront kernel's sums, bit for bit.  One chain per blockIdx.y.
constexpr int LRS_NT = 256;
static __global__ void __launch_bounds__(LRS_NT) k_lr_partials_staged(Layout L, const LRBlock* __restrict__ blk, int sel,
                                                               const long long* __restrict__ ent_off,
                                                               const double* __restrict__ ent_val,
                                                               const double* __restrict__ dense_val,
                                                               const double* __restrict__ v, double* __restrict__ part,
                                                               long long cs, int nblk) {
    __shared__ double prod[LR_BLK];
    const int b = blockIdx.x;
    const int ch = blockIdx.y;
    const int tid = threadIdx.x;
    const LRBlock c = blk[b];
    const int cnt = c.cnt;  // entries of this block
    const double s = sel ? c.sc[1] : c.sc[0];  // (a static index: no private-memory copy of c)
    const double* vc = v + ch * cs;
    constexpr int PER = LR_BLK / LRS_NT;
    if (c.dense >= 0) {
        const double* dv = dense_val + (long long)c.dense * L.nstore;
        // every entry's vertex directly (the 256-entry carry walked up to 8 rows per step on the small
        // levels); positions past the column's end are clamped to its first entry, never stored
        const double rnx = 1.0 / (double)(L.nx - 1), rny = 1.0 / (double)(L.ny - 1);
        long long p[PER];
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int e = tid + t * LRS_NT;
            p[t] = lr_entry_pos(L, c.e0 + (e < cnt ? e : 0), rnx, rny);
        }
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int e = tid + t * LRS_NT;
            if (e < cnt) prod[e] = (s * (c.cflag ? c.cval : dv[p[t]])) * vc[p[t]];
        }
    } else {
#pragma unroll
        for (int t = 0; t < PER; ++t) {
            const int e = tid + t * LRS_NT;
            if (e < cnt) {
                const long long q = c.ent0 + e;
                prod[e] = (s * ent_val[q]) * vc[ent_off[q]];
            }
        }
    }
    __syncthreads();
    if (tid >= 64) return;
    // lane l: entries l, l + 64, ... in order, their LDS reads issued 8 at a time
    double acc = 0.0;
    int e = tid;
    for (; e + 7 * 64 < cnt; e += 8 * 64) {
        double t8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t8[u] = prod[e + u * 64];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = acc + t8[u];
    }
    for (; e < cnt; e += 64) acc = acc + prod[e];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
    if (tid == 0) part[(long long)ch * nblk + b] = acc;
}

// ---- dot products, stage 2: one wavefront per column ----
static __global__ void __launch_bounds__(64) k_lr_totals(const LRColMeta* __restrict__ meta, const double* __restrict__ part,
                                                   double* __restrict__ out, int nblk, int m) {
    const int k = blockIdx.x;
    const int lane = threadIdx.x;
    const LRColMeta c = meta[k];
    part += (long long)blockIdx.z * nblk;  // batched chains (blockIdx.z): part nblk, out m apart
    out += (long long)blockIdx.z * m;
    // lane l adds partials l, l + 64, ... in order; the loads of U of them are issued together
    // (the fine level's dense column has ~4000 blocks: 63 dependent round trips per lane otherwise)
    const double* pc = part + c.blk0;
    double acc = 0.0;
    int b = lane;
    constexpr int U = 8;
    for (; b + (U - 1) * 64 < c.nblk; b += U * 64) {
        double t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = pc[b + u * 64];
#pragma unroll
        for (int u = 0; u < U; ++u) acc = acc + t[u];
    }
    for (; b < c.nblk; b += 64) acc = acc + pc[b];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
    if (lane == 0) out[k] = acc;
}

// ---- patch a vector on the rows of B with e = B s ----
//   mode 0: sampler noise  f_save = f, f = f + B s  with s_k = sq_k xi'_k drawn here
//   mode 1: residual       f_save = f, f = f - B t  (t = Sigma^{-1} B^T x, precomputed)
//   mode 2: operator       y = y + B t
enum { LR_PATCH_NOISE = 0, LR_PATCH_RESIDUAL = 1, LR_PATCH_APPLY = 2 };

// The patch of one row of B: y +/- e, e = 0.0 + sum_k B_ik s_k over the row's columns in ascending k
// (Eigen's sparse-times-dense order).  On a level with a split column g (LowRankDev::split_g: its one
// dense column, every value one number -- the fine level's global average) the column is added last
// and on its own: (y +/- e_loc) +/- e_g, e_loc = 0.0 + sum_{k != g} (applied only on a row with such
// a k), e_g = 0.0 + B_ig s_g -- the same sum in another order (the oracle's MULTICOLOUR patch follows
// it).  defer: e_g is left out, the consumer kernel adds it (LRRhsArg).
__device__ __forceinline__ double lr_row_patch(double y, bool minus, uint64_t msk, const double* cf,
                                               const double* s, int m, int g, bool defer) {
    double e = 0.0;
    bool any = false;
    for (int k = 0; k < m; ++k)
        if (k != g && ((msk >> k) & 1)) {
            e = e + cf[k] * s[k];
            any = true;
        }
    if (g < 0) return minus ? y - e : y + e;
    double t = y;
    if (any) t = minus ? t - e : t + e;
    if (!defer && ((msk >> g) & 1)) {
        const double eg = 0.0 + cf[g] * s[g];
        t = minus ? t - eg : t + eg;
    }
    return t;
}

struct LRPatchArgs {
    int m, nrows;
    const long long* off;    // padded offsets of the rows of B
    const double* coef;      // nrows x m, B_ik (0 where absent)
    const uint64_t* mask;    // bit k: column k has an entry in the row
    const double* t;         // mode 1/2: the m-vector
    const double* sq;        // mode 0: sqrt(1 / Sigma_k)
    RngKey key;
    uint32_t tag;
    const uint64_t* sample;
    double* y;
    double* save;
    int mode;
    long long cs;               // batched chains (blockIdx.z): y cs, save nrows, t m apart
    uint32_t chain0, seed_hi;   // chain c's Philox key: (key.k0, lo32(chain0 + c) ^ seed_hi)
    int split_g;                // the level's split column (lr_row_patch), -1: none (and LR_PATCH_APPLY)
    // non-null (a level read in place, LRRhsArg): the rows defer e_g, and eout[c] = chain c's
    // +/-(0.0 + bgc s_g), the term every row's consumer adds (bgc = B_g's one number)
    double* eout;
    double bgc;
};

__device__ __forceinline__ RngKey lr_chain_key(RngKey key, uint32_t chain0, uint32_t seed_hi, int ch) {
    if (ch) key.k1 = (chain0 + (uint32_t)ch) ^ seed_hi;
    return key;
}

static __global__ void __launch_bounds__(256) k_lr_patch(LRPatchArgs a) {
    {
        const int ch = batch_chain();
        a.y += ch * a.cs;
        a.save += (long long)ch * a.nrows;
        if (a.t) a.t += ch * a.m;
        a.key = lr_chain_key(a.key, a.chain0, a.seed_hi, ch);
    }
    __shared__ double s[LR_MAX_M];
    if (a.mode == LR_PATCH_NOISE) {
        const int t = threadIdx.x;
        if (2 * t < a.m) {
            const uint64_t sample = *a.sample;
            const Philox4 r = philox4x32_10(LR_PAIR0 + (uint32_t)t, a.tag, (uint32_t)sample, (uint32_t)(sample >> 32),
                                            a.key.k0, a.key.k1);
            double z0, z1;
            normal_pair(r, &z0, &z1);
            s[2 * t] = a.sq[2 * t] * z0;
            if (2 * t + 1 < a.m) s[2 * t + 1] = a.sq[2 * t + 1] * z1;
        }
    } else if ((int)threadIdx.x < a.m) {
        s[threadIdx.x] = a.t[threadIdx.x];
    }
    __syncthreads();
    if (a.eout && blockIdx.x == 0 && threadIdx.x == 0) {
        const double e = 0.0 + a.bgc * s[a.split_g];
        a.eout[batch_chain()] = a.mode == LR_PATCH_RESIDUAL ? -e : e;  // (y - e == y + (-e))
    }
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= a.nrows) return;
    const long long p = a.off[u];
    const double y = a.y[p];
    if (a.mode != LR_PATCH_APPLY) a.save[u] = y;
    a.y[p] = lr_row_patch(y, a.mode == LR_PATCH_RESIDUAL, a.mask[u], a.coef + (long long)u * a.m, s, a.m, a.split_g,
                          a.eout != nullptr);
}

// ---- smoother fix x -= B_bar w on B_bar's rows; optionally restore f on the rows of B ----
// Batched chains: every row of B_bar is read once and applied to all nch chains (x, f cs apart, w m
// apart, the saved f nrest apart) -- the (N x m) (m x C) product of the chain batch, each chain's
// entry the single-chain fma chain over k ascending.
constexpr int LR_MAX_CH = 16;  // chains of one batched handle (w of every chain in LDS)
static __global__ void __launch_bounds__(256) k_lr_update(int m, int nbar, const long long* __restrict__ bar_off,
                                                    const double* __restrict__ bar_val, const double* __restrict__ w,
                                                    double* __restrict__ x, int nrest,
                                                    const long long* __restrict__ rest_off,
                                                    const double* __restrict__ rest_val, double* __restrict__ f,
                                                    int nch, long long cs) {
    __shared__ double ws[LR_MAX_CH * LR_MAX_M];
    for (int q = threadIdx.x; q < nch * m; q += blockDim.x) ws[q] = w[q];
    __syncthreads();
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < nbar) {
        const double* bv = bar_val + (long long)u * m;  // from HBM once, then from L1 for chains 1..
        const long long p = bar_off[u];
        for (int ch = 0; ch < nch; ++ch) {
            double acc = 0.0;
            for (int k = 0; k < m; ++k) acc = fma(bv[k], ws[ch * m + k], acc);
            double* xc = x + ch * cs;
            xc[p] = xc[p] - acc;
        }
    }
    if (u < nrest)
        for (int ch = 0; ch < nch; ++ch) f[ch * cs + rest_off[u]] = rest_val[(long long)ch * nrest + u];
}

// ---- restore f on the rows of B ----
static __global__ void __launch_bounds__(256) k_lr_restore(int n, const long long* __restrict__ off,
                                                     const double* __restrict__ save, double* __restrict__ f,
                                                     long long cs) {
    save += (long long)blockIdx.z * n;  // batched chains (blockIdx.z)
    f += blockIdx.z * cs;
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u < n) f[off[u]] = save[u];
}

// ---- after a residual + restriction: every f update until the level's next sweeps, one launch ----
// Job 0 (the fine level of the restriction): restore f, and with `noise` set patch it at once with
// the noise of its first post-sweep -- f is not touched again before that sweep (the coarse-grid
// correction writes only coarser f and this level's x), and save[] already holds the true f, so
// the patched values equal the separate restore + k_lr_patch bit for bit.  Job 1 (the coarse level):
// the noise patch of its first pre-sweep (k_lr_patch, LR_PATCH_NOISE).  Blocks [0, nb0) run job 0.
struct LRJob {
    int m, nrows;
    const long long* off;
    const double* coef;
    const uint64_t* mask;
    const double* sq;
    uint32_t tag;
    double* f;
    double* save;
    int restore;  // 1: f = save (+ noise)
    int noise;    // 1: + B Sigma^{-1/2} xi'
    int split_g;   // the level's split column (lr_row_patch), -1: none
    double* eout;  // non-null (noise, a level read in place): rows defer e_g, eout[c] = 0.0 + bgc s_g (k_lr_patch)
    double bgc;
};

struct LRRestorePatchArgs {
    LRJob job[2];
    int nb0;
    RngKey key;
    const uint64_t* sample;
    long long cs[2];            // batched chains (blockIdx.z): f of job 0 / 1 cs apart, save nrows apart
    uint32_t chain0, seed_hi;
};

static __global__ void __launch_bounds__(256) k_lr_restore_patch(LRRestorePatchArgs a) {
    __shared__ double s[LR_MAX_M];
    const bool second = (int)blockIdx.x >= a.nb0;
    const int ch = batch_chain();
    a.key = lr_chain_key(a.key, a.chain0, a.seed_hi, ch);
    LRJob j = a.job[second ? 1 : 0];
    j.f += ch * a.cs[second ? 1 : 0];
    j.save += (long long)ch * j.nrows;
    const int u = (second ? (int)blockIdx.x - a.nb0 : (int)blockIdx.x) * blockDim.x + threadIdx.x;
    if (j.noise) {
        const int t = threadIdx.x;
        if (2 * t < j.m) {
            const uint64_t sample = *a.sample;
            const Philox4 r =
                philox4x32_10(LR_PAIR0 + (uint32_t)t, j.tag, (uint32_t)sample, (uint32_t)(sample >> 32), a.key.k0,
                              a.key.k1);
            double z0, z1;
            normal_pair(r, &z0, &z1);
            s[2 * t] = j.sq[2 * t] * z0;
            if (2 * t + 1 < j.m) s[2 * t + 1] = j.sq[2 * t + 1] * z1;
        }
        __syncthreads();
        if (j.eout && u == 0) j.eout[ch] = 0.0 + j.bgc * s[j.split_g];
    }
    if (u >= j.nrows) return;
    const long long p = j.off[u];
    if (!j.noise) {
        j.f[p] = j.save[u];
        return;
    }
    double y;
    if (j.restore) {
        y = j.save[u];
    } else {
        y = j.f[p];
        j.save[u] = y;
    }
    j.f[p] = lr_row_patch(y, false, j.mask[u], j.coef + (long long)u * j.m, s, j.m, j.split_g, j.eout != nullptr);
}

// ---- dense-column path: one dense column g of B (the global average measurement) ----
// A dense column makes every row a row of B and of B_bar, and the row lists above then cost
// 8 (m + 2) bytes per vertex and launch.  But on every row where only column g of B (and of
// Y = (L + D/omega)^{-1} B) is nonzero -- all rows except a few dozen around each point
// measurement -- both are one number per vertex:
//   * patch  e_i = 0.0 + B_ig s_g                (the row's mask holds only bit g)
//   * B_bar  B_bar_ik = fma(Y_ig, Minv_gk, 0.0)   (the setup's fma chain over l, Y_il = 0 for l != g)
// so those "dense-only" rows stream B_g / Y_g over the padded store (coalesced; bit p of `skip`
// set = not a dense-only interior vertex) and only the remaining "local" rows keep the row lists
// -- the same arithmetic, bit for bit.  The patched right-hand side goes to a separate vector
// (out = f +/- e) which the level's sweep / residual reads: no saved copy, no restore.
// Batched chains: every thread loops over the chains (f, out, x cs apart), B_g / Y_g and the row
// lists are read once for all of them.
// threads per block, 16-byte pairs of the padded store per thread (L.nstore and every chain / column
// offset are multiples of 16 doubles), store entries per block
constexpr int LRD_NT = 256, LRD_PER = tune::LR_DENSE_PER, LRD_ELEMS = 2 * LRD_PER * LRD_NT;

// the pairs of one thread: p[r] (even) clamped into [0, n), ok[r][h] = a dense-only vertex p + h
__device__ __forceinline__ void lrd_pairs(const uint32_t* __restrict__ skip, long long n, int nbs, long long p[LRD_PER],
                                          bool ok[LRD_PER][2]) {
    const long long q0 = 2 * ((long long)((int)blockIdx.x - nbs) * (LRD_PER * LRD_NT) + threadIdx.x);
#pragma unroll
    for (int r = 0; r < LRD_PER; ++r) {
        const long long q = q0 + 2ll * r * LRD_NT;
        p[r] = q < n ? q : n - 2;
        const uint32_t w = skip[p[r] >> 5] >> (p[r] & 31);  // p even: both bits in one word
        ok[r][0] = q < n && !(w & 1);
        ok[r][1] = q < n && !(w & 2);
    }
}

struct LRDenseArgs {
    int m, g, mode, nch;      // mode: LR_PATCH_NOISE / RESIDUAL (out = f -/+ e) / APPLY (out == f, +=)
    long long cs;             // chain stride of f, out, x
    uint32_t chain0, seed_hi;
    RngKey key;
    uint32_t tag;
    const uint64_t* sample;
    const double* sq;         // noise: sqrt(1 / Sigma_k)
    const double* t;          // residual / apply: the m dots of every chain, m apart
    const double* f;
    double* out;
    double* out2;             // RESIDUAL with out2: also out2 = f + B Sigma^{-1/2} xi' of sweep tag2
    uint32_t tag2;            //   (the level's first post-sweep: f is not written in between)
    // local rows (blocks [0, nbs)): padded offsets, m coefficients, column masks
    int nrows, nbs;
    const long long* off;
    const double* coef;
    const uint64_t* mask;
    // dense-only rows (blocks [nbs, ...)): padded range [0, n)
    long long n;
    const uint32_t* skip;
    const double* bg;         // B_g over the padded store, or null: every B_g entry is bgc
    double bgc;
    int split_g;              // local rows: lr_row_patch's split column (-1: none, and LR_PATCH_APPLY)
};

// s[ch * m + k] = sq_k xi'_k of sweep `tag` for every chain (only k = g, g's pair, if !all)
__device__ __forceinline__ void lrd_noise(const LRDenseArgs& a, uint32_t tag, bool all, double* s) {
    const int m = a.m, np = (m + 1) / 2;
    const uint64_t sample = *a.sample;
    for (int q = threadIdx.x; q < a.nch * np; q += LRD_NT) {
        const int ch = q / np, pr = q - ch * np;
        if (!all && pr != a.g / 2) continue;  // dense-only rows need s_g alone
        const RngKey k = lr_chain_key(a.key, a.chain0, a.seed_hi, ch);
        const Philox4 r =
            philox4x32_10(LR_PAIR0 + (uint32_t)pr, tag, (uint32_t)sample, (uint32_t)(sample >> 32), k.k0, k.k1);
        double z0, z1;
        normal_pair(r, &z0, &z1);
        s[ch * m + 2 * pr] = a.sq[2 * pr] * z0;
        if (2 * pr + 1 < m) s[ch * m + 2 * pr + 1] = a.sq[2 * pr + 1] * z1;
    }
}

static __global__ void __launch_bounds__(LRD_NT) k_lr_dense_rhs(LRDenseArgs a) {
    __shared__ double s[LR_MAX_CH * LR_MAX_M];
    __shared__ double s2[LR_MAX_CH * LR_MAX_M];
    const bool local = (int)blockIdx.x < a.nbs;
    const int m = a.m;
    const bool two = a.out2 != nullptr;
    if (a.mode == LR_PATCH_NOISE) {
        lrd_noise(a, a.tag, local, s);
    } else {
        for (int q = threadIdx.x; q < a.nch * m; q += LRD_NT) s[q] = a.t[q];
        if (two) lrd_noise(a, a.tag2, local, s2);
    }
    __syncthreads();
    const bool minus = a.mode == LR_PATCH_RESIDUAL;
    if (local) {
        const int u = blockIdx.x * LRD_NT + threadIdx.x;
        if (u >= a.nrows) return;
        const long long p = a.off[u];
        const uint64_t msk = a.mask[u];
        const double* cf = a.coef + (long long)u * m;
        for (int ch = 0; ch < a.nch; ++ch) {
            const double y = a.f[ch * a.cs + p];
            a.out[ch * a.cs + p] = lr_row_patch(y, minus, msk, cf, s + ch * m, m, a.split_g, false);
            if (two) a.out2[ch * a.cs + p] = lr_row_patch(y, false, msk, cf, s2 + ch * m, m, a.split_g, false);
        }
        return;
    }
    // 16-byte pairs, every load unconditional (p clamped into the store), the stores masked
    long long p[LRD_PER];
    bool ok[LRD_PER][2];
    lrd_pairs(a.skip, a.n, a.nbs, p, ok);
    double2 bv[LRD_PER];
#pragma unroll
    for (int r = 0; r < LRD_PER; ++r) bv[r] = a.bg ? *(const double2*)(a.bg + p[r]) : make_double2(a.bgc, a.bgc);
    for (int ch = 0; ch < a.nch; ++ch) {
        const double sg = s[ch * m + a.g];
        const double* fc = a.f + ch * a.cs;
        double* oc = a.out + ch * a.cs;
        double2 y[LRD_PER];
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) y[r] = *(const double2*)(fc + p[r]);
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) {
            const double e0 = 0.0 + bv[r].x * sg, e1 = 0.0 + bv[r].y * sg;
            double2 o;
            o.x = minus ? y[r].x - e0 : y[r].x + e0;
            o.y = minus ? y[r].y - e1 : y[r].y + e1;
            if (ok[r][0] && ok[r][1]) *(double2*)(oc + p[r]) = o;
            else if (ok[r][0]) oc[p[r]] = o.x;
            else if (ok[r][1]) oc[p[r] + 1] = o.y;
        }
        if (two) {
            const double sg2 = s2[ch * m + a.g];
            double* o2c = a.out2 + ch * a.cs;
#pragma unroll
            for (int r = 0; r < LRD_PER; ++r) {
                double2 o;
                o.x = y[r].x + (0.0 + bv[r].x * sg2);
                o.y = y[r].y + (0.0 + bv[r].y * sg2);
                if (ok[r][0] && ok[r][1]) *(double2*)(o2c + p[r]) = o;
                else if (ok[r][0]) o2c[p[r]] = o.x;
                else if (ok[r][1]) o2c[p[r] + 1] = o.y;
            }
        }
    }
}

// smoother fix x -= B_bar w: local rows from the row list (blocks [0, nbs)), dense-only rows
// with B_bar_ik = fma(Y_ig, Minv_gk, 0.0) recomputed on the fly
struct LRDenseUpdateArgs {
    int m, g, nch;
    long long cs;
    const double* w;          // the m dots of every chain, m apart
    double* x;
    int nbar, nbs;
    const long long* bar_off;
    const double* bar_val;
    long long n;
    const uint32_t* skip;
    const double* yg;
    const uint8_t* ykey;      // non-null: Y_g = ytab[ykey[p]] (LowRankDev::ykey), yg is not read
    const double* ytab;
    const double* minv_g;     // row g of Minv
    // the restore of f on the rows of B (a right-hand side patched in place, LRRhsArg), with the
    // local blocks: f[rest_off[u]] = rest_val[u] for u < nrest (k_lr_update's)
    int nrest;
    const long long* rest_off;
    const double* rest_val;
    double* f;
};

static __global__ void __launch_bounds__(LRD_NT) k_lr_dense_update(LRDenseUpdateArgs a) {
    __shared__ double ws[LR_MAX_CH * LR_MAX_M];
    __shared__ double mg[LR_MAX_M];
    __shared__ double dt[LR_MAX_CH * 128];  // ykey: the fix of every key and chain, sum_k B_bar_ik w_k
    const int m = a.m;
    for (int q = threadIdx.x; q < a.nch * m; q += LRD_NT) ws[q] = a.w[q];
    for (int q = threadIdx.x; q < m; q += LRD_NT) mg[q] = a.minv_g[q];
    __syncthreads();
    if (a.ykey && (int)blockIdx.x >= a.nbs)
        // a dense-only row's fix depends on its Y_g (one of the table's values) and the chain alone:
        // the per-vertex loop below, computed once per key
        for (int q = threadIdx.x; q < a.nch * 128; q += LRD_NT) {
            const int ch = q >> 7;
            const double y = a.ytab[q & 127];
            double acc = 0.0;
            for (int k = 0; k < m; ++k) acc = fma(fma(y, mg[k], 0.0), ws[ch * m + k], acc);
            dt[q] = acc;
        }
    __syncthreads();
    if ((int)blockIdx.x < a.nbs) {
        const int u = blockIdx.x * LRD_NT + threadIdx.x;
        if (u < a.nbar) {
            const double* bv = a.bar_val + (long long)u * m;
            const long long p = a.bar_off[u];
            for (int ch = 0; ch < a.nch; ++ch) {
                double acc = 0.0;
                for (int k = 0; k < m; ++k) acc = fma(bv[k], ws[ch * m + k], acc);
                double* xc = a.x + ch * a.cs;
                xc[p] = xc[p] - acc;
            }
        }
        if (u < a.nrest)
            for (int ch = 0; ch < a.nch; ++ch) a.f[ch * a.cs + a.rest_off[u]] = a.rest_val[(long long)ch * a.nrest + u];
        return;
    }
    long long p[LRD_PER];
    bool ok[LRD_PER][2];
    lrd_pairs(a.skip, a.n, a.nbs, p, ok);
    if (a.ykey) {
        uint16_t kk[LRD_PER];
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) kk[r] = *(const uint16_t*)(a.ykey + p[r]);  // p even: both keys in one load
        for (int ch = 0; ch < a.nch; ++ch) {
            double* xc = a.x + ch * a.cs;
            const double* d = dt + ch * 128;
            double2 xv[LRD_PER];
#pragma unroll
            for (int r = 0; r < LRD_PER; ++r) xv[r] = *(const double2*)(xc + p[r]);
#pragma unroll
            for (int r = 0; r < LRD_PER; ++r) {
                double2 o;
                o.x = xv[r].x - d[kk[r] & 0xff];
                o.y = xv[r].y - d[kk[r] >> 8];
                if (ok[r][0] && ok[r][1]) *(double2*)(xc + p[r]) = o;
                else if (ok[r][0]) xc[p[r]] = o.x;
                else if (ok[r][1]) xc[p[r] + 1] = o.y;
            }
        }
        return;
    }
    double2 yv[LRD_PER];
    {
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) yv[r] = *(const double2*)(a.yg + p[r]);
    }
    for (int ch = 0; ch < a.nch; ++ch) {
        double* xc = a.x + ch * a.cs;
        double2 xv[LRD_PER];
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) xv[r] = *(const double2*)(xc + p[r]);
#pragma unroll
        for (int r = 0; r < LRD_PER; ++r) {
            double acc0 = 0.0, acc1 = 0.0;
            for (int k = 0; k < m; ++k) {
                const double wk = ws[ch * m + k], mk = mg[k];
                acc0 = fma(fma(yv[r].x, mk, 0.0), wk, acc0);
                acc1 = fma(fma(yv[r].y, mk, 0.0), wk, acc1);
            }
            double2 o;
            o.x = xv[r].x - acc0;
            o.y = xv[r].y - acc1;
            if (ok[r][0] && ok[r][1]) *(double2*)(xc + p[r]) = o;
            else if (ok[r][0]) xc[p[r]] = o.x;
            else if (ok[r][1]) xc[p[r] + 1] = o.y;
        }
    }
}

// ---- one workgroup for everything between two sweeps of a level with a small low-rank part ----
// (every column sparse with <= LR_BLK entries, few B_bar rows): the fix after a sweep, the restore
// of f, and the patch the next op of the level needs (noise of the next sweep, or the posterior
// residual's f - B Sigma^{-1} B^T x) -- one launch instead of up to six.  Same arithmetic as the
// separate kernels: the single-block dot is the block butterfly followed by the totals butterfly
// over (partial, 0, 0, ...).
enum { LR_NEXT_NONE = 0, LR_NEXT_NOISE = 1, LR_NEXT_RESIDUAL = 2 };

struct LRSmallArgs {
    int m;
    const LRColMeta* meta;
    const long long* ent_off;
    const double* ent_val;
    const double* sc_one;
    const double* sc_inv;
    const double* sq;
    double* x;  // state after the sweep
    int nbar;
    const long long* bar_off;
    const double* bar_val;
    int nrows;  // rows of B
    const long long* rows_off;
    const double* coef;
    const uint64_t* mask;
    double* save;
    double* f;
    int restore;  // f is noise-patched on the rows of B; save holds the true f
    int next;     // LR_NEXT_*
    RngKey key;
    uint32_t tag;  // sweep tag of the next sweep (LR_NEXT_NOISE)
    const uint64_t* sample;
    long long cs;               // batched chains: one workgroup per chain, x / f cs apart, save nrows apart
    uint32_t chain0, seed_hi;
};

__device__ __forceinline__ void lr_small_chain(LRSmallArgs& a) {
    const int ch = blockIdx.x;
    a.x += ch * a.cs;
    a.f += ch * a.cs;
    a.save += (long long)ch * a.nrows;
    a.key = lr_chain_key(a.key, a.chain0, a.seed_hi, ch);
}

__device__ __forceinline__ double lr_wave_dot(const LRColMeta& c, const long long* __restrict__ ent_off,
                                              const double* __restrict__ ent_val, double sc,
                                              const double* __restrict__ v, int lane) {
    // the lane's entries in order, U at a time with their loads issued together (a dense column of
    // a small level has up to 64 per lane: that many dependent round trips otherwise)
    constexpr int U = 8;
    double acc = 0.0;
    long long e = lane;
    for (; e + (U - 1) * 64 < c.n; e += U * 64) {
        long long o[U];
        double bv[U], xv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            o[u] = ent_off[c.ent0 + e + u * 64];
            bv[u] = ent_val[c.ent0 + e + u * 64];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) xv[u] = v[o[u]];
#pragma unroll
        for (int u = 0; u < U; ++u) acc = acc + (sc * bv[u]) * xv[u];
    }
    for (; e < c.n; e += 64) {
        const long long q = c.ent0 + e;
        acc = acc + (sc * ent_val[q]) * v[ent_off[q]];
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
    double tot = lane == 0 ? 0.0 + acc : 0.0;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) tot = tot + __shfl_xor(tot, off, 64);
    return tot;
}

static __global__ void __launch_bounds__(1024) k_lr_small(LRSmallArgs a) {
    lr_small_chain(a);
    __shared__ double ws[LR_MAX_M], ts[LR_MAX_M];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nwave = blockDim.x >> 6;
    // 1. w = B^T x
    for (int k = wave; k < a.m; k += nwave) {
        const double t = lr_wave_dot(a.meta[k], a.ent_off, a.ent_val, a.sc_one[k], a.x, lane);
        if (lane == 0) ws[k] = t;
    }
    __syncthreads();
    // 2. x -= B_bar w
    for (int u = tid; u < a.nbar; u += blockDim.x) {
        const double* bv = a.bar_val + (long long)u * a.m;
        double acc = 0.0;
        for (int k = 0; k < a.m; ++k) acc = fma(bv[k], ws[k], acc);
        const long long p = a.bar_off[u];
        a.x[p] = a.x[p] - acc;
    }
    // 3. the next op's vector: Sigma^{-1} B^T x of the fixed state, or the next sweep's noise
    if (a.next == LR_NEXT_RESIDUAL) {
        __syncthreads();  // the fixed x rows of other waves
        for (int k = wave; k < a.m; k += nwave) {
            const double t = lr_wave_dot(a.meta[k], a.ent_off, a.ent_val, a.sc_inv[k], a.x, lane);
            if (lane == 0) ts[k] = t;
        }
    } else if (a.next == LR_NEXT_NOISE && 2 * tid < a.m) {
        const uint64_t sample = *a.sample;
        const Philox4 r = philox4x32_10(LR_PAIR0 + (uint32_t)tid, a.tag, (uint32_t)sample, (uint32_t)(sample >> 32),
                                        a.key.k0, a.key.k1);
        double z0, z1;
        normal_pair(r, &z0, &z1);
        ts[2 * tid] = a.sq[2 * tid] * z0;
        if (2 * tid + 1 < a.m) ts[2 * tid + 1] = a.sq[2 * tid + 1] * z1;
    }
    __syncthreads();
    // 4. f on the rows of B: restore and / or patch
    for (int u = tid; u < a.nrows; u += blockDim.x) {
        const long long p = a.rows_off[u];
        const double base = a.restore ? a.save[u] : a.f[p];
        if (a.next == LR_NEXT_NONE) {
            if (a.restore) a.f[p] = base;
            continue;
        }
        const uint64_t msk = a.mask[u];
        const double* cf = a.coef + (long long)u * a.m;
        double e = 0.0;
        for (int k = 0; k < a.m; ++k)
            if ((msk >> k) & 1) e = e + cf[k] * ts[k];
        if (!a.restore) a.save[u] = base;
        a.f[p] = a.next == LR_NEXT_NOISE ? base + e : base - e;
    }
}

// ---- k_lr_small with its independent loads issued up front ----
// k_lr_small is a chain of dependent global round trips (column metadata -> entries -> x, then
// B_bar rows, the second dot's metadata and entries, the rows of B), each ~1 us.  When every column
// has <= 64 entries (one per lane), m <= M and each thread owns <= PR rows of B_bar and of B, all of
// those loads do not depend on anything this kernel writes and go first; what is left is entries ->
// x, the fix's read-modify-write of x, (the residual's second read of x), the write of f.  Same
// arithmetic: one entry per lane is the lane sum 0.0 + (sc B_ek) x_e, the fix is the fma chain over
// k ascending, the patch the masked mul+add chain.
template <int M, int PR>
__global__ void __launch_bounds__(1024) k_lr_small_pf(LRSmallArgs a) {
    lr_small_chain(a);
    __shared__ double ws[LR_MAX_M], ts[LR_MAX_M];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nt = blockDim.x;
    const int m = a.m;
    // 0. independent loads
    long long eoff = 0;
    double evs = 0.0, evi = 0.0;
    bool have_e = false;
    if (wave < m) {
        const LRColMeta c = a.meta[wave];
        if (lane < c.n) {
            const long long q = c.ent0 + lane;
            const double v = a.ent_val[q];
            eoff = a.ent_off[q];
            evs = a.sc_one[wave] * v;
            evi = a.sc_inv[wave] * v;
            have_e = true;
        }
    }
    double bv[PR][M];
    long long boff[PR];
    double cf[PR][M];
    uint64_t msk[PR];
    long long roff[PR];
    double base[PR];
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        const int u = tid + r * nt;
        boff[r] = 0;
        roff[r] = 0;
        msk[r] = 0;
        base[r] = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) bv[r][k] = cf[r][k] = 0.0;
        if (u < a.nbar) {
            boff[r] = a.bar_off[u];
#pragma unroll
            for (int k = 0; k < M; ++k)
                if (k < m) bv[r][k] = a.bar_val[(long long)u * m + k];
        }
        if (u < a.nrows) {
            roff[r] = a.rows_off[u];
            msk[r] = a.mask[u];
#pragma unroll
            for (int k = 0; k < M; ++k)
                if (k < m) cf[r][k] = a.coef[(long long)u * m + k];
            base[r] = a.restore ? a.save[u] : a.f[roff[r]];
        }
    }
    auto wave_total = [&](double acc) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
        double tot = lane == 0 ? 0.0 + acc : 0.0;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) tot = tot + __shfl_xor(tot, off, 64);
        return tot;
    };
    // 1. w = B^T x
    if (wave < m) {
        const double acc = have_e ? 0.0 + evs * a.x[eoff] : 0.0;
        const double t = wave_total(acc);
        if (lane == 0) ws[wave] = t;
    }
    __syncthreads();
    // 2. x -= B_bar w
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        const int u = tid + r * nt;
        if (u < a.nbar) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < M; ++k)
                if (k < m) acc = fma(bv[r][k], ws[k], acc);
            a.x[boff[r]] = a.x[boff[r]] - acc;
        }
    }
    // 3. the next op's vector
    if (a.next == LR_NEXT_RESIDUAL) {
        __syncthreads();
        if (wave < m) {
            const double acc = have_e ? 0.0 + evi * a.x[eoff] : 0.0;
            const double t = wave_total(acc);
            if (lane == 0) ts[wave] = t;
        }
    } else if (a.next == LR_NEXT_NOISE && 2 * tid < m) {
        const uint64_t sample = *a.sample;
        const Philox4 rr = philox4x32_10(LR_PAIR0 + (uint32_t)tid, a.tag, (uint32_t)sample, (uint32_t)(sample >> 32),
                                         a.key.k0, a.key.k1);
        double z0, z1;
        normal_pair(rr, &z0, &z1);
        ts[2 * tid] = a.sq[2 * tid] * z0;
        if (2 * tid + 1 < m) ts[2 * tid + 1] = a.sq[2 * tid + 1] * z1;
    }
    __syncthreads();
    // 4. f on the rows of B
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        const int u = tid + r * nt;
        if (u >= a.nrows) continue;
        if (a.next == LR_NEXT_NONE) {
            if (a.restore) a.f[roff[r]] = base[r];
            continue;
        }
        double e = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k)
            if (k < m && ((msk[r] >> k) & 1)) e = e + cf[r][k] * ts[k];
        if (!a.restore) a.save[u] = base[r];
        a.f[roff[r]] = a.next == LR_NEXT_NOISE ? base[r] + e : base[r] - e;
    }
}

// ============================================================================================
// host side: the same orders, for the B_bar setup (M = Sigma + B^T Y needs the dots of Y)
// ============================================================================================
struct LRColumn {
    std::vector<std::pair<long long, double>> ent;  // (row in reference order, value), rows ascending
    bool dense = false;
};

inline double lr_butterfly64_host(double* v) {
    for (int off = 32; off >= 1; off >>= 1) {
        double t[64];
        for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
        std::copy(t, t + 64, v);
    }
    return v[0];
}

// sum_e (sc B_ek) v_e in the device order (v in reference order)
inline double lr_dot_host(const LRColumn& col, double sc, const double* v) {
    const long long n = (long long)col.ent.size();
    const long long nblk = (n + LR_BLK - 1) / LR_BLK;
    std::vector<double> part((size_t)nblk);
    double acc[64];
    for (long long b = 0; b < nblk; ++b) {
        const long long end = std::min(n, (b + 1) * LR_BLK);
        for (int l = 0; l < 64; ++l) {
            acc[l] = 0.0;
            for (long long e = b * LR_BLK + l; e < end; e += 64)
                acc[l] = acc[l] + (sc * col.ent[e].second) * v[col.ent[e].first];
        }
        part[b] = lr_butterfly64_host(acc);
    }
    for (int l = 0; l < 64; ++l) {
        acc[l] = 0.0;
        for (long long b = l; b < nblk; b += 64) acc[l] = acc[l] + part[b];
    }
    return lr_butterfly64_host(acc);
}

// inverse of a small dense row-major m x m matrix: Gauss-Jordan with partial pivoting (the
// oracle's small_inverse, operation for operation); returns false if singular
inline bool lr_small_inverse(std::vector<double> M, int m, std::vector<double>& I) {
    I.assign((size_t)m * m, 0.0);
    for (int i = 0; i < m; ++i) I[(size_t)i * m + i] = 1.0;
    for (int c = 0; c < m; ++c) {
        int piv = c;
        for (int r = c + 1; r < m; ++r)
            if (std::fabs(M[(size_t)r * m + c]) > std::fabs(M[(size_t)piv * m + c])) piv = r;
        if (piv != c)
            for (int q = 0; q < m; ++q) {
                std::swap(M[(size_t)c * m + q], M[(size_t)piv * m + q]);
                std::swap(I[(size_t)c * m + q], I[(size_t)piv * m + q]);
            }
        const double d = M[(size_t)c * m + c];
        if (d == 0.0 || !std::isfinite(d)) return false;
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
    return true;
}

}  // namespace mgmc
