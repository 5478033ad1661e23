// mgmc_zsweep.hpp -- z-marching fused red-black Gibbs sweep of the fine 3D 7-point level.
//
// One launch = one full SOR Gibbs sweep (both colours) = SORSampler::apply with nsmooth = 1
// (sampler/sor_sampler.cc:37-59) in red-black order.  The colour-pass kernels of
// mgmc_kernels.hpp read x and f twice per sweep (48 B/unknown of HBM traffic); this kernel reads
// x and f once and writes x once (24 B/unknown, the algorithmic minimum):
//
//  * Out of place: every new value is a pure function of (x_in, f, Philox counter), so tiles are
//    independent and may recompute each other's halo; x_out never aliases x_in.
//  * Each workgroup owns a tile of XP x-pairs x TY rows and marches a z-chunk.  At step p it
//    updates the first colour on plane p (over the tile plus a one-vertex halo, recomputed) and
//    the second colour on plane p-1 (tile only), which then is final and is stored.  A red update
//    on plane p only reads black values of planes p-1..p+1 (still old), a black update on p-1 only
//    reads red values of planes p-2..p (already new): this is exactly the two-pass result.
//  * Planes live in an LDS ring (4 slots of x, 2 of f); global traffic is 16-byte pair loads and
//    stores, one pass over x_in, f and x_out (+ halo re-reads that hit L2 / Infinity Cache).
//  * The two vertices of an x-pair share one Philox block: the first-colour update consumes one
//    Box-Muller branch and parks the other in LDS for the second-colour update one step later.
//  * Optional fused prolongate-add on the input: x_old = x_in + alpha P x_c, evaluated exactly as
//    k_prolongate_add (so the post-sampler needs no separate prolongation pass).
// Per-vertex arithmetic is the reference's (see mgmc_kernels.hpp); results are bitwise equal to
// the two colour passes.
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

struct ZSweepArgs {
    Layout L;                  // fine level
    const double* xin;
    double* xout;
    const double* f;
    const double* xc;          // coarse correction (PROLONG only)
    Layout Lc;
    double alpha;
    StencilArg S;
    GibbsArg G;                // colour field = first colour (0 forward, 1 backward)
    int tz;                    // planes per z-chunk
    int ntx, nty, ntz;         // tile counts
};

// prolongate-add gather of one fine vertex (identical arithmetic to k_prolongate_add)
__device__ __forceinline__ double prolong_gather(double v, const double* __restrict__ xc, const Layout& Lc, int i,
                                                 int j, int k, double alpha) {
    const int i0 = i >> 1, j0 = j >> 1, k0 = k >> 1;
    const int ni = (i & 1) ? 2 : 1, nj = (j & 1) ? 2 : 1, nk = (k & 1) ? 2 : 1;
    for (int a = 0; a < nk; ++a) {
        const int kk = k0 + a;
        if (kk < 1 || kk > Lc.nz - 1) continue;
        for (int b = 0; b < nj; ++b) {
            const int jj = j0 + b;
            if (jj < 1 || jj > Lc.ny - 1) continue;
            for (int c = 0; c < ni; ++c) {
                const int ii = i0 + c;
                if (ii < 1 || ii > Lc.nx - 1) continue;
                double w = 1.0;
                w *= w1(i - 2 * ii);
                w *= w1(j - 2 * jj);
                w *= w1(k - 2 * kk);
                v += alpha * w * xc[Lc.at(ii, jj, kk)];
            }
        }
    }
    return v;
}

template <int XP, int TY, int NT, bool PROLONG>
__global__ void __launch_bounds__(NT) k_zsweep_rb7(ZSweepArgs a) {
    constexpr int W = 2 * XP + 8;  // LDS columns: positions [2*q0-3, 2*q0+2*XP+4]
    constexpr int WP = W / 2;      // pairs per LDS row
    constexpr int R = TY + 4;      // rows j0-2 .. j0+TY+1
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                   // [4][R][W]
    double* fs = xs + 4 * R * W;         // [2][R][W]   (rows j0-2 .. j0+TY+1, only R_1 used)
    double* ns = fs + 2 * R * W;         // [2][TY][XP] parked second-colour normals

    const Layout& L = a.L;
    // XCD-aware tile order: blocks b and b+8 share an XCD, give them neighbouring tiles
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);
    const int txi = tile % a.ntx;
    const int tyi = (tile / a.ntx) % a.nty;
    const int tzi = tile / (a.ntx * a.nty);
    if (tzi >= a.ntz) return;
    const int q0 = txi * XP;          // first core pair; core positions 2q0+1 .. 2q0+2XP
    const int j0 = 1 + tyi * TY;      // first core row
    const int k0 = 1 + tzi * a.tz;    // first core plane
    const int k1 = min(k0 + a.tz, L.nz);  // one past the last core plane
    const int ibase = 2 * q0 - 3;     // position of LDS column 0
    const int fc = a.G.colour;        // first colour
    const double omega = a.G.omega, sd = a.G.sd;
    const double diag = a.S.a[13];
    const uint64_t sample = *a.G.sample;
    const int tid = threadIdx.x;

    auto slot = [](int p) { return (p + 8) & 3; };
    auto interior_row = [&](int j) { return j >= 1 && j <= L.ny - 1; };
    auto interior_plane = [&](int k) { return k >= 1 && k <= L.nz - 1; };

    // load plane k of x_in (rows j0-2..j0+TY+1, all LDS columns) into slot(k)
    auto load_x = [&](int k) {
        double* dst = xs + slot(k) * R * W;
        for (int it = tid; it < R * WP; it += NT) {
            const int r = it / WP, c2 = it - r * WP;
            const int j = j0 - 2 + r;
            const int i = ibase + 2 * c2;
            double2 v = make_double2(0.0, 0.0);
            if (interior_plane(k) && interior_row(j)) {
                v = *reinterpret_cast<const double2*>(a.xin + L.at(i, j, k));
                if (PROLONG) {
                    if (i >= 1 && i <= L.nx - 1) v.x = prolong_gather(v.x, a.xc, a.Lc, i, j, k, a.alpha);
                    if (i + 1 >= 1 && i + 1 <= L.nx - 1) v.y = prolong_gather(v.y, a.xc, a.Lc, i + 1, j, k, a.alpha);
                }
            }
            *reinterpret_cast<double2*>(dst + r * W + 2 * c2) = v;
        }
    };
    auto load_f = [&](int k) {
        double* dst = fs + (k & 1) * R * W;
        for (int it = tid; it < (R - 2) * WP; it += NT) {
            const int r = 1 + it / WP, c2 = it % WP;
            const int j = j0 - 2 + r;
            const int i = ibase + 2 * c2;
            double2 v = make_double2(0.0, 0.0);
            if (interior_plane(k) && interior_row(j)) v = *reinterpret_cast<const double2*>(a.f + L.at(i, j, k));
            *reinterpret_cast<double2*>(dst + r * W + 2 * c2) = v;
        }
    };
    auto store_x = [&](int k) {
        if (k < k0 || k >= k1) return;
        const double* src = xs + slot(k) * R * W;
        for (int it = tid; it < TY * XP; it += NT) {
            const int r = 2 + it / XP, c2 = 2 + it % XP;
            const int j = j0 - 2 + r;
            if (!interior_row(j)) continue;
            const int i = ibase + 2 * c2;
            *reinterpret_cast<double2*>(a.xout + L.at(i, j, k)) = *reinterpret_cast<const double2*>(src + r * W + 2 * c2);
        }
    };
    // ascending-column-order stencil sum at LDS (r, c) of plane k
    auto row_sum = [&](int k, int r, int c) {
        const double* sm = xs + slot(k - 1) * R * W;
        const double* s0 = xs + slot(k) * R * W;
        const double* sp = xs + slot(k + 1) * R * W;
        double res = 0.0;
        res += a.S.a[4] * sm[r * W + c];
        res += a.S.a[10] * s0[(r - 1) * W + c];
        res += a.S.a[12] * s0[r * W + c - 1];
        res += a.S.a[13] * s0[r * W + c];
        res += a.S.a[14] * s0[r * W + c + 1];
        res += a.S.a[16] * s0[(r + 1) * W + c];
        res += a.S.a[22] * sp[r * W + c];
        return res;
    };

    // first-colour update on plane k over rows R_1 and pairs [1, WP-1)
    auto first_colour = [&](int k) {
        if (!interior_plane(k)) return;
        double* s0 = xs + slot(k) * R * W;
        const double* fk = fs + (k & 1) * R * W;
        double* park = ns + (k & 1) * TY * XP;
        const uint64_t rowbase = (uint64_t)(k - 1) * (uint64_t)(L.ny - 1);
        for (int it = tid; it < (R - 2) * (WP - 2); it += NT) {
            const int r = 1 + it / (WP - 2), c2 = 1 + it % (WP - 2);
            const int j = j0 - 2 + r;
            if (!interior_row(j)) continue;
            const int i = ibase + 2 * c2;  // odd position: pair (i, i+1)
            const int e = ((i + j + k) & 1) == fc ? 0 : 1;  // element of the first colour
            const int ie = i + e;
            const bool in0 = i >= 1 && i <= L.nx - 1, in1 = i + 1 >= 1 && i + 1 <= L.nx - 1;
            if (!in0 && !in1) continue;
            const uint32_t pair = (uint32_t)((rowbase + (uint64_t)(j - 1)) * (uint64_t)(L.nx / 2) + (uint64_t)((i - 1) >> 1));
            const Philox4 rnd = philox4x32_10(pair, a.G.tag, (uint32_t)sample, (uint32_t)(sample >> 32), a.G.key.k0, a.G.key.k1);
            double z0, z1;
            normal_pair(rnd, &z0, &z1);  // z0: odd position i, z1: even position i+1
            const bool core = r >= 2 && r < 2 + TY && c2 >= 2 && c2 < 2 + XP;
            if (core) park[(r - 2) * XP + (c2 - 2)] = e == 0 ? z1 : z0;
            if (ie < 1 || ie > L.nx - 1) continue;
            const int c = 2 * c2 + e;
            const double res = row_sum(k, r, c);
            const double cr = sd * (e == 0 ? z0 : z1) + fk[r * W + c];
            s0[r * W + c] += omega * (cr - res) / diag;
        }
    };
    // second-colour update on plane k over the core tile
    auto second_colour = [&](int k) {
        if (!interior_plane(k) || k < k0 || k >= k1) return;
        double* s0 = xs + slot(k) * R * W;
        const double* fk = fs + (k & 1) * R * W;
        const double* park = ns + (k & 1) * TY * XP;
        for (int it = tid; it < TY * XP; it += NT) {
            const int r = 2 + it / XP, c2 = 2 + it % XP;
            const int j = j0 - 2 + r;
            if (!interior_row(j)) continue;
            const int i = ibase + 2 * c2;
            const int e = ((i + j + k) & 1) == fc ? 1 : 0;  // element of the second colour
            const int ie = i + e;
            if (ie < 1 || ie > L.nx - 1) continue;
            const int c = 2 * c2 + e;
            const double res = row_sum(k, r, c);
            const double cr = sd * park[(r - 2) * XP + (c2 - 2)] + fk[r * W + c];
            s0[r * W + c] += omega * (cr - res) / diag;
        }
    };

    load_x(k0 - 2);
    load_x(k0 - 1);
    for (int p = k0 - 1; p <= k1; ++p) {
        store_x(p - 2);
        load_x(p + 1);
        load_f(p);
        __syncthreads();
        first_colour(p);
        __syncthreads();
        second_colour(p - 1);
        __syncthreads();
    }
    store_x(k1 - 1);
}

inline size_t zsweep_lds_bytes(int XP, int TY) {
    const int W = 2 * XP + 8, R = TY + 4;
    return (size_t)(4 * R * W + 2 * R * W + 2 * TY * XP) * sizeof(double);
}

}  // namespace mgmc
