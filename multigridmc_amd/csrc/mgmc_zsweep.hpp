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
// Per-vertex arithmetic is that of mgmc_kernels.hpp (fused Gibbs update); results are bitwise
// equal to the two colour passes.
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
    constexpr int NCORE = TY * XP;                 // core pairs (both colours)
    constexpr int NHALO = 2 * (XP + 2) + 2 * TY;   // first-colour halo ring pairs
    static_assert(NCORE % NT == 0, "core pairs must divide evenly over the workgroup");
    constexpr int NC = NCORE / NT;                 // core pairs per thread
    constexpr int NH = (NHALO + NT - 1) / NT;      // halo pairs per thread
    constexpr int NLX = (R * WP + NT - 1) / NT;    // pair loads of one x plane per thread
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                 // [4][R][W] ring of x planes (p-2 .. p+1)
    double* tab = xs + 4 * R * W;      // [3][64] log reduction table (rc, hi, lo)
    for (int q = threadIdx.x; q < 64; q += NT) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }

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
    const int q0 = txi * XP;              // first core pair; core positions 2q0+1 .. 2q0+2XP
    const int j0 = 1 + tyi * TY;          // first core row
    const int k0 = 1 + tzi * a.tz;        // first core plane
    const int k1 = min(k0 + a.tz, L.nz);  // one past the last core plane
    const int ibase = 2 * q0 - 3;         // position of LDS column 0
    const int fc = a.G.colour;            // first colour
    const double sd = a.G.sd, wd = a.G.wd;
    const uint64_t sample = *a.G.sample;
    const int tid = threadIdx.x;

    auto slot = [](int p) { return (p + 8) & 3; };
    auto interior_row = [&](int j) { return j >= 1 && j <= L.ny - 1; };
    auto interior_plane = [&](int k) { return k >= 1 && k <= L.nz - 1; };

    // item -> (LDS row r, LDS pair column c2)
    int cr[NC], cc[NC];
#pragma unroll
    for (int u = 0; u < NC; ++u) {
        const int it = tid + u * NT;
        cr[u] = 2 + it / XP;
        cc[u] = 2 + it % XP;
    }
    int hr[NH], hc[NH];
#pragma unroll
    for (int u = 0; u < NH; ++u) {
        int it = tid + u * NT;
        if (it >= NHALO) { hr[u] = -1; hc[u] = 0; continue; }
        if (it < XP + 2) { hr[u] = 1; hc[u] = 1 + it; continue; }
        it -= XP + 2;
        if (it < XP + 2) { hr[u] = R - 2; hc[u] = 1 + it; continue; }
        it -= XP + 2;
        hr[u] = 2 + (it >> 1);
        hc[u] = (it & 1) ? WP - 2 : 1;
    }

    // ---- global <-> LDS / registers ----
    double2 px[NLX];
    auto issue_x = [&](int k) {
#pragma unroll
        for (int u = 0; u < NLX; ++u) {
            const int it = tid + u * NT;
            px[u] = make_double2(0.0, 0.0);
            if (it < R * WP) {
                const int r = it / WP, c2 = it - r * WP;
                const int j = j0 - 2 + r;
                if (interior_plane(k) && interior_row(j))
                    px[u] = *reinterpret_cast<const double2*>(a.xin + L.at(ibase + 2 * c2, j, k));
            }
        }
    };
    auto deposit_x = [&](int k) {
        double* dst = xs + slot(k) * R * W;
#pragma unroll
        for (int u = 0; u < NLX; ++u) {
            const int it = tid + u * NT;
            if (it < R * WP) {
                const int r = it / WP, c2 = it - r * WP;
                double2 v = px[u];
                if (PROLONG && interior_plane(k)) {
                    const int j = j0 - 2 + r, i = ibase + 2 * c2;
                    if (interior_row(j)) {
                        if (i >= 1 && i <= L.nx - 1) v.x = prolong_gather(v.x, a.xc, a.Lc, i, j, k, a.alpha);
                        if (i + 1 >= 1 && i + 1 <= L.nx - 1) v.y = prolong_gather(v.y, a.xc, a.Lc, i + 1, j, k, a.alpha);
                    }
                }
                *reinterpret_cast<double2*>(dst + r * W + 2 * c2) = v;
            }
        }
    };
    auto store_x = [&](int k) {
        if (k < k0 || k >= k1) return;
        const double* src = xs + slot(k) * R * W;
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            const int j = j0 - 2 + cr[u];
            if (!interior_row(j)) continue;
            *reinterpret_cast<double2*>(a.xout + L.at(ibase + 2 * cc[u], j, k)) =
                *reinterpret_cast<const double2*>(src + cr[u] * W + 2 * cc[u]);
        }
    };
    // f pairs of the core items (used by both colours) and f of the halo items
    auto load_fcore = [&](int k, double2* out) {
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            const int j = j0 - 2 + cr[u];
            out[u] = make_double2(0.0, 0.0);
            if (interior_plane(k) && interior_row(j))
                out[u] = *reinterpret_cast<const double2*>(a.f + L.at(ibase + 2 * cc[u], j, k));
        }
    };
    auto load_fhalo = [&](int k, double2* out) {
#pragma unroll
        for (int u = 0; u < NH; ++u) {
            out[u] = make_double2(0.0, 0.0);
            if (hr[u] < 0) continue;
            const int j = j0 - 2 + hr[u];
            if (interior_plane(k) && interior_row(j))
                out[u] = *reinterpret_cast<const double2*>(a.f + L.at(ibase + 2 * hc[u], j, k));
        }
    };

    // ascending-column-order stencil sum at LDS (r, c) of plane k
    auto row_sum = [&](int k, int r, int c) {
        const double* sm = xs + slot(k - 1) * R * W;
        const double* s0 = xs + slot(k) * R * W;
        const double* sp = xs + slot(k + 1) * R * W;
        double res = a.S.a[4] * sm[r * W + c];
        res = fma(a.S.a[10], s0[(r - 1) * W + c], res);
        res = fma(a.S.a[12], s0[r * W + c - 1], res);
        res = fma(a.S.a[13], s0[r * W + c], res);
        res = fma(a.S.a[14], s0[r * W + c + 1], res);
        res = fma(a.S.a[16], s0[(r + 1) * W + c], res);
        res = fma(a.S.a[22], sp[r * W + c], res);
        return res;
    };
    // first-colour update of the pair at LDS (r, c2) on plane k; returns the other normal
    auto first_pair = [&](int k, int r, int c2, double2 fv) -> double {
        const int j = j0 - 2 + r;
        if (!interior_row(j)) return 0.0;
        const int i = ibase + 2 * c2;  // odd position: pair (i, i+1)
        const int e = ((i + j + k) & 1) == fc ? 0 : 1;
        const bool in0 = i >= 1 && i <= L.nx - 1, in1 = i + 1 >= 1 && i + 1 <= L.nx - 1;
        if (!in0 && !in1) return 0.0;
        const uint32_t pair = (uint32_t)(((uint64_t)(k - 1) * (uint64_t)(L.ny - 1) + (uint64_t)(j - 1)) *
                                             (uint64_t)(L.nx / 2) + (uint64_t)((i - 1) >> 1));
        const Philox4 rnd = philox4x32_10(pair, a.G.tag, (uint32_t)sample, (uint32_t)(sample >> 32), a.G.key.k0,
                                          a.G.key.k1);
        double z0, z1;
        normal_pair_t(rnd, &z0, &z1, tab, tab + 64, tab + 128);  // z0: odd position i, z1: even i+1
        if ((e == 0 && in0) || (e == 1 && in1)) {
            const int c = 2 * c2 + e;
            const double res = row_sum(k, r, c);
            const double crhs = fma(sd, e == 0 ? z0 : z1, e == 0 ? fv.x : fv.y);
            double* s0 = xs + slot(k) * R * W;
            s0[r * W + c] = fma(wd, crhs - res, s0[r * W + c]);
        }
        return e == 0 ? z1 : z0;
    };
    auto second_pair = [&](int k, int r, int c2, double2 fv, double z) {
        const int j = j0 - 2 + r;
        if (!interior_row(j)) return;
        const int i = ibase + 2 * c2;
        const int e = ((i + j + k) & 1) == fc ? 1 : 0;
        const int ie = i + e;
        if (ie < 1 || ie > L.nx - 1) return;
        const int c = 2 * c2 + e;
        const double res = row_sum(k, r, c);
        const double crhs = fma(sd, z, e == 0 ? fv.x : fv.y);
        double* s0 = xs + slot(k) * R * W;
        s0[r * W + c] = fma(wd, crhs - res, s0[r * W + c]);
    };

    // register pipeline: f(p) core pairs are loaded at step p-1 and used at steps p (first colour)
    // and p+1 (second colour); x(p+2) is loaded at step p and deposited at step p+1.
    double2 fnext[NC], fcur[NC], fprev[NC], fh_next[NH], fh_cur[NH];
    double zpark_new[NC], zpark_old[NC];
#pragma unroll
    for (int u = 0; u < NC; ++u) {
        fcur[u] = fprev[u] = make_double2(0.0, 0.0);
        zpark_new[u] = zpark_old[u] = 0.0;
    }
    // prologue: planes k0-2, k0-1 in LDS, x(k0) and f(k0-1) in flight
    {
        const int kk[2] = {k0 - 2, k0 - 1};
        for (int q = 0; q < 2; ++q) {
            issue_x(kk[q]);
            deposit_x(kk[q]);
        }
    }
    issue_x(k0);
    load_fcore(k0 - 1, fnext);
    load_fhalo(k0 - 1, fh_next);
    for (int p = k0 - 1; p <= k1; ++p) {
        deposit_x(p + 1);
#pragma unroll
        for (int u = 0; u < NC; ++u) {
            fprev[u] = fcur[u];
            fcur[u] = fnext[u];
            zpark_old[u] = zpark_new[u];
        }
#pragma unroll
        for (int u = 0; u < NH; ++u) fh_cur[u] = fh_next[u];
        store_x(p - 2);
        issue_x(p + 2);
        load_fcore(p + 1, fnext);
        load_fhalo(p + 1, fh_next);
        __syncthreads();
        if (interior_plane(p)) {
#pragma unroll
            for (int u = 0; u < NC; ++u) zpark_new[u] = first_pair(p, cr[u], cc[u], fcur[u]);
#pragma unroll
            for (int u = 0; u < NH; ++u)
                if (hr[u] >= 0) (void)first_pair(p, hr[u], hc[u], fh_cur[u]);
        }
        __syncthreads();
        if (p - 1 >= k0 && interior_plane(p - 1)) {
#pragma unroll
            for (int u = 0; u < NC; ++u) second_pair(p - 1, cr[u], cc[u], fprev[u], zpark_old[u]);
        }
        __syncthreads();
    }
    store_x(k1 - 1);
}

inline size_t zsweep_lds_bytes(int XP, int TY) {
    const int W = 2 * XP + 8, R = TY + 4;
    return (size_t)(4 * R * W + 3 * 64) * sizeof(double);
}

}  // namespace mgmc
