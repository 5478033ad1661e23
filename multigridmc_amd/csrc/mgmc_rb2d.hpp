// mgmc_rb2d.hpp -- one launch per red-black Gibbs sweep of a 2D 5-point (FD) level.
//
// sampler/sor_sampler.cc:37-59 + smoother/sor_smoother.cc:56-78 under the red-black splitting: the
// first colour is updated from the old second colour, then the second from the new first.  The 2D
// fine level (1023^2 unknowns at BASELINE config 2) is launch-bound: two colour passes of ~6.5 us.
// Here a workgroup stages a 128 x 16 tile of the old state with a 2-vertex halo in LDS, updates the
// first colour on the tile plus a 1-vertex ring (the ring's values are the neighbouring tiles' own
// results: same inputs, same arithmetic), then the second colour on the tile, and writes the tile to
// the other buffer (out of place: neighbouring workgroups still read the old values).  Each update is
// gibbs_point's arithmetic: c = fma(sd, xi, f) with xi the cos / sin branch of the Philox pair
// (odd i, i+1) of the sweep's tag, x = fma(omega/diag, c - S, x), S the stencil fma chain.
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

constexpr int RB2_TW = 128, RB2_TH = 16;                 // tile columns, rows
constexpr int RB2_W = RB2_TW + 4, RB2_H = RB2_TH + 4;    // staged region: 2-vertex halo
constexpr int RB2_NT = 1024;                            // threads: about one item per thread per phase
constexpr int RB2_HW = RB2_W / 2;                       // LDS rows are colour-split: [even c | odd c]

// LDS index of region row r, column c: the vertices of one colour in a row are consecutive doubles,
// so a colour pass reads without bank conflicts (the natural layout's stride 2 was 44% conflict
// cycles, PMC)
__device__ __forceinline__ int rb2_lidx(int r, int c) { return r * RB2_W + (c & 1) * RB2_HW + (c >> 1); }

template <bool NOISE>
__global__ void __launch_bounds__(RB2_NT) k_rb2d(Layout L, const double* __restrict__ xin, double* __restrict__ xout,
                                              const double* __restrict__ f, StencilArg S, GibbsArg G, int c1,
                                              int ntx, long long chs) {
    {  // batched chains (blockIdx.z)
        const int ch = batch_chain();
        xin += ch * chs;
        xout += ch * chs;
        f += ch * chs;
        G.key = chain_key(G, ch);
    }
    __shared__ double xs[RB2_H * RB2_W];
    __shared__ double cs[RB2_H * RB2_W];  // right hand sides c = fma(sd, xi, f) of the updated vertices
    const int tid = threadIdx.x;
    const int tx = (int)blockIdx.x % ntx, ty = (int)blockIdx.x / ntx;
    const int i0 = 1 + tx * RB2_TW, j0 = 1 + ty * RB2_TH;
    const int ib = i0 - 2, jb = j0 - 2;  // lattice coordinates of LDS (0, 0)
    const uint64_t sample = NOISE ? *G.sample : 0;
    // all global loads of the workgroup first (the old state with its 2-vertex halo, f of the
    // updated vertices), then the Box-Muller draws while they are in flight, then the LDS deposits
    // -- the draws no longer wait behind the loads (same values, same arithmetic)
    constexpr int NSX = (RB2_H * RB2_W + RB2_NT - 1) / RB2_NT;
    double xv[NSX];
#pragma unroll
    for (int u = 0; u < NSX; ++u) {
        const int q = tid + u * RB2_NT;
        const int r = q / RB2_W, c = q - r * RB2_W;
        const int i = ib + c, j = jb + r;
        xv[u] = (q < RB2_H * RB2_W && i >= 0 && i <= L.nx && j >= 0 && j <= L.ny) ? xin[L.at(i, j, 0)] : 0.0;
    }
    // right hand sides of every vertex the two passes update (rows [j0-1, j0+TH], columns [i0-1,
    // i0+TW]): f does not change during the sweep, so they are evaluated up front, one Box-Muller per
    // pair (odd i, i+1) -- the values point_normal gives each vertex
    constexpr int NP = RB2_TW / 2 + 2;  // pairs with odd i from i0-2 to i0+TW
    constexpr int NPI = (NP * (RB2_TH + 2) + RB2_NT - 1) / RB2_NT;
    double fa[NPI], fb[NPI];
    bool wa[NPI], wb[NPI];
    int ja[NPI], ia[NPI];
#pragma unroll
    for (int u = 0; u < NPI; ++u) {
        const int q = tid + u * RB2_NT;
        const int r = q / NP, m = q - r * NP;
        const int j = j0 - 1 + r, io = i0 - 2 + 2 * m;
        const bool row = q < NP * (RB2_TH + 2) && j >= 1 && j <= L.ny - 1;
        ja[u] = j;
        ia[u] = io;
        wa[u] = row && io >= 1 && io <= L.nx - 1 && io >= i0 - 1;
        wb[u] = row && io + 1 >= 1 && io + 1 <= L.nx - 1 && io + 1 <= i0 + RB2_TW;
        fa[u] = wa[u] ? f[L.at(io, j, 0)] : 0.0;
        fb[u] = wb[u] ? f[L.at(io + 1, j, 0)] : 0.0;
    }
    double za[NPI], zb[NPI];
#pragma unroll
    for (int u = 0; u < NPI; ++u) {
        const int q = tid + u * RB2_NT;
        const int j = ja[u], io = ia[u];
        za[u] = zb[u] = 0.0;
        if (NOISE && q < NP * (RB2_TH + 2) && j >= 1 && j <= L.ny - 1 && io >= 1 && io <= L.nx - 1) {
            const Philox4 rnd = philox4x32_10(pair_id<2>(L, io, j, 0), G.tag, (uint32_t)sample,
                                              (uint32_t)(sample >> 32), G.key.k0, G.key.k1);
            normal_pair(rnd, &za[u], &zb[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < NSX; ++u) {
        const int q = tid + u * RB2_NT;
        if (q < RB2_H * RB2_W) {
            const int r = q / RB2_W, c = q - r * RB2_W;
            xs[rb2_lidx(r, c)] = xv[u];
        }
    }
#pragma unroll
    for (int u = 0; u < NPI; ++u) {
        if (wa[u]) cs[rb2_lidx(ja[u] - jb, ia[u] - ib)] = NOISE ? fma(G.sd, za[u], fa[u]) : fa[u];
        if (wb[u]) cs[rb2_lidx(ja[u] - jb, ia[u] + 1 - ib)] = NOISE ? fma(G.sd, zb[u], fb[u]) : fb[u];
    }
    __syncthreads();
    // one colour on columns [ia, ia + w) x rows [ja, ja + h) (interior vertices only)
    auto colour_pass = [&](int colour, int ia, int ja, int w, int h) {
        const int per_row = (w + 1) / 2;
        for (int q = tid; q < per_row * h; q += RB2_NT) {
            const int r = q / per_row, k = q - r * per_row;
            const int j = ja + r;
            const int i = ia + (((ia + j) & 1) != colour ? 1 : 0) + 2 * k;
            if (i >= ia + w || i < 1 || i > L.nx - 1 || j < 1 || j > L.ny - 1) continue;
            const int r2 = j - jb, c2 = i - ib;
            const int p = rb2_lidx(r2, c2);
            // stencil_fma<2, 5>'s chain: south, west, centre, east, north
            double res = S.a[1] * xs[p - RB2_W];
            res = fma(S.a[3], xs[rb2_lidx(r2, c2 - 1)], res);
            res = fma(S.a[4], xs[p], res);
            res = fma(S.a[5], xs[rb2_lidx(r2, c2 + 1)], res);
            res = fma(S.a[7], xs[p + RB2_W], res);
            xs[p] = fma(G.wd, cs[p] - res, xs[p]);
        }
    };
    colour_pass(c1, i0 - 1, j0 - 1, RB2_TW + 2, RB2_TH + 2);
    __syncthreads();
    colour_pass(1 - c1, i0, j0, RB2_TW, RB2_TH);
    __syncthreads();
    for (int q = tid; q < RB2_TW * RB2_TH; q += RB2_NT) {
        const int r = q / RB2_TW, c = q - r * RB2_TW;
        const int i = i0 + c, j = j0 + r;
        if (i <= L.nx - 1 && j <= L.ny - 1) xout[L.at(i, j, 0)] = xs[rb2_lidx(r + 2, c + 2)];
    }
}

}  // namespace mgmc
