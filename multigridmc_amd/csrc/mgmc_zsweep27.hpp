// mgmc_zsweep27.hpp -- one launch per 2^3-colour Gibbs sweep of a 3D Galerkin (27-point) level.
//
// SORSampler::apply (sampler/sor_sampler.cc:37-59) on a coarse level in the 8-colour order of
// k_sweep_mc / k_sweep_pairs: colour bit 0 = parity of i, bit 1 = of j, bit 2 = of k; forward
// colours 0..7, backward 7..0.  The pair passes read x four times per sweep (one pass per (j, k)
// parity, 512^3 level 1: 4 x 41 us); this kernel reads it once.
//
// z-march.  Write K1 for the plane parity updated first (even forward, odd backward) and K2 for the
// other.  A K1 plane's colours read only old K2 planes; a K2 plane's colours read the new K1 planes
// on either side.  So the march takes one K1 plane q and the K2 plane q-1 per step: the four colours
// of q (rows of parity J1, then J2; within a row the pair trick of k_sweep_pairs), then the four of
// q-1, whose neighbours q-2 (previous step) and q are new by then.  Four LDS plane slots hold
// q-2 (new), q-1, q, q+1; the loads of q+2, q+3 are in flight during the step.
//
// Tiles.  A workgroup stages a 64 x 64 (i, j) slab of every plane and updates it in place in LDS.
// Updated values near the slab edge are wrong (their neighbours outside the slab are missing); each
// colour step moves the edge of the valid region one vertex inward along the dimensions its
// dependences cross -- after the eighth colour the K2 values are valid 8 vertices in from the
// edge in i and 4 in j (the K1 values 4 and 2).  The workgroup stores its core, 46 columns x 56 rows (SR = 64);
// the neighbouring workgroups recompute the overlap from the same old values (out of place:
// x_in -> x_out) with the same arithmetic.  In z, a chunk of planes [k0, k1) recomputes the K1
// planes k0-1 / k1 when they lie outside the chunk.
//
// Arithmetic is k_sweep_pairs' per vertex (stencil fma chain in ascending column order from the
// register window, c = fma(sd, xi, f), x = fma(omega/diag, c - sum, x), the Box-Muller pair of the
// Philox pair (odd i, i+1) with the sweep's tag): bitwise the colour passes and the oracle.
#pragma once
#include "mgmc_kernels.hpp"

#ifndef MGMC_Z27_EXP  // timing decomposition (wrong results): 1 no Philox, 2 one stencil column, 4 no mid-phase barrier
#define MGMC_Z27_EXP 0
#endif

namespace mgmc {

constexpr int Z27_SW = 64;                 // slab columns: LDS column c is lattice i = ib + c (ib even)
constexpr int Z27_RS = 68;                 // LDS row stride (doubles)
#ifndef MGMC_Z27_SR
#define MGMC_Z27_SR 64
#endif
constexpr int Z27_SR = MGMC_Z27_SR;        // slab rows: LDS row r is lattice j = jb + r
constexpr int Z27_CX = 46, Z27_C0 = 9;     // core columns [9, 55): pairs (odd, even) 16-byte aligned
constexpr int Z27_CY = Z27_SR - 8, Z27_R0 = 4;  // core rows [4, SR - 4)
constexpr int Z27_NT = 16 * Z27_SR;        // 32 pairs x SR/2 rows of one parity
constexpr int Z27_SLOT = Z27_SR * Z27_RS;  // doubles per plane slot
constexpr size_t z27_lds_bytes() { return (size_t)4 * Z27_SLOT * sizeof(double); }

struct Z27Args {
    Layout L;
    const double* xin;
    double* xout;
    const double* f;
    StencilArg S;
    GibbsArg G;
    int ntx, nty, ntz, kz;  // tiles in i, j, z-chunks; planes per chunk
    long long cs;           // batched chains: doubles between chains (blockIdx.z = chain)
};

template <bool BACKWARD>
__global__ void __launch_bounds__(Z27_NT) k_zsweep27(Z27Args a) {
    extern __shared__ __attribute__((aligned(16))) double sl[];  // [4][SR][RS]
    {
        const int ch = batch_chain();
        a.xin += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        a.G.key = chain_key(a.G, ch);
    }
    const Layout& L = a.L;
    const int nb = gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);  // blocks b, b+8 share an XCD
    const int tx = tile % a.ntx, ty = (tile / a.ntx) % a.nty, tz = tile / (a.ntx * a.nty);
    if (tz >= a.ntz) return;
    const int ib = Z27_CX * tx - (Z27_C0 - 1);  // core column 9 is lattice i = 1 + 46 tx
    const int jb = Z27_CY * ty - (Z27_R0 - 1);  // core row 4 is lattice j = 1 + CY ty
    const int k0 = 1 + tz * a.kz, k1 = min(k0 + a.kz, L.nz);  // output planes [k0, k1)
    constexpr int K1 = BACKWARD ? 1 : 0, J1 = BACKWARD ? 1 : 0;
    constexpr int s1 = BACKWARD ? 1 : 2, s2 = 3 - s1;  // window position of the first / second vertex
    const int tid = threadIdx.x, m = tid & 31, u = tid >> 5;
    const int i0 = ib + 2 * m + 1;  // odd lattice position of the thread's pair (LDS columns 2m+1, 2m+2)
    const uint64_t sample = *a.G.sample;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    const double sd = a.G.sd, wd = a.G.wd;
    const bool pair_core = m >= Z27_C0 / 2 && 2 * m + 2 < Z27_C0 + Z27_CX;
    const bool odd_col = i0 >= 1 && i0 <= L.nx - 1, even_col = i0 + 1 >= 1 && i0 + 1 <= L.nx - 1;

    auto slot = [&](int k) { return sl + ((k + 4) & 3) * Z27_SLOT; };
    // plane k of x_in: rows u, u + 32 as (odd, even) pairs at LDS columns 2m+1, 2m+2, column 0 of
    // row tid (tid < 64); rows / planes outside the level read as zero.  Columns outside [0, nx]
    // hold whatever the store has there: only vertices that are never updated read them.
    double2 pv[2][2];
    double p0[2];
    auto issue = [&](int k, int h) {
        const bool kin = k >= 0 && k <= L.nz;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = jb + u + (Z27_SR / 2) * e;
            pv[h][e] = (kin && j >= 0 && j <= L.ny) ? *reinterpret_cast<const double2*>(a.xin + L.at(i0, j, k))
                                                   : make_double2(0.0, 0.0);
        }
        const int j = jb + tid;
        p0[h] = (tid < Z27_SR && kin && j >= 0 && j <= L.ny) ? a.xin[L.at(ib, j, k)] : 0.0;
    };
    auto deposit = [&](int k, int h) {
        double* s = slot(k);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            double* row = s + (u + (Z27_SR / 2) * e) * Z27_RS;
            row[2 * m + 1] = pv[h][e].x;
            row[2 * m + 2] = pv[h][e].y;
        }
        if (tid < Z27_SR) s[tid * Z27_RS] = p0[h];
    };
    // f of the thread's pair in the rows of parity P of plane k (zero outside the interior)
    auto row_of = [&](int P) { return 2 * u + ((P - jb) & 1); };
    auto load_f = [&](int k, int P) {
        const int j = jb + row_of(P);
        const bool in = k >= 1 && k <= L.nz - 1 && j >= 1 && j <= L.ny - 1 && odd_col && m < 31;
        return in ? *reinterpret_cast<const double2*>(a.f + L.at(i0, j, k)) : make_double2(0.0, 0.0);
    };

    // the colours of the rows of parity P of plane k (the first vertex of each pair, exchange, the
    // second); stores the core to x_out when `out`
    // the Box-Muller pair of the thread's pair in the rows of parity P of plane k (0 where the
    // pair's odd vertex is not updated)
    auto noise = [&](int k, int P) {
        const int r = row_of(P);
        const int j = jb + r;
        const bool odd_in = k >= 1 && k <= L.nz - 1 && m < 31 && r >= 1 && r <= Z27_SR - 2 && j >= 1 &&
                            j <= L.ny - 1 && odd_col;
        double2 z = make_double2(0.0, 0.0);
        if (odd_in && !(MGMC_Z27_EXP & 1)) {
            const Philox4 rnd = philox4x32_10(pair_id<3>(L, i0, j, k), a.G.tag, s_lo, s_hi, a.G.key.k0, a.G.key.k1);
            normal_pair(rnd, &z.x, &z.y);
        }
        return z;
    };
    // one phase with the noise zc of its own pairs (computed during the phase before); the noise
    // of the next phase (plane nk, rows of parity nP) is computed here, between the exchange read
    // and the second vertex's chain, where it overlaps the LDS latency instead of stalling the
    // phase after the barrier
    auto phase = [&](int k, int P, double2 fv, bool out, double2 zc, int nk, int nP, double2& zn) {
        const int r = row_of(P);
        const int j = jb + r;
        const bool act = k >= 1 && k <= L.nz - 1 && m < 31 && r >= 1 && r <= Z27_SR - 2 && j >= 1 && j <= L.ny - 1;
        const bool odd_in = act && odd_col, even_in = act && even_col;
        double* own = slot(k) + r * Z27_RS;
        // stencil rows (dz, dy) in ascending order, each read as two aligned pairs (positions 2m ..
        // 2m+3); the first vertex's chain takes every row, the second vertex's chain its rows before
        // the centre row here and the rest after the exchange (its centre row holds the new first
        // vertex and the neighbouring pair's new vertex), so only the rows from the centre on stay
        // in registers across the barrier
        auto row_vals = [&](int rr, double (&v)[4]) {
            const int dz = rr / 3 - 1, dy = rr % 3 - 1;
            const double* q = slot(k + dz) + (r + dy) * Z27_RS + 2 * m;
            const double2 lo = *reinterpret_cast<const double2*>(q);
            const double2 hi = *reinterpret_cast<const double2*>(q + 2);
            v[0] = lo.x;
            v[1] = lo.y;
            v[2] = hi.x;
            v[3] = hi.y;
        };
        constexpr int C = 4;  // centre row (dz, dy) = (0, 0)
        double keep[5][4];    // rows 4 .. 8
        double res1 = 0.0, res2 = 0.0;
        if (act) {
#pragma unroll
            for (int rr = 0; rr < 9; ++rr) {
                double v[4];
                row_vals(rr, v);
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) {
                    const int q = rr * 3 + dx + 1;
                    if ((MGMC_Z27_EXP & 2) && dx != 0) continue;
                    if (q == 0) {
                        res1 = a.S.a[0] * v[s1 - 1];
                        res2 = a.S.a[0] * v[s2 - 1];
                    } else {
                        res1 = fma(a.S.a[q], v[s1 + dx], res1);
                        if (rr < C) res2 = fma(a.S.a[q], v[s2 + dx], res2);
                    }
                }
                if (rr >= C) {
#pragma unroll
                    for (int c = 0; c < 4; ++c) keep[rr - C][c] = v[c];
                }
            }
        } else {
#pragma unroll
            for (int rr = 0; rr < 5; ++rr) keep[rr][0] = keep[rr][1] = keep[rr][2] = keep[rr][3] = 0.0;
        }
        const double z0 = zc.x, z1 = zc.y;  // cos -> odd position, sin -> even position
        const bool in1 = s1 == 1 ? odd_in : even_in, in2 = s1 == 1 ? even_in : odd_in;
        double v1 = keep[0][s1];
        if (in1) {
            const double c = fma(sd, s1 == 1 ? z0 : z1, s1 == 1 ? fv.x : fv.y);
            v1 = fma(wd, c - res1, v1);
            own[2 * m + s1] = v1;
        }
        if (!(MGMC_Z27_EXP & 4)) __syncthreads();
        keep[0][s1] = v1;
        if (act) {
            if (s1 == 1) keep[0][3] = own[2 * m + 3];  // second = even 2m+2: the next pair's new odd vertex
            else keep[0][0] = own[2 * m];              // second = odd 2m+1: the previous pair's new even vertex
        }
        zn = noise(nk, nP);
        double v2 = keep[0][s2];
        if (in2) {
#pragma unroll
            for (int rr = C; rr < 9; ++rr)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx)
                    if (!(MGMC_Z27_EXP & 2) || dx == 0) res2 = fma(a.S.a[rr * 3 + dx + 1], keep[rr - C][s2 + dx], res2);
            const double c = fma(sd, s1 == 1 ? z1 : z0, s1 == 1 ? fv.y : fv.x);
            v2 = fma(wd, c - res2, v2);
            own[2 * m + s2] = v2;
        }
        if (out && pair_core && r >= Z27_R0 && r < Z27_R0 + Z27_CY && odd_in) {
            const double vo = s1 == 1 ? v1 : v2, ve = s1 == 1 ? v2 : v1;
            double* dst = a.xout + L.at(i0, j, k);
            if (even_in) *reinterpret_cast<double2*>(dst) = make_double2(vo, ve);
            else dst[0] = vo;
        }
        __syncthreads();
    };

    // K1 planes q from the first >= k0 - 1 to the last <= k1
    const int qa = (k0 - 1) + (((k0 - 1) & 1) != K1 ? 1 : 0);
    const int qb = k1 - ((k1 & 1) != K1 ? 1 : 0);
    issue(qa - 1, 0);
    issue(qa, 1);
    deposit(qa - 1, 0);
    deposit(qa, 1);
    issue(qa + 1, 0);
    deposit(qa + 1, 0);
    issue(qa + 2, 0);
    issue(qa + 3, 1);
    __syncthreads();
    // f of each phase is loaded one phase ahead (its latency hides behind the phase before)
    double2 fa = load_f(qa, J1);
    double2 z = noise(qa, J1);
    for (int q = qa; q <= qb; q += 2) {
        const bool two = q - 1 >= k0;  // the K2 plane q-1 (neighbours q-2, q new)
        double2 fb = load_f(q, 1 - J1);
        phase(q, J1, fa, q >= k0 && q < k1, z, q, 1 - J1, z);
        double2 fc = two ? load_f(q - 1, J1) : make_double2(0.0, 0.0);
        if (two) {
            phase(q, 1 - J1, fb, q >= k0 && q < k1, z, q - 1, J1, z);
            double2 fd = load_f(q - 1, 1 - J1);
            phase(q - 1, J1, fc, true, z, q - 1, 1 - J1, z);
            fa = load_f(q + 2, J1);
            phase(q - 1, 1 - J1, fd, true, z, q + 2, J1, z);
        } else {
            phase(q, 1 - J1, fb, q >= k0 && q < k1, z, q + 2, J1, z);
            fa = load_f(q + 2, J1);
        }
        if (q + 2 <= qb) {  // planes q+2, q+3 into the slots of q-2, q-1
            deposit(q + 2, 0);
            deposit(q + 3, 1);
            issue(q + 4, 0);
            issue(q + 5, 1);
        }
        __syncthreads();
    }
}

}  // namespace mgmc
