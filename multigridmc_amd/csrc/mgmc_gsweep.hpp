// mgmc_gsweep.hpp -- pair passes of the 2^d-colour Gibbs sweep of a Galerkin (9/27-point) level.
//
// One SOR Gibbs sweep of a coarse level (SORSampler::apply, sampler/sor_sampler.cc:37-59) in the
// 2^d-colour order of k_sweep_mc (colour bit d = parity of coordinate d; forward = colours 0..2^d-1,
// backward = reversed) takes 2^(d-1) passes instead of 2^d:
//
//  * Colours c and c^1 differ only in the parity of i.  A c^1 vertex reads c vertices only at i-1 and
//    i+1 in its own row (every other neighbour changes the parity of j or k), and neither colour
//    reads any other vertex of the pass's rows.  So one pass updates both colours of the rows of
//    parity (jp, kp): a thread owns the Philox pair (2m+1, 2m+2), updates the vertex of the first
//    colour, trades the new value with its row neighbour through LDS (one barrier), then updates
//    the vertex of the second colour.  Rows are independent, so the pass runs in place.
//  * The two vertices of a pair take the cos / sin branch of one Box-Muller draw: one evaluation per
//    pair and sweep, no recomputation.
//  * Whole rows sit in one workgroup (nx/2 threads per row), so the exchange never leaves it.
// Arithmetic is gibbs_point's (stencil fma chain in ascending column order, c = fma(sd, xi, f),
// x = fma(omega/diag, c - sum, x)) with the Philox pair ids / tags of k_sweep_mc: bitwise equal to
// the colour passes.
#pragma once
#include <type_traits>

#include "mgmc_kernels.hpp"

namespace mgmc {

struct PairPassArgs {
    Layout L;
    double* x;
    const double* f;
    StencilArg S;
    GibbsArg G;
    int jp, kp;        // row parities of the pass (kp unused in 2D)
    int rows_per_block, nrows_j, nrows;  // pass rows: j = 2 - jp + 2 t (t < nrows_j), k likewise
    long long cs;      // batched chains: doubles between chains (blockIdx.z = chain)
};

// FIRST_ODD: the odd position (i parity 1) is updated first (backward sweeps).  A template parameter,
// so every index into the register window below is static.
template <int DIM, bool FIRST_ODD, bool SYM = false>  // SYM: stencil_coef's fold (3D, same bits)
__global__ void __launch_bounds__(256) k_sweep_pairs(PairPassArgs a) {
    constexpr int NPTS = DIM == 3 ? 27 : 9;
    __shared__ double xnew[256 + 2];  // new first-colour values, [1 + tid]; zero guards at both ends
    {
        const int ch = batch_chain();
        a.x += ch * a.cs;
        a.f += ch * a.cs;
        a.G.key = chain_key(a.G, ch);
    }
    const Layout& L = a.L;
    const int npair = L.nx / 2;
    const int tid = threadIdx.x;
    const int rloc = tid / npair, m = tid - rloc * npair;
    const int row = blockIdx.x * a.rows_per_block + rloc;
    const bool active = rloc < a.rows_per_block && row < a.nrows;
    const int tj = active ? row % a.nrows_j : 0, tk = active ? row / a.nrows_j : 0;
    const int j = 2 - a.jp + 2 * tj;
    const int k = DIM == 3 ? 2 - a.kp + 2 * tk : 0;
    const int i0 = 2 * m + 1;  // odd position of the pair
    if (tid < 2) xnew[tid == 0 ? 0 : 257] = 0.0;
    const long long p0 = active ? L.at(i0, j, k) : 0;  // offset of the odd vertex

    // vertex values around the pair: rows (dz, dy) x positions 2m .. 2m+3 (3 aligned pairs loaded)
    constexpr int NR = DIM == 3 ? 9 : 3;
    double w[NR][4];
    double2 fv = make_double2(0.0, 0.0);
    if (active) {
#pragma unroll
        for (int rr = 0; rr < NR; ++rr) {
            const int dz = DIM == 3 ? rr / 3 - 1 : 0, dy = rr % 3 - 1;
            const double* q = a.x + p0 + (long long)dz * L.sp + (long long)dy * L.sx;
            const double2 lo = *reinterpret_cast<const double2*>(q - 2);
            const double2 mid = *reinterpret_cast<const double2*>(q);
            const double2 hi = *reinterpret_cast<const double2*>(q + 2);
            w[rr][0] = lo.y;   // 2m
            w[rr][1] = mid.x;  // 2m+1
            w[rr][2] = mid.y;  // 2m+2
            w[rr][3] = hi.x;   // 2m+3
        }
        fv = *reinterpret_cast<const double2*>(a.f + p0);
    }
    constexpr int C = DIM == 3 ? 4 : 1;  // row index (dz, dy) = (0, 0)
    // stencil fma chain of the vertex at window position s (1: odd 2m+1, 2: even 2m+2)
    auto chain = [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        double res = stencil_coef<SYM>(a.S, 0) * w[0][s - 1];
#pragma unroll
        for (int q = 1; q < NPTS; ++q) {
            const int rr = q / 3, dx = q % 3 - 1;
            res = fma(stencil_coef<SYM>(a.S, q), w[rr][s + dx], res);
        }
        return res;
    };

    double z0 = 0.0, z1 = 0.0;  // Box-Muller pair: cos -> odd position, sin -> even position
    const bool odd_in = active && i0 <= L.nx - 1;
    const bool even_in = active && i0 + 1 <= L.nx - 1;
    if (odd_in) {
        const uint32_t pair = pair_id<DIM>(L, i0, j, k);
        const Philox4 rnd = philox4x32_10(pair, a.G.tag, (uint32_t)*a.G.sample, (uint32_t)(*a.G.sample >> 32),
                                          a.G.key.k0, a.G.key.k1);
        normal_pair(rnd, &z0, &z1);
    }
    const double sd = a.G.sd, wd = a.G.wd;
    // first colour
    constexpr int s1 = FIRST_ODD ? 1 : 2;
    const bool in1 = FIRST_ODD ? odd_in : even_in;
    double v1 = w[C][s1];
    if (in1) {
        const double res = chain(std::integral_constant<int, s1>{});
        const double c = fma(sd, FIRST_ODD ? z0 : z1, FIRST_ODD ? fv.x : fv.y);
        v1 = fma(wd, c - res, v1);
    }
    xnew[1 + tid] = v1;
    __syncthreads();
    // second colour: its row neighbours are first-colour vertices (own pair + adjacent pair)
    constexpr int s2 = 3 - s1;
    const bool in2 = FIRST_ODD ? even_in : odd_in;
    w[C][s1] = v1;
    if (FIRST_ODD) {  // second = even 2m+2, neighbours 2m+1 (own) and 2m+3 (next pair's odd)
        w[C][3] = (m + 1 < npair) ? xnew[2 + tid] : 0.0;
    } else {            // second = odd 2m+1, neighbours 2m (previous pair's even) and 2m+2 (own)
        w[C][0] = (m > 0) ? xnew[tid] : 0.0;
    }
    double v2 = w[C][s2];
    if (in2) {
        const double res = chain(std::integral_constant<int, s2>{});
        const double c = fma(sd, FIRST_ODD ? z1 : z0, FIRST_ODD ? fv.y : fv.x);
        v2 = fma(wd, c - res, v2);
    }
    if (active)
        *reinterpret_cast<double2*>(a.x + p0) = FIRST_ODD ? make_double2(v1, v2) : make_double2(v2, v1);
}

// ---- both colour pairs of one k parity in one launch (2 launches per 3D sweep, 1 in 2D) ----
//
// The pair passes of a sweep come in k-parity halves: forward (0,1), (2,3) | (4,5), (6,7).  Within a
// half the second pair's rows (parity jp2) read the first pair's rows (parity jp1) only at j-1 and j+1
// of their own plane; everything else they read belongs to the other k parity (not touched in this
// half).  A workgroup takes 2T+1 consecutive full rows of one plane: rows of parity jp1 at local rows
// 0, 2, ..., 2T, rows of parity jp2 in between.  Phase 1 runs the first pair on the jp1 rows (one of
// them is the neighbouring workgroup's row, recomputed and not stored), the new rows go to LDS, phase 2
// runs the second pair on the jp2 rows with those rows substituted into its window.
// Out of place (x_in -> x_out), so the recomputed row sees the old values whatever the other
// workgroups have written: the first half reads x_in and writes its planes of x_out, the second half
// reads its own planes from x_in and the first half's (new) planes from x_out.  Each vertex sees
// exactly the values of the separate pair passes and the same arithmetic, so the result is bitwise the
// same; x is read once per half instead of once per pair pass.
struct QuadPassArgs {
    Layout L;
    const double* x0;   // rows of the pass's own planes (old values)
    const double* xz;   // rows of the planes k-1, k+1 (other parity: old in the first half, new in the second)
    double* xout;
    const double* f;
    StencilArg S;
    GibbsArg G;
    int jp1, kp;        // row parity of the first pair (first colour's bit 1), plane parity (bit 2)
    int T;              // rows of parity jp2 per workgroup (2T+1 rows in all)
    int nblk_y;         // workgroups along j
    long long cs;       // batched chains: doubles between chains (blockIdx.z = chain)
    const double2* zb;  // PZ: the sweep's Box-Muller pairs, drawn earlier (pair id order; one chain)
};

// 64-bit value of the neighbouring lane (wave_shr:1: lane l - 1's, wave_shl:1: lane l + 1's; 0 past the
// wavefront's ends), two 32-bit DPP moves
__device__ __forceinline__ double lane_prev(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_next(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

// SYM: stencil_coef's fold (3D, same bits).  XZ: the input x is known zero (the level's first pre-sweep,
// mgmc_capi.hip mark_zero_inputs): 1 = every x row is the constant 0.0 (first half), 2 = the own planes'
// rows are (second half) -- not loaded.
// LANES (3D, npair dividing 64: every wavefront holds whole rows, thread = row * npair + pair): each
// lane loads only its own pair (2m+1, 2m+2) of a window row; the outer columns 2m and 2m+3 are the
// neighbouring lanes' pairs (lane_prev / lane_next), or the zero guards at positions 0 and nx+1 for the
// row's first / last pair -- one 16-byte load per row instead of three (the passes are bound by the
// vector-memory instructions' address / L1 throughput, not by HBM: the window's 27 loads mostly hit)
// PZ: the Box-Muller pairs come from a.zb (k_tail's spare workgroups, mgmc_tail.hpp tail_post_noise)
template <int DIM, bool FIRST_ODD, bool SYM = false, int XZ = 0, bool LANES = false, bool PZ = false>
__global__ void __launch_bounds__(1024) k_sweep_quads(QuadPassArgs a) {
    static_assert(!LANES || DIM == 3, "LANES: 3D levels");
    {
        const int ch = batch_chain();
        a.x0 += ch * a.cs;
        a.xz += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        a.G.key = chain_key(a.G, ch);
    }
    // T+1 thread rows of npair threads: thread row t runs the first pair on local row 2t (phase 1),
    // then the second pair on local row 2t+1 (phase 2, t < T)
    constexpr int NPTS = DIM == 3 ? 27 : 9;
    extern __shared__ __attribute__((aligned(16))) double rowbuf[];  // [2T+1][nx+2] new row values by position
    const Layout& L = a.L;
    const int npair = L.nx / 2;
    const int RW = L.nx + 2;
    const int nrow = 2 * a.T + 1;
    const int tid = threadIdx.x;
    const int t = tid / npair, m = tid - t * npair;
    const int by = blockIdx.x % a.nblk_y, tk = blockIdx.x / a.nblk_y;
    const int jbase = 2 * a.T * by + a.jp1;  // row of local row 0
    const int k = DIM == 3 ? 2 - a.kp + 2 * tk : 0;
    const int i0 = 2 * m + 1;
    for (int q = tid; q < nrow; q += blockDim.x) {  // zero guards: positions 0, nx, nx+1 of every row
        rowbuf[q * RW] = 0.0;
        rowbuf[q * RW + L.nx] = 0.0;
        rowbuf[q * RW + L.nx + 1] = 0.0;
    }
    constexpr int NR = DIM == 3 ? 9 : 3;
    constexpr int C = DIM == 3 ? 4 : 1;
    constexpr int s1 = FIRST_ODD ? 1 : 2, s2 = 3 - s1;
    const double sd = a.G.sd, wd = a.G.wd;
    double w[NR][4];
    auto chain = [&](auto sc) {
        constexpr int s = decltype(sc)::value;
        double res = stencil_coef<SYM>(a.S, 0) * w[0][s - 1];
#pragma unroll
        for (int q = 1; q < NPTS; ++q) {
            const int rr = q / 3, dx = q % 3 - 1;
            res = fma(stencil_coef<SYM>(a.S, q), w[rr][s + dx], res);
        }
        return res;
    };
    // one colour pair on local row lr (go: this thread has a row in this phase; the barrier is for all)
    auto pair_pass = [&](bool go, int lr, bool from_lds) {
        const int j = jbase + lr;
        const bool inrow = go && j >= 1 && j <= L.ny - 1;
        const bool own = inrow && ((lr & 1) ? true : (a.jp1 == 0 ? lr > 0 : lr < 2 * a.T));
        const long long p0 = inrow ? L.at(i0, j, k) : 0;
        double2 fv = make_double2(0.0, 0.0);
        double2 zzv = make_double2(0.0, 0.0);  // PZ: the pair's noise, loaded with f
        if constexpr (LANES) {
            // own pairs of the window rows (the whole wavefront takes part in the lane shifts below:
            // lanes of rows outside the pass hold zeros, and a row's first / last lane never uses a
            // neighbouring row's value)
            double2 mid[NR];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int dz = rr / 3 - 1, dy = rr % 3 - 1;
                mid[rr] = make_double2(0.0, 0.0);
                if (!inrow || (from_lds && dz == 0 && dy != 0) || XZ == 1 || (XZ == 2 && dz == 0)) continue;
                mid[rr] = *reinterpret_cast<const double2*>((dz == 0 ? a.x0 : a.xz) + p0 + (long long)dz * L.sp +
                                                            (long long)dy * L.sx);
            }
            if (inrow) fv = *reinterpret_cast<const double2*>(a.f + p0);
            if (PZ && inrow) zzv = a.zb[pair_id<DIM>(L, i0, j, k)];
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int dz = rr / 3 - 1, dy = rr % 3 - 1;
                if (from_lds && dz == 0 && dy != 0) {  // the new first-pair rows of this plane
                    const double* q = rowbuf + (lr + dy) * RW + 2 * m;
                    w[rr][0] = q[0];
                    w[rr][1] = q[1];
                    w[rr][2] = q[2];
                    w[rr][3] = q[3];
                    continue;
                }
                const double l = lane_prev(mid[rr].y), r = lane_next(mid[rr].x);
                w[rr][0] = m == 0 ? 0.0 : l;
                w[rr][1] = mid[rr].x;
                w[rr][2] = mid[rr].y;
                w[rr][3] = m == npair - 1 ? 0.0 : r;
            }
        } else if (inrow) {
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) {
                const int dz = DIM == 3 ? rr / 3 - 1 : 0, dy = rr % 3 - 1;
                if (from_lds && dz == 0 && dy != 0) {  // the new first-pair rows of this plane
                    const double* q = rowbuf + (lr + dy) * RW + 2 * m;
                    w[rr][0] = q[0];
                    w[rr][1] = q[1];
                    w[rr][2] = q[2];
                    w[rr][3] = q[3];
                    continue;
                }
                if (XZ == 1 || (XZ == 2 && dz == 0)) {
                    w[rr][0] = w[rr][1] = w[rr][2] = w[rr][3] = 0.0;
                    continue;
                }
                const double* q = (dz == 0 ? a.x0 : a.xz) + p0 + (long long)dz * L.sp + (long long)dy * L.sx;
                const double2 lo = *reinterpret_cast<const double2*>(q - 2);
                const double2 mid = *reinterpret_cast<const double2*>(q);
                const double2 hi = *reinterpret_cast<const double2*>(q + 2);
                w[rr][0] = lo.y;
                w[rr][1] = mid.x;
                w[rr][2] = mid.y;
                w[rr][3] = hi.x;
            }
            fv = *reinterpret_cast<const double2*>(a.f + p0);
            if (PZ) zzv = a.zb[pair_id<DIM>(L, i0, j, k)];
        } else {
#pragma unroll
            for (int rr = 0; rr < NR; ++rr) w[rr][0] = w[rr][1] = w[rr][2] = w[rr][3] = 0.0;
        }
        double z0 = 0.0, z1 = 0.0;
        const bool odd_in = inrow && i0 <= L.nx - 1;
        const bool even_in = inrow && i0 + 1 <= L.nx - 1;
        if (PZ) {
            z0 = zzv.x;
            z1 = zzv.y;
        } else if (odd_in) {
            const uint32_t pair = pair_id<DIM>(L, i0, j, k);
            const Philox4 rnd = philox4x32_10(pair, a.G.tag, (uint32_t)*a.G.sample, (uint32_t)(*a.G.sample >> 32),
                                              a.G.key.k0, a.G.key.k1);
            normal_pair(rnd, &z0, &z1);
        }
        const bool in1 = FIRST_ODD ? odd_in : even_in;
        const bool in2 = FIRST_ODD ? even_in : odd_in;
        double* myrow = rowbuf + lr * RW;
        double v1 = w[C][s1];
        if (in1) {
            const double res = chain(std::integral_constant<int, s1>{});
            const double c = fma(sd, FIRST_ODD ? z0 : z1, FIRST_ODD ? fv.x : fv.y);
            v1 = fma(wd, c - res, v1);
        }
        if (go) myrow[i0 + (s1 - 1)] = v1;
        __syncthreads();
        w[C][s1] = v1;
        if (go) {
            if (FIRST_ODD) w[C][3] = myrow[i0 + 2];   // next pair's odd element (0 past the row end)
            else w[C][0] = myrow[i0 - 1];             // previous pair's even element (0 before the row)
        }
        double v2 = w[C][s2];
        if (in2) {
            const double res = chain(std::integral_constant<int, s2>{});
            const double c = fma(sd, FIRST_ODD ? z1 : z0, FIRST_ODD ? fv.y : fv.x);
            v2 = fma(wd, c - res, v2);
        }
        if (go) myrow[i0 + (s2 - 1)] = v2;
        if (own) *reinterpret_cast<double2*>(a.xout + p0) = FIRST_ODD ? make_double2(v1, v2) : make_double2(v2, v1);
    };
    const bool act = t <= a.T;
    // phase 1: first pair on the jp1 rows; every jp1 row is complete in LDS after the barrier
    pair_pass(act, 2 * t, false);
    __syncthreads();
    // phase 2: second pair on the jp2 rows with the new jp1 rows j-1, j+1 of this plane
    pair_pass(act && t < a.T, 2 * t + 1, true);
}

}  // namespace mgmc
