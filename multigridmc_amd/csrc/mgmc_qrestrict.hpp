// mgmc_qrestrict.hpp -- last pre-sweep + residual + restriction of a 2D Galerkin (9-point) level in
// one launch.
//
//   x <- Gibbs sweep(x)   (sampler/sor_sampler.cc:37-59, four colours as k_sweep_quads)
//   f_c = R (f - A x),  x_c = 0      (sampler/multigridmc_sampler.cc:116-122)
//
// The 2D levels below the fine one are launch-bound: at 1024^2 a 511^2 sweep is 5.7 us and the
// residual + restriction after it 4.8 us, whatever their size.  This kernel does both in one launch.
// A workgroup owns CJ coarse rows J0 .. J0+CJ-1 (all columns).  Their restriction needs the residual
// on fine rows 2J0-1 .. 2J0+2CJ-1, which needs the swept x on rows 2J0-2 .. 2J0+2CJ; those need the
// first colour pair (rows of parity jp1) on rows 2J0-3 .. 2J0+2CJ+1 and old x on 2J0-4 .. 2J0+2CJ+2.
// So the workgroup stages old x and f of its rows in LDS, runs the four colour passes in place there
// (the rows near its edges recomputed, as the neighbouring workgroups compute them too), evaluates
// the residual rows into LDS, restricts, and stores its own fine rows 2J0-1 .. 2J0+2CJ-2 (the last
// workgroup also row ny-1) out of place (x_in -> x_out, like the quad passes).
//
// Every value is the same function of the same inputs as in the separate kernels, so the result is
// bitwise theirs:
//  * colour passes in k_sweep_quads' order: first pair (rows of parity jp1: colours 0, 1 forward,
//    3, 2 backward), then the second pair (rows jp2); within a pair the element FIRST_ODD picks, then
//    the other.  A colour's vertices read only vertices of other colours, so updating a colour in
//    place between barriers gives exactly the colour-pass values.  Per vertex: one Box-Muller per
//    pair (cos -> odd position, sin -> even), c = fma(sd, xi, f), S the stencil fma chain in
//    ascending column order, x = fma(omega/diag, c - S, x) (gibbs_point);
//  * residual r = f - (0 + sum a x, separate mul and add, ascending), restriction sum over (sy, sx)
//    ascending of (1 w1(sx) w1(sy)) r from 0.0 (k_residual_restrict).
// Global traffic per level vertex: x and f read once (+ the recomputed rows' re-reads, L2 hits),
// x written once, f_c and x_c.
//
// k_prolong_quads2d is the mirror image on the way up: the prolongate-add x += alpha P x_c
// (intergrid_operator.hh:106-120, multigridmc_sampler.cc:124-127) and the first post-sweep in one
// launch.  A workgroup owns fine rows lo .. hi, stages old x on rows lo-2 .. hi+2 and the coarse rows
// under them, adds the prolongation to every staged interior vertex (k_prolongate_pairs' terms and
// order), runs the first colour pair on rows lo-1 .. hi+1 and the second on lo .. hi, and stores its
// own rows out of place.
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

struct QRestrictArgs {
    Layout L, Lc;
    const double* xin;
    double* xout;
    const double* f;
    double* fc;
    double* xc;
    StencilArg S;
    GibbsArg G;
    int CJ;             // coarse rows per workgroup
    long long cs, csc;  // batched chains: doubles between chains of the level / the coarse level
};

// rows of the LDS buffers for CJ coarse rows: old / swept x, f, residual
inline int qr_xrows(int CJ) { return 2 * CJ + 7; }
inline int qr_frows(int CJ) { return 2 * CJ + 5; }
inline int qr_rrows(int CJ) { return 2 * CJ + 1; }
// LDS row: positions -1 .. nx+2 at index i + 1 (nx + 4 doubles)
inline size_t qrestrict_lds_bytes(int nx, int CJ) {
    return (size_t)(qr_xrows(CJ) + qr_frows(CJ) + qr_rrows(CJ)) * (size_t)(nx + 4) * sizeof(double);
}

// NT >= (CJ + 3) * nx / 2: one pair item per thread in every colour phase
template <int NT, bool FIRST_ODD>
__global__ void __launch_bounds__(NT) k_quads_restrict2d(QRestrictArgs a) {
    {
        const int ch = batch_chain();
        a.xin += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        a.fc += ch * a.csc;
        a.xc += ch * a.csc;
        a.G.key = chain_key(a.G, ch);
    }
    extern __shared__ __attribute__((aligned(16))) double qsm[];
    const Layout& L = a.L;
    const Layout& Lc = a.Lc;
    const int CJ = a.CJ;
    const int npair = L.nx / 2;
    const int RW = L.nx + 4;
    const int NXR = 2 * CJ + 7, NFR = 2 * CJ + 5, NRR = 2 * CJ + 1;
    double* xs = qsm;               // rows xr0 .. xr0 + NXR - 1
    double* fs = xs + NXR * RW;     // rows xr0 + 1 .. xr0 + NFR
    double* rs = fs + NFR * RW;     // rows 2J0-1 .. 2J0+2CJ-1
    const int J0 = 1 + (int)blockIdx.x * CJ;
    const int xr0 = 2 * J0 - 4;     // fine row of LDS x row 0 (f row 0 is xr0 + 1)
    const int tid = threadIdx.x;
    const int jp1 = FIRST_ODD ? 1 : 0;  // forward: colours (0,1) on even rows first; backward (3,2) on odd rows
    auto X = [&](int j, int i) -> double& { return xs[(j - xr0) * RW + i + 1]; };

    // ---- stage old x (rows xr0 .. xr0+NXR-1) and f (rows xr0+1 .. xr0+NFR) as 16-byte pairs
    // (i odd, i+1) from i = -1; rows outside [0, ny] are clamped onto the zero boundary rows ----
    const int ppr = npair + 2;  // pairs per staged row: starts -1, 1, ..., nx+1
    for (int it = tid; it < (NXR + NFR) * ppr; it += NT) {
        const bool isf = it >= NXR * ppr;
        const int u = isf ? it - NXR * ppr : it;
        const int r = u / ppr, c = u - r * ppr;
        const int j = xr0 + r + (isf ? 1 : 0);
        const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
        const double* src = (isf ? a.f : a.xin) + L.at(2 * c - 1, jc, 0);
        const double2 v = *reinterpret_cast<const double2*>(src);
        double* dst = (isf ? fs : xs) + r * RW + 2 * c;
        dst[0] = v.x;
        dst[1] = v.y;
    }

    // ---- the Box-Muller pairs of this thread's item in each of the two phases (no data needed) ----
    const int m = tid % npair, trow = tid / npair;
    const int i0 = 2 * m + 1;
    auto phase_row = [&](int ph) {  // fine row of this thread's item in phase ph (0: jp1 rows, 1: jp2)
        const int lo = ph == 0 ? 2 * J0 - 3 : 2 * J0 - 2;
        const int par = ph == 0 ? jp1 : 1 - jp1;
        return lo + ((lo & 1) != par ? 1 : 0) + 2 * trow;
    };
    auto phase_hi = [&](int ph) { return ph == 0 ? 2 * J0 + 2 * CJ + 1 : 2 * J0 + 2 * CJ; };
    const uint64_t sample = *a.G.sample;
    double z[2][2];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
        const int j = phase_row(ph);
        z[ph][0] = z[ph][1] = 0.0;
        if (j >= 1 && j <= L.ny - 1 && j <= phase_hi(ph)) {
            const Philox4 rnd = philox4x32_10(pair_id<2>(L, i0, j, 0), a.G.tag, (uint32_t)sample,
                                              (uint32_t)(sample >> 32), a.G.key.k0, a.G.key.k1);
            normal_pair(rnd, &z[ph][0], &z[ph][1]);
        }
    }
    __syncthreads();

    const double sd = a.G.sd, wd = a.G.wd;
    // one vertex update at (j, i) in LDS, Box-Muller value zv
    auto update = [&](int j, int i, double zv) {
        double res = a.S.a[0] * X(j - 1, i - 1);
#pragma unroll
        for (int q = 1; q < 9; ++q) res = fma(a.S.a[q], X(j + q / 3 - 1, i + q % 3 - 1), res);
        const double c = fma(sd, zv, fs[(j - xr0 - 1) * RW + i + 1]);
        X(j, i) = fma(wd, c - res, X(j, i));
    };
    // ---- four colour passes: (phase, element) = (0, first), (0, second), (1, first), (1, second) ----
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
        const int j = phase_row(ph);
        const bool go = j >= 1 && j <= L.ny - 1 && j <= phase_hi(ph);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool odd = (e == 0) == FIRST_ODD;  // this pass updates the odd position i0
            const int i = odd ? i0 : i0 + 1;
            if (go && i <= L.nx - 1) update(j, i, odd ? z[ph][0] : z[ph][1]);
            __syncthreads();
        }
    }

    // ---- residual of rows 2J0-1 .. 2J0+2CJ-1 (interior columns) ----
    const int rr0 = 2 * J0 - 1;
    for (int it = tid; it < NRR * (L.nx - 1); it += NT) {
        const int r = it / (L.nx - 1), i = 1 + it - r * (L.nx - 1);
        const int j = rr0 + r;
        double y = 0.0;
#pragma unroll
        for (int q = 0; q < 9; ++q) y += a.S.a[q] * X(j + q / 3 - 1, i + q % 3 - 1);
        rs[r * RW + i + 1] = fs[(j - xr0 - 1) * RW + i + 1] - y;
    }
    __syncthreads();

    // ---- restriction of coarse rows J0 .. J0+CJ-1: f_c, x_c = 0 ----
    const int ncx = Lc.nx - 1;
    for (int it = tid; it < CJ * ncx; it += NT) {
        const int cj = it / ncx, I = 1 + it - cj * ncx;
        const int J = J0 + cj;
        if (J > Lc.ny - 1) continue;
        const double* rc = rs + (2 * J - rr0) * RW + 2 * I + 1;
        double result = 0.0;
#pragma unroll
        for (int sy = -1; sy <= 1; ++sy)
#pragma unroll
            for (int sx = -1; sx <= 1; ++sx) {
                double w = 1.0;
                w *= w1(sx);
                w *= w1(sy);
                result += w * rc[sy * RW + sx];
            }
        const long long pc = Lc.at(I, J, 0);
        a.fc[pc] = result;
        a.xc[pc] = 0.0;
    }

    // ---- own fine rows out of place: pairs (i odd, i+1), i = 1 .. nx-1 ----
    const int olo = 2 * J0 - 1;
    const int ohi = (J0 + CJ - 1 >= Lc.ny - 1) ? L.ny : 2 * (J0 + CJ) - 1;  // one past the last own row
    for (int it = tid; it < (ohi - olo) * npair; it += NT) {
        const int r = it / npair, mm = it - r * npair;
        const int j = olo + r;
        const double* s = &X(j, 2 * mm + 1);
        *reinterpret_cast<double2*>(a.xout + L.at(2 * mm + 1, j, 0)) = make_double2(s[0], s[1]);
    }
}

// ---- prolongate-add + first post-sweep (2D Galerkin level) ----
struct QProlongArgs {
    Layout L, Lc;
    const double* xin;  // x before the prolongation
    double* xout;
    const double* f;
    const double* xc;   // coarse correction
    double alpha;       // coarse_scaling
    StencilArg S;
    GibbsArg G;
    int CJ;             // the workgroup's own fine rows: 2 CJ (2J0-1 .. 2J0+2CJ-2), the last one to ny-1
    long long cs, csc;
};

inline int qp_xrows(int CJ) { return 2 * CJ + 5; }
inline int qp_crows(int CJ) { return CJ + 4; }
// fine rows as in k_quads_restrict2d (nx + 4 doubles), coarse rows positions -1 .. nc+2 (nc + 4)
inline size_t qprolong_lds_bytes(int nx, int CJ) {
    return ((size_t)(qp_xrows(CJ) + qp_xrows(CJ) - 2) * (size_t)(nx + 4) + (size_t)qp_crows(CJ) * (nx / 2 + 4)) *
           sizeof(double);
}

// NT >= (CJ + 2) * nx / 2: one pair item per thread in every colour phase
template <int NT, bool FIRST_ODD>
__global__ void __launch_bounds__(NT) k_prolong_quads2d(QProlongArgs a) {
    {
        const int ch = batch_chain();
        a.xin += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        a.xc += ch * a.csc;
        a.G.key = chain_key(a.G, ch);
    }
    extern __shared__ __attribute__((aligned(16))) double qsm[];
    const Layout& L = a.L;
    const Layout& Lc = a.Lc;
    const int CJ = a.CJ;
    const int npair = L.nx / 2;
    const int RW = L.nx + 4, RWC = Lc.nx + 4;
    const int NXR = 2 * CJ + 5, NFR = 2 * CJ + 3, NCR = CJ + 4;
    double* xs = qsm;             // fine rows xr0 .. xr0 + NXR - 1
    double* fs = xs + NXR * RW;   // fine rows xr0 + 1 .. xr0 + NFR
    double* cs = fs + NFR * RW;   // coarse rows cr0 .. cr0 + NCR - 1
    const int J0 = 1 + (int)blockIdx.x * CJ;
    const int lo = 2 * J0 - 1;
    const int hi = (J0 + CJ - 1 >= Lc.ny - 1) ? L.ny - 1 : 2 * J0 + 2 * CJ - 2;  // own rows lo .. hi
    const int xr0 = lo - 2;
    const int cr0 = J0 - 2;       // coarse rows (lo-2)>>1 .. ((hi+2)>>1)+1 lie in cr0 .. cr0+NCR-1
    const int tid = threadIdx.x;
    const int jp1 = FIRST_ODD ? 1 : 0;
    auto X = [&](int j, int i) -> double& { return xs[(j - xr0) * RW + i + 1]; };

    // ---- stage old x, f and the coarse rows (16-byte pairs from position -1, rows clamped) ----
    const int ppr = npair + 2, pprc = Lc.nx / 2 + 2;
    const int nfine = (NXR + NFR) * ppr;
    for (int it = tid; it < nfine + NCR * pprc; it += NT) {
        const double* src;
        double* dst;
        if (it < nfine) {
            const bool isf = it >= NXR * ppr;
            const int u = isf ? it - NXR * ppr : it;
            const int r = u / ppr, c = u - r * ppr;
            const int j = xr0 + r + (isf ? 1 : 0);
            const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
            src = (isf ? a.f : a.xin) + L.at(2 * c - 1, jc, 0);
            dst = (isf ? fs : xs) + r * RW + 2 * c;
        } else {
            const int u = it - nfine;
            const int r = u / pprc, c = u - r * pprc;
            const int jj = cr0 + r;
            const int jc = jj < 0 ? 0 : (jj > Lc.ny ? Lc.ny : jj);
            src = a.xc + Lc.at(2 * c - 1, jc, 0);
            dst = cs + r * RWC + 2 * c;
        }
        const double2 v = *reinterpret_cast<const double2*>(src);
        dst[0] = v.x;
        dst[1] = v.y;
    }
    // ---- Box-Muller pairs of this thread's item in each phase (no data needed) ----
    const int m = tid % npair, trow = tid / npair;
    const int i0 = 2 * m + 1;
    auto phase_row = [&](int ph) {  // phase 0: jp1 rows from lo-1; phase 1: jp2 rows from lo
        const int first = ph == 0 ? lo - 1 : lo;
        const int par = ph == 0 ? jp1 : 1 - jp1;
        return first + ((first & 1) != par ? 1 : 0) + 2 * trow;
    };
    auto phase_hi = [&](int ph) { return ph == 0 ? hi + 1 : hi; };
    const uint64_t sample = *a.G.sample;
    double z[2][2];
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
        const int j = phase_row(ph);
        z[ph][0] = z[ph][1] = 0.0;
        if (j >= 1 && j <= L.ny - 1 && j <= phase_hi(ph)) {
            const Philox4 rnd = philox4x32_10(pair_id<2>(L, i0, j, 0), a.G.tag, (uint32_t)sample,
                                              (uint32_t)(sample >> 32), a.G.key.k0, a.G.key.k1);
            normal_pair(rnd, &z[ph][0], &z[ph][1]);
        }
    }
    __syncthreads();

    // ---- x += alpha P x_c on every staged interior vertex: k_prolongate_pairs' terms in its order
    // (coarse rows jj ascending, parents q then q+1; (alpha w) x_c added, w = 1 * w1(dx) * w1(dy)) ----
    const int ncx = Lc.nx - 1;
    for (int it = tid; it < NXR * npair; it += NT) {
        const int r = it / npair, q = it - r * npair;
        const int j = xr0 + r;
        if (j < 1 || j > L.ny - 1) continue;
        const int i = 2 * q + 1;
        double* px = &X(j, i);
        double vx = px[0], vy = px[1];
        const bool has1 = i + 1 <= L.nx - 1;
        const int j0 = j >> 1, nj = (j & 1) ? 2 : 1;
        for (int b = 0; b < nj; ++b) {
            const int jj = j0 + b;
            if (jj < 1 || jj > Lc.ny - 1) continue;
            const double* row = cs + (jj - cr0) * RWC + 1;  // row[ii] = coarse position ii
            if (q >= 1) {
                double w = 1.0;
                w *= 0.5;
                w *= w1(j - 2 * jj);
                vx += a.alpha * w * row[q];
            }
            if (q + 1 <= ncx) {
                double w = 1.0;
                w *= 0.5;
                w *= w1(j - 2 * jj);
                vx += a.alpha * w * row[q + 1];
                if (has1) {
                    double w2 = 1.0;
                    w2 *= 1.0;
                    w2 *= w1(j - 2 * jj);
                    vy += a.alpha * w2 * row[q + 1];
                }
            }
        }
        px[0] = vx;
        px[1] = vy;
    }
    __syncthreads();

    const double sd = a.G.sd, wd = a.G.wd;
    auto update = [&](int j, int i, double zv) {
        double res = a.S.a[0] * X(j - 1, i - 1);
#pragma unroll
        for (int q = 1; q < 9; ++q) res = fma(a.S.a[q], X(j + q / 3 - 1, i + q % 3 - 1), res);
        const double c = fma(sd, zv, fs[(j - xr0 - 1) * RW + i + 1]);
        X(j, i) = fma(wd, c - res, X(j, i));
    };
#pragma unroll
    for (int ph = 0; ph < 2; ++ph) {
        const int j = phase_row(ph);
        const bool go = j >= 1 && j <= L.ny - 1 && j <= phase_hi(ph);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const bool odd = (e == 0) == FIRST_ODD;
            const int i = odd ? i0 : i0 + 1;
            if (go && i <= L.nx - 1) update(j, i, odd ? z[ph][0] : z[ph][1]);
            __syncthreads();
        }
    }

    // ---- own rows out of place ----
    for (int it = tid; it < (hi - lo + 1) * npair; it += NT) {
        const int r = it / npair, mm = it - r * npair;
        const int j = lo + r;
        const double* sv = &X(j, 2 * mm + 1);
        *reinterpret_cast<double2*>(a.xout + L.at(2 * mm + 1, j, 0)) = make_double2(sv[0], sv[1]);
    }
}

}  // namespace mgmc
