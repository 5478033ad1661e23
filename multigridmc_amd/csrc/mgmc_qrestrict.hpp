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
    // when the coarse level is the coarsest and its SSOR sampler follows (k_coarse_ssor_lds<..., ZBUF>):
    // workgroups nblk_main .. of the grid draw that sampler's Box-Muller pairs into zc (its item
    // order; tags zc_tag, zc_tag + 1, ...), in parallel with the restriction -- they depend on no data
    int nblk_main;
    double2* zc;
    int zc_nsweeps;
    uint32_t zc_tag;
    long long zcs;      // zc doubles2 per chain
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
    if ((int)blockIdx.x >= a.nblk_main) {  // the coarsest level's noise (see QRestrictArgs)
        const Layout& Lc = a.Lc;
        const uint64_t sample = *a.G.sample;
        const int nxi = Lc.nx - 1, nyi = Lc.ny - 1, npair = Lc.nx / 2;
        const int n = a.zc_nsweeps * nyi * npair;
        double2* z = a.zc + batch_chain() * a.zcs;
        for (int t = ((int)blockIdx.x - a.nblk_main) * NT + (int)threadIdx.x; t < n;
             t += ((int)gridDim.x - a.nblk_main) * NT) {
            const int m = t % npair, rt = t / npair;
            const int row = rt % nyi, sw = rt / nyi;
            const int i0 = 2 * m + 1;
            if (i0 > nxi) continue;
            const Philox4 rnd = philox4x32_10(pair_id<2>(Lc, i0, row + 1, 0), a.zc_tag + (uint32_t)sw,
                                              (uint32_t)sample, (uint32_t)(sample >> 32), a.G.key.k0, a.G.key.k1);
            double z0, z1;
            normal_pair(rnd, &z0, &z1);
            z[t] = make_double2(z0, z1);
        }
        return;
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

}  // namespace mgmc
