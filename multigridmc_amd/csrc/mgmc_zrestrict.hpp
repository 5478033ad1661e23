// mgmc_zrestrict.hpp -- z-marching fused residual + restriction for 3D levels.
//
//   f_c = R (f - A x),  x_c = 0           (sampler/multigridmc_sampler.cc:118-122)
//
// Each workgroup owns CX x CY coarse points and marches a chunk of coarse planes K.  The fine
// residual r = f - A x is evaluated exactly once per fine vertex (plus a one-vertex tile overlap)
// into an LDS ring of three residual planes (fine planes 2K-1, 2K, 2K+1; plane 2K+1 is reused by
// coarse plane K+1), from x planes staged in an LDS ring with a one-vertex halo.  The restriction
// then reads the 3^3 weighted residuals from LDS.  Arithmetic is the reference's, in the
// reference's order (A x ascending from 0.0, r = f - Ax, restriction sum sigma with x fastest),
// so f_c is bitwise equal to k_residual_restrict and to the CPU oracle.
// Global traffic: x and f once (16 B per fine vertex) + f_c, x_c (2 B per fine vertex).
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

struct ZRestrictArgs {
    Layout Lf, Lc;
    const double* x;
    const double* f;
    double* fc;
    double* xc;
    StencilArg S;
    int kz;            // coarse planes per chunk
    int ntx, nty, ntz;
};

template <int NPTS, int CX, int CY, int NT>
__global__ void __launch_bounds__(NT) k_zresrestrict(ZRestrictArgs a) {
    // fine x range of the residual region: [2*I0-1, 2*I0+2*CX-1]; as pairs starting at odd
    // positions: RP = CX+1 pairs.  x is staged with one more vertex on each side: positions
    // [2*I0-3, 2*I0+2*CX+2] = XP = CX+3 pairs (starting at an odd position).
    constexpr int RP = CX + 1, RW = 2 * RP;      // residual row: pairs / doubles
    constexpr int RR = 2 * CY + 1;               // residual rows
    constexpr int XPP = CX + 3, XW = 2 * XPP;    // x row: pairs / doubles
    constexpr int XR = 2 * CY + 3;               // x rows
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                 // [4][XR][XW] x planes
    double* rs = xs + 4 * XR * XW;     // [3][RR][RW] residual planes

    const Layout& Lf = a.Lf;
    const Layout& Lc = a.Lc;
    const int nb = gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);
    const int txi = tile % a.ntx;
    const int tyi = (tile / a.ntx) % a.nty;
    const int tzi = tile / (a.ntx * a.nty);
    if (tzi >= a.ntz) return;
    const int I0 = 1 + txi * CX, J0 = 1 + tyi * CY;
    const int K0 = 1 + tzi * a.kz, K1 = min(K0 + a.kz, Lc.nz);  // coarse planes [K0, K1)
    const int xi0 = 2 * I0 - 3;  // fine position of x column 0
    const int xj0 = 2 * J0 - 2;  // fine row of x row 0
    const int ri0 = 2 * I0 - 1;  // fine position of r column 0
    const int rj0 = 2 * J0 - 1;  // fine row of r row 0
    const int tid = threadIdx.x;

    auto xslot = [](int k) { return (k + 8) & 3; };
    auto rslot = [](int k) { return (k + 9) % 3; };
    auto fine_row_in = [&](int j) { return j >= 1 && j <= Lf.ny - 1; };
    auto fine_plane_in = [&](int k) { return k >= 1 && k <= Lf.nz - 1; };

    // ---- register pipeline: x(2K+1), x(2K+2) and f(2K), f(2K+1) of step K are loaded during
    // step K-1 (into registers) and deposited / consumed at step K ----
    constexpr int NLX = (XR * XPP + NT - 1) / NT;  // x pair loads per plane per thread
    constexpr int NLR = (RR * RP + NT - 1) / NT;   // residual pair items per plane per thread
    long long xoff[NLX];
    int xlds[NLX];
#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int it = tid + u * NT;
        xoff[u] = -1;
        xlds[u] = -1;
        if (it < XR * XPP) {
            const int r = it / XPP, c2 = it - r * XPP;
            const int j = xj0 + r;
            xlds[u] = r * XW + 2 * c2;
            if (fine_row_in(j)) xoff[u] = (long long)j * Lf.sx + (xi0 + 2 * c2) + Lf.off;
        }
    }
    long long roff[NLR];
    int rlds[NLR], rflag[NLR];
#pragma unroll
    for (int u = 0; u < NLR; ++u) {
        const int it = tid + u * NT;
        roff[u] = -1;
        rlds[u] = -1;
        rflag[u] = 0;
        if (it < RR * RP) {
            const int r = it / RP, c2 = it - r * RP;
            const int j = rj0 + r, i = ri0 + 2 * c2;
            rlds[u] = r * RW + 2 * c2;
            if (fine_row_in(j)) {
                roff[u] = (long long)j * Lf.sx + i + Lf.off;
                rflag[u] = ((i >= 1 && i <= Lf.nx - 1) ? 1 : 0) | ((i + 1 <= Lf.nx - 1) ? 2 : 0);
            }
        }
    }
    double2 px[2][NLX], pf[2][NLR];
    auto issue_x = [&](int k, double2* dst) {
        const bool kin = fine_plane_in(k);
        const double* base = a.x + (long long)k * Lf.sp;
#pragma unroll
        for (int u = 0; u < NLX; ++u) {
            dst[u] = make_double2(0.0, 0.0);
            if (kin && xoff[u] >= 0) dst[u] = *reinterpret_cast<const double2*>(base + xoff[u]);
        }
    };
    auto deposit_x = [&](int k, const double2* src) {
        double* dst = xs + xslot(k) * XR * XW;
#pragma unroll
        for (int u = 0; u < NLX; ++u)
            if (xlds[u] >= 0) *reinterpret_cast<double2*>(dst + xlds[u]) = src[u];
    };
    auto issue_f = [&](int k, double2* dst) {
        const bool kin = fine_plane_in(k);
        const double* base = a.f + (long long)k * Lf.sp;
#pragma unroll
        for (int u = 0; u < NLR; ++u) {
            dst[u] = make_double2(0.0, 0.0);
            if (kin && roff[u] >= 0) dst[u] = *reinterpret_cast<const double2*>(base + roff[u]);
        }
    };
    // residual of fine plane k over the residual region (vertices outside the fine interior -> 0)
    auto residual = [&](int k, const double2* fv) {
        double* dst = rs + rslot(k) * RR * RW;
        const bool kin = fine_plane_in(k);
        const double* xm = xs + xslot(k - 1) * XR * XW;
        const double* x0 = xs + xslot(k) * XR * XW;
        const double* xp = xs + xslot(k + 1) * XR * XW;
#pragma unroll
        for (int u = 0; u < NLR; ++u) {
            if (rlds[u] < 0) continue;
            double2 out = make_double2(0.0, 0.0);
            if (kin) {
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    if (!(rflag[u] & (1 << e))) continue;
                    const int r = rlds[u] / RW, c = rlds[u] - r * RW + e;
                    const int o = (r + 1) * XW + c + 2;  // x LDS offset of the same vertex
                    double y = 0.0;
                    if (NPTS == 7) {
                        y += a.S.a[4] * xm[o];
                        y += a.S.a[10] * x0[o - XW];
                        y += a.S.a[12] * x0[o - 1];
                        y += a.S.a[13] * x0[o];
                        y += a.S.a[14] * x0[o + 1];
                        y += a.S.a[16] * x0[o + XW];
                        y += a.S.a[22] * xp[o];
                    } else {
                        const double* pl[3] = {xm, x0, xp};
#pragma unroll
                        for (int dz = 0; dz < 3; ++dz)
#pragma unroll
                            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                                for (int dx = -1; dx <= 1; ++dx)
                                    y += a.S.a[dz * 9 + (dy + 1) * 3 + (dx + 1)] * pl[dz][o + dy * XW + dx];
                    }
                    const double rv = (e == 0 ? fv[u].x : fv[u].y) - y;
                    if (e == 0) out.x = rv; else out.y = rv;
                }
            }
            *reinterpret_cast<double2*>(dst + rlds[u]) = out;
        }
    };
    auto restrict_plane = [&](int K) {
        const double* rm = rs + rslot(2 * K - 1) * RR * RW;
        const double* r0 = rs + rslot(2 * K) * RR * RW;
        const double* rp = rs + rslot(2 * K + 1) * RR * RW;
        const double* pl[3] = {rm, r0, rp};
        for (int it = tid; it < CX * CY; it += NT) {
            const int cy = it / CX, cx = it - cy * CX;
            const int I = I0 + cx, J = J0 + cy;
            if (I > Lc.nx - 1 || J > Lc.ny - 1) continue;
            const int o = (2 * cy + 1) * RW + 2 * cx + 1;  // r LDS offset of fine (2I, 2J)
            double result = 0.0;
#pragma unroll
            for (int sz = 0; sz < 3; ++sz)
#pragma unroll
                for (int sy = -1; sy <= 1; ++sy)
#pragma unroll
                    for (int sx = -1; sx <= 1; ++sx) {
                        double w = 1.0;
                        w *= w1(sx);
                        w *= w1(sy);
                        w *= w1(sz - 1);
                        result += w * pl[sz][o + sy * RW + sx];
                    }
            const long long pc = Lc.at(I, J, K);
            a.fc[pc] = result;
            a.xc[pc] = 0.0;
        }
    };

    // prologue: x planes 2K0-2 .. 2K0 and residual plane 2K0-1; step K0's loads in flight
    issue_x(2 * K0 - 2, px[0]);
    deposit_x(2 * K0 - 2, px[0]);
    issue_x(2 * K0 - 1, px[0]);
    deposit_x(2 * K0 - 1, px[0]);
    issue_x(2 * K0, px[0]);
    deposit_x(2 * K0, px[0]);
    issue_f(2 * K0 - 1, pf[0]);
    __syncthreads();
    residual(2 * K0 - 1, pf[0]);
    __syncthreads();  // the first deposit below overwrites the slot of x(2K0-2) read just above
    issue_x(2 * K0 + 1, px[0]);
    issue_x(2 * K0 + 2, px[1]);
    issue_f(2 * K0, pf[0]);
    issue_f(2 * K0 + 1, pf[1]);
    for (int K = K0; K < K1; ++K) {
        // x planes 2K-1, 2K in LDS; deposit 2K+1, 2K+2 (slots of 2K-3, 2K-2, free since the last barrier)
        deposit_x(2 * K + 1, px[0]);
        deposit_x(2 * K + 2, px[1]);
        double2 fa[NLR], fb[NLR];
#pragma unroll
        for (int u = 0; u < NLR; ++u) {
            fa[u] = pf[0][u];
            fb[u] = pf[1][u];
        }
        if (K + 1 < K1) {  // next step's loads, in flight during this step's compute
            issue_x(2 * K + 3, px[0]);
            issue_x(2 * K + 4, px[1]);
            issue_f(2 * K + 2, pf[0]);
            issue_f(2 * K + 3, pf[1]);
        }
        __syncthreads();
        residual(2 * K, fa);
        residual(2 * K + 1, fb);
        __syncthreads();
        restrict_plane(K);
        __syncthreads();
    }
}

inline size_t zrestrict_lds_bytes(int CX, int CY) {
    const int XW = 2 * (CX + 3), XR = 2 * CY + 3, RW = 2 * (CX + 1), RR = 2 * CY + 1;
    return (size_t)(4 * XR * XW + 3 * RR * RW) * sizeof(double);
}

}  // namespace mgmc
