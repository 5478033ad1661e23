// mgmc_zsweepres.hpp -- fine 3D 7-point level: the last pre-sweep fused with the residual and the
// restriction, in one z-march over x and f.
//
//   x  <- one SOR Gibbs sweep of x (sampler/sor_sampler.cc:37-59, red-black order)
//   f_c = R (f - A x),  x_c = 0           (sampler/multigridmc_sampler.cc:118-122)
//
// k_zsweep_rb7 followed by k_zresrestrict reads x and f twice (24 + 16 B per fine unknown); this
// kernel reads them once (24 B + 2 B for f_c and x_c).  Every value is computed with the arithmetic of
// those two kernels, so the result is bitwise the same.
//
// Tiling.  A workgroup owns CX x CY coarse points of a chunk of kz coarse planes.  Its fine region:
//  * output (stored x): pair columns [0, CX) x rows [0, 2CY) x planes [2K0-1, 2K1-2], pair column c
//    holding positions (2I0-1+2c, 2I0+2c), row r the fine row 2J0-1+r -- a partition of the fine
//    interior (the last tile of a direction also owns the one position / row / plane past it when the
//    coarse points end exactly at the boundary);
//  * residual: columns [0, CX], rows [0, 2CY], planes [2K0-1, 2K1-1] (the 3^3 restriction footprint);
//  * final x (both colours) is needed one vertex further: second-colour updates on columns [-1, CX] x
//    rows [-1, 2CY+1] x planes [2K0-2, 2K1]; first colour on columns [-1, CX+1] x rows [-2, 2CY+2];
//    old x staged on columns [-2, CX+1] x rows [-3, 2CY+3].  Halo values are recomputed, tiles are
//    independent (x_out never aliases x_in).
// The z-march is that of k_zsweep_rb7: step p updates the first colour on plane p and the second
// colour on plane p-1, in a 3-slot LDS plane ring.  Here the second-colour values are written back
// into the ring (no update reads an old second-colour value after that point), so plane p-1 is final
// in LDS for the residual.  The residual of plane q is accumulated in registers in the reference's
// term order as its planes become final: 0 + a4 x(q-1) at step q, the five in-plane terms at step q+1,
// + a22 x(q+1) and r = f - y at step q+2 (f(q) is kept two steps in registers).  Residuals of a plane
// go to one LDS plane and every coarse point adds its 9 weighted terms per plane to a register
// accumulator, sz outermost: exactly k_zresrestrict's (and the reference's) order.
#pragma once
#include "mgmc_zsweep.hpp"

namespace mgmc {

struct ZSweepResArgs {
    Layout L, Lc;
    const double* xin;
    double* xout;
    const double* f;
    double* fc;
    double* xc;
    StencilArg S;
    GibbsArg G;
    int kz;  // coarse planes per chunk
    int ntx, nty, ntz;
};

template <int CX, int CY, int NT>
__global__ void __launch_bounds__(NT) k_zsweep_res7(ZSweepResArgs a) {
    constexpr int WP = CX + 4;                       // staged pair columns [-2, CX+1]
    constexpr int RS = 2 * WP + 2;                   // LDS row [odd | even | 2 pad]
    constexpr int R = 2 * CY + 7;                    // staged rows [-3, 2CY+3]
    constexpr int PS = R * RS;
    constexpr int NRES = (CX + 1) * (2 * CY + 1);    // residual items
    constexpr int NSEC = (CX + 2) * (2 * CY + 3);    // second-colour items (residual items first)
    constexpr int NFIR = (CX + 3) * (2 * CY + 5);    // first-colour items (second-colour items first)
    constexpr int NI = (NFIR + NT - 1) / NT;         // item slots per thread
    constexpr int NLX = (R * WP + NT - 1) / NT;      // x pair loads per plane per thread
    constexpr int RP = CX + 1, RSr = 2 * RP + 2;     // residual plane row (odd | even | pad)
    constexpr int NCP = (CX * CY + NT - 1) / NT;     // coarse points per thread
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                         // [3][R][RS] x planes p-1, p, p+1
    double* rs = xs + 3 * PS;                  // [2CY+1][RSr] residual plane
    double* tab = rs + (2 * CY + 1) * RSr;     // log (rc, hi, lo) + sincos tables
    for (int q = threadIdx.x; q < 64; q += NT) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }
    for (int q = threadIdx.x; q < 130; q += NT) tab[192 + q] = SINCOS_TAB[q];

    const Layout& L = a.L;
    const Layout& Lc = a.Lc;
    const int nb = gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);  // XCD-aware order
    const int txi = tile % a.ntx;
    const int tyi = (tile / a.ntx) % a.nty;
    const int tzi = tile / (a.ntx * a.nty);
    if (tzi >= a.ntz) return;
    const int I0 = 1 + txi * CX, J0 = 1 + tyi * CY;
    const int K0 = 1 + tzi * a.kz, K1 = min(K0 + a.kz, Lc.nz);  // coarse planes [K0, K1)
    const int i0 = 2 * I0 - 1;  // odd position of pair column 0
    const int j0 = 2 * J0 - 1;  // fine row of row 0
    const int kq0 = 2 * K0 - 1, kq1 = 2 * K1 - 1;             // residual planes [kq0, kq1]
    const int ko0 = kq0, ko1 = (kq1 == L.nz - 1) ? kq1 : kq1 - 1;  // owned planes [ko0, ko1]
    const int fc = a.G.colour;
    const double sd = a.G.sd, wd = a.G.wd;
    const uint64_t sample = *a.G.sample;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    const uint32_t plane_pairs = (uint32_t)((uint64_t)(L.ny - 1) * (uint64_t)(L.nx / 2));
    const int tid = threadIdx.x;

    auto slot = [](int p) { return (p + 9) % 3; };
    auto interior_plane = [&](int k) { return k >= 1 && k <= L.nz - 1; };
    auto plane_base = [&](const double* v, int k) { return v + (long long)(k < 0 ? 0 : (k > L.nz ? L.nz : k)) * L.sp; };

    // ---- items: flags bit0 row interior, bit1 i interior, bit2 i+1 interior, bit3 parity (i+j)&1,
    //      bit4 second-colour item, bit5 residual item, bit6 first-colour item, bit7 stored (owned) ----
    constexpr int F_SEC = 16, F_RES = 32, F_FIR = 64, F_OWN = 128;
    long long igoff[NI];
    uint32_t ipb[NI];
    int ilds[NI], iflg[NI], irs[NI];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        int it = tid + u * NT;
        int c = 0, r = 0, fl = 0;
        if (it < NRES) {
            r = it / (CX + 1);
            c = it - r * (CX + 1);
            fl = F_RES | F_SEC | F_FIR;
        } else if (it < NSEC) {
            it -= NRES;
            if (it < CX + 2) { r = -1; c = it - 1; }
            else if (it < 2 * (CX + 2)) { r = 2 * CY + 1; c = it - (CX + 2) - 1; }
            else { r = it - 2 * (CX + 2); c = -1; }
            fl = F_SEC | F_FIR;
        } else if (it < NFIR) {
            it -= NSEC;
            if (it < CX + 3) { r = -2; c = it - 1; }
            else if (it < 2 * (CX + 3)) { r = 2 * CY + 2; c = it - (CX + 3) - 1; }
            else { r = it - 2 * (CX + 3) - 1; c = CX + 1; }
            fl = F_FIR;
        }
        const int i = i0 + 2 * c, j = j0 + r;
        const bool rin = j >= 1 && j <= L.ny - 1;
        const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
        igoff[u] = (long long)jc * L.sx + i + L.off;
        ipb[u] = (uint32_t)((uint64_t)(j - 1) * (uint64_t)(L.nx / 2) + (uint64_t)((i - 1) >> 1));
        ilds[u] = (r + 3) * RS + (c + 2);
        irs[u] = r * RSr + c;
        const bool colown = (c >= 0 && c < CX) || (c == CX && i == L.nx - 1);
        const bool rowown = (r >= 0 && r < 2 * CY) || (r == 2 * CY && j == L.ny - 1);
        if (fl & F_SEC && colown && rowown) fl |= F_OWN;
        if (fl) fl |= (rin ? 1 : 0) | ((i >= 1 && i <= L.nx - 1) ? 2 : 0) | ((i + 1 >= 1 && i + 1 <= L.nx - 1) ? 4 : 0) |
                      (((i + j) & 1) << 3);
        iflg[u] = fl;
    }
    long long xoff[NLX];
    int xlds[NLX];
#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int it = tid + u * NT;
        xoff[u] = L.off + 1;  // spare threads load a zero pad pair and deposit nothing
        xlds[u] = -1;
        if (it < R * WP) {
            const int rr = it / WP, c2 = it - rr * WP;
            const int j = j0 - 3 + rr;
            const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
            xlds[u] = rr * RS + c2;
            xoff[u] = (long long)jc * L.sx + (i0 - 4 + 2 * c2) + L.off;
        }
    }
    int cpo[NCP];
    long long cpg[NCP];
    bool cpin[NCP];
#pragma unroll
    for (int u = 0; u < NCP; ++u) {
        const int it = tid + u * NT;
        const int cy = it / CX, cx = it - cy * CX;
        cpin[u] = it < CX * CY && I0 + cx <= Lc.nx - 1 && J0 + cy <= Lc.ny - 1;
        cpo[u] = (2 * cy + 1) * RSr + cx;
        cpg[u] = cpin[u] ? Lc.at(I0 + cx, J0 + cy, 0) : 0;
    }

    double2 px[NLX];
    auto issue_x = [&](int k) {
        const double* base = plane_base(a.xin, k);
#pragma unroll
        for (int u = 0; u < NLX; ++u) px[u] = *reinterpret_cast<const double2*>(base + xoff[u]);
    };
    auto deposit_x = [&](int k) {
        double* dst = xs + slot(k) * PS;
#pragma unroll
        for (int u = 0; u < NLX; ++u) {
            if (xlds[u] < 0) continue;
            dst[xlds[u]] = px[u].x;
            dst[xlds[u] + WP] = px[u].y;
        }
    };
    auto load_f = [&](int k, double2 (&dst)[NI]) {
        const double* base = plane_base(a.f, k);
#pragma unroll
        for (int u = 0; u < NI; ++u) dst[u] = *reinterpret_cast<const double2*>(base + igoff[u]);
    };

    // Gibbs sweep arithmetic: that of k_zsweep_rb7 (folded symmetric 7-point stencil, fma chain)
    const double cz = a.S.a[4], cy = a.S.a[10], cx = a.S.a[12], cc = a.S.a[13];
    auto row_sum = [&](int k, int o, int e, double below) {
        const double* s0 = xs + slot(k) * PS;
        const double* sp = xs + slot(k + 1) * PS;
        const int xm = e ? o - WP : o + WP - 1;
        double res = cz * below;
        res = fma(cy, s0[o - RS], res);
        res = fma(cx, s0[xm], res);
        res = fma(cc, s0[o], res);
        res = fma(cx, s0[xm + 1], res);
        res = fma(cy, s0[o + RS], res);
        res = fma(cz, sp[o], res);
        return res;
    };
    auto first_pair = [&](int k, int u, double2 fv) -> double {
        const int fl = iflg[u];
        if (!(fl & F_FIR) || !(fl & 1) || !(fl & 6)) return 0.0;
        const int e = (((fl >> 3) ^ k) & 1) == fc ? 0 : 1;
        const uint32_t pair = (uint32_t)(k - 1) * plane_pairs + ipb[u];
        uint32_t key0 = a.G.key.k0, key1 = a.G.key.k1;
        asm volatile("" : "+s"(key0), "+s"(key1));
        const Philox4 rnd = philox4x32_10(pair, a.G.tag, s_lo, s_hi, key0, key1);
        double z0, z1;
        normal_pair_t(rnd, &z0, &z1, tab, tab + 64, tab + 128, tab + 192);
        if (fl & (2 << e)) {
            const int o = ilds[u] + (e ? WP : 0);
            const double res = row_sum(k, o, e, xs[slot(k - 1) * PS + o]);
            const double crhs = fma(sd, e == 0 ? z0 : z1, e == 0 ? fv.x : fv.y);
            double* s0 = xs + slot(k) * PS;
            s0[o] = fma(wd, crhs - res, s0[o]);
        }
        return e == 0 ? fma(sd, z1, fv.y) : fma(sd, z0, fv.x);
    };

    // residual terms (k_zresrestrict order): y = 0 + a4 x(k-1); y += a10, a12, a13, a14, a16 terms
    // of plane k; y += a22 x(k+1); r = f - y
    const double r4 = a.S.a[4], r10 = a.S.a[10], r12 = a.S.a[12], r13 = a.S.a[13], r14 = a.S.a[14],
                 r16 = a.S.a[16], r22 = a.S.a[22];
    auto accumulate = [&](double (&acc)[NCP], int sz) {
#pragma unroll
        for (int u = 0; u < NCP; ++u) {
            double result = acc[u];
#pragma unroll
            for (int sy = -1; sy <= 1; ++sy)
#pragma unroll
                for (int sx = -1; sx <= 1; ++sx) {
                    double w = 1.0;
                    w *= w1(sx);
                    w *= w1(sy);
                    w *= w1(sz - 1);
                    result += w * rs[cpo[u] + sy * RSr + (sx < 0 ? 0 : (sx == 0 ? RP : 1))];
                }
            acc[u] = result;
        }
    };
    auto finish = [&](const double (&acc)[NCP], int K) {
        const long long pk = (long long)K * Lc.sp;
#pragma unroll
        for (int u = 0; u < NCP; ++u)
            if (cpin[u]) {
                a.fc[pk + cpg[u]] = acc[u];
                a.xc[pk + cpg[u]] = 0.0;
            }
    };

    // registers carried between steps (p = current step)
    double2 fnxt[NI], fcur[NI], fm1[NI], fm2[NI];  // f(p+1), f(p), f(p-1), f(p-2) at the items
    double pk[NI], fb[NI];                          // second-colour rhs of plane p-1; first colour of p-2
    double2 ya[NI], yb[NI];                         // residual partial sums of planes p-2 (a) and p-1 (b)
    double acc[NCP];
#pragma unroll
    for (int u = 0; u < NI; ++u) {
        pk[u] = fb[u] = 0.0;
        ya[u] = yb[u] = make_double2(0.0, 0.0);
        fm1[u] = fm2[u] = make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < NCP; ++u) acc[u] = 0.0;

    const int ps = kq0 - 2, pe = kq1 + 2;  // first colour from plane 2K0-3; the last step finishes r(2K1-1)
    issue_x(ps - 1);
    deposit_x(ps - 1);
    issue_x(ps);
    deposit_x(ps);
    issue_x(ps + 1);
    load_f(ps, fcur);
    for (int p = ps; p <= pe; ++p) {
        // P1: stage x(p+1), x(p+2) and f(p+1) in flight
        deposit_x(p + 1);
        issue_x(p + 2);
        load_f(p + 1, fnxt);
        __syncthreads();
        // P2: first colour on plane p
        double pko[NI];
        if (interior_plane(p)) {
#pragma unroll
            for (int u = 0; u < NI; ++u) pko[u] = first_pair(p, u, fcur[u]);
        } else {
#pragma unroll
            for (int u = 0; u < NI; ++u) pko[u] = 0.0;
        }
        __syncthreads();
        // P3: second colour on plane k = p-1 (written back: plane k is final in the ring), store
        const int k = p - 1;
        const bool need = k >= kq0 - 1 && k <= kq1 + 1 && interior_plane(k);
        const bool own = k >= ko0 && k <= ko1;
        double* sk = xs + slot(k) * PS;
        double* obase = a.xout + (long long)k * L.sp;
#pragma unroll
        for (int u = 0; u < NI; ++u) {
            const int fl = iflg[u];
            if (!(fl & F_SEC)) continue;
            const int ef = (((fl >> 3) ^ k) & 1) == fc ? 0 : 1;  // first-colour element on plane k
            const int e = 1 - ef;                                  // second-colour element
            const int o = ilds[u] + (e ? WP : 0);
            const double fv = sk[ilds[u] + (ef ? WP : 0)];
            double sv = sk[o];
            if (need && (fl & 1) && (fl & (2 << e))) {
                sv = fma(wd, pk[u] - row_sum(k, o, e, fb[u]), sv);
                sk[o] = sv;
            }
            fb[u] = fv;
            if (own && (fl & F_OWN) && (fl & 1)) {
                const double2 out = ef == 0 ? make_double2(fv, sv) : make_double2(sv, fv);
                __builtin_nontemporal_store(out.x, obase + igoff[u]);
                __builtin_nontemporal_store(out.y, obase + igoff[u] + 1);
            }
        }
        __syncthreads();
        // P4: residuals.  finish plane p-2, in-plane terms of plane p-1, start plane p
        const bool fin = p - 2 >= kq0 && p - 2 <= kq1;
        const bool mid = k >= kq0 && k <= kq1;
        const bool sta = p >= kq0 && p <= kq1;
#pragma unroll
        for (int u = 0; u < NI; ++u) {
            const int fl = iflg[u];
            if (!(fl & F_RES)) continue;
            const int o0 = ilds[u], o1 = ilds[u] + WP;
            const double x0 = sk[o0], x1 = sk[o1];
            if (fin) {
                double y0 = ya[u].x, y1 = ya[u].y;
                y0 += r22 * x0;
                y1 += r22 * x1;
                rs[irs[u]] = ((fl & 1) && (fl & 2)) ? fm2[u].x - y0 : 0.0;
                rs[irs[u] + RP] = ((fl & 1) && (fl & 4)) ? fm2[u].y - y1 : 0.0;
            }
            if (mid) {
                const int m0 = o0 + WP - 1, m1 = o1 - WP;
                double y0 = yb[u].x, y1 = yb[u].y;
                y0 += r10 * sk[o0 - RS];
                y1 += r10 * sk[o1 - RS];
                y0 += r12 * sk[m0];
                y1 += r12 * sk[m1];
                y0 += r13 * x0;
                y1 += r13 * x1;
                y0 += r14 * sk[m0 + 1];
                y1 += r14 * sk[m1 + 1];
                y0 += r16 * sk[o0 + RS];
                y1 += r16 * sk[o1 + RS];
                ya[u] = make_double2(y0, y1);
            }
            if (sta) {
                double y0 = 0.0, y1 = 0.0;
                y0 += r4 * x0;
                y1 += r4 * x1;
                yb[u] = make_double2(y0, y1);
            }
        }
        // the next step's deposit overwrites the slot of plane p-1 read above; the residual plane is read below
        __syncthreads();
        if (fin) {
            // P5: restriction terms of residual plane q = p-2 (sz = 0, 1, 2 of coarse plane q>>1 ...)
            const int q = p - 2;
            if (q == kq0) {
                accumulate(acc, 0);
            } else if (!(q & 1)) {
                accumulate(acc, 1);
            } else {
                accumulate(acc, 2);
                finish(acc, (q - 1) >> 1);
#pragma unroll
                for (int u = 0; u < NCP; ++u) acc[u] = 0.0;
                accumulate(acc, 0);
            }
        }
        // rotate the carried registers
#pragma unroll
        for (int u = 0; u < NI; ++u) {
            pk[u] = pko[u];
            fm2[u] = fm1[u];
            fm1[u] = fcur[u];
            fcur[u] = fnxt[u];
        }
    }
}

inline size_t zsweepres_lds_bytes(int CX, int CY) {
    const int RS = 2 * (CX + 4) + 2, R = 2 * CY + 7, RSr = 2 * (CX + 1) + 2;
    return (size_t)(3 * R * RS + (2 * CY + 1) * RSr + 3 * 64 + 130) * sizeof(double);
}

}  // namespace mgmc
