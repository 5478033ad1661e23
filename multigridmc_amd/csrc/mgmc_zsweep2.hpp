// mgmc_zsweep2.hpp -- the fine post-sweep of cycle n and the fine pre-sweep of cycle n+1 in one
// z-march (temporal blocking across the cycle boundary).
//
// Between the post-sampler of one MGMC cycle (SORSampler::apply backward, with the prolongation of
// the coarse correction, multigridmc_sampler.cc:120-128) and the pre-sampler of the next cycle
// (forward, :117) nothing reads the fine state but the QoI record (driver_mgmc.cc:76).  With red-black
// colours A = 1 (first of the backward sweep) and B = 0 the four colour passes are
//     P1: A | post(n), P2: B | post(n), P3: B | pre(n+1), P4: A | pre(n+1)
// and P2 / P3 update the same B vertex twice from the same A neighbours, so they run as one phase.
// One launch of this kernel reads x, f and the coarse correction once and writes x once for both
// sweeps (the two separate kernels read and write the fine level twice: 24 + 25 B against ~32 B per
// unknown of this one, halo included).
//
//  * Out of place (xin -> xout); every value is a pure function of (xin, xc, f, the Philox counters),
//    so a workgroup recomputes the halo it needs: P1 over the core tile plus a 2-vertex ring, P2/P3
//    over the core plus a 1-vertex ring, P4 on the core, which is then final and stored.
//  * Step p: P1 on plane p, P2/P3 on plane p-1, P4 on plane p-2 (each reads planes +-1 of the
//    previous phase); planes p-3 .. p+1 live in a 6-slot LDS ring (in place: each phase overwrites
//    only its own colour), three barriers per step.  The prolongation x_old = xin + alpha P xc is
//    applied as each plane is staged, in k_prolongate_pairs' term order (same bits as
//    mgmc_zsweep.hpp's fused prolongation).
//  * One thread per pair item of the P1 region (fixed for the whole march): the post-sweep draw of
//    the pair (tag of the post-sweep, sample s) is made in P1 and its second branch carried to P2; the
//    pre-sweep draw (tag of the pre-sweep, sample s+1) in P2/P3 with its second branch carried to P4.
//  * The post-sweep value of the QoI vertex (or the lattice-centre guard vertex) is captured into
//    cap[chain] for the QoI record, which runs after this kernel.
// Per-vertex arithmetic is gibbs_point's (fma chain in ascending column order, c = fma(sd, xi, f),
// x = fma(omega/diag, c - S, x)); P2 and P3 share the first three terms of the chain (the same values
// in the same order), so the results are bitwise those of the two separate sweeps.
#pragma once
#include "mgmc_kernels.hpp"

namespace mgmc {

struct ZSweep2Args {
    Layout L;              // fine level
    const double* xin;
    double* xout;
    const double* f;
    const double* xc;      // coarse correction
    Layout Lc;
    double alpha;
    StencilArg S;
    GibbsArg G;            // tag = the post-sweep's tag; sample word = s (pre-sweep: s + 1)
    uint32_t tag_pre;      // tag of the next cycle's pre-sweep
    const uint64_t* ctrl;  // [2] QoI offset (>= 0) or -1 (guard vertex ctrl[6])
    double* cap;           // [chain] post-sweep value at that vertex
    int tz;                // planes per z-chunk (even)
    int ntx, nty, ntz;
    long long cs, csc;     // batched chains
};

constexpr int zs2_threads(int XP, int TY) { return 256 * (((TY + 4) * (XP + 2) + 255) / 256); }

template <int XP, int TY, int NT, int PROLONG>
__global__ void __launch_bounds__(NT) k_zsweep2_rb7(ZSweep2Args a) {
    static_assert(NT == zs2_threads(XP, TY) && TY % 2 == 0, "tile shape");
    constexpr int WP = XP + 4;     // pairs per LDS row: 2 halo pairs per side
    constexpr int RS = 2 * WP + 2;  // [odd positions | even positions | pad]
    constexpr int R = TY + 6;       // rows j0-3 .. j0+TY+2
    constexpr int PS = R * RS;
    constexpr int NSLOT = 6;
    constexpr int NX1 = XP + 2;     // P1 columns per row (pairs 1 .. XP+2)
    constexpr int NI1 = (TY + 4) * NX1;
    constexpr int NLX = (R * WP + NT - 1) / NT;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;
    double* tab = xs + NSLOT * PS;
    for (int q = threadIdx.x; q < 64; q += NT) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }
    for (int q = threadIdx.x; q < 130; q += NT) tab[192 + q] = SINCOS_TAB[q];
    // coarse ring: 3 planes x rows [Jst, Jst + CR) x columns [q0-3, q0+XP+4]
    constexpr int CW = XP + 8, CWP = CW / 2, CR = TY / 2 + 4, CPS = CR * CW;
    constexpr int NLC = PROLONG ? (CR * CWP + NT - 1) / NT : 1;
    double* cring = tab + 322;

    const int ch = batch_chain();
    a.xin += ch * a.cs;
    a.xout += ch * a.cs;
    a.f += ch * a.cs;
    a.xc += ch * a.csc;
    const RngKey key = chain_key(a.G, ch);
    const Layout& L = a.L;
    const Layout& Lc = a.Lc;
    const int nb = gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);
    const int txi = tile % a.ntx, tyi = (tile / a.ntx) % a.nty, tzi = tile / (a.ntx * a.nty);
    if (tzi >= a.ntz) return;
    const int q0 = txi * XP;               // first core pair
    const int j0 = 1 + tyi * TY;           // first core row
    const int k0 = 1 + tzi * a.tz;         // first core plane (odd)
    const int k1 = min(k0 + a.tz, L.nz);
    const int ibase = 2 * q0 - 3;          // position of LDS pair 0's odd element
    const double sd = a.G.sd, wd = a.G.wd;
    const uint64_t sample = *a.G.sample;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    const uint64_t sample1 = sample + 1;
    const uint32_t t_lo = (uint32_t)sample1, t_hi = (uint32_t)(sample1 >> 32);
    const uint32_t plane_pairs = (uint32_t)((uint64_t)(L.ny - 1) * (uint64_t)(L.nx / 2));
    const long long qcap = (long long)a.ctrl[2] >= 0 ? (long long)a.ctrl[2] : (long long)a.ctrl[6];
    const int tid = threadIdx.x;
    auto slot = [](int k) { return (k + 6) % 6; };
    auto interior_plane = [&](int k) { return k >= 1 && k <= L.nz - 1; };
    auto clamp_row = [&](int j) { return j < 0 ? 0 : (j > L.ny ? L.ny : j); };
    auto plane_base = [&](const double* v, int k) { return v + (long long)(k < 0 ? 0 : (k > L.nz ? L.nz : k)) * L.sp; };

    // ---- this thread's pair item (P1 region: rows 1 .. R-2, pairs 1 .. XP+2) ----
    const bool item = tid < NI1;
    const int r = item ? 1 + tid / NX1 : 1, c = item ? 1 + tid % NX1 : 1;
    const int j = j0 - 3 + r, i0 = ibase + 2 * c;  // the pair (i0, i0+1), i0 odd
    const bool rowin = item && j >= 1 && j <= L.ny - 1;
    const bool in0 = rowin && i0 >= 1 && i0 <= L.nx - 1, in1 = rowin && i0 + 1 >= 1 && i0 + 1 <= L.nx - 1;
    const bool r23 = item && r >= 2 && r <= R - 3;                        // P2/P3 region
    const bool r4 = item && r >= 3 && r <= R - 4 && c >= 2 && c <= XP + 1;  // core (P4, store)
    const int lo = r * RS + c;                                            // odd element; even at +WP
    const int goff = (int)((long long)clamp_row(j) * L.sx + i0 + L.off);
    const uint32_t pbase = (uint32_t)((uint64_t)(j - 1) * (uint64_t)(L.nx / 2) + (uint64_t)((i0 - 1) >> 1));

    // ---- staging (x planes with the prolongation, coarse planes) ----
    int xoff[NLX], xlds[NLX], pcro[NLX];
#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int it = tid + u * NT;
        xoff[u] = L.off + 1;
        xlds[u] = -1;
        pcro[u] = 0;
        if (it < R * WP) {
            const int rr = it / WP, cc = it - rr * WP;
            const int jj = j0 - 3 + rr;
            xlds[u] = rr * RS + cc;
            xoff[u] = (int)((long long)clamp_row(jj) * L.sx + ibase + 2 * cc + L.off);
            // ring column of coarse column (i-1)/2 = q0-2+cc: cc+1; ring row of coarse row jj>>1
            pcro[u] = 2 * ((cc + 1) + ((jj >> 1) - ((j0 - 3) >> 1)) * CW) + (jj & 1);
        }
    }
    const int Jst = (j0 - 3) >> 1;
    int coff[NLC], clds[NLC];
    double2 pcv[NLC];
#pragma unroll
    for (int u = 0; u < NLC; ++u) {
        const int it = tid + u * NT;
        clds[u] = (PROLONG && it < CR * CWP) ? 2 * it : -1;
        const int rr = it / CWP, cc = 2 * (it % CWP);
        const int jr = Jst + rr;
        const int jc = jr < 0 ? 0 : (jr > Lc.ny ? Lc.ny : jr);
        coff[u] = clds[u] >= 0 ? (int)((long long)jc * Lc.sx + (q0 - 3 + cc) + Lc.off) : Lc.off + 1;
    }
    auto cslot = [](int K) { return (K + 3) % 3; };
    auto issue_c = [&](int K) {
        const double* base = a.xc + (long long)(K < 0 ? 0 : (K > Lc.nz ? Lc.nz : K)) * Lc.sp;
#pragma unroll
        for (int u = 0; u < NLC; ++u) pcv[u] = *reinterpret_cast<const double2*>(base + coff[u]);
    };
    auto deposit_c = [&](int K) {
        double* dst = cring + cslot(K) * CPS;
#pragma unroll
        for (int u = 0; u < NLC; ++u)
            if (clds[u] >= 0) {
                dst[clds[u]] = pcv[u].x;
                dst[clds[u] + 1] = pcv[u].y;
            }
    };
    const double al0 = a.alpha, al1 = a.alpha * 0.5;
    // x_old + alpha P x_c at a staged pair: the terms of k_prolongate_pairs in its order (see
    // mgmc_zsweep.hpp prolong_pair; parents on the coarse boundary are zeros of the layout)
    auto prolong_pair = [&](double2 v, int jodd, int k, int cro) {
        const int K0 = k >> 1, kodd = k & 1;
        const double awx = ldexp(al1, -(jodd + kodd)), awy = ldexp(al0, -(jodd + kodd));
        for (int aa = 0; aa < 1 + kodd; ++aa) {
            const double* cp = cring + cslot(K0 + aa) * CPS + cro;
            for (int bb = 0; bb < 1 + jodd; ++bb) {
                const double c0 = cp[bb * CW], c1 = cp[bb * CW + 1];
                if (PROLONG == 2) {
                    v.x = fma(awx, c0, v.x);
                    v.x = fma(awx, c1, v.x);
                    v.y = fma(awy, c1, v.y);
                } else {
                    v.x = v.x + awx * c0;
                    v.x = v.x + awx * c1;
                    v.y = v.y + awy * c1;
                }
            }
        }
        return v;
    };
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
            double2 v = px[u];
            if (PROLONG && interior_plane(k)) v = prolong_pair(v, pcro[u] & 1, k, pcro[u] >> 1);
            dst[xlds[u]] = v.x;
            dst[xlds[u] + WP] = v.y;
        }
    };
    auto load_f = [&](int k) {
        return item ? *reinterpret_cast<const double2*>(plane_base(a.f, k) + goff) : make_double2(0.0, 0.0);
    };

    const double cz = a.S.a[4], cy = a.S.a[10], cx = a.S.a[12], cc = a.S.a[13];
    // the first three terms of the chain (z below, y below, x below) and the rest from a centre value
    auto head = [&](const double* s0, const double* sm, int o, int e) {
        const int xm = e ? o - WP : o + WP - 1;
        double res = cz * sm[o];
        res = fma(cy, s0[o - RS], res);
        return fma(cx, s0[xm], res);
    };
    auto tail = [&](double res, const double* s0, const double* sp, int o, int e, double centre) {
        const int xm = e ? o - WP : o + WP - 1;
        res = fma(cc, centre, res);
        res = fma(cx, s0[xm + 1], res);
        res = fma(cy, s0[o + RS], res);
        return fma(cz, sp[o], res);
    };
    auto draw = [&](int k, uint32_t tag, uint32_t slo, uint32_t shi) -> double2 {
        const uint32_t pair = (uint32_t)(k - 1) * plane_pairs + pbase;
        uint32_t k0r = key.k0, k1r = key.k1;
        asm volatile("" : "+s"(k0r), "+s"(k1r));
        const Philox4 rnd = philox4x32_10(pair, tag, slo, shi, k0r, k1r);
        double z0, z1;
        normal_pair_t(rnd, &z0, &z1, tab, tab + 64, tab + 128, tab + 192);
        return make_double2(z0, z1);
    };

    // ---- prologue: coarse planes for the first stagings, fine planes k0-3, k0-2; k0-1 in flight ----
    int kc_dep = (k0 - 3) >> 1;  // highest coarse plane in the ring
    if (PROLONG) {
        issue_c((k0 - 3) >> 1);
        deposit_c((k0 - 3) >> 1);
        issue_c(((k0 - 3) >> 1) + 1);
        deposit_c(((k0 - 3) >> 1) + 1);
        kc_dep = ((k0 - 3) >> 1) + 1;
        __syncthreads();
    }
    issue_x(k0 - 3);
    deposit_x(k0 - 3);
    issue_x(k0 - 2);
    deposit_x(k0 - 2);
    issue_x(k0 - 1);
    if (PROLONG && (((k0 - 2) + 3) >> 1) > kc_dep) issue_c(kc_dep + 1);
    double2 fcur = load_f(k0 - 2), fprev = make_double2(0.0, 0.0);
    double pkB = 0.0, pkBprev = 0.0;  // post-sweep rhs of the B element (P1 -> P2, one step)
    double pkA = 0.0, pkAprev = 0.0;  // pre-sweep rhs of the A element (P2/P3 -> P4, one step)

    for (int p = k0 - 2; p <= k1 + 1; ++p) {
        // stage plane p+1 (and the coarse plane its successor needs), issue p+2
        if (PROLONG && ((p + 3) >> 1) > kc_dep) {
            deposit_c(kc_dep + 1);
            ++kc_dep;
        }
        deposit_x(p + 1);
        issue_x(p + 2);
        if (PROLONG && ((p + 4) >> 1) > kc_dep) issue_c(kc_dep + 1);
        const double2 fnext = load_f(p + 1);
        __syncthreads();
        // P1: colour A of the post-sweep on plane p (core + 2-ring)
        {
            const int eA = (j + p) & 1;
            const bool inA = eA ? in1 : in0, inB = eA ? in0 : in1;
            double pk = 0.0;
            if (interior_plane(p) && (inA || inB)) {
                const double2 z = draw(p, a.G.tag, s_lo, s_hi);
                double* s0 = xs + slot(p) * PS;
                if (inA) {
                    const int o = lo + eA * WP;
                    const double h = head(s0, xs + slot(p - 1) * PS, o, eA);
                    const double res = tail(h, s0, xs + slot(p + 1) * PS, o, eA, s0[o]);
                    const double crhs = fma(sd, eA ? z.y : z.x, eA ? fcur.y : fcur.x);
                    s0[o] = fma(wd, crhs - res, s0[o]);
                }
                pk = fma(sd, eA ? z.x : z.y, eA ? fcur.x : fcur.y);
            }
            pkBprev = pkB;
            pkB = pk;
        }
        __syncthreads();
        // P2 + P3: colour B on plane p-1, post-sweep then pre-sweep (core + 1-ring)
        {
            const int k = p - 1;
            const int eB = 1 - ((j + k) & 1);
            const bool inB = eB ? in1 : in0, inA = eB ? in0 : in1;
            double pk = 0.0;
            if (r23 && interior_plane(k) && (inA || inB)) {
                const double2 z = draw(k, a.tag_pre, t_lo, t_hi);
                if (inB) {
                    const int o = lo + eB * WP;
                    double* s0 = xs + slot(k) * PS;
                    const double* sm = xs + slot(k - 1) * PS;
                    const double* sp = xs + slot(k + 1) * PS;
                    const double h = head(s0, sm, o, eB);
                    double v = s0[o];
                    v = fma(wd, pkBprev - tail(h, s0, sp, o, eB, v), v);  // post-sweep
                    if (r4 && k >= k0 && k < k1 && (long long)k * L.sp + goff + eB == qcap) a.cap[ch] = v;
                    const double crhs = fma(sd, eB ? z.y : z.x, eB ? fprev.y : fprev.x);
                    v = fma(wd, crhs - tail(h, s0, sp, o, eB, v), v);     // pre-sweep
                    s0[o] = v;
                }
                pk = fma(sd, eB ? z.x : z.y, eB ? fprev.x : fprev.y);
            }
            pkAprev = pkA;
            pkA = pk;
        }
        __syncthreads();
        // P4: colour A of the pre-sweep on plane p-2 (core); the plane is final: store it
        {
            const int k = p - 2;
            if (r4 && rowin && k >= k0 && k < k1) {
                const int eA = (j + k) & 1;
                const bool inA = eA ? in1 : in0;
                const int o = lo + eA * WP;
                const double* s0 = xs + slot(k) * PS;
                double v = s0[o];
                if ((long long)k * L.sp + goff + eA == qcap) a.cap[ch] = v;  // post-sweep value of A
                if (inA) {
                    const double h = head(s0, xs + slot(k - 1) * PS, o, eA);
                    v = fma(wd, pkAprev - tail(h, s0, xs + slot(k + 1) * PS, o, eA, v), v);
                }
                const double vb = s0[lo + (1 - eA) * WP];
                const double2 out = eA ? make_double2(vb, v) : make_double2(v, vb);
                double* dst = a.xout + (long long)k * L.sp + goff;
                __builtin_nontemporal_store(out.x, dst);
                __builtin_nontemporal_store(out.y, dst + 1);
            }
        }
        fprev = fcur;
        fcur = fnext;
    }
}

inline size_t zsweep2_lds_bytes(int XP, int TY, bool prolong) {
    const int RS = 2 * (XP + 4) + 2, R = TY + 6;
    const int coarse = prolong ? 3 * (TY / 2 + 4) * (XP + 8) : 0;
    return (size_t)(6 * R * RS + 3 * 64 + 130 + coarse) * sizeof(double);
}

}  // namespace mgmc
