// mgmc_zrestrict.hpp -- z-marching fused residual + restriction for 3D levels.
//
//   f_c = R (f - A x),  x_c = 0           (sampler/multigridmc_sampler.cc:118-122)
//
// Each workgroup owns CX x CY coarse points and marches fine planes k = 2K0-1 .. 2K1-1 of a chunk
// of coarse planes [K0, K1).  Per fine plane: the residual r = f - A x of the plane is evaluated
// once per fine vertex (plus a one-vertex tile overlap) into one LDS plane, from x planes staged in
// a 3-slot LDS ring with a one-vertex halo; then every coarse point adds the 9 weighted residuals of
// its 3x3 fine neighbourhood in that plane to a register accumulator.  The restriction sums over
// (sz, sy, sx) with sz outermost, so plane-by-plane accumulation adds exactly the reference's terms
// in the reference's order: fine plane 2K-1 is sz = 0 of coarse plane K, 2K is sz = 1, and 2K+1 is
// sz = 2 of K (which is then final) and sz = 0 of K+1.  Arithmetic: A x ascending from 0.0 as the
// reference's (the 7-point fine level and non-symmetric 27-point levels) or class-folded (fold27, the
// reflection-symmetric 27-point levels); r = f - Ax, restriction weights multiplied x, y, z; f_c is
// bitwise equal to k_residual_restrict's and to the CPU oracle's.
//
// LDS rows are colour-split as in mgmc_zsweep.hpp -- [odd positions | even positions | pad] -- so
// lanes owning consecutive pairs (residual) or consecutive coarse points (restriction) read
// consecutive doubles.  All global loads are unconditional: rows / planes outside the level are
// clamped onto the zero boundary rows / planes, columns past a row end onto the zero pair (nx+1, nx+2).
// Global traffic: x and f once (16 B per fine vertex) + f_c, x_c (2 B per fine vertex).
#pragma once
#include "mgmc_kernels.hpp"
#include "mgmc_tail.hpp"
#include "mgmc_tuning.hpp"
#include <type_traits>

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
    long long csf, csc;  // batched chains: doubles between chains on the fine / coarse level
    // ZN: workgroups nblk_main .. of the grid draw the next op's (k_tail's) Box-Muller pairs instead
    // (they depend on no data): jobs[0 .. njobs) into zb (zbs items per chain)
    int nblk_main;
    const TailNoiseJob* jobs;
    int njobs;
    double2* zb;
    long long zbs;
    RngKey key;                // chain c's key: (key.k0, lo32(chain0 + c) ^ seed_hi)
    uint32_t chain0, seed_hi;
    const uint64_t* sample;
    LRRhsArg lr;               // LRF: the right-hand side is f patched in place (mgmc_kernels.hpp)
    // pn.dst (non-null): every workgroup also draws its share of the Box-Muller pairs of the coarse level's
    // first pre-sweep (pair q -> pn.dst[q], chain 0's key: one chain), after its own march
    PostNoiseJob pn;
};

// One plane's 3 x 4 window of a residual pair item (rows dy = -1, 0, 1 at byte offsets 0, RB, 2 RB from
// `base`, the LDS byte address of row dy = -1's odd element i): per row x(i), x(i+2), x(i-1), x(i+1) at
// byte offsets 0, 8, EV - 8, EV (EV = the even block's offset).  Twelve single ds_read_b64 with immediate
// offsets in one statement that ends in the wait: the compiler otherwise pairs them into ds_read2_b64,
// which moves 8 bytes per lane at half the LDS rate (MI355X_MICROARCH.md, LDS table) -- the level-1
// residual + restriction reads 36 values per pair item from LDS and was bound by those reads.
#define ZR_RD(n, o) "ds_read_b64 %" #n ", %12 offset:" #o "\n"
template <int RB, int EV>
__device__ __forceinline__ void zr_plane12(uint32_t base, double (&v)[12]) {
    static_assert(2 * RB + EV < 65536 && EV >= 8, "ds offsets");
    asm volatile(ZR_RD(0, 0) ZR_RD(1, 8) ZR_RD(2, %c13) ZR_RD(3, %c14)
                 ZR_RD(4, %c15) ZR_RD(5, %c16) ZR_RD(6, %c17) ZR_RD(7, %c18)
                 ZR_RD(8, %c19) ZR_RD(9, %c20) ZR_RD(10, %c21) ZR_RD(11, %c22) "s_waitcnt lgkmcnt(0)"
                 : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                   "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11])
                 : "v"(base), "i"(EV - 8), "i"(EV), "i"(RB), "i"(RB + 8), "i"(RB + EV - 8), "i"(RB + EV),
                   "i"(2 * RB), "i"(2 * RB + 8), "i"(2 * RB + EV - 8), "i"(2 * RB + EV)
                 : "memory");
}
#undef ZR_RD

// SYM: a fold level (reflection-symmetric 27-point stencil): the residual's sum is fold27's
// LRF: a low-rank level whose right-hand side is read in place (a.lr: f + e, lr_rhs_pair)
template <int NPTS, int CX, int CY, int NT, bool ZN = false, bool SYM = false, bool LRF = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NPTS == 27 && SYM && CX >= 48 ? tune::ZR27_MINW : 1)))
k_zresrestrict(ZRestrictArgs a) {
    if (ZN && (int)blockIdx.x >= a.nblk_main) {  // the tail's noise (see ZRestrictArgs)
        const int ch = batch_chain();
        RngKey key = a.key;
        if (ch) key.k1 = (a.chain0 + (uint32_t)ch) ^ a.seed_hi;
        const uint64_t sample = *a.sample;
        double2* z = a.zb + ch * a.zbs;
        const int nw = ((int)gridDim.x - a.nblk_main) * NT;
        const int w0 = ((int)blockIdx.x - a.nblk_main) * NT + (int)threadIdx.x;
        for (int jb = 0; jb < a.njobs; ++jb) {
            const TailNoiseJob J = a.jobs[jb];
            const int npair = J.nx / 2, nyi = J.ny - 1;
            const int n = npair * nyi * (J.nz - 1);
            for (int q = w0; q < n; q += nw) {
                const int m = q % npair, row = q / npair;
                const int i0 = 2 * m + 1;
                if (i0 > J.nx - 1) continue;
                const int j = row % nyi + 1, k = row / nyi + 1;
                const uint32_t pair = (uint32_t)(((uint64_t)(k - 1) * (uint64_t)nyi + (uint64_t)(j - 1)) * (uint64_t)npair +
                                                 (uint64_t)m);  // pair_id<3>
                const Philox4 rnd = philox4x32_10(pair, J.tag, (uint32_t)sample, (uint32_t)(sample >> 32), key.k0, key.k1);
                double z0, z1;
                normal_pair(rnd, &z0, &z1);
                z[J.zoff + q] = make_double2(z0, z1);
            }
        }
        return;
    }
    // fine x range of the residual region: [2*I0-1, 2*I0+2*CX-1] = RP pairs from an odd position.
    // x is staged with one more vertex on each side: positions [2*I0-3, 2*I0+2*CX+2] = XPP pairs.
    constexpr int RP = CX + 1;                   // residual pairs per row
    constexpr int RR = 2 * CY + 1;               // residual rows
    constexpr int RSr = 2 * RP + 2;              // residual row stride (odd | even | pad)
    constexpr int XPP = CX + 3;                  // x pairs per row
    constexpr int XR = 2 * CY + 3;               // x rows
    constexpr int XS = 2 * XPP + 2;              // x row stride (odd | even | pad)
    constexpr int XPS = XR * XS;                 // x plane
    constexpr int NLX = (XR * XPP + NT - 1) / NT;  // x pair loads per plane per thread
    constexpr int NLR = (RR * RP + NT - 1) / NT;   // residual pair items per plane per thread
    constexpr int NCP = (CX * CY + NT - 1) / NT;   // coarse points per thread
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                 // [3][XR][XS] x planes k-1, k, k+1
    double* rs = xs + 3 * XPS;         // [RR][RSr] residual of plane k

    {  // batched chains (blockIdx.z)
        const int ch = batch_chain();
        a.x += ch * a.csf;
        a.f += ch * a.csf;
        a.fc += ch * a.csc;
        a.xc += ch * a.csc;
        if (LRF) a.lr.e += ch;
    }
    const double lre = LRF ? *a.lr.e : 0.0;
    const Layout& Lf = a.Lf;
    const Layout& Lc = a.Lc;
    const int nb = ZN ? a.nblk_main : (int)gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);
    const int txi = tile % a.ntx;
    const int tyi = (tile / a.ntx) % a.nty;
    const int tzi = tile / (a.ntx * a.nty);
    // the coarse level's first pre-sweep's pairs (a.pn): workgroup b draws q = b NT + tid + r nb NT
    auto draw_pn = [&]() {
        if (!a.pn.dst) return;
        const uint64_t sample = *a.sample;
        const uint32_t n = (uint32_t)(a.pn.nx / 2) * (uint32_t)(a.pn.ny - 1) * (uint32_t)(a.pn.nz - 1);
        const uint32_t nw = (uint32_t)nb * NT;
        for (uint32_t q = (uint32_t)b * NT + threadIdx.x; q < n; q += nw) {
            const Philox4 r = philox4x32_10(q, a.pn.tag, (uint32_t)sample, (uint32_t)(sample >> 32), a.key.k0, a.key.k1);
            double z0, z1;
            normal_pair(r, &z0, &z1);
            a.pn.dst[q] = make_double2(z0, z1);
        }
    };
    if (tzi >= a.ntz) {
        draw_pn();
        return;
    }
    const int I0 = 1 + txi * CX, J0 = 1 + tyi * CY;
    const int K0 = 1 + tzi * a.kz, K1 = min(K0 + a.kz, Lc.nz);  // coarse planes [K0, K1)
    const int xi0 = 2 * I0 - 3;  // fine position of x pair column 0 (odd)
    const int xj0 = 2 * J0 - 2;  // fine row of x row 0
    const int ri0 = 2 * I0 - 1;  // fine position of residual pair column 0 (odd)
    const int rj0 = 2 * J0 - 1;  // fine row of residual row 0
    const int tid = threadIdx.x;

    auto xslot = [](int k) { return (k + 9) % 3; };
    auto clamp_row = [&](int j) { return j < 0 ? 0 : (j > Lf.ny ? Lf.ny : j); };
    // pairs past the row end read the zero pair (nx+1, nx+2) of the row padding: the last tile's
    // columns can run up to 2 CX - 2 past nx (nx - 1 = 1 mod CX), beyond the padding; the positions
    // involved are outside the lattice, their values only reach residuals that are forced to 0
    // (mgmc_layout_check.hpp)
    auto clamp_col = [&](int i) { return i > Lf.nx + 1 ? Lf.nx + 1 : i; };
    auto plane_ptr = [&](const double* v, int k) { return v + (long long)(k < 0 ? 0 : (k > Lf.nz ? Lf.nz : k)) * Lf.sp; };

    int xoff[NLX], xlds[NLX];
#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int it = tid + u * NT;
        xoff[u] = Lf.off + 1;  // spare threads load a zero pad pair and deposit nothing
        xlds[u] = -1;
        if (it < XR * XPP) {
            const int r = it / XPP, c2 = it - r * XPP;
            xlds[u] = r * XS + c2;
            xoff[u] = (int)((long long)clamp_row(xj0 + r) * Lf.sx + clamp_col(xi0 + 2 * c2) + Lf.off);
        }
    }
    int roff[NLR], rlds[NLR], rflag[NLR], rxo[NLR];
#pragma unroll
    for (int u = 0; u < NLR; ++u) {
        const int it = tid + u * NT;
        roff[u] = Lf.off + 1;
        rlds[u] = -1;
        rflag[u] = 0;
        rxo[u] = XS + 1;  // spare items read (and discard) an in-range LDS neighbourhood
        if (it < RR * RP) {
            const int r = it / RP, c2 = it - r * RP;
            const int j = rj0 + r, i = ri0 + 2 * c2;
            rlds[u] = r * RSr + c2;
            rxo[u] = (r + 1) * XS + (c2 + 1);  // x LDS offset of the same odd vertex
            roff[u] = (int)((long long)clamp_row(j) * Lf.sx + clamp_col(i) + Lf.off);
            const bool rin = j >= 1 && j <= Lf.ny - 1;
            rflag[u] = (rin && i >= 1 && i <= Lf.nx - 1 ? 1 : 0) | (rin && i + 1 <= Lf.nx - 1 ? 2 : 0);
        }
    }
    // coarse points: (I, J) and the residual LDS offset of the odd element left of the centre 2I
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

    double2 px[NLX], pf[NLR];
    // the chunk stages x planes 2 K0 - 2 .. 2 K1 and f planes 2 K0 - 1 .. 2 K1 - 1: the last step's loads one
    // plane ahead reload those (never used) instead of fetching the next chunk's planes
    const int kx_last = 2 * K1, kf_last = 2 * K1 - 1;
    auto issue_x = [&](int k) {
        const double* base = plane_ptr(a.x, k > kx_last ? kx_last : k);
#pragma unroll
        for (int u = 0; u < NLX; ++u) px[u] = *reinterpret_cast<const double2*>(base + xoff[u]);
    };
    auto deposit_x = [&](int k) {
        double* dst = xs + xslot(k) * XPS;
#pragma unroll
        for (int u = 0; u < NLX; ++u)
            if (xlds[u] >= 0) {
                dst[xlds[u]] = px[u].x;
                dst[xlds[u] + XPP] = px[u].y;
            }
    };
    auto issue_f = [&](int k) {
        const double* base = plane_ptr(a.f, k > kf_last ? kf_last : k);
#pragma unroll
        for (int u = 0; u < NLR; ++u) pf[u] = *reinterpret_cast<const double2*>(base + roff[u]);
    };
    // residual of fine plane k over the residual region (vertices outside the fine interior -> 0).
    // The two vertices of a pair advance together through the stencil terms, so their dependent
    // adds interleave; each chain still adds its terms in ascending column order from 0.0.
    auto residual = [&](int k, const double2 (&fv)[NLR]) {
        const bool kin = k >= 1 && k <= Lf.nz - 1;
        const double* pl[3] = {xs + xslot(k - 1) * XPS, xs + xslot(k) * XPS, xs + xslot(k + 1) * XPS};
#pragma unroll
        for (int u = 0; u < NLR; ++u) {
            if (rlds[u] < 0) continue;
            const int o0 = rxo[u], o1 = rxo[u] + XPP;  // odd / even vertex
            const int m0 = o0 + XPP - 1, m1 = o1 - XPP;   // their x-1 neighbours (x+1 = m + 1; 7-point)
            double y0 = 0.0, y1 = 0.0;
            if (NPTS == 7) {
                y0 += a.S.a[4] * pl[0][o0];
                y1 += a.S.a[4] * pl[0][o1];
                y0 += a.S.a[10] * pl[1][o0 - XS];
                y1 += a.S.a[10] * pl[1][o1 - XS];
                y0 += a.S.a[12] * pl[1][m0];
                y1 += a.S.a[12] * pl[1][m1];
                y0 += a.S.a[13] * pl[1][o0];
                y1 += a.S.a[13] * pl[1][o1];
                y0 += a.S.a[14] * pl[1][m0 + 1];
                y1 += a.S.a[14] * pl[1][m1 + 1];
                y0 += a.S.a[16] * pl[1][o0 + XS];
                y1 += a.S.a[16] * pl[1][o1 + XS];
                y0 += a.S.a[22] * pl[2][o0];
                y1 += a.S.a[22] * pl[2][o1];
            } else if constexpr (SYM) {  // a fold level: the class-folded sum (fold27), each plane's window by
                                         // zr_plane12 (512^3 level 1: 96 -> 81 us against the compiler's read2 pairs)
                double s0[8], s1[8];
#pragma unroll
                for (int dz = 0; dz < 3; ++dz) {
                    double v[12];
                    zr_plane12<XS * 8, XPP * 8>(lds_addr(pl[dz] - XS + o0), v);
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const int c = dz * 9 + r * 3;
                        // row by row, (i-1, i, i+1) for the odd vertex and (i, i+1, i+2) for the even one
                        fold27_acc(s0, c, v[4 * r + 2]);
                        fold27_acc(s1, c, v[4 * r + 0]);
                        fold27_acc(s0, c + 1, v[4 * r + 0]);
                        fold27_acc(s1, c + 1, v[4 * r + 3]);
                        fold27_acc(s0, c + 2, v[4 * r + 3]);
                        fold27_acc(s1, c + 2, v[4 * r + 1]);
                    }
                }
                y0 = fold27_finish(s0, a.S.a);
                y1 = fold27_finish(s1, a.S.a);
            } else {  // the reference's CSR order: ascending columns from 0.0, separate multiply and add
#pragma unroll
                for (int dz = 0; dz < 3; ++dz) {
                    double v[12];
                    zr_plane12<XS * 8, XPP * 8>(lds_addr(pl[dz] - XS + o0), v);
#pragma unroll
                    for (int r = 0; r < 3; ++r) {
                        const int c = dz * 9 + r * 3;
                        y0 += a.S.a[c] * v[4 * r + 2];
                        y1 += a.S.a[c] * v[4 * r + 0];
                        y0 += a.S.a[c + 1] * v[4 * r + 0];
                        y1 += a.S.a[c + 1] * v[4 * r + 3];
                        y0 += a.S.a[c + 2] * v[4 * r + 3];
                        y1 += a.S.a[c + 2] * v[4 * r + 1];
                    }
                }
            }
            double2 f = fv[u];
            if constexpr (LRF) f = lr_rhs_pair(f, lre);
            rs[rlds[u]] = (kin && (rflag[u] & 1)) ? f.x - y0 : 0.0;
            rs[rlds[u] + RP] = (kin && (rflag[u] & 2)) ? f.y - y1 : 0.0;
        }
    };
    // acc += the 9 terms (sy, sx ascending) of restriction plane index sz from the residual plane
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
                if (a.xc) a.xc[pk + cpg[u]] = 0.0;  // (null: the coarse level's first sweep takes x_c = 0 as given)
            }
    };

    // One fine plane k: deposit x(k+1), issue x(k+2) | barrier | residual(k), issue f(k+1) | barrier |
    // accumulate.  The next step's residual writes the residual plane only after its own first
    // barrier, i.e. after every thread accumulated; x(k+2) overwrites the slot of x(k-1), last read
    // by residual(k) before the second barrier.
    double acc[NCP], accn[NCP];
    // f(k) is in pf when residual(k) runs; f(k+1) is issued once it has used it (one register set)
    auto step = [&](int k) __attribute__((always_inline)) {
        deposit_x(k + 1);
        issue_x(k + 2);
        __syncthreads();
        residual(k, pf);
        issue_f(k + 1);
        __syncthreads();
    };
    // prologue: x planes 2K0-2, 2K0-1 in LDS, x(2K0) and f(2K0-1) in flight
    issue_x(2 * K0 - 2);
    deposit_x(2 * K0 - 2);
    issue_x(2 * K0 - 1);
    deposit_x(2 * K0 - 1);
    issue_x(2 * K0);
    issue_f(2 * K0 - 1);
#pragma unroll
    for (int u = 0; u < NCP; ++u) acc[u] = 0.0;
    step(2 * K0 - 1);
    accumulate(acc, 0);  // sz = 0 of coarse plane K0
    for (int K = K0; K < K1; ++K) {
        step(2 * K);
        accumulate(acc, 1);
        step(2 * K + 1);
        accumulate(acc, 2);
        finish(acc, K);
#pragma unroll
        for (int u = 0; u < NCP; ++u) accn[u] = 0.0;
        accumulate(accn, 0);  // sz = 0 of coarse plane K+1
#pragma unroll
        for (int u = 0; u < NCP; ++u) acc[u] = accn[u];
    }
    draw_pn();
}

inline size_t zrestrict_lds_bytes(int CX, int CY) {
    const int XS = 2 * (CX + 3) + 2, XR = 2 * CY + 3, RSr = 2 * (CX + 1) + 2, RR = 2 * CY + 1;
    return (size_t)(3 * XR * XS + RR * RSr) * sizeof(double);
}

}  // namespace mgmc
