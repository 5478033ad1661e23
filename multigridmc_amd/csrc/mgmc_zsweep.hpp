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
//  * Planes live in a 4-slot LDS ring (p-2 .. p+1) in a colour-split row layout; global traffic is
//    16-byte pair loads and stores, one pass over x_in, f and x_out (+ halo re-reads that hit L2 /
//    Infinity Cache).  Second-colour results never return to LDS (no update reads them), they go
//    straight to the store; the z-below values of the second colour come from registers.  With four
//    slots the deposit of plane p+2 never touches a plane the second colour still reads, so a step
//    needs two barriers.
//  * The two vertices of an x-pair share one Philox block: the first-colour update consumes one
//    Box-Muller branch and keeps the other's right-hand side in a register for the second-colour
//    update one step later.  The noise of plane p+1 is drawn in the second-colour phase of step p
//    (it depends on no data), which evens the arithmetic out over the phases between barriers.
//  * One pair item per thread: TY/2 core waves (rows of one parity per wave, so which element of a
//    pair takes the first colour is a wave-uniform branch, not a per-lane select), two waves for the
//    first-colour halo ring (row j0-1 with the columns of the odd core rows, row j0+TY with those of
//    the even ones), idle waves up to a multiple of four (the dispatcher places a workgroup's waves
//    round-robin over the four SIMDs: other sizes strand wave slots).
//  * Optional fused prolongate-add on the input: x_old = x_in + alpha P x_c, evaluated exactly as
//    k_prolongate_add (so the post-sampler needs no separate prolongation pass).
// Per-vertex arithmetic is that of mgmc_kernels.hpp (fused Gibbs update); results are bitwise
// equal to the two colour passes.
#pragma once
#include <type_traits>

#include "mgmc_kernels.hpp"
#include "mgmc_tuning.hpp"

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
    int zpairs;                // plain sweep: z-chunks in pairs marching towards each other (below)
    long long cs, csc;         // batched chains: doubles between chains of the level / coarse level
    LRRhsArg lr;               // LRF: the right-hand side is f patched in place (mgmc_kernels.hpp)
};

// One pair item of a tile: LDS offset, plane-independent global offset, Philox pair base,
// position parity and interior flags, all computed once per workgroup.
struct ZItem {
    int goff;        // j*sx + i + off  (add k*sp for plane k; a plane is < 2^31 doubles)
    uint32_t pbase;  // (j-1)*(nx/2) + (i-1)/2
    int lds;         // r*RS + c2 (odd element; even element at +WP)
    int flags;       // bit0 row interior, bit1 i interior, bit2 i+1 interior, bit3 parity (i+j)&1
};

// PROLONG: 0 plain sweep; 1 fused prolongation, terms v + (alpha w) x_c (any alpha); 2 the same with
// v = fma(alpha w, x_c, v), selected when alpha is a power of two: alpha w x_c is then exact, so the
// fma rounds once like the separate add and the bits are the same.
// MINW: minimum waves per SIMD the register allocation must allow (1 = unconstrained)
// LRF: a low-rank level whose right-hand side is read in place (a.lr: f + e, lr_rhs_pair)
struct RunE0 {
    int value;
};

// threads of a TY-row tile: TY/2 core waves + 2 halo waves, rounded up to a multiple of 4 waves
constexpr int zs_threads(int TY) { return 256 * ((TY / 2 + 2 + 3) / 4); }

// XP must be 32 (a wave = two rows of 32 pairs); TY a multiple of 4, <= 32
template <int XP, int TY, int NT, int PROLONG, int MINW, bool LRF = false>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MINW))) k_zsweep_rb7(ZSweepArgs a) {
    static_assert(XP == 32 && TY % 4 == 0 && TY <= 32 && NT == zs_threads(TY), "tile shape");
    // pairs per LDS row: positions [2*q0-1, 2*q0+2*XP+2] -- the core pairs and one halo pair per side.
    // The halo ring's column items need only their element next to the tile (the even one on the left,
    // the odd one on the right), whose x neighbours are staged; their other element's update reads a
    // wrapped-around slot and lands in a slot no update of this tile ever reads.
    constexpr int WP = XP + 2;
    // LDS row = [odd positions of the WP pairs | even positions | 2 pad]: lanes owning consecutive
    // pairs read consecutive doubles (conflict-free); the row stride (2XP+6 doubles = 12 mod 64 banks)
    // spreads the column accesses of the x-halo items over the banks
    constexpr int RS = 2 * WP + 2;
    constexpr int R = TY + 4;      // rows j0-2 .. j0+TY+1
    constexpr int PS = R * RS;     // LDS plane
    constexpr int NSLOT = 4;
    constexpr int NCW = TY / 2;    // core waves
    constexpr int NLX = (R * WP + NT - 1) / NT;    // pair loads of one x plane per thread
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;                  // [4][R][RS] ring of x planes
    double* tab = xs + NSLOT * PS;      // [3][64] log reduction table (rc, hi, lo) + [130] cos/sin table
    for (int q = threadIdx.x; q < 64; q += NT) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }
    for (int q = threadIdx.x; q < 130; q += NT) tab[192 + q] = SINCOS_TAB[q];
    // waves 0-2 write the tables, every wave reads them in its first noise draw, which the plain sweep
    // makes before the march's first barrier (the fused-prolongation sweep has a prologue barrier
    // first): without this barrier a wave dispatched ahead of waves 0-2 reads whatever the CU's LDS held
    if (!PROLONG) __syncthreads();
    // PROLONG: ring of two coarse planes (slot K & 1) over the tile's coarse footprint, coarse
    // columns [q0-3, q0+XP+4] (starting on an even storage index: 16-byte pair loads) x rows
    // [(j0-3)/2, (j0+TY+1)/2]
    constexpr int CW = XP + 8, CWP = CW / 2, CR = TY / 2 + 3, CPS = CR * CW;
    constexpr int NLC = PROLONG ? (CR * CWP + NT - 1) / NT : 1;
    double* cring = tab + 322;

    {  // batched chains: this launch's chain (blockIdx.z), its vectors and its Philox key
        const int ch = batch_chain();
        a.xin += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        if (PROLONG) a.xc += ch * a.csc;
        a.G.key = chain_key(a.G, ch);
        if (LRF) a.lr.e += ch;
    }
    const double lre = LRF ? *a.lr.e : 0.0;
    const Layout& L = a.L;
    // XCD-aware tile order: blocks b and b+8 share an XCD, give them neighbouring tiles
    const int nb = gridDim.x;
    const int b = blockIdx.x;
    const int per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);
    // x fastest: a workgroup's x neighbours run next to it on the same XCD and share the partial
    // 128-B lines of the x halo through L2 (y fastest: 1.49x algorithmic traffic against 1.21x)
    int txi = tile % a.ntx;
    int tyi = (tile / a.ntx) % a.nty;
    int tzi = tile / (a.ntx * a.nty);
    // zpairs (plain sweep): z-chunks 2m and 2m+1 of a column are neighbouring tiles (same XCD, same
    // round of workgroups); chunk 2m marches up and 2m+1 down, so both reach their shared boundary
    // planes at the end of their march, and those planes' second read is an L2 hit instead of an HBM
    // re-read one round later.  The march direction does not change a value: every vertex sees the
    // same old / new neighbours either way.
    bool down = false;
    if (!PROLONG && a.zpairs) {
        const int nxy = a.ntx * a.nty;
        const int zp = tile / (2 * nxy), rem = tile - zp * 2 * nxy;
        txi = (rem >> 1) % a.ntx;
        tyi = (rem >> 1) / a.ntx;
        tzi = 2 * zp + (rem & 1);
        down = (rem & 1) != 0;
    }
    if (tzi >= a.ntz) return;
    const int q0 = txi * XP;              // first core pair; core positions 2q0+1 .. 2q0+2XP
    const int j0 = 1 + tyi * TY;          // first core row
    const int k0 = 1 + tzi * a.tz;        // first core plane
    const int k1 = min(k0 + a.tz, L.nz);  // one past the last core plane
    const int ibase = 2 * q0 - 1;         // position of LDS column 0
    const int fc = a.G.colour;            // first colour
    const double sd = a.G.sd, wd = a.G.wd;
    const uint64_t sample = *a.G.sample;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    const uint32_t plane_pairs = (uint32_t)((uint64_t)(L.ny - 1) * (uint64_t)(L.nx / 2));
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;

    auto slot = [](int p) { return (p + 4) & 3; };
    auto interior_plane = [&](int k) { return k >= 1 && k <= L.nz - 1; };
    auto make_item = [&](int r, int c2) {
        ZItem t;
        const int j = j0 - 2 + r, i = ibase + 2 * c2;
        const bool rin = j >= 1 && j <= L.ny - 1;
        // rows outside [0, ny] are clamped onto the zero boundary rows 0 / ny, so every load is
        // unconditional and reads exactly the zeros the guarded form produced (columns past either
        // end of a row land in the zero padding of the layout)
        const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
        t.goff = (int)((long long)jc * L.sx + i + L.off);
        t.pbase = (uint32_t)((uint64_t)(j - 1) * (uint64_t)(L.nx / 2) + (uint64_t)((i - 1) >> 1));
        t.lds = r * RS + c2;  // odd element; the even element is at +WP
        t.flags = (rin ? 1 : 0) | ((i >= 1 && i <= L.nx - 1) ? 2 : 0) | ((i + 1 >= 1 && i + 1 <= L.nx - 1) ? 4 : 0) |
                  (((i + j) & 1) << 3);
        return t;
    };

    // ---- this thread's pair item ----
    const bool core_wave = wave < NCW, active_wave = wave < NCW + 2;  // wave-uniform
    int ir = 2, ic = 1;
    if (core_wave) {
        ir = 2 + 4 * (wave >> 1) + (wave & 1) + (lane >= 32 ? 2 : 0);  // rows r, r + 2: one parity
        ic = 1 + (lane & 31);
    } else if (active_wave) {
        const int h = wave - NCW;
        // lanes past the halo items mirror lane 0's item: the same arithmetic writes the same bits
        // to the same LDS word, so the duplicate is harmless
        const int l = (lane < 32 + TY) ? lane : 0;
        if (l < 32) {
            ir = h == 0 ? 1 : R - 2;
            ic = 1 + l;
        } else {  // left / right column of the core rows of the row's parity
            const int m = l - 32;
            ir = (h == 0 ? 3 : 2) + 2 * (m >> 1);
            ic = (m & 1) ? WP - 1 : 0;
        }
    }
    const ZItem t = make_item(ir, ic);
    // (i + j) & 1 of the wave's items (all i odd, rows of one parity): wave-uniform
    const int wpar = __builtin_amdgcn_readfirstlane((t.flags >> 3) & 1);
    // element (0 odd position, 1 even) taking the first colour on plane k: wave-uniform.  Chunks
    // start on odd planes, so it is E0 on the steps p = k0-1, k0+1, ... (even p) and 1 - E0 on the
    // others (a downward march starts on plane k1: its first step's element is E0d).  The plain sweep compiles the z march below once per value of E0 and runs the steps in
    // pairs, so every element choice in it is a compile-time constant: no selects, and pair loads
    // and stores stay 16-byte accesses (the two copies execute the same sequence of barriers).  The
    // fused-prolongation sweep keeps one copy with wave-uniform selects (its registers are the
    // binding limit: 2 workgroups of 12 waves per CU need <= 80 VGPRs).
    const int E0 = __builtin_amdgcn_readfirstlane(((wpar ^ (k0 - 1)) & 1) == fc ? 0 : 1);
    const int E0d = __builtin_amdgcn_readfirstlane(((wpar ^ k1) & 1) == fc ? 0 : 1);
    // the odd / even element is an interior vertex (per lane; boundary vertices are never written)
    const bool rowin = (t.flags & 1) != 0;
    const bool in0 = rowin && (t.flags & 2), in1 = rowin && (t.flags & 4);

    int xoff[NLX];
    int xlds[NLX];
#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int it = tid + u * NT;
        xoff[u] = L.off + 1;  // threads without an item load a zero pad pair and deposit nothing
        xlds[u] = -1;
        if (it < R * WP) {
            // rows of one parity first: a wavefront's pairs then share the row parity, so the
            // prolongation's odd-row terms (PROLONG) are skipped by whole wavefronts
            constexpr int NE = (R + 1) / 2;  // rows r = 0, 2, 4, ...
            const int r = it < NE * WP ? 2 * (it / WP) : 2 * ((it - NE * WP) / WP) + 1;
            const ZItem q = make_item(r, it % WP);
            xlds[u] = q.lds;
            xoff[u] = q.goff;
        }
    }
    // PROLONG: per staged pair, the row parity and the coarse-ring offset of its first parent
    // (coarse column q = (i-1)/2 = q0-1+c2, coarse row j>>1)
    int pcro[NLX];  // 2 x (coarse-ring offset) + row parity
    // planes outside [0, nz] are clamped onto the zero boundary planes 0 / nz
    auto plane_base = [&](const double* v, int k) { return v + (long long)(k < 0 ? 0 : (k > L.nz ? L.nz : k)) * L.sp; };

    // ---- PROLONG: coarse planes (loads one step ahead, deposited into the coarse ring) ----
    const Layout& Lc = a.Lc;
    const int Jst = (j0 - 2) >> 1;  // first coarse row of the footprint
    int coff[NLC], clds[NLC];
    double2 pcv[NLC];
#pragma unroll
    for (int u = 0; u < NLC; ++u) {
        const int it = tid + u * NT;
        clds[u] = (PROLONG && it < CR * CWP) ? 2 * it : -1;  // pair it: row it / CWP, columns 2 (it % CWP) + {0, 1}
        const int r = it / CWP, c = 2 * (it % CWP);
        const int jr = Jst + r;
        const int jc = jr < 0 ? 0 : (jr > Lc.ny ? Lc.ny : jr);
        coff[u] = clds[u] >= 0 ? (int)((long long)jc * Lc.sx + (q0 - 3 + c) + Lc.off) : Lc.off + 1;
    }
    auto issue_c = [&](int K) {
        const double* base = a.xc + (long long)(K < 0 ? 0 : (K > Lc.nz ? Lc.nz : K)) * Lc.sp;
#pragma unroll
        for (int u = 0; u < NLC; ++u) pcv[u] = *reinterpret_cast<const double2*>(base + coff[u]);
    };
    auto deposit_c = [&](int K) {
        double* dst = cring + (K & 1) * CPS;
#pragma unroll
        for (int u = 0; u < NLC; ++u)
            if (clds[u] >= 0) {
                dst[clds[u]] = pcv[u].x;
                dst[clds[u] + 1] = pcv[u].y;
            }
    };
    // x_old + alpha P x_c at the fine pair (i odd, i+1) of row j, plane k, from the coarse ring.  The
    // same terms in the same order as k_prolongate_pairs: coarse parents in ascending (kk, jj, ii),
    // each added as v += (alpha w) x_c.  No existence tests: a parent on the coarse boundary (index 0
    // or n_c) is a zero of the padded layout (boundary vertices and pads are zero, and the ring's
    // clamped rows / planes are boundary rows / planes), so its term adds +0 and leaves v unchanged
    // -- the reference skips it (intergrid_operator.hh:106-120); the two agree bit for bit except for
    // the sign of an exact zero (-0 + 0 = +0).  Fine positions outside the domain (staged halo
    // columns / rows past the boundary) only ever combine zero parents or are never read.  The plane
    // parents (kk) depend on k only, the row parents on the row, both uniform across a wavefront.
    // alpha w = alpha 2^-(#odd of j, k) / 2 (odd position) or alpha 2^-(...) (even position): exact
    // scalings, equal to the reference's products alpha * w.
    const double al0 = a.alpha, al1 = a.alpha * 0.5;
    // KO: k & 1 when known at compile time (the z march: chunks start on odd planes), else -1
    auto prolong_pair = [&](double2 v, int jodd, int k, int cro, auto KO) {
        const int K0 = k >> 1;
        const int kodd = decltype(KO)::value >= 0 ? decltype(KO)::value : (k & 1);
        const double awx = ldexp(al1, -(jodd + kodd)), awy = ldexp(al0, -(jodd + kodd));
        const double* cp0 = cring + cro;
#pragma unroll
        for (int aa = 0; aa < 2; ++aa) {
            if (aa == 1 && !kodd) break;
            const double* cp = cp0 + ((K0 + aa) & 1) * CPS;
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                if (bb == 1 && !jodd) break;
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

#pragma unroll
    for (int u = 0; u < NLX; ++u) {
        const int c2 = xlds[u] < 0 ? 0 : xlds[u] % RS, j = xlds[u] < 0 ? j0 : j0 - 2 + xlds[u] / RS;
        pcro[u] = 2 * (c2 + 2 + ((j >> 1) - Jst) * CW) + (j & 1);  // ring column of coarse q0-1+c2
    }

    // ---- global <-> LDS / registers ----
    // The fused-prolongation sweep (PF2) loads x planes two steps ahead (one register set per plane
    // parity, chosen at compile time from the step's parity) and f unconditionally (idle waves load a
    // zero pad pair): its 0.686 -> 0.677 ms (round 3, interleaved A/B).  The plain sweep has no
    // registers to spare for the second set (it spills at its 80-VGPR budget).
    constexpr bool PF2 = PROLONG != 0;
    double2 pxb[PF2 ? 2 : 1][NLX];
#define ZS_PX(B) pxb[PF2 ? (B) : 0]
    // planes past the chunk's last deposited plane k1 + 1 (the loads issued one / two steps ahead in the
    // chunk's last steps) are never used: they load plane k1 + 1 again (an L2 hit) instead of the next
    // chunk's planes from HBM; likewise f past k1
    auto issue_x = [&](int k, auto Bc) {
        // (downward march: below k0 - 2)
        const double* base =
            plane_base(a.xin, k > k1 + 1 ? k1 + 1 : (k < k0 - 2 ? k0 - 2 : k));
#pragma unroll
        for (int u = 0; u < NLX; ++u) ZS_PX(decltype(Bc)::value)[u] = *reinterpret_cast<const double2*>(base + xoff[u]);
    };
    auto deposit_x = [&](int k, auto KO, auto Bc) {
        double* dst = xs + slot(k) * PS;
#pragma unroll
        for (int u = 0; u < NLX; ++u) {
            if (xlds[u] < 0) continue;
            double2 v = ZS_PX(decltype(Bc)::value)[u];
            if (PROLONG && interior_plane(k)) v = prolong_pair(v, pcro[u] & 1, k, pcro[u] >> 1, KO);
            dst[xlds[u]] = v.x;
            dst[xlds[u] + WP] = v.y;
        }
    };
    // f of the item on plane k: (first-colour element, other element) -- two 8-byte loads at
    // wave-uniform element offsets instead of a pair load and per-lane selects
    const int foff = PF2 ? (active_wave ? t.goff : L.off + 1) : t.goff;  // (PF2: idle waves load a zero pad pair)
    auto load_f = [&](int k) {
        return *reinterpret_cast<const double2*>(
            plane_base(a.f, k > k1 ? k1 : (k < k0 - 1 ? k0 - 1 : k)) + foff);
    };

    // fma-chain stencil sum (ascending column order) at LDS offset o of plane k.  The fine FD
    // stencil is symmetric (launch_zsweep checks a[4]=a[22], a[10]=a[16], a[12]=a[14]), so four
    // coefficients serve the seven terms -- same values, same order, same bits.
    const double cz = a.S.a[4], cy = a.S.a[10], cx = a.S.a[12], cc = a.S.a[13];
    // o = LDS offset of the vertex, e = 0 (odd position) / 1 (even position): the x neighbours are
    // the even elements of pairs c-1, c (e = 0) or the odd elements of pairs c, c+1 (e = 1)
    // below = the value at (i, j, k-1): from LDS for the first colour, from a register for the second
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
    // the same sum with the value above (i, j, k+1) from a register (second colour of a downward march)
    auto row_sum_ba = [&](int k, int o, int e, double below, double above) {
        const double* s0 = xs + slot(k) * PS;
        const int xm = e ? o - WP : o + WP - 1;
        double res = cz * below;
        res = fma(cy, s0[o - RS], res);
        res = fma(cx, s0[xm], res);
        res = fma(cc, s0[o], res);
        res = fma(cx, s0[xm + 1], res);
        res = fma(cy, s0[o + RS], res);
        res = fma(cz, above, res);
        return res;
    };
    // the Box-Muller pair of this item on plane k (z.x: odd position i, z.y: even i+1)
    auto noise = [&](int k) -> double2 {
        const uint32_t pair = (uint32_t)(k - 1) * plane_pairs + t.pbase;
        uint32_t key0 = a.G.key.k0, key1 = a.G.key.k1;
        asm volatile("" : "+s"(key0), "+s"(key1));  // keep the round-key schedule out of the SGPR budget
        const Philox4 rnd = philox4x32_10(pair, a.G.tag, s_lo, s_hi, key0, key1);
        double z0, z1;
        normal_pair_t(rnd, &z0, &z1, tab, tab + 64, tab + 128, tab + 192);
        return make_double2(z0, z1);
    };
    // One z step p (LDS ring = planes p-2 .. p+1):
    //   deposit x(p+1) (into the slot plane p-3 left), issue x(p+2) and f(p+1)   | barrier
    //   (PF2: issue x(p+3); f(p+2) is issued once this step has used f(p))
    //   first colour on plane p (core + halo ring)                              | barrier
    //   second colour on plane p-1 (core); plane p-1 is final: store it from the new second-colour
    //   values (registers) and the first-colour values (LDS), and keep the latter as the next
    //   step's z-below values; draw the noise of plane p+1
    // (the next step's deposit writes the slot of plane p-2, which nothing reads any more).
    // f(p) arrives in fcur (loaded one step earlier), f(p+1) goes to fnxt; the second colour's right
    // hand side of plane p goes to pk_out, that of plane p-1 comes from pk_in.  The loop runs the
    // steps in pairs with the register sets swapped, so nothing is copied.
    // PROLONG, coarse ring: the deposit of fine plane p+1 reads coarse planes (p+1)>>1 .. (p+2)>>1;
    // even steps (p even: chunks start on odd planes) issue coarse plane (p+4)/2, odd steps deposit it
    // (its slot held plane (p-1)/2, last read at step p-1).
    double2 z = make_double2(0.0, 0.0);
    double fb = 0.0;  // first-colour value below (plane p-2) at the second-colour position of p-1
    // E0c: std::integral_constant (E0 known at compile time in this copy of the march) or RunE0 (a
    // wave-uniform run-time value: the fused-prolongation sweep, one copy, fewer registers)
    // DNc: a downward march (zpairs, plain sweep only): steps p = k1, k1 - 1, ..., k0 - 1; deposit x(p-1)
    // into the slot of plane p+3, issue x(p-2) and f(p-1); first colour on p, second colour on p+1, whose
    // below value (plane p, written by this step's first colour) comes from LDS and whose above value
    // (plane p+2, whose slot the next step's deposit overwrites) from a register; ring = planes p-1 .. p+2
    auto run = [&](auto E0c, auto DNc) __attribute__((always_inline)) {
        const int E0c_v = E0c.value;
        constexpr bool DN = decltype(DNc)::value;
        constexpr int dz = DN ? -1 : 1;
        auto step = [&](int p, auto ODDc, double2& fcur, double2& fnxt, double pk_in, double& pk_out)
                        __attribute__((always_inline)) {
            constexpr bool odd_step = decltype(ODDc)::value;
            const int e = odd_step ? 1 - E0c_v : E0c_v;  // first-colour element on plane p
            const int o1 = t.lds + e * WP, o2 = t.lds + (1 - e) * WP;
            const bool inf = e ? in1 : in0;  // (compile-time choice)
            // p even on even steps: plane p+1 odd (register set 1), p+3 too
            using Bp = std::integral_constant<int, odd_step ? 0 : 1>;
            deposit_x(p + dz, std::integral_constant<int, DN ? -1 : (odd_step ? 0 : 1)>{}, Bp{});
            if (PROLONG) {
                if (odd_step) deposit_c((p + 3) / 2);
                else issue_c((p + 4) / 2);
            }
            if constexpr (PF2) {
                issue_x(p + 3, Bp{});  // (past the chunk: clamped planes, loaded and never used)
                (void)fnxt;
            } else {
                issue_x(p + 2 * dz, Bp{});
                if (active_wave) fnxt = load_f(p + dz);
            }
            __syncthreads();
            // first colour on plane p: c = fma(sd, z, f), x = fma(omega/diag, c - S, x); the second
            // colour's right-hand side of the pair, c' = fma(sd, z', f')
            if (interior_plane(p) && active_wave) {
                double2 fv = fcur;
                if constexpr (LRF) fv = lr_rhs_pair(fv, lre);
                if (inf) {
                    const double res = row_sum(p, o1, e, xs[slot(p - 1) * PS + o1]);
                    const double crhs = fma(sd, e ? z.y : z.x, e ? fv.y : fv.x);
                    double* s0 = xs + slot(p) * PS;
                    s0[o1] = fma(wd, crhs - res, s0[o1]);
                }
                pk_out = fma(sd, e ? z.x : z.y, e ? fv.x : fv.y);
            }
            if constexpr (PF2) fcur = load_f(p + 2);  // this step's f is used up: the registers take f(p+2)
            __syncthreads();
            // second colour on plane k = p-1 (DN: p+1; its element is e: the parity flips with the plane)
            const int k = p - dz;
            if (core_wave) {
                const bool own = k >= k0 && k < k1;  // a core plane of this tile (interior)
                const double* s0 = xs + slot(k) * PS;
                const double fv = s0[o2];             // final first-colour value
                if (own && rowin) {
                    double sv = s0[o1];
                    if (inf) {
                        // DN: below = plane p (this step's first colour, LDS), above = plane p+2 (fb); the
                        // slot of p+2 takes the next step's deposit, so it is not read here
                        const double res = DN ? row_sum_ba(k, o1, e, xs[slot(p) * PS + o1], fb) : row_sum(k, o1, e, fb);
                        sv = fma(wd, pk_in - res, sv);
                    }
                    double* dst = a.xout + (long long)k * L.sp + t.goff;
                    // (x, y) = (odd, even) element; the second colour is element e here
                    const double2 out = e ? make_double2(fv, sv) : make_double2(sv, fv);
                    // streaming store: keep the write stream out of L2 (plain stores: pre-sweep 0.641 ->
                    // 0.673 ms)
                    __builtin_nontemporal_store(out.x, dst);
                    __builtin_nontemporal_store(out.y, dst + 1);
                }
                fb = fv;  // the next step's value below (UP) / above (DN) at its second-colour position
            }
            if (active_wave && interior_plane(p + dz)) z = noise(p + dz);
        };
        double2 fA = make_double2(0.0, 0.0), fB = make_double2(0.0, 0.0);
        double pkA = 0.0, pkB = 0.0;
        const int pst = DN ? k1 : k0 - 1;  // first step's plane
        if constexpr (PF2) {
            fA = load_f(k0 - 1);
            fB = load_f(k0);
        } else if (active_wave) {
            fA = load_f(pst);
        }
        if (active_wave && interior_plane(pst)) z = noise(pst);
        if constexpr (DN) {
            for (int p = k1; p >= k0 - 1; p -= 2) {
                step(p, std::integral_constant<bool, false>{}, fA, fB, pkB, pkA);
                if (p - 1 >= k0 - 1) step(p - 1, std::integral_constant<bool, true>{}, fB, fA, pkA, pkB);
            }
        } else {
            for (int p = k0 - 1; p <= k1; p += 2) {
                step(p, std::integral_constant<bool, false>{}, fA, fB, pkB, pkA);
                if (p + 1 <= k1) step(p + 1, std::integral_constant<bool, true>{}, fB, fA, pkA, pkB);
            }
        }
    };

    // prologue: planes k0-2, k0-1 in LDS, x(k0) and f(k0-1) in flight, noise of plane k0-1 (k0 is
    // odd: tz even)
    if (PROLONG) {  // coarse planes (k0-3)/2, (k0-1)/2 for the first two deposits, then (k0+1)/2
        issue_c((k0 - 3) / 2);
        deposit_c((k0 - 3) / 2);
        issue_c((k0 - 1) / 2);
        deposit_c((k0 - 1) / 2);
        __syncthreads();
    }
    // (k0 odd: planes k0-2, k0 take register set 1, k0-1, k0+1 set 0)
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    using UP = std::integral_constant<bool, false>;
    using DOWN = std::integral_constant<bool, true>;
    if (!PROLONG && down) {  // downward march (zpairs): planes k1 + 1, k1 in LDS, x(k1 - 1) in flight
        issue_x(k1 + 1, B1{});
        deposit_x(k1 + 1, std::integral_constant<int, -1>{}, B1{});
        issue_x(k1, B0{});
        deposit_x(k1, std::integral_constant<int, -1>{}, B0{});
        issue_x(k1 - 1, B1{});
        if (E0d) run(std::integral_constant<int, 1>{}, DOWN{});  // block-uniform branches
        else run(std::integral_constant<int, 0>{}, DOWN{});
        return;
    }
    issue_x(k0 - 2, B1{});
    deposit_x(k0 - 2, std::integral_constant<int, -1>{}, B1{});
    issue_x(k0 - 1, B0{});
    deposit_x(k0 - 1, std::integral_constant<int, -1>{}, B0{});
    if (PROLONG) {
        __syncthreads();
        issue_c((k0 + 1) / 2);
        deposit_c((k0 + 1) / 2);
        __syncthreads();
    }
    issue_x(k0, B1{});
    if constexpr (PF2) issue_x(k0 + 1, B0{});
    if (PROLONG) run(RunE0{E0}, UP{});
    else if (E0) run(std::integral_constant<int, 1>{}, UP{});  // wave-uniform branch
    else run(std::integral_constant<int, 0>{}, UP{});
}

#undef ZS_PX

inline size_t zsweep_lds_bytes(int XP, int TY, bool prolong) {
    const int RS = 2 * (XP + 2) + 2, R = TY + 4;
    const int coarse = prolong ? 2 * (TY / 2 + 3) * (XP + 8) : 0;
    return (size_t)(4 * R * RS + 3 * 64 + 130 + coarse) * sizeof(double);
}

}  // namespace mgmc
