// mgmc_tail.hpp -- the coarsest levels' whole sub-cycle in one workgroup, every level in LDS.
//
// Below a certain size a level's kernels are launch-bound: at 512^3 the 15^3 and 7^3 levels took 20
// launches of 4.8-24 us per cycle (pre-sweep colour-pair passes, residual + restriction, coarse SSOR
// sampler, prolongation, post-sweep passes) for 3,718 unknowns; the floor of one launch in the cycle
// graph is ~3.6 us (k_qoi_record, one wavefront).  k_tail replays that stretch of the cycle's op list
// -- every op of one call of build_ops_level(lt), i.e. MultigridMCSampler::apply's recursion from
// level lt down (sampler/multigridmc_sampler.cc:103-138) -- inside one 1024-thread workgroup with x and
// f of every level resident in LDS, __syncthreads between phases instead of kernel boundaries.
//
// Each op does exactly the arithmetic of the kernel it replaces, so the cycle is bitwise the same:
//  * Gibbs sweep (k_sweep_pairs / k_sweep_mc / k_coarse_ssor_lds): colours in order (forward
//    0..2^d-1, backward reversed); c = fma(sd, xi, f) with xi the cos / sin branch of the Philox pair
//    (odd i, i+1) of the sweep's tag; x = fma(omega/diag, c - S, x), S the stencil fma chain in
//    ascending column order.  The right hand sides of a sweep are evaluated first, one Box-Muller per
//    pair for all colours at once (f does not change during a sweep), then the colour passes;
//  * residual + restriction (k_zresrestrict / k_residual_restrict): r = f - (0 + sum a x ascending)
//    at every fine vertex, then f_c = sum over (sz, sy, sx) of (1 w1(sx) w1(sy) w1(sz)) r, x_c = 0;
//  * prolongate-add (k_prolongate_pairs): x += (alpha w) x_c over the interior parents in ascending
//    coarse order.
//  * low-rank levels (posterior Q = A + B Sigma^{-1} B^T with small sparse columns, the k_lr_small
//    path): before a sweep f += B Sigma^{-1/2} xi' on the rows of B (k_lr_patch / k_lr_small noise),
//    after it w = B^T x by one wavefront per column (lr_wave_dot's order) and x -= B_bar w, f restored;
//    before a residual f -= B (Sigma^{-1} B^T x), restored after the restriction
//    (sor_sampler.cc:48-56, sor_smoother.cc:41-53, linear_operator.hh:66-76).
// LDS layout per level: the (nx+1)(ny+1)(nz+1) vertices including the zero boundary, x fastest, rows
// unpadded, 3D planes padded to 8 (mod 16) doubles (tail_layout, mgmc_capi.hip); one scratch array (right hand sides / residuals) of the largest tail level; the saved f
// on the rows of B of every low-rank level.
#pragma once
#include "mgmc_kernels.hpp"
#include "mgmc_lowrank.hpp"

namespace mgmc {

enum TailKind { TAIL_SWEEP = 0, TAIL_RESTRICT = 1, TAIL_PROLONG = 2, TAIL_COARSE = 3 };
constexpr int TAIL_MAX_LEVELS = 4;
constexpr int TAIL_MAX_OPS = 96;

struct TailOp {
    int kind;
    int level;     // index into TailArgs::lv (0 = level lt)
    int dir;       // sweeps: 1 forward, 2 backward (MGMC_FORWARD / MGMC_BACKWARD)
    uint32_t tag;  // first sweep tag
    int nsweeps;   // TAIL_COARSE: forward/backward sweeps, tags tag, tag+1, ...
    int zoff;      // sweeps, with TailArgs::zb: this op's Box-Muller pairs start at zb[zoff] (one sweep's
                   // npair x nrow items after the other, the item order of the right-hand-side loop)
};

// one job of the tail's pre-drawn noise: the pairs of one sweep of one tail level (drawn by spare
// workgroups of the residual + restriction launch before the tail, mgmc_zrestrict.hpp)
struct TailNoiseJob {
    int nx, ny, nz;    // the level's cells (pair ids: pair_id<3>)
    uint32_t tag;
    int zoff;          // first item in zb
};
constexpr int TAIL_MAX_NOISE_JOBS = 24;

// one job of the noise the tail launch draws for a sweep after it (the first post-sweep of each 3D
// Galerkin level between the tail and the fine level, plan_drawn_noise in mgmc_capi.hip): every pair of
// the level's sweep with tag `tag`, pair id q -> dst[q] (pair_id<3> order), drawn by the launch's spare
// workgroups while the tail's one workgroup runs on one CU
struct PostNoiseJob {
    int nx, ny, nz;
    uint32_t tag;
    double2* dst;
};
constexpr int TAIL_MAX_PN_JOBS = 8;

struct TailLevel {
    Layout G;      // LDS layout (off 0, sx = nx+1, sp = sx (ny+1), 3D padded to 8 mod 16)
    int ox, of;    // LDS offsets (doubles) of x and f
    int ncolours;
    int fold;      // a fold level (27-point, reflection-symmetric): the residual's sum is fold27's
    double sd, wd; // sqrt(diag (2-omega)/omega), omega/diag
    StencilArg S;
    // low-rank part (m = 0: none); every offset in the LDS layout G
    int m, nrows, osave;
    int nbar[2];
    const LRColMeta* meta;
    const int* ent_off;
    const double* ent_val;
    const double* sc_one;
    const double* sc_inv;
    const double* sq;
    const int* bar_off[2];
    const double* bar_val[2];
    const int* rows_off;
    const double* coef;
    const uint64_t* mask;
};

struct TailArgs {
    int nlev, nops, oscr, lds_doubles;
    int x_zero;            // level lt's x is known zero on entry (the restriction before the tail zeroed it, lt > 0):
                           // it is not loaded (the LDS fill already holds the zeros)
    double alpha;          // coarse_scaling
    RngKey key;
    const uint64_t* sample;
    double* xg;            // level lt in HBM (its padded layout Lg)
    const double* fg;
    Layout Lg;
    long long cs;          // batched chains: doubles between chains of level lt (one workgroup per chain)
    uint32_t chain0, seed_hi;  // chain c's Philox key: (key.k0, lo32(chain0 + c) ^ seed_hi)
    const double2* zb;     // pre-drawn Box-Muller pairs of the sweeps (nullptr: drawn here), zbs per chain
    long long zbs;
    int npn;               // post-sweep noise jobs (one chain only): drawn by the launch's blocks from nwg on
    PostNoiseJob pn[TAIL_MAX_PN_JOBS];
    TailLevel lv[TAIL_MAX_LEVELS];
    TailOp ops[TAIL_MAX_OPS];
    unsigned long long* prof;  // (timing builds, MGMC_TAIL_PROF: wall-clock stamps per phase; else null)
};

#ifdef MGMC_TAIL_PROF  // timing builds only: one wall-clock stamp per phase from thread 0
#define TAIL_STAMP(slot)                                                          \
    do {                                                                          \
        if (A->prof && threadIdx.x == 0 && blockIdx.x == 0) A->prof[slot] = wall_clock64(); \
    } while (0)
#else
#define TAIL_STAMP(slot) \
    do {                 \
    } while (0)
#endif

// Per-op constants pinned in SGPRs.  The tail's arguments sit in global memory behind a pointer; a
// scalar load the compiler leaves in flight inside a colour pass shares lgkmcnt with the LDS reads and
// returns out of order, so every wait in the pass became lgkmcnt(0) and the 27 window reads ran one at
// a time (0.8-1 us per colour pass, round 4).  An empty asm with a "+s" operand makes the value live
// in an SGPR from here on: the loads complete before the pass, and nothing is re-loaded inside it.
__device__ __forceinline__ void tail_pin(int& v) { asm volatile("" : "+s"(v)); }
__device__ __forceinline__ void tail_pin(uint32_t& v) { asm volatile("" : "+s"(v)); }
__device__ __forceinline__ void tail_pin(long long& v) { asm volatile("" : "+s"(v)); }
__device__ __forceinline__ void tail_pin(double& v) { asm volatile("" : "+s"(v)); }
__device__ __forceinline__ void tail_pin(Layout& G) {
    tail_pin(G.nx);
    tail_pin(G.ny);
    tail_pin(G.nz);
    tail_pin(G.off);
    tail_pin(G.sx);
    tail_pin(G.sp);
}
template <int NPTS, bool SYM>
__device__ __forceinline__ void tail_pin(StencilArg& S) {
#pragma unroll
    for (int q = 0; q < NPTS; ++q)
        if (!SYM || sym_rep(q) == q) tail_pin(S.a[q]);
}

// LDS byte address of a pointer into the dynamic shared array
__device__ __forceinline__ uint32_t lds_addr(const double* p) {
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) double*)p;
}
#define TAIL_RD(n, b, o) "ds_read_b64 %" #n ", %" #b " offset:" #o "\n"
// The 3^d window of x around p (v[q], q = 9 (dz+1) + 3 (dy+1) + dx+1) of an LDS-resident level, read
// as its 3^(d-1) rows, each from one address with the immediate offsets 0 / 8 / 16 bytes, in one asm
// statement that ends in the wait:
//  * every read is issued before the first use (left to itself the compiler read one or two values,
//    waited, multiplied and read the next: the LDS latency 9-14 times per vertex);
//  * one address instruction per row, not two or three per value (a colour pass's address arithmetic
//    was as long as its fma chain);
//  * single ds_read_b64: a paired ds_read2_b64 moves 8 bytes per lane at half the rate
//    (MI355X_MICROARCH.md, LDS table), and each row's aligned pair as one ds_read_b128 doubled the 15^3
//    colour passes' time (round 5).
// The memory clobber keeps the caller's earlier LDS reads (the right-hand side) issued before it.
template <int DIM, int NPTS>
__device__ __forceinline__ void tail_window(const double* __restrict__ x, int p, const Layout& G, double (&v)[NPTS]) {
    const uint32_t px = lds_addr(x) + 8u * (uint32_t)(p - 1);
    if constexpr (NPTS == 27) {
        uint32_t rb[9];
#pragma unroll
        for (int rr = 0; rr < 9; ++rr) rb[rr] = px + 8u * (uint32_t)((rr / 3 - 1) * (int)G.sp + (rr % 3 - 1) * (int)G.sx);
        asm volatile(TAIL_RD(0, 27, 0) TAIL_RD(1, 27, 8) TAIL_RD(2, 27, 16) TAIL_RD(3, 28, 0) TAIL_RD(4, 28, 8)
                     TAIL_RD(5, 28, 16) TAIL_RD(6, 29, 0) TAIL_RD(7, 29, 8) TAIL_RD(8, 29, 16) TAIL_RD(9, 30, 0)
                     TAIL_RD(10, 30, 8) TAIL_RD(11, 30, 16) TAIL_RD(12, 31, 0) TAIL_RD(13, 31, 8) TAIL_RD(14, 31, 16)
                     TAIL_RD(15, 32, 0) TAIL_RD(16, 32, 8) TAIL_RD(17, 32, 16) TAIL_RD(18, 33, 0) TAIL_RD(19, 33, 8)
                     TAIL_RD(20, 33, 16) TAIL_RD(21, 34, 0) TAIL_RD(22, 34, 8) TAIL_RD(23, 34, 16) TAIL_RD(24, 35, 0)
                     TAIL_RD(25, 35, 8) TAIL_RD(26, 35, 16) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                       "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]),
                       "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15]), "=&v"(v[16]), "=&v"(v[17]), "=&v"(v[18]),
                       "=&v"(v[19]), "=&v"(v[20]), "=&v"(v[21]), "=&v"(v[22]), "=&v"(v[23]), "=&v"(v[24]),
                       "=&v"(v[25]), "=&v"(v[26])
                     : "v"(rb[0]), "v"(rb[1]), "v"(rb[2]), "v"(rb[3]), "v"(rb[4]), "v"(rb[5]), "v"(rb[6]), "v"(rb[7]),
                       "v"(rb[8])
                     : "memory");
    } else {
        static_assert(NPTS == 9, "tail stencils are 27- or 9-point");
        const uint32_t r0 = px - 8u * (uint32_t)G.sx, r2 = px + 8u * (uint32_t)G.sx;
        asm volatile(TAIL_RD(0, 9, 0) TAIL_RD(1, 9, 8) TAIL_RD(2, 9, 16) TAIL_RD(3, 10, 0) TAIL_RD(4, 10, 8)
                     TAIL_RD(5, 10, 16) TAIL_RD(6, 11, 0) TAIL_RD(7, 11, 8) TAIL_RD(8, 11, 16) "s_waitcnt lgkmcnt(0)"
                     : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
                       "=&v"(v[7]), "=&v"(v[8])
                     : "v"(r0), "v"(px), "v"(r2)
                     : "memory");
    }
}
#undef TAIL_RD
// one vertex of a colour pass: x_p = fma(wd, c_p - S, x_p) with c_p = scr[p] and S = a_0 x_0, then
// fma(a_k, x_k, .) ascending (= stencil_fma); c_p is read just before the window (one LDS round trip
// per vertex) and x_p is the window's centre
template <int DIM, int NPTS, bool SYM>
__device__ __forceinline__ void tail_gibbs(double* __restrict__ x, const double* __restrict__ scr, int p,
                                           const Layout& G, const StencilArg& S, double wd) {
    const double c = scr[p];
    double v[NPTS];
    tail_window<DIM, NPTS>(x, p, G, v);
    double res = stencil_coef<SYM && NPTS == 27>(S, 0) * v[0];
#pragma unroll
    for (int q = 1; q < NPTS; ++q) res = fma(stencil_coef<SYM && NPTS == 27>(S, q), v[q], res);
    x[p] = fma(wd, c - res, v[NPTS / 2]);
}
// 0.0 + a_0 x_0 + a_1 x_1 + ... ascending, separate multiply and add (= stencil_sum)
template <int DIM, int NPTS, bool SYM>
__device__ __forceinline__ double tail_sum(const double* __restrict__ x, int p, const Layout& G, const StencilArg& S) {
    double v[NPTS];
    tail_window<DIM, NPTS>(x, p, G, v);
    double res = 0.0;
#pragma unroll
    for (int q = 0; q < NPTS; ++q) res += stencil_coef<SYM && NPTS == 27>(S, q) * v[q];
    return res;
}

// The spare workgroups of a tail launch (blocks nwg ..): the Box-Muller pairs of the post-sweep noise
// jobs (PostNoiseJob), pair q of a job -> dst[q], the same Philox counter and arithmetic as the sweep
// kernel would use (normal_pair_t with the tables in LDS), chain 0's key.  Items are dealt round-robin
// over every spare thread, so consecutive lanes store consecutive 16-byte pairs.
__device__ __forceinline__ void tail_post_noise(const TailArgs* __restrict__ A, int nwg, double* tab) {
    for (int q = threadIdx.x; q < 64; q += blockDim.x) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }
    for (int q = threadIdx.x; q < 130; q += blockDim.x) tab[192 + q] = SINCOS_TAB[q];
    __syncthreads();
    const uint64_t sample = *A->sample;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    const RngKey key = A->key;
    const uint32_t nw = (gridDim.x - (uint32_t)nwg) * blockDim.x;
    const uint32_t w0 = (blockIdx.x - (uint32_t)nwg) * blockDim.x + threadIdx.x;
    const int npn = A->npn;
    for (int jb = 0; jb < npn; ++jb) {
        const PostNoiseJob J = A->pn[jb];
        const uint32_t n = (uint32_t)(J.nx / 2) * (uint32_t)(J.ny - 1) * (uint32_t)(J.nz - 1);
        for (uint32_t q = w0; q < n; q += nw) {
            const Philox4 r = philox4x32_10(q, J.tag, s_lo, s_hi, key.k0, key.k1);
            double z0, z1;
            normal_pair_t(r, &z0, &z1, tab, tab + 64, tab + 128, tab + 192);
            J.dst[q] = make_double2(z0, z1);
        }
    }
}

// SYM: every 27-point level of the tail has a reflection-symmetric stencil (stencil_coef)
// nwg: workgroups running the tail (one per chain; a kernel argument, not a field of *A: the tail's first
// read of its arguments would be a dependent miss); blocks from nwg on draw the post-sweep noise
template <int DIM, bool SYM = false>
__global__ void __launch_bounds__(1024) k_tail(const TailArgs* __restrict__ A, int nwg) {
    constexpr int NPTS = DIM == 3 ? 27 : 9;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if ((int)blockIdx.x >= nwg) {  // a spare workgroup: post-sweep noise only
        tail_post_noise(A, nwg, lds);
        return;
    }
    const int tid = threadIdx.x, nt = blockDim.x;
    const int ntot = A->lds_doubles;
    // the arguments' cache lines into L2 by vector loads, one line per thread, behind the LDS fill: the
    // ops' scalar loads of them (each op's fields, then its level's) are otherwise dependent misses to
    // HBM, the cycle's fine-level sweeps having flushed the caches (44 -> 42 us at 512^3, round 5)
    uint32_t pre = 0;
    if (tid * 64 < (int)sizeof(TailArgs)) pre = reinterpret_cast<const uint32_t*>(A)[tid * 16];
    for (int q = tid; q < ntot; q += nt) lds[q] = 0.0;
    asm volatile("" ::"v"(pre));
    __syncthreads();
    const uint64_t sample = *A->sample;
    const int ch = blockIdx.x;  // batched chains: one workgroup per chain
    double* const xg = A->xg + ch * A->cs;
    const double* const fg = A->fg + ch * A->cs;
    RngKey key = A->key;
    if (ch) key.k1 = (A->chain0 + (uint32_t)ch) ^ A->seed_hi;
    const uint32_t s_lo = (uint32_t)sample, s_hi = (uint32_t)(sample >> 32);
    double* scr = lds + A->oscr;
    TAIL_STAMP(0);

    __shared__ double lr_s[LR_MAX_M];
    const int wave = tid >> 6, lane = tid & 63, nwave = nt >> 6;
    // w_k = sc_k (B^T x)_k, one wavefront per column (lr_wave_dot with LDS offsets)
    auto lr_dots = [&](const TailLevel& t, const double* sc, const double* x) {
        for (int k = wave; k < t.m; k += nwave) {
            const LRColMeta c = t.meta[k];
            const double sk = sc[k];
            double acc = 0.0;
            for (int e = lane; e < (int)c.n; e += 64) {
                const long long q = c.ent0 + e;
                acc = acc + (sk * t.ent_val[q]) * x[t.ent_off[q]];
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) acc = acc + __shfl_xor(acc, off, 64);
            double tot = lane == 0 ? 0.0 + acc : 0.0;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) tot = tot + __shfl_xor(tot, off, 64);
            if (lane == 0) lr_s[k] = tot;
        }
    };
    // f on the rows of B: save it, then f + B s (sign +1) or f - B s (sign -1), s = lr_s
    auto lr_patch_rows = [&](const TailLevel& t, double* f, int sign) {
        double* save = lds + t.osave;
        for (int u = tid; u < t.nrows; u += nt) {
            const int p = t.rows_off[u];
            const uint64_t msk = t.mask[u];
            const double* cf = t.coef + (long long)u * t.m;
            double e = 0.0;
            for (int k = 0; k < t.m; ++k)
                if ((msk >> k) & 1) e = e + cf[k] * lr_s[k];
            const double y = f[p];
            save[u] = y;
            f[p] = sign > 0 ? y + e : y - e;
        }
    };
    auto lr_restore_rows = [&](const TailLevel& t, double* f) {
        const double* save = lds + t.osave;
        for (int u = tid; u < t.nrows; u += nt) f[t.rows_off[u]] = save[u];
    };

    // body(i, j, k) for every interior vertex of a level, threads strided over a power-of-two box: bit
    // fields instead of integer divisions (each a ~40-instruction sequence on the device), with the
    // box's vertices outside the interior skipped.  The order is immaterial: vertices are independent.
    auto bits_of = [](int n) { return 32 - __builtin_clz((unsigned)(n - 1 > 0 ? n - 1 : 1)); };
    auto for_interior = [&](const Layout& G, auto&& body) __attribute__((always_inline)) {
        const int bx = bits_of(G.nx), by = bits_of(G.ny), bz = DIM == 3 ? bits_of(G.nz) : 0;
        const int tot = 1 << (bx + by + bz);
        for (int q = tid; q < tot; q += nt) {
            const int i = q & ((1 << bx) - 1), j = (q >> bx) & ((1 << by) - 1), k = DIM == 3 ? q >> (bx + by) : 0;
            if (i < 1 || i > G.nx - 1 || j < 1 || j > G.ny - 1 || (DIM == 3 && (k < 1 || k > G.nz - 1))) continue;
            body(i, j, k);
        }
    };

    {  // level lt from HBM (boundary entries stay 0)
        const TailLevel& t0 = A->lv[0];
        for_interior(t0.G, [&](int i, int j, int k) {
            if (!A->x_zero) lds[t0.ox + (int)t0.G.at(i, j, k)] = xg[A->Lg.at(i, j, k)];
            lds[t0.of + (int)t0.G.at(i, j, k)] = fg[A->Lg.at(i, j, k)];
        });
    }
    __syncthreads();

    TAIL_STAMP(1);
    const double2* zb = A->zb ? A->zb + ch * A->zbs : nullptr;
    [[maybe_unused]] int stamp_op = 0;  // (MGMC_TAIL_PROF: the op being run)
    // one Gibbs sweep of level t: right hand sides of every vertex, then the colour passes
    auto sweep = [&](const TailLevel& t, int dir, uint32_t tag, int zoff) {
        Layout G = t.G;
        StencilArg S = t.S;
        double sd = t.sd, wd = t.wd;
        int ox = t.ox, of = t.of, nc = t.ncolours, lrm = t.m;
        tail_pin(G);
        tail_pin<NPTS, SYM>(S);
        tail_pin(sd);
        tail_pin(wd);
        tail_pin(ox);
        tail_pin(of);
        tail_pin(nc);
        tail_pin(lrm);
        double* x = lds + ox;
        double* f = lds + of;
        if (lrm > 0) {  // f += B Sigma^{-1/2} xi' (the sweep's m extra normals)
            if (2 * tid < t.m) {
                const Philox4 r = philox4x32_10(LR_PAIR0 + (uint32_t)tid, tag, s_lo, s_hi, key.k0, key.k1);
                double z0, z1;
                normal_pair(r, &z0, &z1);
                lr_s[2 * tid] = t.sq[2 * tid] * z0;
                if (2 * tid + 1 < t.m) lr_s[2 * tid + 1] = t.sq[2 * tid + 1] * z1;
            }
            __syncthreads();
            lr_patch_rows(t, f, 1);
            __syncthreads();
        }
        const int npair = G.nx / 2;
        // pairs (i0 = 2m + 1, i0 + 1) over a power-of-two box (bit fields, no divisions); q = the pair's
        // item index in the pre-drawn noise (row-major over (k, j), m fastest)
        const int bm = bits_of(npair), by = bits_of(G.ny), bz = DIM == 3 ? bits_of(G.nz) : 0;
        for (int qq = tid; qq < (1 << (bm + by + bz)); qq += nt) {
            const int m = qq & ((1 << bm) - 1), j = (qq >> bm) & ((1 << by) - 1), k = DIM == 3 ? qq >> (bm + by) : 0;
            if (m >= npair || j < 1 || j > G.ny - 1 || (DIM == 3 && (k < 1 || k > G.nz - 1))) continue;
            const int q = ((DIM == 3 ? k - 1 : 0) * (G.ny - 1) + (j - 1)) * npair + m;
            const int i0 = 2 * m + 1;
            if (i0 > G.nx - 1) continue;
            double z0, z1;
            if (zb) {
                const double2 zz = zb[zoff + q];
                z0 = zz.x;
                z1 = zz.y;
            } else {
                const Philox4 rnd = philox4x32_10(pair_id<DIM>(G, i0, j, k), tag, s_lo, s_hi, key.k0, key.k1);
                normal_pair(rnd, &z0, &z1);
            }
            const int p = (int)G.at(i0, j, k);
            scr[p] = fma(sd, z0, f[p]);
            if (i0 + 1 <= G.nx - 1) scr[p + 1] = fma(sd, z1, f[p + 1]);
        }
        __syncthreads();
        TAIL_STAMP(2 + 2 * stamp_op);
        // vertices of colour c: coordinate d = 2 - bit_d(c) + 2 t_d, t_d < the class size along d.
        // Small levels (every class <= 8 x 8 x 16, 2D 32 x 32 vertices): thread bits are the class
        // coordinates.  3D: tid = ti | tk0 << 3 | tj << 4 | (tk >> 1) << 7, so a half-wave holds class
        // planes tk and tk+1 (vertex planes 2 apart, 16 bank pairs apart with the padded plane stride of
        // tail_layout): 2-way banks.  Each thread's vertex of every colour (an offset from pb) and the
        // colours it has (bits of vm) are worked out once per sweep: class sizes and bounds per pass were
        // ~40 scalar instructions and six branches in every wavefront, half of a pass's time.
        const int cmi = (G.nx - 2) / 2 + 1, cmj = (G.ny - 2) / 2 + 1, cmk = DIM == 3 ? (G.nz - 2) / 2 + 1 : 1;
        const bool fast = DIM == 3 ? (cmi <= 8 && cmj <= 8 && cmk * 64 <= nt) : (cmi <= 32 && cmj * 32 <= nt);
        const int ti = DIM == 3 ? (tid & 7) : (tid & 31);
        const int tj = DIM == 3 ? ((tid >> 4) & 7) : (tid >> 5);
        const int tk = DIM == 3 ? (((tid >> 3) & 1) | ((tid >> 7) << 1)) : 0;
        const int pb = (int)G.at(2 + 2 * ti, 2 + 2 * tj, DIM == 3 ? 2 + 2 * tk : 0);
        uint32_t vm = 0;
#pragma unroll
        for (int c = 0; c < (DIM == 3 ? 8 : 4); ++c) {
            const bool in = 2 - (c & 1) + 2 * ti <= G.nx - 1 && 2 - ((c >> 1) & 1) + 2 * tj <= G.ny - 1 &&
                            (DIM == 2 || 2 - ((c >> 2) & 1) + 2 * tk <= G.nz - 1);
            vm |= (uint32_t)in << c;
        }
        for (int cc = 0; cc < nc; ++cc) {
            const int c = dir == 1 ? cc : nc - 1 - cc;
            if (fast) {
                if ((vm >> c) & 1) {
                    const int p = pb - (c & 1) - ((c >> 1) & 1) * (int)G.sx - (DIM == 3 ? ((c >> 2) & 1) * (int)G.sp : 0);
                    tail_gibbs<DIM, NPTS, SYM>(x, scr, p, G, S, wd);
                }
            } else {
                const int fi = 2 - (c & 1), fj = 2 - ((c >> 1) & 1), fk = DIM == 3 ? 2 - ((c >> 2) & 1) : 0;
                const int ci = fi > G.nx - 1 ? 0 : (G.nx - 1 - fi) / 2 + 1;
                const int cj = fj > G.ny - 1 ? 0 : (G.ny - 1 - fj) / 2 + 1;
                const int ck = DIM == 3 ? (fk > G.nz - 1 ? 0 : (G.nz - 1 - fk) / 2 + 1) : 1;
                for (int q = tid; q < ci * cj * ck; q += nt) {
                    const int i = fi + 2 * (q % ci), r = q / ci;
                    const int j = fj + 2 * (r % cj), k = DIM == 3 ? fk + 2 * (r / cj) : 0;
                    tail_gibbs<DIM, NPTS, SYM>(x, scr, (int)G.at(i, j, k), G, S, wd);
                }
            }
            __syncthreads();
        }
        if (lrm > 0) {  // x -= B_bar (B^T x), f restored
            lr_dots(t, t.sc_one, x);
            lr_restore_rows(t, f);
            __syncthreads();
            const int d = dir == 1 ? 0 : 1;
            const int* boff = t.bar_off[d];
            const double* bval = t.bar_val[d];
            for (int u = tid; u < t.nbar[d]; u += nt) {
                const double* bv = bval + (long long)u * t.m;
                double acc = 0.0;
                for (int k = 0; k < t.m; ++k) acc = fma(bv[k], lr_s[k], acc);
                const int p = boff[u];
                x[p] = x[p] - acc;
            }
            __syncthreads();
        }
    };

    for (int o = 0; o < A->nops; ++o) {
        TailOp op = A->ops[o];
        tail_pin(op.kind);
        tail_pin(op.level);
        tail_pin(op.dir);
        tail_pin(op.tag);
        tail_pin(op.nsweeps);
        tail_pin(op.zoff);
        const TailLevel& t = A->lv[op.level];
        stamp_op = o;
        if (op.kind == TAIL_SWEEP) {
            sweep(t, op.dir, op.tag, op.zoff);
        } else if (op.kind == TAIL_COARSE) {
            for (int s = 0; s < op.nsweeps; ++s) {
                const int npair = t.G.nx / 2, nrow = (t.G.ny - 1) * (DIM == 3 ? t.G.nz - 1 : 1);
                sweep(t, (s & 1) ? 2 : 1, op.tag + (uint32_t)s, op.zoff + s * npair * nrow);
            }
        } else if (op.kind == TAIL_RESTRICT) {
            const TailLevel& c = A->lv[op.level + 1];
            Layout G = t.G, Gc = c.G;
            StencilArg S = t.S;
            int ox = t.ox, of = t.of, cox = c.ox, cof = c.of, lrm = t.m;
            tail_pin(G);
            tail_pin(Gc);
            tail_pin<NPTS, SYM>(S);
            tail_pin(ox);
            tail_pin(of);
            tail_pin(cox);
            tail_pin(cof);
            tail_pin(lrm);
            const double* x = lds + ox;
            double* f = lds + of;
            if (lrm > 0) {  // r = (f - B Sigma^{-1} B^T x) - A x
                lr_dots(t, t.sc_inv, x);
                __syncthreads();
                lr_patch_rows(t, f, -1);
                __syncthreads();
            }
            if (DIM == 3 && NPTS == 27 && t.fold) {
                // runs of TSEG vertices along x per thread: each of the 9 window rows is read once over
                // TSEG + 2 columns (9 (TSEG + 2) LDS reads instead of 27 TSEG) and its values go straight
                // into the vertices' class sums -- rows ascending, columns ascending: fold27's member
                // order, so the same bits
                constexpr int TSEG = 2;
                const int nseg = (G.nx - 1 + TSEG - 1) / TSEG;
                const int bs = bits_of(nseg), by = bits_of(G.ny), bz = bits_of(G.nz);
                for (int q = tid; q < (1 << (bs + by + bz)); q += nt) {
                    const int sg = q & ((1 << bs) - 1), j = (q >> bs) & ((1 << by) - 1), k = q >> (bs + by);
                    if (sg >= nseg || j < 1 || j > G.ny - 1 || k < 1 || k > G.nz - 1) continue;
                    const int i0 = 1 + TSEG * sg;
                    const int p0 = (int)G.at(i0, j, k);
                    double cs[TSEG][8];
#pragma unroll
                    for (int rr = 0; rr < 9; ++rr) {
                        double w[TSEG + 2];  // columns i0 - 1 .. i0 + TSEG (past the row end: the next
                                             // row's zero boundary vertex, used by no interior vertex)
#pragma unroll
                        for (int c = 0; c < TSEG + 2; ++c) {
                            int idx = p0 + (rr / 3 - 1) * (int)G.sp + (rr % 3 - 1) * (int)G.sx + c - 1;
                            asm volatile("" : "+v"(idx));
                            w[c] = x[idx];
                        }
#pragma unroll
                        for (int e = 0; e < TSEG; ++e)
#pragma unroll
                            for (int dx = 0; dx < 3; ++dx) {
                                const int t27 = 3 * rr + dx, cl = fold_class(t27);
                                if (fold_rep(cl) == t27) cs[e][cl] = w[e + dx];
                                else cs[e][cl] = cs[e][cl] + w[e + dx];
                            }
                    }
#pragma unroll
                    for (int e = 0; e < TSEG; ++e) {
                        if (i0 + e > G.nx - 1) break;
                        double y = S.a[fold_rep(7)] * cs[e][7];
#pragma unroll
                        for (int cl = 6; cl >= 0; --cl) y = fma(S.a[fold_rep(cl)], cs[e][cl], y);
                        scr[p0 + e] = f[p0 + e] - y;
                    }
                }
            } else {
                for_interior(G, [&](int i, int j, int k) {
                    const long long p = G.at(i, j, k);
                    scr[p] = f[p] - tail_sum<DIM, NPTS, SYM>(x, (int)p, G, S);
                });
            }
            __syncthreads();
            for_interior(Gc, [&](int I, int J, int K) {
                const int pf = (int)G.at(2 * I, 2 * J, 2 * K);
                double rv[NPTS];  // the 3^d residuals (tail_window)
                tail_window<DIM, NPTS>(scr, pf, G, rv);
                double result = 0.0;
                const int zr = DIM == 3 ? 1 : 0;
#pragma unroll
                for (int sz = -zr; sz <= zr; ++sz)
#pragma unroll
                    for (int sy = -1; sy <= 1; ++sy)
#pragma unroll
                        for (int sx = -1; sx <= 1; ++sx) {
                            double w = 1.0;
                            w *= w1(sx);
                            w *= w1(sy);
                            if (DIM == 3) w *= w1(sz);
                            result += w * rv[(sz + zr) * 9 + (sy + 1) * 3 + (sx + 1)];
                        }
                const long long pc = Gc.at(I, J, K);
                lds[cof + pc] = result;
                lds[cox + pc] = 0.0;
            });
            if (lrm > 0) lr_restore_rows(t, f);
            __syncthreads();
        } else {  // TAIL_PROLONG: x_l += alpha P x_{l+1}
            const TailLevel& c = A->lv[op.level + 1];
            Layout G = t.G, Gc = c.G;
            int ox = t.ox, cox = c.ox;
            double alpha = A->alpha;
            tail_pin(G);
            tail_pin(Gc);
            tail_pin(ox);
            tail_pin(cox);
            tail_pin(alpha);
            double* x = lds + ox;
            const double* xc = lds + cox;
            // every vertex takes the 2^d candidate parents (d >> 1, (d + 1) >> 1) per axis in the
            // reference's order (kk, jj, ii ascending), with weight 0 where the two coincide (d even):
            // those terms add an exact 0, and parents on the coarse boundary are zeros of the LDS
            // layout, so the sum of the present parents' terms is unchanged (only a zero's sign can
            // differ) -- and no lane diverges on the parent count
            for_interior(G, [&](int i, int j, int k) {
                const long long p = G.at(i, j, k);
                double v = x[p];
                const int ia = i >> 1, ja = j >> 1, ka = DIM == 3 ? k >> 1 : 0;
                const double wi[2] = {(i & 1) ? 0.5 : 1.0, (i & 1) ? 0.5 : 0.0};
                const double wj[2] = {(j & 1) ? 0.5 : 1.0, (j & 1) ? 0.5 : 0.0};
                const double wk[2] = {(DIM == 3 && (k & 1)) ? 0.5 : 1.0, (DIM == 3 && (k & 1)) ? 0.5 : 0.0};
                double c[2][2][2];
                const int pc0 = (int)Gc.at(ia, ja, ka);
#pragma unroll
                for (int aa = 0; aa < (DIM == 3 ? 2 : 1); ++aa)
#pragma unroll
                    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                        for (int cc = 0; cc < 2; ++cc) c[aa][bb][cc] = xc[pc0 + aa * (int)Gc.sp + bb * (int)Gc.sx + cc];
#pragma unroll
                for (int aa = 0; aa < (DIM == 3 ? 2 : 1); ++aa)
#pragma unroll
                    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                        for (int cc = 0; cc < 2; ++cc) {
                            double w = 1.0;
                            w *= wi[cc];
                            w *= wj[bb];
                            if (DIM == 3) w *= wk[aa];
                            v += alpha * w * c[aa][bb][cc];
                        }
                x[p] = v;
            });
            __syncthreads();
        }
        TAIL_STAMP(3 + 2 * o);
    }

    {  // level lt back to HBM
        const TailLevel& t0 = A->lv[0];
        for_interior(t0.G, [&](int i, int j, int k) { xg[A->Lg.at(i, j, k)] = lds[t0.ox + (int)t0.G.at(i, j, k)]; });
    }
    TAIL_STAMP(2 + 2 * A->nops);
}

}  // namespace mgmc
