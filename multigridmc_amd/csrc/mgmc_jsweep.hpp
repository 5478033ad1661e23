// mgmc_jsweep.hpp -- j-marching half-sweeps of the 8-colour Gibbs sweep of a 3D Galerkin-shaped
// (27-point) level with rows of NP = 128 or 256 pairs (level 1 of the 512^3 hierarchy; the FEM prior's
// fine level at 512^3): both colour pairs of one k parity in one launch, x read about 1.5 times per
// half instead of once per colour-pair pass.
//
// A sweep's four colour-pair passes (mgmc_gsweep.hpp: forward (0,1), (2,3) | (4,5), (6,7), backward
// reversed) come in k-parity halves.  Within a half (own planes k of parity kp), the second pair's rows
// (parity jB) read the first pair's rows (parity jA) of their own plane at j-1 and j+1; everything else
// is old in the half (rows of their own parity, planes k +- 1 of the other parity).  One workgroup
// marches a chunk of one own plane in j, two rows per step, pipelined:
//
//   step s, a = 2 s + jA:  A-row a       first pair  (threads 0..NP-1: rows a-1, a, a+1, old)
//                          B-row a - 3   second pair (threads NP..2NP-1: rows a-4 and a-2 new, a-3 old)
//
// Both rows run in the same two phases (first colour | barrier | second colour with the new values of
// the first, exchanged through LDS | barrier), one pair per thread, as the pair passes do within a row.
// The rows a-4 .. a+1 of planes k-1, k, k+1 sit in an 8-row LDS ring (colour-split rows: odd positions,
// then even ones, zero guards at both ends, so consecutive lanes read consecutive doubles); each thread
// reads its pair's 9 x 4 window once per step.  The next step's rows a+2, a+3 are written into the
// ring's free slots at the end of a step; their loads were issued into registers JS_D - 1 steps
// earlier.  New first-pair values are written into the ring (the second pair and the chunk's later
// steps read them); every row of the chunk is stored to xout.  Barriers wait for LDS only (js_barrier),
// and the Box-Muller tables sit in LDS, so nothing drains the prefetched loads early.
//
// Tiles are (own plane, chunk of steps).  A chunk that stores the A-rows of steps [s0, s1) and the
// B-rows below them runs steps s0 - 1 .. s1: step s0 - 1 recomputes the A-row the chunk's first B-row
// needs (same inputs, same arithmetic, not stored), step s1 only completes the last B-row.  Out of place,
// as k_sweep_quads: own planes read from xo (old), planes k +- 1 from xz (old in the first half, the
// first half's new planes in the second).  Per vertex the arithmetic is gibbs_point's / the pair
// passes' (a plain product, then the stencil fma chain in ascending column order; c = fma(sd, xi, f);
// x = fma(omega/diag, c - sum, x)) with the pair ids and the sweep tag of the pair passes: bitwise
// equal to them and to the oracle.
#pragma once
#include <type_traits>

#include "mgmc_kernels.hpp"
#include "mgmc_tuning.hpp"

namespace mgmc {

// NP pairs per row (nx = 2 NP); 2 NP threads (A-row pairs, B-row pairs); ring rows of stride 2 NP + 8: odd pairs [0, NP) and the guard at NP, then
// the even block from NP + 1: its guard (position 0) first, even pair m at NP + 2 + m
constexpr int JS_RING = 8;           // rows per plane in the LDS ring
constexpr int JS_D = tune::JS_D;     // global loads run this many steps ahead (2 .. 4)
static_assert(JS_D >= 2 && JS_D <= 4, "JS_D");

struct JSweepArgs {
    Layout L;
    const double* xo;  // own planes, old values
    const double* xz;  // planes k -+ 1
    double* xout;
    const double* f;
    StencilArg S;
    GibbsArg G;
    int kp, jA;        // own plane parity (k = 2 - kp + 2 t), first pair's row parity
    int nk;            // own planes of the half
    int nsteps;        // steps per plane: s = 0 .. (ny - jA) / 2
    int spc;           // steps per chunk
    int nchunk;        // chunks per plane
    long long cs;      // batched chains: doubles between chains (blockIdx.z = chain)
};

// workgroup barrier that waits for this wave's LDS operations only: the prefetched global loads stay in
// flight across it (__syncthreads() would drain them with vmcnt(0) first); the "memory" clobber keeps
// the compiler from moving LDS accesses across it
__device__ __forceinline__ void js_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

constexpr int JS_TAB = 322;  // Box-Muller tables in LDS: log reduction (rc, hi, lo) x 64 + cos/sin 130
inline size_t jsweep_lds_bytes(int np) { return (size_t)(JS_RING * 3 * (2 * np + 8) + JS_TAB) * sizeof(double); }

// XZ: the sweep's input x is known zero (the level's first pre-sweep, mgmc_capi.hip mark_zero_inputs):
// 1 = every x row is the constant 0.0 (the first half), 2 = the own planes' rows are (the second half;
// planes k +- 1 hold the first half's new values) -- those rows are not loaded at all
template <int NP, bool FIRST_ODD, bool SYM = false, int XZ = 0>
__global__ void __launch_bounds__(2 * NP) k_jsweep_half(JSweepArgs a) {
    constexpr int JS_NP = NP, JS_NT = 2 * NP, JS_RS = 2 * NP + 8, JS_EV = NP + 1;
    {
        const int ch = batch_chain();
        a.xo += ch * a.cs;
        a.xz += ch * a.cs;
        a.xout += ch * a.cs;
        a.f += ch * a.cs;
        a.G.key = chain_key(a.G, ch);
    }
    extern __shared__ __attribute__((aligned(16))) double ring[];  // [JS_RING rows][3 planes][JS_RS]
    const Layout& L = a.L;
    const int nb = gridDim.x, b = blockIdx.x, per = nb >> 3;
    const int tile = (nb & 7) ? b : (b & 7) * per + (b >> 3);  // XCD-aware: neighbouring planes on one XCD
    if (tile >= a.nk * a.nchunk) return;
    const int chunk = tile / a.nk, kk = tile - chunk * a.nk;
    const int k = 2 - a.kp + 2 * kk;
    const int s0 = chunk * a.spc, s1 = min(s0 + a.spc, a.nsteps);
    const int tid = threadIdx.x;
    // 0: A-row, 1: B-row -- uniform across a wavefront (NP is a multiple of 64): readfirstlane lets the
    // compiler keep everything that depends only on the role (rows, ring slots, row offsets, the step's
    // go / store flags) in SGPRs, so the per-lane work is the pair's column arithmetic
    const int role = __builtin_amdgcn_readfirstlane(tid / JS_NP);
    const int m = tid & (JS_NP - 1);  // pair of the row
    const int i0 = 2 * m + 1;
    const uint64_t sample = *a.G.sample;
    const double sd = a.G.sd, wd = a.G.wd;

    auto slot = [](int j) { return ((j % JS_RING) + JS_RING) % JS_RING; };
    auto rowp = [&](int j, int dz) { return ring + (slot(j) * 3 + dz) * JS_RS; };  // dz: plane index 0..2
    // staging: thread t moves pair t % NP of item 2 q + t / NP, q = 0..2 (6 items: 2 rows x 3 planes)
    // Loads are unconditional (rows clamped onto the lattice: an out-of-range row reads the zero
    // boundary row, exactly its zeros): a conditional load merges into its register through a copy,
    // and the copy waits for the load right away
    // Rows past the chunk's last window row a(s1) + 1 are never deposited (the loop's idle steps and the
    // prefetches JS_D steps past s1): they are loaded from that last row instead of the next chunk's
    // rows, which would be fetched from HBM only to be dropped (their values are never used)
    const int jlast = 2 * s1 + a.jA + 1, flast = 2 * s1 + a.jA;
    auto load_pair = [&](int j, int dz) -> double2 {
        if (XZ == 1 || (XZ == 2 && dz == 1)) return make_double2(0.0, 0.0);
        j = j > jlast ? jlast : j;
        const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
        const double* src = (dz == 1 ? a.xo : a.xz) + L.at(i0, jc, k + dz - 1);
        return *reinterpret_cast<const double2*>(src);
    };
    // (rows outside [0, ny] were loaded from the clamped boundary rows 0 / ny: already zeros)
    auto deposit = [&](int j, int dz, double2 v) {
        double* r = rowp(j, dz);
        r[m] = v.x;               // odd position 2m+1
        r[JS_EV + 1 + m] = v.y;   // even position 2m+2
    };
    auto guards = [&](int j) {  // zero guards of a ring row index (positions 0 and nx + 1)
        if (tid < 3) {
            double* r = rowp(j, tid);
            r[JS_NP] = 0.0;
            r[JS_EV] = 0.0;
        }
    };
    // prologue: rows a(s0-1) - 1 .. a(s0-1) + 1 (the first step's A-row window) and their guards
    const int a0 = 2 * (s0 - 1) + a.jA;
#pragma unroll
    for (int q = 0; q < 9; q += 2) {
        const int item = q + role;  // (row, plane) item of this thread: 9 items, two per pass
        if (item < 9) {
            const int j = a0 - 1 + item / 3, dz = item % 3;
            deposit(j, dz, load_pair(j, dz));
        }
    }
    for (int j = a0 - 4; j <= a0 + 3; ++j) guards(j);
    // B-row window of the first step: rows a0 - 4 .. a0 - 2 are never read there (no B-row at s0 - 1).
    // The Box-Muller tables go to LDS: a table load from global memory would be a vector load, and
    // waiting for it (in-order vmcnt) would also wait for the prefetched rows
    double* tab = ring + JS_RING * 3 * JS_RS;
    for (int q = tid; q < 64; q += JS_NT) {
        tab[q] = LOGTAB_RC[q];
        tab[64 + q] = LOGTAB_HI[q];
        tab[128 + q] = LOGTAB_LO[q];
    }
    for (int q = tid; q < 130; q += JS_NT) tab[192 + q] = SINCOS_TAB[q];
    js_barrier();

    // the pair's window: rows (dz, dy) = rr / 3, rr % 3 - 1 at positions 2m .. 2m+3, read from the ring
    // once per step (only the own row changes between the two colours)
    double w[9][4];
    auto load_window = [&](int j) {
#pragma unroll
        for (int rr = 0; rr < 9; ++rr) {
            const double* r = rowp(j + rr % 3 - 1, rr / 3);
            w[rr][0] = r[JS_EV + m];      // 2m (position 0: the guard)
            w[rr][1] = r[m];              // 2m+1
            w[rr][2] = r[JS_EV + 1 + m];  // 2m+2
            w[rr][3] = r[m + 1];          // 2m+3 (position nx+1: the guard)
        }
    };
    // 27-term chain of window element e (1: odd position 2m+1, 2: even 2m+2)
    auto chain = [&](auto ec) {
        constexpr int e = decltype(ec)::value;
        double res = stencil_coef<SYM>(a.S, 0) * w[0][e - 1];
#pragma unroll
        for (int t = 1; t < 27; ++t) res = fma(stencil_coef<SYM>(a.S, t), w[t / 3][e + t % 3 - 1], res);
        return res;
    };

    // Loads run JS_D steps ahead: at step s (index t = s - s0 + 1) the rows a + 2 JS_D, a + 2 JS_D + 1
    // (3 planes) go into P[(t + JS_D - 1) % JS_D], written into the ring at the end of step s + JS_D - 1;
    // the right-hand side of step s + JS_D goes into F[t % JS_D] once step s has taken its own.  The
    // loop is unrolled by JS_D so that the buffers are static registers.
    double2 P[JS_D][3], F[JS_D];
    auto frow = [&](int s) { return role == 0 ? 2 * s + a.jA : 2 * s + a.jA - 3; };
    auto load_f = [&](int j) -> double2 {  // (rows outside the lattice or past flast: never used)
        j = j > flast ? flast : j;
        const int jc = j < 1 ? 1 : (j > L.ny - 1 ? L.ny - 1 : j);
        return *reinterpret_cast<const double2*>(a.f + L.at(i0, jc, k));
    };
    auto load_rows = [&](double2 (&dst)[3], int j0) {  // rows j0, j0 + 1 of the 3 planes: items 2 q + role
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int item = 2 * q + role;
            dst[q] = load_pair(j0 + item / 3, item % 3);
        }
    };
    auto step = [&](auto par_c, int s) __attribute__((always_inline)) {
        constexpr int par = decltype(par_c)::value;  // (s - s0 + 1) % JS_D
        const int ar = 2 * s + a.jA;
        const double2 fcur = F[par];
        F[par] = load_f(frow(s + JS_D));  // (past the chunk: loaded, never used)
        load_rows(P[(par + JS_D - 1) % JS_D], ar + 2 * JS_D);
        // this thread's row: A-row ar (steps s0-1 .. s1-1) or B-row ar - 3 (steps s0 + 1 .. s1, i.e. the
        // B-rows of steps s0 .. s1-1)
        const int j = role == 0 ? ar : ar - 3;
        const bool go = (role == 0 ? s < s1 : (s > s0 && s <= s1)) && j >= 1 && j <= L.ny - 1;
        const bool store = go && (role == 1 || s >= s0);
        double z0 = 0.0, z1 = 0.0;
        if (go) {
            const Philox4 rnd = philox4x32_10(pair_id<3>(L, i0, j, k), a.G.tag, (uint32_t)sample,
                                              (uint32_t)(sample >> 32), a.G.key.k0, a.G.key.k1);
            normal_pair_t(rnd, &z0, &z1, tab, tab + 64, tab + 128, tab + 192);
        }
        const bool odd_in = go;                       // i0 <= nx - 1 always
        const bool even_in = go && i0 + 1 <= L.nx - 1;
        double* own = rowp(j, 1);
        load_window(j);
        // first colour (a first-colour vertex reads only second-colour positions of its row besides its
        // own, so the new value goes straight into the ring)
        constexpr int e1 = FIRST_ODD ? 1 : 2, e2 = 3 - e1;
        double v1 = w[4][e1];
        if (FIRST_ODD ? odd_in : even_in) {
            const double res = chain(std::integral_constant<int, e1>{});
            const double c = fma(sd, FIRST_ODD ? z0 : z1, FIRST_ODD ? fcur.x : fcur.y);
            v1 = fma(wd, c - res, v1);
            if (FIRST_ODD) own[m] = v1;
            else own[JS_EV + 1 + m] = v1;
        }
        js_barrier();
        // second colour: its row neighbours are first-colour vertices (own pair and the neighbouring one)
        w[4][e1] = v1;
        if (FIRST_ODD) w[4][3] = own[m + 1];        // next pair's odd element (the guard past the row)
        else w[4][0] = own[JS_EV + m];              // previous pair's even element (the guard before it)
        double v2 = w[4][e2];
        if (FIRST_ODD ? even_in : odd_in) {
            const double res = chain(std::integral_constant<int, e2>{});
            const double c = fma(sd, FIRST_ODD ? z1 : z0, FIRST_ODD ? fcur.y : fcur.x);
            v2 = fma(wd, c - res, v2);
            if (role == 0) {  // A-rows are read by later B-rows
                if (FIRST_ODD) own[JS_EV + 1 + m] = v2;
                else own[m] = v2;
            }
        }
        if (store) {
            double* dst = a.xout + L.at(i0, j, k);
            __builtin_nontemporal_store(FIRST_ODD ? v1 : v2, dst);  // streaming stores
            __builtin_nontemporal_store(FIRST_ODD ? v2 : v1, dst + 1);
        }
        // the next step's rows (ar + 2, ar + 3) into the slots of rows ar - 6, ar - 5 (read by no one)
        if (s < s1) {
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                const int item = 2 * q + role;
                deposit(ar + 2 + item / 3, item % 3, P[par][q]);
            }
            guards(ar + 2);
            guards(ar + 3);
        }
        js_barrier();
    };
    // steps s0 - 1 .. s1 in groups of JS_D (idle steps at the end), buffers by step index from the chunk
    // start, so the loop carries its registers without copies (a copy of an in-flight load would wait
    // for it)
#pragma unroll
    for (int t = 0; t + 1 < JS_D; ++t) load_rows(P[t], a0 + 2 + 2 * t);
#pragma unroll
    for (int t = 0; t < JS_D; ++t) F[t] = load_f(frow(s0 - 1 + t));
    for (int s = s0 - 1; s <= s1; s += JS_D) {
        step(std::integral_constant<int, 0>{}, s);
        step(std::integral_constant<int, 1>{}, s + 1);
        if constexpr (JS_D > 2) step(std::integral_constant<int, 2>{}, s + 2);
        if constexpr (JS_D > 3) step(std::integral_constant<int, 3>{}, s + 3);
    }
}

}  // namespace mgmc
