// mgmc_layout_check.hpp -- host-side bounds check of the padded level layouts (no device code).
//
// Every kernel addresses a level's vectors as L.at(i, j, k) + chain * L.nstore with unconditional
// loads: coordinates outside the interior land on the zero boundary rows / planes and in the row
// padding.  That is only safe while the extreme coordinates each kernel family
// can form stay inside [0, L.nstore) of every chain's copy.  A reach-2 operator read one row and one
// plane before the allocation in round 2 and faulted a GPU; this check makes such a layout a host
// error instead.  The extents below restate the index arithmetic of each family:
//
//   point kernels, reach r (k_sweep_rb / k_sweep_mc / k_residual_restrict / k_operator_apply /
//     k_restrict / k_prolongate_pairs, field kernels k_fsweep / k_fresidual / k_fapply):
//     interior vertices and their neighbours: i in [1-r, nx-1+r], j likewise, k likewise (3D)
//   colour-pair / quad passes (mgmc_gsweep.hpp): double2 loads at q-2, q, q+2 around the odd vertex
//     i0 in [1, nx-1] of rows j+-1, planes k+-1: i in [-1, nx+2], j in [0, ny], k in [0, nz]
//   fused z-sweep (mgmc_zsweep.hpp): pair columns 2 q0 - 1 .. 2 q0 + 2 XP + 2 of 64-wide tiles
//     (nx % 64 == 0): i in [-1, nx+2]; rows / planes clamped onto [0, ny] / [0, nz].  Its fused
//     prolongation reads coarse columns q0 - 3 .. q0 + XP + 4: i_c in [-3, nc+4], clamped rows /
//     planes
//     The post-sweep's two-step-ahead prefetch (PF2) issues x planes p + 3 past the chunk end and f
//     planes p + 2: both through plane_base's clamp onto [0, nz]; its idle waves load f at L.off + 1
//     (vertex (1, 0, 0), a zero boundary pair) -- inside the same box
//   z-marching residual + restriction (mgmc_zrestrict.hpp): x pairs from 2 I0 - 3, f pairs from
//     2 I0 - 1 over CX coarse points per tile, columns clamped to nx + 1 (the pair (nx+1, nx+2));
//     rows / planes clamped
//   one-launch 2D red-black sweep (mgmc_rb2d.hpp): guarded to i in [0, nx], j in [0, ny]
//   j-marching half-sweeps (mgmc_jsweep.hpp, round 3): pairs (i0, i0 + 1), i0 = 2m + 1, m < nx / 2: i in
//     [1, nx]; ring rows clamped onto [0, ny] (load_pair), f rows onto [1, ny - 1] (load_f), own planes
//     k = 2 - kp + 2 kk (kk < nk) and k +- 1.  Beyond the box, jsweep_grid_check replays the kernel's
//     whole grid -- the tile order, the chunk's steps s0 - 1 .. s1, the idle steps of the unrolled
//     loop and every prefetch JS_D steps ahead -- with the launch plan of launch_jsweep
//   2D last pre-sweep + residual + restriction (mgmc_qrestrict.hpp, round 3): staged pairs from
//     i = -1 to nx + 2 on rows clamped onto [0, ny]; stores on interior rows / coarse interior points
//   whole-store kernels (k_tail staging, k_coarse_ssor_lds, low-rank dense columns): [0, nstore)
//   the tail's pre-drawn noise (k_zresrestrict<..., ZN> writes, k_tail reads): job items
//     [zoff, zoff + items) inside the buffer's [0, zbs), pairwise disjoint (tail_noise_check)
//
// Double2 accesses start on an even offset: the upper column of a pair is included in the ranges.
#pragma once
#include <algorithm>
#include <string>
#include <vector>

#include "mgmc_kernels.hpp"

namespace mgmc {

enum LayoutFamily : unsigned {
    LF_POINT = 1u,      // reach-r point kernels
    LF_PAIRS = 2u,      // colour-pair / quad passes
    LF_ZSWEEP = 4u,     // fused z-marching red-black sweep (fine side)
    LF_ZSWEEP_C = 8u,   // ... its prolongation reads on the coarse level (coarse side)
    LF_ZRESTRICT = 16u, // z-marching residual + restriction (fine side)
    LF_RB2D = 32u,      // 2D one-launch red-black sweep
    LF_JSWEEP = 64u,    // 3D j-marching half-sweeps (box + grid replay)
    LF_QRESTRICT = 128u,  // 2D fused last pre-sweep + residual + restriction
};

// launch plan of one k_jsweep_half launch (launch_jsweep): shared by the launch and the check
struct JSweepPlan {
    int kp, jA, nk, nsteps, spc, nchunk, nb;
};
inline JSweepPlan jsweep_plan(const Layout& L, bool forward, int half, int num_cu, size_t lds_bytes, int rounds) {
    JSweepPlan p;
    const int slots = (int)std::max<size_t>(1, (160 * 1024) / lds_bytes) * num_cu * rounds;
    p.jA = forward ? 0 : 1;
    p.nsteps = (L.ny - p.jA) / 2 + 1;
    p.kp = forward ? half : 1 - half;
    const int first = 2 - p.kp;
    p.nk = first > L.nz - 1 ? 0 : (L.nz - 1 - first) / 2 + 1;
    p.spc = p.nchunk = p.nb = 0;
    if (p.nk == 0) return p;
    const int nchunk = std::max(1, std::min(p.nsteps, slots / p.nk));
    p.spc = (p.nsteps + nchunk - 1) / nchunk;
    p.nchunk = (p.nsteps + p.spc - 1) / p.spc;
    p.nb = (p.nk * p.nchunk + 7) / 8 * 8;
    return p;
}

// Replay of k_jsweep_half's addressing over its whole grid (host).  Every global access of the kernel
// is (i0 or i0 + 1, row, plane) with i0 = 2m + 1 < nx; this returns the extreme (row, plane) it forms
// for x loads, f loads and stores, or an error if the tile order misses or repeats a tile, a store
// leaves the interior, or a row / plane leaves [0, ny] x [0, nz].  js_d: the kernel's JS_D.
inline std::string jsweep_grid_check(const Layout& L, const JSweepPlan& p, int js_d) {
    if (p.nk == 0) return "";
    if (L.nx % 2 || L.dim != 3) return "j-sweep: not a 3D level with even nx";
    std::vector<char> seen((size_t)p.nk * p.nchunk, 0);
    const int per = p.nb >> 3;
    auto bad = [&](const char* what, int j, int k) {
        return std::string("j-sweep ") + what + ": row " + std::to_string(j) + ", plane " + std::to_string(k) +
               " outside the level (" + std::to_string(L.nx) + " x " + std::to_string(L.ny) + " x " +
               std::to_string(L.nz) + ")";
    };
    for (int b = 0; b < p.nb; ++b) {
        const int tile = (p.nb & 7) ? b : (b & 7) * per + (b >> 3);
        if (tile >= p.nk * p.nchunk) continue;
        if (seen[tile]++) return "j-sweep: tile " + std::to_string(tile) + " mapped twice";
        const int chunk = tile / p.nk, kk = tile - chunk * p.nk;
        const int k = 2 - p.kp + 2 * kk;
        const int s0 = chunk * p.spc, s1 = std::min(s0 + p.spc, p.nsteps);
        const int a0 = 2 * (s0 - 1) + p.jA;
        const int jlast = 2 * s1 + p.jA + 1, flast = 2 * s1 + p.jA;  // (the kernel's clamps past the chunk)
        auto xrow = [&](int j, int dz) -> std::string {  // load_pair: clamped row, plane k + dz - 1
            j = j > jlast ? jlast : j;
            const int jc = j < 0 ? 0 : (j > L.ny ? L.ny : j);
            const int kz = k + dz - 1;
            if (jc < 0 || jc > L.ny || kz < 0 || kz > L.nz) return bad("x load", jc, kz);
            return "";
        };
        auto frow_ok = [&](int j) -> std::string {  // load_f: row clamped onto [1, ny - 1], plane k
            j = j > flast ? flast : j;
            const int jc = j < 1 ? 1 : (j > L.ny - 1 ? L.ny - 1 : j);
            if (jc < 1 || jc > L.ny - 1 || k < 1 || k > L.nz - 1) return bad("f load", jc, k);
            return "";
        };
        std::string e;
        for (int item = 0; item < 9 && e.empty(); ++item) e = xrow(a0 - 1 + item / 3, item % 3);
        auto frow = [&](int s, int role) { return role == 0 ? 2 * s + p.jA : 2 * s + p.jA - 3; };
        for (int t = 0; t + 1 < js_d && e.empty(); ++t)
            for (int item = 0; item < 6 && e.empty(); ++item) e = xrow(a0 + 2 + 2 * t + item / 3, item % 3);
        for (int t = 0; t < js_d && e.empty(); ++t)
            for (int role = 0; role < 2 && e.empty(); ++role) e = frow_ok(frow(s0 - 1 + t, role));
        // the unrolled loop runs steps s0 - 1 .. in groups of js_d (idle steps past s1 included)
        const int nst = s1 - (s0 - 1) + 1;
        const int last = s0 - 1 + (nst + js_d - 1) / js_d * js_d - 1;
        for (int s = s0 - 1; s <= last && e.empty(); ++s) {
            const int ar = 2 * s + p.jA;
            for (int role = 0; role < 2 && e.empty(); ++role) {
                e = frow_ok(frow(s + js_d, role));
                for (int item = role; item < 6 && e.empty(); item += 2) e = xrow(ar + 2 * js_d + item / 3, item % 3);
                const int j = role == 0 ? ar : ar - 3;
                const bool go = (role == 0 ? s < s1 : (s > s0 && s <= s1)) && j >= 1 && j <= L.ny - 1;
                const bool store = go && (role == 1 || s >= s0);
                if (store && e.empty() && (j < 1 || j > L.ny - 1 || k < 1 || k > L.nz - 1)) e = bad("store", j, k);
                // the clamps past the chunk never touch a row that is used: deposited rows (steps
                // s < s1: ar + 2, ar + 3) stay <= jlast, the f row of a computed row stays <= flast
                if (e.empty() && s < s1 && ar + 3 > jlast) e = bad("deposit past the chunk's last row", ar + 3, k);
                if (e.empty() && go && frow(s, role) > flast) e = bad("f row past the chunk's last row", frow(s, role), k);
            }
        }
        if (!e.empty()) return e;
    }
    for (size_t t = 0; t < seen.size(); ++t)
        if (!seen[t]) return "j-sweep: tile " + std::to_string(t) + " not covered by the grid";
    return "";
}

// the tail's pre-drawn noise: job q's items [zoff_q, zoff_q + items_q) inside [0, zbs), disjoint
inline std::string tail_noise_check(const std::vector<long long>& zoff, const std::vector<long long>& items, long long zbs) {
    for (size_t q = 0; q < zoff.size(); ++q) {
        if (zoff[q] < 0 || items[q] < 0 || zoff[q] + items[q] > zbs)
            return "tail noise job " + std::to_string(q) + ": items [" + std::to_string(zoff[q]) + ", " +
                   std::to_string(zoff[q] + items[q]) + ") outside the buffer [0, " + std::to_string(zbs) + ")";
        for (size_t r = 0; r < q; ++r)
            if (zoff[q] < zoff[r] + items[r] && zoff[r] < zoff[q] + items[q])
                return "tail noise jobs " + std::to_string(r) + " and " + std::to_string(q) + " overlap";
    }
    return "";
}

struct IndexBox {
    long long i0, i1, j0, j1, k0, k1;
};

// the offsets a box addresses in one chain's copy must lie in [0, nstore)
inline std::string check_box(const Layout& L, const IndexBox& b, const char* what) {
    const bool three = L.dim == 3;
    const long long lo = (three ? b.k0 * L.sp : 0) + b.j0 * L.sx + b.i0 + L.off;
    const long long hi = (three ? b.k1 * L.sp : 0) + b.j1 * L.sx + b.i1 + L.off;
    if (lo >= 0 && hi < L.nstore) return "";
    return std::string(what) + ": offsets [" + std::to_string(lo) + ", " + std::to_string(hi) +
           "] leave the level store [0, " + std::to_string(L.nstore) + ") (lattice " + std::to_string(L.nx) + " x " +
           std::to_string(L.ny) + (three ? " x " + std::to_string(L.nz) : std::string()) + ")";
}

// zrestrict_cx: coarse points per tile in x of the residual + restriction kernel on this (fine) level
// (0: not used); legacy_zrestrict: the column range before the clamp (round 2 layout)
inline std::string check_level_layout(const Layout& L, unsigned families, int reach, int zrestrict_cx,
                                      bool legacy_zrestrict = false) {
    const bool three = L.dim == 3;
    const long long nx = L.nx, ny = L.ny, nz = three ? L.nz : 0;
    std::string e;
    auto box = [&](long long i0, long long i1, long long j0, long long j1, long long k0, long long k1, const char* w) {
        if (e.empty()) e = check_box(L, IndexBox{i0, i1, j0, j1, three ? k0 : 0, three ? k1 : 0}, w);
    };
    if (families & LF_POINT) box(1 - reach, nx - 1 + reach, 1 - reach, ny - 1 + reach, 1 - reach, nz - 1 + reach,
                                 "point kernels");
    if (families & LF_PAIRS) box(-1, nx + 2, 0, ny, 0, nz, "colour-pair passes");
    if (families & LF_ZSWEEP) box(-1, nx + 2, 0, ny, 0, nz, "z-sweep");
    if (families & LF_ZSWEEP_C) box(-3, nx + 4, 0, ny, 0, nz, "z-sweep prolongation (coarse level)");
    if ((families & LF_ZRESTRICT) && zrestrict_cx > 0) {
        const long long nc = nx / 2, cx = zrestrict_cx;
        const long long ntx = (nc - 1 + cx - 1) / cx;
        const long long i0max = 1 + (ntx - 1) * cx;  // first coarse point of the last tile
        long long xhi = 2 * i0max + 2 * cx + 2, fhi = 2 * i0max + 2 * cx;
        if (!legacy_zrestrict) {
            xhi = xhi > nx + 2 ? nx + 2 : xhi;
            fhi = fhi > nx + 2 ? nx + 2 : fhi;
        }
        box(-1, xhi, 0, ny, 0, nz, "residual + restriction (x)");
        box(1, fhi, 0, ny, 0, nz, "residual + restriction (f)");
    }
    if (families & LF_RB2D) box(0, nx, 0, ny, 0, 0, "2D red-black sweep");
    if (families & LF_JSWEEP) box(1, nx, 0, ny, 0, nz, "j-marching half-sweep");
    if (families & LF_QRESTRICT) box(-1, nx + 2, 0, ny, 0, 0, "2D sweep + residual + restriction");
    return e;
}

}  // namespace mgmc
