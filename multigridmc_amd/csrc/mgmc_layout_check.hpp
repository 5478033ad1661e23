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
//   z-marching residual + restriction (mgmc_zrestrict.hpp): x pairs from 2 I0 - 3, f pairs from
//     2 I0 - 1 over CX coarse points per tile, columns clamped to nx + 1 (the pair (nx+1, nx+2));
//     rows / planes clamped
//   one-launch 2D red-black sweep (mgmc_rb2d.hpp): guarded to i in [0, nx], j in [0, ny]
//   whole-store kernels (k_tail staging, k_coarse_ssor_lds, low-rank dense columns): [0, nstore)
//
// Double2 accesses start on an even offset: the upper column of a pair is included in the ranges.
#pragma once
#include <string>

#include "mgmc_kernels.hpp"

namespace mgmc {

enum LayoutFamily : unsigned {
    LF_POINT = 1u,      // reach-r point kernels
    LF_PAIRS = 2u,      // colour-pair / quad passes
    LF_ZSWEEP = 4u,     // fused z-marching red-black sweep (fine side)
    LF_ZSWEEP_C = 8u,   // ... its prolongation reads on the coarse level (coarse side)
    LF_ZRESTRICT = 16u, // z-marching residual + restriction (fine side)
    LF_RB2D = 32u,      // 2D one-launch red-black sweep
};

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
    return e;
}

}  // namespace mgmc
