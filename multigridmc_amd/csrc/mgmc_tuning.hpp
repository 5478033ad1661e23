// mgmc_tuning.hpp -- the library's launch-shape constants, in one place.
//
// Every value here is bitwise-neutral: it sets tile shapes, chunk depths, thread counts and launch
// thresholds, never an arithmetic order, so the results do not depend on it (the -m gpu suite holds at
// any setting; the layout check of mgmc_layout_check.hpp covers every shape).  The values are the ones
// measured fastest on MI355X; the losing alternatives and their timings are in docs/HISTORY.md and
// DESIGN.md 3i.  Timing experiments (scripts/build_exp.sh) build a copy of the sources with edited
// values here; the product build has no override switches.
#pragma once

namespace mgmc {
namespace tune {

// fine 3D 7-point z-sweep (mgmc_zsweep.hpp): 32 x-pairs x ZS_TY rows per tile, z-chunks of ZS_TZ
// planes, at least ZS_MINW waves per SIMD (2 workgroups of 12 waves per CU, <= 80 VGPRs)
constexpr int ZS_TY = 20;
constexpr int ZS_MINW = 6;
constexpr int ZS_TZ = 32;
// ... the fused-prolongation post-sweep: 16-row tiles (its registers bind first), 128-plane chunks
constexpr int ZS_TYP = 16;
constexpr int ZS_MINWP = 6;
constexpr int ZS_TZP = 128;

// quad passes (k_sweep_quads) on 3D Galerkin levels with rows of at most QUADS_MAXPAIR pairs;
// workgroup threads: 2D levels, 3D rows of more than 32 pairs, 3D rows of at most 32 pairs
constexpr int QUADS_MAXPAIR = 64;
constexpr int QUADS_NT = 128;
constexpr int QUADS_NT_WIDE = 256;
constexpr int QUADS_NT3 = 128;
// 3D quad passes on rows of npair dividing 64 read one pair per window row and shift the outer columns
// in from the neighbouring lanes (k_sweep_quads LANES); 0: three pair loads per row
constexpr int QUADS_LANES = 1;

// j-marching half-sweeps (mgmc_jsweep.hpp): global loads this many steps ahead (2 .. 4), workgroups
// per half = this many rounds of the resident slots
constexpr int JS_D = 3;
constexpr int JS_ROUNDS = 1;

// residual + restriction (mgmc_zrestrict.hpp): coarse points per tile in x of the symmetric 27-point
// instance; coarse nx below which the one-wavefront 16 x 4 tiles are used
constexpr int ZR27_CX = 64;
// ... its coarse rows per tile and minimum waves per SIMD (register budget: 4 = <= 128 VGPRs)
constexpr int ZR27_CY = 4;
constexpr int ZR27_MINW = 1;
constexpr int ZR_SMALL_NX = 32;
// the 7-point (fine level) instance with 64 x 8 coarse points per 512-thread workgroup (else 64 x 4
// per 256 threads) from this many 64 x 8 tiles up (512^3: 32,768)
constexpr int ZR7_WIDE_MIN_TILES = 16 * 1024;

// z-marching prolongation (k_prolongate_z): fine planes per thread on big 3D levels, and below 2^21
// fine pair items
constexpr int PROLONG_Z = 8;
constexpr int PROLONG_Z_SMALL = 4;

// spare workgroups of a tail launch drawing the post-sweep noise (plan_drawn_noise; 0: one per other CU).
// Each adds to the launch: 512^3 tail 43.5 us alone, 44.3 / 46.9 / 47.4 us with 32 / 64 / 255 of them; 32
// draw the 1.15 M pairs of the 127^3-31^3 post-sweeps inside the tail's own time
constexpr int TAIL_PN_WG = 32;

// ---- low-rank dot products (mgmc_lowrank.hpp) ----
// levels whose partials need fewer wavefronts than this take the staged kernel (a block's loads
// spread over a 256-thread workgroup), the others one wavefront per block
constexpr int LR_STAGED_MAX_WAVES = 512;
// entries per lane whose loads k_lr_partials issues together
constexpr int LR_PART_U = 8;
// chains per wavefront of k_lr_partials (batched chains: a column value loaded once for them)
constexpr int LR_PART_CH = 1;
// 16-byte pairs per thread of the dense-column kernels (k_lr_dense_rhs / _update)
constexpr int LR_DENSE_PER = 8;

}  // namespace tune
}  // namespace mgmc
