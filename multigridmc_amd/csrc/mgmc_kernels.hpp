// mgmc_kernels.hpp -- HIP kernels of the MGMC V-cycle for gfx950 (CDNA4).
//
// Data layout in HBM (every level): the (n+1)^d lattice vertices INCLUDING the Dirichlet
// boundary are stored, boundary values are zero and never written, so every stencil is
// branch-free.  Vertex (i,j,k), 0 <= i <= nx, sits at  k*sp + j*sx + i + off  with off = 7
// (interior i=1 is 64-byte aligned) and sx a multiple of 8 doubles.
//
// Per-point arithmetic (compiled with -ffp-contract=off, every fma explicit):
//   * Gibbs/SOR update: the reference's  x += omega * (c - sum_k a_k x_k) / a_c  with
//     c = sqrt(a_c(2-w)/w)*xi + f  (smoother/sor_smoother.cc:66-76, sampler/sor_sampler.cc:42-46)
//     evaluated in fused form  c = fma(sd, xi, f),  x = fma(omega/a_c, c - S, x),  S the fma chain
//     over the row in ascending column order -- mathematically identical, ~1 ulp apart, and
//     replayed bit for bit by the oracle's MULTICOLOUR mode;
//   * residual  r = f - A x  with A x accumulated in ascending column order
//     (linear_operator/linear_operator.hh:66-76, Eigen ColMajor SpMV);
//   * restriction  sum_sigma w_sigma r(2i+sigma), sigma with x fastest
//     (intergrid/intergrid_operator.hh:74-88, intergrid_operator_linear.cc:13-29);
//   * prolongate-add  x += (alpha*w) * xc  in ascending coarse index
//     (intergrid/intergrid_operator.hh:106-120) -- evaluated in gather form, which visits the
//     coarse contributions of a fine vertex in exactly the scatter order of the reference.
// What differs from the reference is the visiting order of the Gibbs updates (multicolour
// instead of lexicographic) and the noise stream (Philox, see philox_normal.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "philox_normal.h"

namespace mgmc {

struct Layout {
    int dim;
    int nx, ny, nz;  // cells
    int off;
    int pad_;
    long long sx, sp, nstore;
    __host__ __device__ long long at(int i, int j, int k) const {
        return (long long)k * sp + (long long)j * sx + (long long)i + off;
    }
};

// The first interior vertex of every row sits on a 128-byte line (row stride a multiple of 16
// doubles, off = 15, odd, so interior x-pairs (i odd, i+1) sit on 16-byte boundaries).
// reach2: operators coupling vertices two apart (the squared FD operator's field levels) read one
// row and one plane beyond the zero boundary on either side; the storage then starts one plane + one
// row earlier and ends one plane + one row later (zeros), so those reads stay inside the allocation.
inline Layout make_layout(int dim, const int n[3], bool reach2 = false) {
    Layout L;
    L.dim = dim;
    L.nx = n[0];
    L.ny = n[1];
    L.nz = dim == 3 ? n[2] : 0;
    L.pad_ = 0;
    L.sx = ((long long)L.nx + 16 + 15) / 16 * 16;  // >= nx + 16: columns -2 .. nx + 2 stay in the row
    L.sp = L.sx * (L.ny + 1);
    const long long margin = reach2 ? (dim == 3 ? L.sp : 0) + L.sx : 0;  // multiple of 16
    L.off = 15 + (int)margin;
    L.nstore = (dim == 3 ? L.sp * (L.nz + 1) : L.sp) + 64 + 2 * margin;
    return L;
}


struct StencilArg {
    double a[27];
};

// Reflection-symmetric 27-point stencils (a[dz][dy][dx] bitwise equal under each of dx, dy, dz -> 2 - d:
// the Galerkin levels of the cubic FD hierarchies, checked on the host by stencil_reflection_symmetric)
// hold at most 8 distinct values.  A kernel instantiated with SYM reads coefficient t from the lowest
// index of its class: the same bits, but only 8 doubles live in SGPRs instead of 27 (the full set
// spills into VGPR lanes and costs a v_readlane per use).
constexpr int sym_rep(int t) {
    const int dz = t / 9, dy = (t / 3) % 3, dx = t % 3;
    return (dz == 2 ? 0 : dz) * 9 + (dy == 2 ? 0 : dy) * 3 + (dx == 2 ? 0 : dx);
}
template <bool SYM>
__host__ __device__ inline double stencil_coef(const StencilArg& S, int t) {
    return S.a[SYM ? sym_rep(t) : t];
}
inline bool stencil_reflection_symmetric(const double* a, int npoints) {
    if (npoints != 27) return false;
    for (int t = 0; t < 27; ++t) {  // bit for bit (a +0 / -0 pair would not do)
        uint64_t u, v;
        __builtin_memcpy(&u, a + t, 8);
        __builtin_memcpy(&v, a + sym_rep(t), 8);
        if (u != v) return false;
    }
    return true;
}

// Class-folded residual sum of a reflection-symmetric 27-point stencil (the "fold" levels: every
// 3D Galerkin level of the cubic FD hierarchies).  The 27 window values v[t], t = (dz+1) 9 + (dy+1) 3
// + (dx+1), fall into 8 coefficient classes c = [dx == 0] + 2 [dy == 0] + 4 [dz == 0] (class
// representative sym_rep(t), its lowest offset index).  Each class sums its members in ascending t
// (s_c = v_rep, then s_c + v_t), then y = a_7 s_7 (the centre) and y = fma(a_c, s_c, y) for c = 6 .. 0.
// 19 adds + 1 multiply + 7 fma instead of 27 multiplies + 27 dependent adds, and a dependency depth
// of about 9 instead of 27: the 27-point residual + restriction kernels are latency / issue bound on
// that chain.  It is not the reference's CSR order (linear_operator.hh:66-76), so the
// fold levels' residuals agree with the FAITHFUL arithmetic to rounding (tests/test_gpu_parity.py,
// tolerance stated there) and bitwise with the MULTICOLOUR oracle, which folds the same way
// (oracle/refcpu.cpp folded_row_sum).
constexpr int fold_class(int t) { return (t % 3 == 1 ? 1 : 0) + ((t / 3) % 3 == 1 ? 2 : 0) + (t / 9 == 1 ? 4 : 0); }
constexpr int fold_rep(int c) { return (c & 1) + 3 * ((c >> 1) & 1) + 9 * ((c >> 2) & 1); }
__host__ __device__ __forceinline__ double fold27(const double (&v)[27], const double* a) {
    double s[8];
#pragma unroll
    for (int t = 0; t < 27; ++t) {
        const int c = fold_class(t);
        if (fold_rep(c) == t) s[c] = v[t];
        else s[c] = s[c] + v[t];
    }
    double y = a[fold_rep(7)] * s[7];
#pragma unroll
    for (int c = 6; c >= 0; --c) y = fma(a[fold_rep(c)], s[c], y);
    return y;
}
// fold27 one value at a time, in ascending t (the same operations in the same order): a caller that
// walks the window row by row keeps 8 class sums live instead of 27 values
__device__ __forceinline__ void fold27_acc(double (&s)[8], int t, double v) {
    const int c = fold_class(t);
    if (fold_rep(c) == t) s[c] = v;
    else s[c] = s[c] + v;
}
__device__ __forceinline__ double fold27_finish(const double (&s)[8], const double* a) {
    double y = a[fold_rep(7)] * s[7];
#pragma unroll
    for (int c = 6; c >= 0; --c) y = fma(a[fold_rep(c)], s[c], y);
    return y;
}

struct GibbsArg {
    double omega;
    double sd;  // sqrt(diag*(2-omega)/omega)
    double wd;  // omega/diag
    RngKey key;  // chain 0 of a batched launch
    uint32_t tag;
    int colour;
    const uint64_t* sample;  // device word holding the sample index
    uint32_t chain0, seed_hi;  // Philox key of chain c: (lo32(seed), lo32(chain0 + c) ^ hi32(seed))
};

// Batched chains (mgmc_create_batch): a handle's C chains share the hierarchy and run every kernel
// of the cycle in one launch, chain c = blockIdx.z / zper of the launch (zper = blocks of the
// kernel's own z dimension); chain c's vectors start c * stride doubles after chain 0's.
__device__ __forceinline__ int batch_chain(int zper = 1) { return (int)blockIdx.z / zper; }
__device__ __forceinline__ RngKey chain_key(const GibbsArg& G, int c) {
    RngKey k = G.key;
    if (c) k.k1 = (G.chain0 + (uint32_t)c) ^ G.seed_hi;
    return k;
}

// The right-hand side of a low-rank level with a split column g read in place (LowRankDev::
// rhs_inplace): every interior row carries B_g = one number, so the patch of row i is
// (f_i +/- e_loc,i) +/- e_g (lr_row_patch).  f is patched in place with the first term on the rows
// with other columns (k_lr_patch / k_lr_restore_patch, deferring e_g) and the sweep / residual kernel
// adds the chain's e = +/-(0.0 + B_g s_g) to every f it reads -- y - e_g taken as y + (-e_g), the same
// IEEE operation.  (Boundary and padding positions get it too; their right-hand side is never used.)
struct LRRhsArg {
    const double* e;  // e of chain c at e[c]; null: f itself is the right-hand side
};
__device__ __forceinline__ double2 lr_rhs_pair(double2 f, double e) { return make_double2(f.x + e, f.y + e); }

// ascending-column-order row sum  sum_k a_k x_k  starting from 0.0 (SYM: stencil_coef's fold)
template <int DIM, int NPTS, bool SYM = false>
__device__ __forceinline__ double stencil_sum(const double* __restrict__ x, long long p, const Layout& L,
                                              const StencilArg& S) {
    double res = 0.0;
    if (NPTS == 7) {
        res += S.a[4] * x[p - L.sp];
        res += S.a[10] * x[p - L.sx];
        res += S.a[12] * x[p - 1];
        res += S.a[13] * x[p];
        res += S.a[14] * x[p + 1];
        res += S.a[16] * x[p + L.sx];
        res += S.a[22] * x[p + L.sp];
    } else if (NPTS == 5) {
        res += S.a[1] * x[p - L.sx];
        res += S.a[3] * x[p - 1];
        res += S.a[4] * x[p];
        res += S.a[5] * x[p + 1];
        res += S.a[7] * x[p + L.sx];
    } else if (NPTS == 27) {
#pragma unroll
        for (int dz = -1; dz <= 1; ++dz)
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx)
                    res += stencil_coef<SYM>(S, (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1)) * x[p + dz * L.sp + dy * L.sx + dx];
    } else {  // 9
#pragma unroll
        for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
            for (int dx = -1; dx <= 1; ++dx) res += S.a[(dy + 1) * 3 + (dx + 1)] * x[p + dy * L.sx + dx];
    }
    return res;
}

// the same row sum as an fma chain (Gibbs updates): a_0 x_0, then fma(a_k, x_k, .) ascending
template <int DIM, int NPTS, bool SYM = false>
__device__ __forceinline__ double stencil_fma(const double* __restrict__ x, long long p, const Layout& L,
                                              const StencilArg& S) {
    double res;
    if (NPTS == 7) {
        res = S.a[4] * x[p - L.sp];
        res = fma(S.a[10], x[p - L.sx], res);
        res = fma(S.a[12], x[p - 1], res);
        res = fma(S.a[13], x[p], res);
        res = fma(S.a[14], x[p + 1], res);
        res = fma(S.a[16], x[p + L.sx], res);
        res = fma(S.a[22], x[p + L.sp], res);
    } else if (NPTS == 5) {
        res = S.a[1] * x[p - L.sx];
        res = fma(S.a[3], x[p - 1], res);
        res = fma(S.a[4], x[p], res);
        res = fma(S.a[5], x[p + 1], res);
        res = fma(S.a[7], x[p + L.sx], res);
    } else if (NPTS == 27) {
        res = stencil_coef<SYM>(S, 0) * x[p - L.sp - L.sx - 1];
#pragma unroll
        for (int q = 1; q < 27; ++q) {
            const int dz = q / 9 - 1, dy = (q / 3) % 3 - 1, dx = q % 3 - 1;
            res = fma(stencil_coef<SYM>(S, q), x[p + dz * L.sp + dy * L.sx + dx], res);
        }
    } else {  // 9
        res = S.a[0] * x[p - L.sx - 1];
#pragma unroll
        for (int q = 1; q < 9; ++q) {
            const int dy = q / 3 - 1, dx = q % 3 - 1;
            res = fma(S.a[q], x[p + dy * L.sx + dx], res);
        }
    }
    return res;
}

template <int DIM>
__device__ __forceinline__ double centre(const StencilArg& S) {
    return DIM == 3 ? S.a[13] : S.a[4];
}

// Philox pair id of vertex (i,j,k) and whether it takes the cos branch
template <int DIM>
__device__ __forceinline__ uint32_t pair_id(const Layout& L, int i, int j, int k) {
    const uint64_t row = (DIM == 3) ? (uint64_t)(k - 1) * (uint64_t)(L.ny - 1) + (uint64_t)(j - 1) : (uint64_t)(j - 1);
    return (uint32_t)(row * (uint64_t)(L.nx / 2) + (uint64_t)((i - 1) >> 1));
}

template <int DIM, int NPTS, bool NOISE>
__device__ __forceinline__ void gibbs_point(double* __restrict__ x, const double* __restrict__ f, long long p,
                                            const Layout& L, const StencilArg& S, const GibbsArg& G, uint64_t sample,
                                            int i, int j, int k) {
    // SOR/Gibbs update (sor_smoother.cc:70-75, sor_sampler.cc:44-45) in fused form:
    //   c = fma(sd, xi, f),  x = fma(omega/diag, c - sum_k a_k x_k, x)
    const double res = stencil_fma<DIM, NPTS>(x, p, L, S);
    double c = f[p];
    if (NOISE) {
        const double xi = point_normal(G.key, pair_id<DIM>(L, i, j, k), (i & 1) != 0, G.tag, sample);
        c = fma(G.sd, xi, f[p]);
    }
    x[p] = fma(G.wd, c - res, x[p]);
}

// ---- red-black sweep pass of the fine 5/7-point level: vertices with (i+j+k)&1 == colour ----
template <int DIM, int NPTS, bool NOISE>
__global__ void __launch_bounds__(256) k_sweep_rb(Layout L, double* __restrict__ x, const double* __restrict__ f,
                                                  StencilArg S, GibbsArg G) {
    const int tx = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (j > L.ny - 1) return;
    const int i = 1 + (((1 + j + k) ^ G.colour) & 1) + 2 * tx;
    if (i > L.nx - 1) return;
    const uint64_t sample = NOISE ? *G.sample : 0;
    gibbs_point<DIM, NPTS, NOISE>(x, f, L.at(i, j, k), L, S, G, sample, i, j, k);
}

// ---- 2^d-colour sweep pass of a Galerkin 9/27-point level: colour bit d = parity of coord d ----
template <int DIM, int NPTS, bool NOISE>
__global__ void __launch_bounds__(256) k_sweep_mc(Layout L, double* __restrict__ x, const double* __restrict__ f,
                                                  StencilArg S, GibbsArg G) {
    const int i = 2 - (G.colour & 1) + 2 * (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int j = 2 - ((G.colour >> 1) & 1) + 2 * (int)(blockIdx.y * blockDim.y + threadIdx.y);
    const int k = (DIM == 3) ? 2 - ((G.colour >> 2) & 1) + 2 * (int)blockIdx.z : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    if (DIM == 3 && k > L.nz - 1) return;
    const uint64_t sample = NOISE ? *G.sample : 0;
    gibbs_point<DIM, NPTS, NOISE>(x, f, L.at(i, j, k), L, S, G, sample, i, j, k);
}

// colour of a vertex under the scheme used for a level with NPTS points
template <int DIM, int NPTS>
__device__ __forceinline__ int colour_of(int i, int j, int k) {
    if (NPTS == 7 || NPTS == 5) return (i + j + k) & 1;
    return (i & 1) | ((j & 1) << 1) | ((k & 1) << 2);
}

// ---- whole coarse-level SSOR sampler in one workgroup, state in LDS ----
// nsweeps sweeps alternating forward/backward (SSORSampler::apply, ssor_sampler.cc:9-15),
// sweep s uses tag0 + s.  PRE: every right hand side c = fma(sd, xi, f) of every sweep is
// evaluated up front by all threads at once (f does not change during the sampler), so a colour pass
// is only the stencil and the update -- one Philox + Box-Muller latency for the whole sampler instead
// of one per colour pass.  The same operations as gibbs_point, so the same bits.
// ZBUF (with PRE): the Box-Muller pairs come from zb[t] (t = the item index below; chains zs apart),
// drawn by spare workgroups of the launch before (k_quads_restrict2d) with the same Philox blocks and
// normal_pair, so the bits are the same
template <int DIM, int NPTS, bool PRE, bool ZBUF = false>
__global__ void __launch_bounds__(1024) k_coarse_ssor_lds(Layout L, double* __restrict__ xg,
                                                          const double* __restrict__ fg, StencilArg S, GibbsArg G,
                                                          int nsweeps, int ncolours, long long chs,
                                                          const double2* __restrict__ zb = nullptr, long long zs = 0) {
    constexpr bool precompute = PRE;  // a template parameter: the colour passes carry no Philox code
    {  // batched chains (blockIdx.z)
        const int ch = batch_chain();
        xg += ch * chs;
        fg += ch * chs;
        G.key = chain_key(G, ch);
        if (ZBUF) zb += ch * zs;
    }
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xs = smem;
    double* fs = smem + L.nstore;
    double* cs = fs + L.nstore;  // [nsweeps][ndof] right hand sides (precompute)
    // the level's x and f: the first MAXS loads of every thread are issued before the Box-Muller
    // draws below and deposited after them, so the draws overlap the loads' latency
    constexpr int MAXS = 6;
    double sx[MAXS], sf[MAXS];
#pragma unroll
    for (int u = 0; u < MAXS; ++u) {
        const long long q = threadIdx.x + (long long)u * blockDim.x;
        sx[u] = q < L.nstore ? xg[q] : 0.0;
        sf[u] = q < L.nstore ? fg[q] : 0.0;
    }
    const uint64_t sample = *G.sample;
    const int nxi = L.nx - 1, nyi = L.ny - 1;
    const long long ndof = (long long)nxi * nyi * (DIM == 3 ? (L.nz - 1) : 1);
    const int npair = L.nx / 2;
    const int nrow = nyi * (DIM == 3 ? (L.nz - 1) : 1);
    // one Philox block and Box-Muller per pair (odd i, i+1) and sweep: cos -> odd, sin -> even,
    // the values point_normal gives each vertex (the first MAXP items of every thread here)
    // 32-bit index arithmetic: an LDS-resident level has far fewer than 2^31 items
    constexpr int MAXP = precompute ? 4 : 1;
    double pz0[MAXP], pz1[MAXP];
    if constexpr (precompute) {
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            const int t = (int)threadIdx.x + u * (int)blockDim.x;
            pz0[u] = pz1[u] = 0.0;
            if (t >= nsweeps * nrow * npair) continue;
            const int m = t % npair;
            const int rt = t / npair;
            const int row = rt % nrow;
            const int sw = rt / nrow;
            const int i0 = 2 * m + 1;
            if (i0 > nxi) continue;
            const int j = row % nyi + 1;
            const int k = (DIM == 3) ? row / nyi + 1 : 0;
            if (ZBUF) {
                const double2 zz = zb[t];
                pz0[u] = zz.x;
                pz1[u] = zz.y;
                continue;
            }
            const Philox4 rnd = philox4x32_10(pair_id<DIM>(L, i0, j, k), G.tag + (uint32_t)sw, (uint32_t)sample,
                                              (uint32_t)(sample >> 32), G.key.k0, G.key.k1);
            normal_pair(rnd, &pz0[u], &pz1[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < MAXS; ++u) {
        const long long q = threadIdx.x + (long long)u * blockDim.x;
        if (q < L.nstore) {
            xs[q] = sx[u];
            fs[q] = sf[u];
        }
    }
    for (long long q = threadIdx.x + (long long)MAXS * blockDim.x; q < L.nstore; q += blockDim.x) {
        xs[q] = xg[q];
        fs[q] = fg[q];
    }
    __syncthreads();
    if constexpr (precompute) {
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            const int t = (int)threadIdx.x + u * (int)blockDim.x;
            if (t >= nsweeps * nrow * npair) continue;
            const int m = t % npair;
            const int rt = t / npair;
            const int row = rt % nrow;
            const int sw = rt / nrow;
            const int i0 = 2 * m + 1;
            if (i0 > nxi) continue;
            const int j = row % nyi + 1;
            const int k = (DIM == 3) ? row / nyi + 1 : 0;
            const long long q = (long long)sw * ndof + (long long)row * nxi + (i0 - 1);
            const long long p = L.at(i0, j, k);
            cs[q] = fma(G.sd, pz0[u], fs[p]);
            if (i0 + 1 <= nxi) cs[q + 1] = fma(G.sd, pz1[u], fs[p + 1]);
        }
        for (int t = threadIdx.x + MAXP * blockDim.x; t < nsweeps * nrow * npair; t += blockDim.x) {
            const int m = t % npair;
            const int rt = t / npair;
            const int row = rt % nrow;
            const int sw = rt / nrow;
            const int i0 = 2 * m + 1;
            if (i0 > nxi) continue;
            const int j = row % nyi + 1;
            const int k = (DIM == 3) ? row / nyi + 1 : 0;
            double z0, z1;
            if (ZBUF) {
                const double2 zz = zb[t];
                z0 = zz.x;
                z1 = zz.y;
            } else {
                const Philox4 rnd = philox4x32_10(pair_id<DIM>(L, i0, j, k), G.tag + (uint32_t)sw, (uint32_t)sample,
                                                  (uint32_t)(sample >> 32), G.key.k0, G.key.k1);
                normal_pair(rnd, &z0, &z1);
            }
            const long long q = (long long)sw * ndof + (long long)row * nxi + (i0 - 1);
            const long long p = L.at(i0, j, k);
            cs[q] = fma(G.sd, z0, fs[p]);
            if (i0 + 1 <= nxi) cs[q + 1] = fma(G.sd, z1, fs[p + 1]);
        }
        __syncthreads();
    }
    // up to MAXV vertices per thread: coordinates, offset and colour computed once (the colour passes
    // then do no index arithmetic); larger levels take the generic loop
    constexpr int MAXV = 4;
    const bool cached = ndof <= MAXV * (long long)blockDim.x;
    int vi[MAXV], vj[MAXV], vk[MAXV], vp[MAXV], vc[MAXV];
#pragma unroll
    for (int u = 0; u < MAXV; ++u) {
        const int q = (int)threadIdx.x + u * (int)blockDim.x;
        vc[u] = -1;
        vi[u] = vj[u] = vk[u] = vp[u] = 0;
        if (cached && q < ndof) {
            vi[u] = q % nxi + 1;
            vj[u] = (q / nxi) % nyi + 1;
            vk[u] = (DIM == 3) ? q / (nxi * nyi) + 1 : 0;
            vp[u] = (int)L.at(vi[u], vj[u], vk[u]);
            vc[u] = colour_of<DIM, NPTS>(vi[u], vj[u], vk[u]);
        }
    }
    // 2^d-colour levels with right-hand sides precomputed: thread t takes the t-th vertex of each
    // colour class, so every colour pass runs on full wavefronts (with the per-thread vertex cache a
    // pass ran each of its MAXV slots with about 1/ncolours of the lanes active)
    constexpr int NCMAX = DIM == 3 ? 8 : 4;
    const bool bycolour = precompute && (NPTS == 9 || NPTS == 27) && ncolours == NCMAX;
    int cp[NCMAX], cq[NCMAX];
    bool all_fit = true;
#pragma unroll
    for (int c = 0; c < NCMAX; ++c) {
        cp[c] = -1;
        cq[c] = 0;
        const int fi = 2 - (c & 1), fj = 2 - ((c >> 1) & 1), fk = DIM == 3 ? 2 - ((c >> 2) & 1) : 0;
        const int ci = fi > nxi ? 0 : (nxi - fi) / 2 + 1;
        const int cj = fj > nyi ? 0 : (nyi - fj) / 2 + 1;
        const int ck = DIM == 3 ? (fk > L.nz - 1 ? 0 : (L.nz - 1 - fk) / 2 + 1) : 1;
        all_fit = all_fit && ci * cj * ck <= (int)blockDim.x;
        const int t = threadIdx.x;
        if (bycolour && t < ci * cj * ck) {
            const int i = fi + 2 * (t % ci), j = fj + 2 * ((t / ci) % cj), k = DIM == 3 ? fk + 2 * (t / (ci * cj)) : 0;
            cp[c] = (int)L.at(i, j, k);
            cq[c] = (DIM == 3 ? (k - 1) * nxi * nyi : 0) + (j - 1) * nxi + (i - 1);
        }
    }
    GibbsArg g = G;
    auto update = [&](int s, long long q, int i, int j, int k, long long p) {
        if constexpr (precompute) {
            const double res = stencil_fma<DIM, NPTS>(xs, p, L, S);
            xs[p] = fma(g.wd, cs[s * ndof + q] - res, xs[p]);
        } else {
            gibbs_point<DIM, NPTS, true>(xs, fs, p, L, S, g, sample, i, j, k);
        }
    };
    for (int s = 0; s < nsweeps; ++s) {
        g.tag = G.tag + (uint32_t)s;
        const bool backward = (s & 1) != 0;
        for (int cc = 0; cc < ncolours; ++cc) {
            const int colour = backward ? ncolours - 1 - cc : cc;
            if (bycolour && all_fit) {
#pragma unroll
                for (int c = 0; c < NCMAX; ++c)
                    if (c == colour && cp[c] >= 0) update(s, cq[c], 0, 0, 0, cp[c]);
            } else if (cached) {
#pragma unroll
                for (int u = 0; u < MAXV; ++u)
                    if (vc[u] == colour) update(s, (int)threadIdx.x + u * (int)blockDim.x, vi[u], vj[u], vk[u], vp[u]);
            } else {
                for (long long q = threadIdx.x; q < ndof; q += blockDim.x) {
                    const int i = (int)(q % nxi) + 1;
                    const int j = (int)((q / nxi) % nyi) + 1;
                    const int k = (DIM == 3) ? (int)(q / ((long long)nxi * nyi)) + 1 : 0;
                    if (colour_of<DIM, NPTS>(i, j, k) != colour) continue;
                    update(s, q, i, j, k, L.at(i, j, k));
                }
            }
            __syncthreads();
        }
    }
    for (long long q = threadIdx.x; q < L.nstore; q += blockDim.x) xg[q] = xs[q];
}

// ---- fused residual + restriction: fc = R (f - A x), xc = 0 (multigridmc_sampler.cc:118-122) ----
__device__ __forceinline__ double w1(int s) { return s == 0 ? 1.0 : 0.5; }

// FOLD: a fold level (27-point, reflection-symmetric): the residual's sum is fold27's
template <int DIM, int NPTS, bool FOLD = false>
__global__ void __launch_bounds__(256) k_residual_restrict(Layout Lf, Layout Lc, const double* __restrict__ xf,
                                                           const double* __restrict__ ff, double* __restrict__ fc,
                                                           double* __restrict__ xc, StencilArg S, int zero_xc) {
    const int I = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int J = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int K = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (I > Lc.nx - 1 || J > Lc.ny - 1) return;
    const long long pf = Lf.at(2 * I, 2 * J, 2 * K);
    double result = 0.0;
    const int zr = (DIM == 3) ? 1 : 0;
#pragma unroll
    for (int sz = -zr; sz <= zr; ++sz)
#pragma unroll
        for (int sy = -1; sy <= 1; ++sy)
#pragma unroll
            for (int sx = -1; sx <= 1; ++sx) {
                const long long q = pf + sz * Lf.sp + sy * Lf.sx + sx;
                double y;
                if constexpr (FOLD && DIM == 3 && NPTS == 27) {
                    double v[27];
#pragma unroll
                    for (int t = 0; t < 27; ++t) v[t] = xf[q + (t / 9 - 1) * Lf.sp + ((t / 3) % 3 - 1) * Lf.sx + (t % 3 - 1)];
                    y = fold27(v, S.a);
                } else {
                    y = stencil_sum<DIM, NPTS>(xf, q, Lf, S);
                }
                const double r = ff[q] - y;
                double w = 1.0;
                w *= w1(sx);
                w *= w1(sy);
                if (DIM == 3) w *= w1(sz);
                result += w * r;
            }
    const long long pc = Lc.at(I, J, K);
    fc[pc] = result;
    if (zero_xc) xc[pc] = 0.0;
}

// ---- restriction only (tests): rc = R r ----
template <int DIM>
__global__ void __launch_bounds__(256) k_restrict(Layout Lf, Layout Lc, const double* __restrict__ r,
                                                  double* __restrict__ rc) {
    const int I = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int J = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int K = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (I > Lc.nx - 1 || J > Lc.ny - 1) return;
    const long long pf = Lf.at(2 * I, 2 * J, 2 * K);
    double result = 0.0;
    const int zr = (DIM == 3) ? 1 : 0;
    for (int sz = -zr; sz <= zr; ++sz)
        for (int sy = -1; sy <= 1; ++sy)
            for (int sx = -1; sx <= 1; ++sx) {
                double w = 1.0;
                w *= w1(sx);
                w *= w1(sy);
                if (DIM == 3) w *= w1(sz);
                result += w * r[pf + sz * Lf.sp + sy * Lf.sx + sx];
            }
    rc[Lc.at(I, J, K)] = result;
}

// ---- prolongate-add in gather form: x += alpha * P xc ----
template <int DIM>
__global__ void __launch_bounds__(256) k_prolongate_add(Layout Lf, Layout Lc, double* __restrict__ x,
                                                        const double* __restrict__ xc, double alpha) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (i > Lf.nx - 1 || j > Lf.ny - 1) return;
    const long long p = Lf.at(i, j, k);
    double v = x[p];
    // coarse coordinates contributing along each axis, ascending
    const int i0 = i >> 1, j0 = j >> 1, k0 = k >> 1;
    const int ni = (i & 1) ? 2 : 1, nj = (j & 1) ? 2 : 1, nk = (DIM == 3 && (k & 1)) ? 2 : 1;
    for (int a = 0; a < nk; ++a) {
        const int kk = k0 + a;
        if (DIM == 3 && (kk < 1 || kk > Lc.nz - 1)) continue;
        for (int b = 0; b < nj; ++b) {
            const int jj = j0 + b;
            if (jj < 1 || jj > Lc.ny - 1) continue;
            for (int c = 0; c < ni; ++c) {
                const int ii = i0 + c;
                if (ii < 1 || ii > Lc.nx - 1) continue;
                double w = 1.0;
                w *= w1(i - 2 * ii);
                w *= w1(j - 2 * jj);
                if (DIM == 3) w *= w1(k - 2 * kk);
                v += alpha * w * xc[Lc.at(ii, jj, DIM == 3 ? kk : 0)];
            }
        }
    }
    x[p] = v;
}

// ---- prolongate-add, one thread per fine x-pair (i odd, i+1): 16-byte load / store of x, the
// coarse values from L2.  Contributions are added in ascending coarse index (kk, jj, ii), exactly
// as k_prolongate_add / the reference's scatter order. ----
template <int DIM>
__global__ void __launch_bounds__(256) k_prolongate_pairs(Layout Lf, Layout Lc, double* __restrict__ x,
                                                          const double* __restrict__ xc, double alpha, int zper,
                                                          long long csf, long long csc) {
    const int ch = batch_chain(zper);  // batched chains: blockIdx.z = ch * zper + plane block
    x += ch * csf;
    xc += ch * csc;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z - ch * zper + 1 : 0;
    const int i = 2 * q + 1;
    if (i > Lf.nx - 1 || j > Lf.ny - 1) return;
    const long long p = Lf.at(i, j, k);
    double2 v = *reinterpret_cast<const double2*>(x + p);
    const bool has1 = i + 1 <= Lf.nx - 1;
    const int j0 = j >> 1, nj = (j & 1) ? 2 : 1;
    const int k0 = k >> 1, nk = (DIM == 3 && (k & 1)) ? 2 : 1;
    for (int a = 0; a < nk; ++a) {
        const int kk = k0 + a;
        if (DIM == 3 && (kk < 1 || kk > Lc.nz - 1)) continue;
        for (int b = 0; b < nj; ++b) {
            const int jj = j0 + b;
            if (jj < 1 || jj > Lc.ny - 1) continue;
            const double* row = xc + Lc.at(0, jj, DIM == 3 ? kk : 0);
            double wyz = 1.0;  // weights multiply x first, then y, then z (intergrid_operator_linear.cc:22-27)
            // element 0: i odd -> coarse ii = q (sigma = +1), q+1 (sigma = -1), weight 1/2 each
            if (q >= 1) {
                double w = 1.0;
                w *= 0.5;
                w *= w1(j - 2 * jj);
                if (DIM == 3) w *= w1(k - 2 * kk);
                v.x += alpha * w * row[q];
            }
            if (q + 1 <= Lc.nx - 1) {
                double w = 1.0;
                w *= 0.5;
                w *= w1(j - 2 * jj);
                if (DIM == 3) w *= w1(k - 2 * kk);
                v.x += alpha * w * row[q + 1];
                // element 1: i+1 even -> coarse ii = q+1 (sigma = 0), weight 1
                if (has1) {
                    double w2 = 1.0;
                    w2 *= 1.0;
                    w2 *= w1(j - 2 * jj);
                    if (DIM == 3) w2 *= w1(k - 2 * kk);
                    v.y += alpha * w2 * row[q + 1];
                }
            }
            (void)wyz;
        }
    }
    *reinterpret_cast<double2*>(x + p) = v;
}

// ---- 3D prolongate-add, z-marching: each thread owns one fine x-pair (i odd, i+1) of one fine row j
// and marches TZ fine planes, keeping the coarse values of the row's parents in registers (a fine
// plane k reads coarse planes k>>1 and, for odd k, (k>>1)+1; two fine planes share each coarse plane),
// with the next plane's fine pair loaded one step ahead.  Per fine vertex the terms and their order are
// k_prolongate_pairs' (coarse planes ascending, rows ascending, then q, q+1): bitwise equal. ----
template <int TZ>
__global__ void __launch_bounds__(256) k_prolongate_z(Layout Lf, Layout Lc, double* __restrict__ x,
                                                      const double* __restrict__ xc, double alpha, int nzc,
                                                      long long csf, long long csc) {
    const int ch = (int)blockIdx.z / nzc;  // batched chains: blockIdx.z = chain * nzc + z chunk
    x += ch * csf;
    xc += ch * csc;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int i = 2 * q + 1;
    const int k0 = 1 + ((int)blockIdx.z - ch * nzc) * TZ;
    const int k1 = min(k0 + TZ, Lf.nz);  // one past the last fine plane
    if (i > Lf.nx - 1 || j > Lf.ny - 1) return;
    const bool has1 = i + 1 <= Lf.nx - 1;
    const bool hq0 = q >= 1, hq1 = q + 1 <= Lc.nx - 1;
    const int j0 = j >> 1, nj = (j & 1) ? 2 : 1;
    const bool hj[2] = {j0 >= 1 && j0 <= Lc.ny - 1, j0 + 1 >= 1 && j0 + 1 <= Lc.ny - 1};
    const double wj[2] = {w1(j - 2 * j0), w1(j - 2 * j0 - 2)};
    // coarse values (rows j0, j0 + 1; columns q, q + 1) of coarse plane K (zero where a parent does
    // not exist -- never added: the existence tests below are k_prolongate_pairs')
    auto coarse = [&](int K, double (&c)[2][2]) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int jj = j0 + b;
            const bool ok = b < nj && hj[b] && K >= 1 && K <= Lc.nz - 1;
            const double* row = xc + Lc.at(0, ok ? jj : 0, ok ? K : 0);
            c[b][0] = ok && hq0 ? row[q] : 0.0;
            c[b][1] = ok && hq1 ? row[q + 1] : 0.0;
        }
    };
    double cA[2][2], cB[2][2];  // coarse planes K, K + 1 around the current fine plane
    int K = k0 >> 1;
    coarse(K, cA);
    coarse(K + 1, cB);
    double2 vn = *reinterpret_cast<const double2*>(x + Lf.at(i, j, k0));
    for (int k = k0; k < k1; ++k) {
        const long long p = Lf.at(i, j, k);
        double2 v = vn;
        if (k + 1 < k1) vn = *reinterpret_cast<const double2*>(x + p + Lf.sp);
        if ((k >> 1) != K) {  // advance the coarse window by one plane
            K = k >> 1;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                cA[b][0] = cB[b][0];
                cA[b][1] = cB[b][1];
            }
            coarse(K + 1, cB);
        }
        const int nk = (k & 1) ? 2 : 1;
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            if (a >= nk) break;
            const int kk = K + a;
            if (kk < 1 || kk > Lc.nz - 1) continue;
            const double(&c)[2][2] = a == 0 ? cA : cB;
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                if (b >= nj || !hj[b]) continue;
                if (hq0) {
                    double w = 1.0;
                    w *= 0.5;
                    w *= wj[b];
                    w *= w1(k - 2 * kk);
                    v.x += alpha * w * c[b][0];
                }
                if (hq1) {
                    double w = 1.0;
                    w *= 0.5;
                    w *= wj[b];
                    w *= w1(k - 2 * kk);
                    v.x += alpha * w * c[b][1];
                    if (has1) {
                        double w2 = 1.0;
                        w2 *= 1.0;
                        w2 *= wj[b];
                        w2 *= w1(k - 2 * kk);
                        v.y += alpha * w2 * c[b][1];
                    }
                }
            }
        }
        *reinterpret_cast<double2*>(x + p) = v;
    }
}

// ---- y = A x (tests, LinearOperator::apply) ----
template <int DIM, int NPTS>
__global__ void __launch_bounds__(256) k_operator_apply(Layout L, const double* __restrict__ x, double* __restrict__ y,
                                                        StencilArg S) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    const long long p = L.at(i, j, k);
    y[p] = stencil_sum<DIM, NPTS>(x, p, L, S);
}

// ---- reference (lexicographic interior) layout <-> padded layout ----
template <int DIM>
__global__ void __launch_bounds__(256) k_pack(Layout L, const double* __restrict__ lex, double* __restrict__ pad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    const long long row = (DIM == 3) ? (long long)(k - 1) * (L.ny - 1) + (j - 1) : (long long)(j - 1);
    pad[L.at(i, j, k)] = lex[row * (L.nx - 1) + (i - 1)];
}

template <int DIM>
__global__ void __launch_bounds__(256) k_unpack(Layout L, const double* __restrict__ pad, double* __restrict__ lex) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y * blockDim.y + threadIdx.y + 1;
    const int k = (DIM == 3) ? (int)blockIdx.z + 1 : 0;
    if (i > L.nx - 1 || j > L.ny - 1) return;
    const long long row = (DIM == 3) ? (long long)(k - 1) * (L.ny - 1) + (j - 1) : (long long)(j - 1);
    lex[row * (L.nx - 1) + (i - 1)] = pad[L.at(i, j, k)];
}

// ---- QoI record + running moments; advances the sample index (driver_mgmc.cc:72-78, :86-94) ----
// ctrl[0] = sample index, ctrl[1] = series length, ctrl[2] = QoI storage index (int64, <0 = off),
// ctrl[5] = non-finite guard (0, or 1 + the sample index at which the watched value first was NaN /
// Inf), ctrl[6] = storage index watched when no QoI is recorded (the lattice centre)
static __global__ void k_qoi_record(const double* __restrict__ x, uint64_t* ctrl, double* series, uint64_t capacity,
                             double* mom, int nchains, long long cs) {
    // thread c records chain c (series and moments chain c * capacity / c * 4 on); the control words
    // are advanced once, after every chain has read them
    __shared__ int bad;
    const int c = threadIdx.x;
    if (c == 0) bad = 0;
    __syncthreads();
    const long long q = (long long)ctrl[2];
    const uint64_t n = ctrl[1], s0 = ctrl[0];
    if (c < nchains) {
        const double z = x[(long long)c * cs + (q >= 0 ? q : (long long)ctrl[6])];
        if (!isfinite(z)) bad = 1;
        if (q >= 0) {
            double* m = mom + 4 * c;
            if (n < capacity) series[(long long)c * capacity + n] = z;
            const double cnt = m[0] + 1.0;
            const double delta = z - m[1];
            const double mean = m[1] + delta / cnt;
            m[2] = m[2] + delta * (z - mean);
            m[1] = mean;
            m[0] = cnt;
        }
    }
    __syncthreads();
    if (c == 0) {
        if (bad && ctrl[5] == 0) ctrl[5] = s0 + 1;
        if (q >= 0) ctrl[1] = n + 1;
        ctrl[0] = s0 + 1;
    }
}

// ---- QoI vector z = b^T x per chain (mgmc_set_qoi_vector; the radius > 0 measurement vector of
// measured_operator.cc:92-171, dotted with the sample as driver_mgmc.cc:76 does) in the fixed order of
// the low-rank dots: entries ascending in 4096-entry blocks, lane l of a wavefront sums entries
// l, l+64, ... of its block from 0.0, the lanes combine by the xor butterfly; k_qoi_record_vec combines
// the block partials the same way.  The oracle's blocked_dot is the same sequence. ----
constexpr int QV_BLK = 4096;
__device__ inline double butterfly64(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = v + __shfl_xor(v, o, 64);
    return v;
}
static __global__ void __launch_bounds__(64) k_qoi_dot(const double* __restrict__ x, const long long* __restrict__ off,
                                                const double* __restrict__ val, long long n, const uint64_t* ctrl,
                                                double* __restrict__ part, int nblk, long long cs) {
    if ((long long)ctrl[2] != -2) return;  // not recording the vector in this call (uniform)
    const int b = blockIdx.x, c = blockIdx.y, l = threadIdx.x;
    const double* xc = x + (long long)c * cs;
    const long long e0 = (long long)b * QV_BLK, e1 = min(n, e0 + (long long)QV_BLK);
    double acc = 0.0;
    constexpr int U = 8;  // products of U entries in flight, then added in entry order
    for (long long e = e0 + l; e < e1; e += 64 * U) {
        double pr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long q = e + 64LL * u;
            pr[u] = q < e1 ? val[q] * xc[off[q]] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (e + 64LL * u < e1) acc = acc + pr[u];
    }
    acc = butterfly64(acc);
    if (l == 0) part[(long long)c * nblk + b] = acc;
}
// k_qoi_record with one wavefront per chain: z = x at the QoI vertex (ctrl[2] >= 0), the centre
// guard (-1), or the combined block partials of k_qoi_dot (-2)
static __global__ void k_qoi_record_vec(const double* __restrict__ x, uint64_t* ctrl, double* series, uint64_t capacity,
                                 double* mom, int nchains, long long cs, const double* __restrict__ part, int nblk) {
    __shared__ int bad;
    const int c = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const long long q = (long long)ctrl[2];
    const uint64_t n = ctrl[1], s0 = ctrl[0];
    if (c < nchains) {
        double z;
        if (q == -2) {
            double acc = 0.0;
            for (int b = l; b < nblk; b += 64) acc = acc + part[(long long)c * nblk + b];
            z = butterfly64(acc);
        } else {
            z = x[(long long)c * cs + (q >= 0 ? q : (long long)ctrl[6])];
        }
        if (l == 0) {
            if (!isfinite(z)) bad = 1;
            if (q >= 0 || q == -2) {
                double* m = mom + 4 * c;
                if (n < capacity) series[(long long)c * capacity + n] = z;
                const double cnt = m[0] + 1.0;
                const double delta = z - m[1];
                const double mean = m[1] + delta / cnt;
                m[2] = m[2] + delta * (z - mean);
                m[1] = mean;
                m[0] = cnt;
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (bad && ctrl[5] == 0) ctrl[5] = s0 + 1;
        if (q >= 0 || q == -2) ctrl[1] = n + 1;
        ctrl[0] = s0 + 1;
    }
}

// ---- normals for the RNG parity test ----
static __global__ void k_normals(RngKey key, uint64_t pair0, uint64_t npairs, uint32_t tag, uint64_t sample,
                          double* __restrict__ out) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= npairs) return;
    const Philox4 r = philox4x32_10((uint32_t)(pair0 + q), tag, (uint32_t)sample, (uint32_t)(sample >> 32), key.k0,
                                    key.k1);
    double z0, z1;
    normal_pair(r, &z0, &z1);
    out[2 * q] = z0;
    out[2 * q + 1] = z1;
}

}  // namespace mgmc
