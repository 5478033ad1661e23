// mgmc_capi.hip -- C-ABI implementation of include/mgmc.h on gfx950.
//
// One handle = one MCMC chain on one GPU.  All per-level state (x_l, f_l) stays resident in HBM
// across calls (the reference keeps it in `mutable` per-level vectors,
// sampler/multigridmc_sampler.hh:66-72).  One sample = one MGMC cycle
// (sampler/multigridmc_sampler.cc:103-138) = a fixed sequence of kernel launches, captured once
// into a hipGraph and replayed; the RNG counter (sample index) is read from device memory so
// the frozen graph produces fresh noise on every replay.
#include "mgmc_internal.hpp"

namespace mgmc_host {
std::mutex g_err_mutex;
std::string g_last_error;
std::atomic<int> g_live_handles{0};
void set_global_error(const std::string& s) {
    std::lock_guard<std::mutex> lock(g_err_mutex);
    g_last_error = s;
}
}  // namespace mgmc_host

namespace {
constexpr int LDS_POISON_DOUBLES = 80 * 1024 / 8;  // two 1024-thread workgroups of 80 KB fill a CU's 160 KB
__global__ void __launch_bounds__(1024) k_lds_poison() {
    extern __shared__ double lds[];
    const double nan = __builtin_nan("");
    for (int q = threadIdx.x; q < LDS_POISON_DOUBLES; q += blockDim.x) lds[q] = nan;
    __syncthreads();
    // a read the compiler cannot drop keeps the stores alive
    if (lds[(threadIdx.x * 7) % LDS_POISON_DOUBLES] == 0.0) asm volatile("" ::: "memory");
}
// NaN into every interior vertex of one level vector (the zero boundary and pad stay zero): in poison
// mode the coarse x a restriction with Op::xzero leaves unwritten (it holds the previous cycle's
// values until the post-sweep rewrites it) -- a later op that read it would trip the guard
__global__ void __launch_bounds__(256) k_poison_interior(Layout L, double* __restrict__ x) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x + 1;
    const int j = blockIdx.y + 1;
    const int k = L.dim == 3 ? (int)blockIdx.z + 1 : 0;
    if (i <= L.nx - 1) x[L.at(i, j, k)] = __builtin_nan("");
}
}  // namespace

// ------------------------------------------------------------------------------------------
// launch helpers
// ------------------------------------------------------------------------------------------
namespace mgmc_host {

dim3 grid3(int nthreads_x, int nrows_y, int nz_blocks, dim3 block) {
    return dim3((unsigned)((nthreads_x + block.x - 1) / block.x), (unsigned)((nrows_y + block.y - 1) / block.y),
                (unsigned)std::max(nz_blocks, 1));
}

GibbsArg make_gibbs(const mgmc_handle* h, const Level& lv, uint32_t tag, int colour, const uint64_t* sample) {
    GibbsArg g;
    g.omega = h->cfg.omega;
    const double diag = lv.spec.diag();
    g.sd = sqrt(diag * (2. - h->cfg.omega) / h->cfg.omega);  // sor_sampler.cc:26
    g.wd = h->cfg.omega / diag;
    g.key = h->key;
    g.tag = tag;
    g.colour = colour;
    g.sample = sample;
    g.chain0 = (uint32_t)h->chain;
    g.seed_hi = (uint32_t)(h->seed >> 32);
    return g;
}

// chain c of a batch: its Philox key (make_key(seed, chain0 + c)) and its copy of a level vector
RngKey chain_key_host(const GibbsArg& g, int c) {
    RngKey k = g.key;
    if (c) k.k1 = (g.chain0 + (uint32_t)c) ^ g.seed_hi;
    return k;
}
template <class T>
T* chain_ptr(T* v, const Level& lv, int c) {
    return v ? v + (long long)c * lv.L.nstore : v;
}

template <int DIM, int NPTS, bool NOISE>
void launch_sweep_t(const Level& lv, double* x, const double* f, const GibbsArg& g0, int direction,
                    hipStream_t s) {
    const Layout& L = lv.L;
    const int nc = lv.spec.ncolours;
    dim3 block(64, 4, 1);
    for (int cc = 0; cc < nc; ++cc) {
        GibbsArg g = g0;
        g.colour = (direction == MGMC_FORWARD) ? cc : nc - 1 - cc;
        if (NPTS == 5 || NPTS == 7) {
            dim3 grid = grid3(L.nx / 2, L.ny - 1, DIM == 3 ? L.nz - 1 : 1, block);
            hipLaunchKernelGGL((k_sweep_rb<DIM, NPTS, NOISE>), grid, block, 0, s, L, x, f, lv.S, g);
        } else {
            dim3 grid = grid3(L.nx / 2, L.ny / 2, DIM == 3 ? L.nz / 2 : 1, block);
            hipLaunchKernelGGL((k_sweep_mc<DIM, NPTS, NOISE>), grid, block, 0, s, L, x, f, lv.S, g);
        }
    }
}

// colour passes of a field level (mgmc_field.hpp): colours ascending forward, descending backward
void launch_fsweep(const Level& lv, double* x, const double* f, const GibbsArg& g0, int direction, bool noise,
                   hipStream_t s) {
    const Layout& L = lv.L;
    const int nc = lv.F.scheme, dim = lv.spec.dim;
    const int st = nc == 9 || nc == 27 ? 3 : 2;  // vertices of one colour are st apart per direction
    dim3 block(64, 4, 1);
    dim3 grid = nc == 2 ? grid3(L.nx / 2, L.ny - 1, dim == 3 ? L.nz - 1 : 1, block)
                        : grid3((L.nx - 1 + st - 1) / st, (L.ny - 1 + st - 1) / st,
                                dim == 3 ? (L.nz - 1 + st - 1) / st : 1, block);
    for (int cc = 0; cc < nc; ++cc) {
        GibbsArg g = g0;
        g.colour = (direction == MGMC_FORWARD) ? cc : nc - 1 - cc;
        if (dim == 3) {
            if (noise) hipLaunchKernelGGL((k_fsweep<3, true>), grid, block, 0, s, L, x, f, lv.F, g);
            else hipLaunchKernelGGL((k_fsweep<3, false>), grid, block, 0, s, L, x, f, lv.F, g);
        } else {
            if (noise) hipLaunchKernelGGL((k_fsweep<2, true>), grid, block, 0, s, L, x, f, lv.F, g);
            else hipLaunchKernelGGL((k_fsweep<2, false>), grid, block, 0, s, L, x, f, lv.F, g);
        }
    }
}

void launch_sweep(const Level& lv, double* x, const double* f, const GibbsArg& g0, int direction, bool noise,
                  hipStream_t s, int nch) {
    if (nch > 1) {  // batched chains on the generic colour-pass kernels: one launch sequence per chain
        for (int c = 0; c < nch; ++c) {
            GibbsArg g = g0;
            g.key = chain_key_host(g0, c);
            launch_sweep(lv, chain_ptr(x, lv, c), chain_ptr(f, lv, c), g, direction, noise, s, 1);
        }
        return;
    }
    const GibbsArg& g = g0;
    if (lv.field) {
        launch_fsweep(lv, x, f, g, direction, noise, s);
        return;
    }
    const int dim = lv.spec.dim, np = lv.spec.npoints;
#define DISPATCH(D, P)                                                       \
    if (dim == D && np == P) {                                               \
        if (noise)                                                           \
            launch_sweep_t<D, P, true>(lv, x, f, g, direction, s);           \
        else                                                                 \
            launch_sweep_t<D, P, false>(lv, x, f, g, direction, s);          \
        return;                                                              \
    }
    DISPATCH(3, 7) DISPATCH(3, 27) DISPATCH(2, 5) DISPATCH(2, 9)
#undef DISPATCH
}

template <int XP, int TY, int NT, int MINW = 1>
void launch_zsweep_t(const Level& lv, ZSweepArgs a, bool prolong, hipStream_t s, int nch) {
    a.ntx = (lv.L.nx / 2) / XP;
    a.nty = (lv.L.ny - 1 + TY - 1) / TY;
    a.ntz = (lv.L.nz - 1 + a.tz - 1) / a.tz;
    // zpairs: tiles in (column, chunk pair) order, an odd chunk count padded by one empty tile per column
    const int ntiles = a.ntx * a.nty * (a.zpairs ? (a.ntz + 1) / 2 * 2 : a.ntz);
    const int nb = (ntiles + 7) / 8 * 8;
    const size_t lds = zsweep_lds_bytes(XP, TY, prolong);
    // alpha a power of two (coarse_scaling 1): fma prolongation terms, same bits (mgmc_zsweep.hpp)
    int ex;
    const bool pow2 = std::isnormal(a.alpha) && std::frexp(std::fabs(a.alpha), &ex) == 0.5 && ex > -900 && ex < 900;
    const dim3 grid(nb, 1, nch);  // batched chains: blockIdx.z
    const bool lrf = a.lr.e != nullptr;  // the right-hand side read in place (LRRhsArg)
    if (prolong && pow2 && lrf)
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 2, MINW, true>), grid, dim3(NT), lds, s, a);
    else if (prolong && pow2)
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 2, MINW>), grid, dim3(NT), lds, s, a);
    else if (prolong && lrf)
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 1, MINW, true>), grid, dim3(NT), lds, s, a);
    else if (prolong)
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 1, MINW>), grid, dim3(NT), lds, s, a);
    else if (lrf)
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 0, MINW, true>), grid, dim3(NT), lds, s, a);
    else
        hipLaunchKernelGGL((k_zsweep_rb7<XP, TY, NT, 0, MINW>), grid, dim3(NT), lds, s, a);
}

// z-chunk depth of a z-marching sweep: the deepest chunk (fewest prologue steps, 2 per chunk) that still
// keeps 3/4 of the 2 x num_cu workgroup slots busy -- 512^3: 32 (plain) / 128 (post) planes, 256^3: 32 / 32.
// Even: chunks start on odd planes (the first-colour element schedule, the coarse ring)
static int zsweep_depth(const Level& lv, int ty, int tzmax) {
    const long long tiles_xy = (long long)((lv.L.nx / 2) / ZS_XP) * ((lv.L.ny - 1 + ty - 1) / ty);
    int tz = tzmax;
    while (tz > 8 && 4 * tiles_xy * ((lv.L.nz - 1 + tz - 1) / tz) < 3LL * 2 * lv.num_cu) tz /= 2;
    return tz;
}

// rows per tile of the plain z-sweep: a level whose TY-row tiles leave part of the one round of
// 2 x num_cu slots idle runs the TYP-row tiles if those still fit the round (more, shorter columns;
// 256^3: 416 -> 512 workgroups, the pre-sweep 100.5 -> 91.9 us; at 512^3, many rounds, the 20-row
// tiles are faster)
static int zsweep_plain_rows(const Level& lv, int nch) {
    const int tz = zsweep_depth(lv, ZS_TY, ZS_TZ);
    auto ntiles = [&](int ty) {  // (z-chunk pairs: an odd chunk count padded by one empty tile per column)
        const long long nz = (lv.L.nz - 1 + tz - 1) / tz;
        return (long long)((lv.L.nx / 2) / ZS_XP) * ((lv.L.ny - 1 + ty - 1) / ty) * ((nz + 1) / 2 * 2) * nch;
    };
    const long long slots = 2LL * lv.num_cu;
    return (ZS_TYP != ZS_TY && ZS_NTP == ZS_NT && ntiles(ZS_TY) < slots && ntiles(ZS_TYP) <= slots) ? ZS_TYP : ZS_TY;
}

// lr (non-null): the right-hand side is read in place (LRRhsArg, LowRankDev::rhs_inplace)
void launch_zsweep(const Level& lv, const double* xin, double* xout, const double* f, const GibbsArg& g0,
                   int direction, const Level* coarse, const double* xc, double alpha, hipStream_t s, int nch = 1,
                   const LRRhsArg* lr = nullptr) {
    ZSweepArgs a;
    a.lr = lr ? *lr : LRRhsArg{nullptr};
    a.cs = lv.L.nstore;
    a.csc = coarse ? coarse->L.nstore : 0;
    a.L = lv.L;
    a.xin = xin;
    a.xout = xout;
    a.f = f;
    a.xc = xc;
    a.Lc = coarse ? coarse->L : lv.L;
    a.alpha = alpha;
    a.S = lv.S;
    a.G = g0;
    a.G.colour = (direction == MGMC_FORWARD) ? 0 : 1;
    a.zpairs = 0;
    if (coarse) {  // fused-prolongation sweep
        a.tz = zsweep_depth(lv, ZS_TYP, ZS_TZP);
        launch_zsweep_t<ZS_XP, ZS_TYP, ZS_NTP, ZS_MINWP>(lv, a, true, s, nch);
        return;
    }
    a.tz = zsweep_depth(lv, ZS_TY, ZS_TZ);
    a.zpairs = 1;  // z-chunks in up / down pairs (mgmc_zsweep.hpp)
    if (zsweep_plain_rows(lv, nch) != ZS_TY) {
        launch_zsweep_t<ZS_XP, ZS_TYP, ZS_NTP, ZS_MINWP>(lv, a, false, s, nch);
        return;
    }
    launch_zsweep_t<ZS_XP, ZS_TY, ZS_NT, ZS_MINW>(lv, a, false, s, nch);
}

// colour-pair passes of a Galerkin 9/27-point level (in place): forward colours (0,1), (2,3), ...,
// backward (7,6), (5,4), ... -- 2^(d-1) passes per sweep
bool pairs_eligible(const LevelSpec& sp, const Layout& L) {
    return (sp.npoints == 27 || sp.npoints == 9) && L.nx / 2 >= 1 && L.nx / 2 <= 256 && L.nx % 2 == 0;
}

// both colour pairs of a k-parity half per launch (k_sweep_quads): on levels with rows of <= 64
// pairs, where each pair pass is launch-latency bound and halving the launches pays (256^3: 63^3
// level 4 x 5.0 -> 2 x 7.6 us, 31^3 level 4 x 4.8 -> 2 x 6.3 us per sweep; round 4, 127^3 level with
// the folded stencil and xzero: 8 x 8 -> 61 us per cycle, 256^3 cycle -8 us), and on every 2D pair-pass
// level (2D 1024^2 FD cycle 0.135 -> 0.129 ms, FEM 0.147 -> 0.139 ms; A/B in one box call).  On the
// large 3D levels it loses (512^3 level 1: 2 x 105 us against 4 x 41 us per sweep): the
// second pair's loads wait for the first pair's rows.  Levels that k_tail runs are left to it (caller).
bool quads_eligible(const LevelSpec& sp, const Layout& L, uint32_t paths) {
    if (!pairs_eligible(sp, L) || (paths & PATH_NO_QUADS)) return false;
    return sp.dim == 2 || L.nx / 2 <= tune::QUADS_MAXPAIR;
}

// one red-black sweep of a 2D 5-point level, xin -> xout (mgmc_rb2d.hpp)
void launch_rb2d(const Level& lv, const double* xin, double* xout, const double* f, const GibbsArg& g, int direction,
                 bool noise, hipStream_t s, int nch = 1) {
    const int ntx = (lv.L.nx - 1 + RB2_TW - 1) / RB2_TW, nty = (lv.L.ny - 1 + RB2_TH - 1) / RB2_TH;
    const int c1 = direction == MGMC_FORWARD ? 0 : 1;
    const dim3 grid(ntx * nty, 1, nch), block(RB2_NT);
    const long long cs = lv.L.nstore;
    if (noise)
        hipLaunchKernelGGL((k_rb2d<true>), grid, block, 0, s, lv.L, xin, xout, f, lv.S, g, c1, ntx, cs);
    else
        hipLaunchKernelGGL((k_rb2d<false>), grid, block, 0, s, lv.L, xin, xout, f, lv.S, g, c1, ntx, cs);
}

// j-marching half-sweeps (k_jsweep_half): 3D 27-point levels with rows of 128 or 256 pairs (nx = 256: level 1
// at 512^3; nx = 512: the FEM prior's fine level at 512^3), x read about 1.5 times per half instead of once
// per colour-pair pass (DESIGN.md sections 3a, 3c; 512^3 FEM cycle 4.65 -> 3.76 ms).
// With 64-pair rows (512^3 level 2, 256^3 level 1) the kernel is slower than the pair passes (2 x 21 against
// 4 x 8 us per sweep at 127^3, 256^3 cycle 0.484 -> 0.503 ms): those levels are latency-bound, and the
// march's chunks are short.
bool jsweep_eligible(const LevelSpec& sp, const Layout& L, uint32_t paths) {
    return sp.dim == 3 && sp.npoints == 27 && (L.nx == 256 || L.nx == 512) &&
           L.ny >= 2 && L.nz >= 2 &&
           !(paths & PATH_NO_JSWEEP);
}


// xzero: xin is known zero (Op::xzero): the first half takes zeros for every x row, the second for its own
// planes (the neighbouring planes are the first half's new values)
void launch_jsweep(const Level& lv, const double* xin, double* xout, const double* f, const GibbsArg& g, int direction,
                   hipStream_t s, int nch, bool xzero = false) {
    JSweepArgs a;
    a.cs = lv.L.nstore;
    a.L = lv.L;
    a.xo = xin;
    a.xout = xout;
    a.f = f;
    a.S = lv.S;
    a.G = g;
    const int np = lv.L.nx / 2;
    const size_t lds = jsweep_lds_bytes(np);
    const bool fwd = direction == MGMC_FORWARD;
    for (int h = 0; h < 2; ++h) {
        // resident workgroups: LDS-bound (160 KB per CU), one round of them per half (jsweep_plan; the
        // host check mgmc_layout_check.hpp jsweep_grid_check replays the same plan)
        const JSweepPlan p = jsweep_plan(lv.L, fwd, h, lv.num_cu, lds, tune::JS_ROUNDS);
        if (p.nk == 0) continue;
        a.kp = p.kp;
        a.jA = p.jA;  // first pair of a half: colours (0,1) / (4,5) forward, (7,6) / (3,2) backward
        a.nsteps = p.nsteps;
        a.nk = p.nk;
        a.spc = p.spc;
        a.nchunk = p.nchunk;
        a.xz = h == 0 ? xin : xout;  // the second half reads the first half's new planes
        const dim3 grid(p.nb, 1, nch), block(2 * np);
#define MGMC_JS_LAUNCH_XZ(NPV, SYMV, XZ)                                                            \
    do {                                                                                            \
        if (fwd) hipLaunchKernelGGL((k_jsweep_half<NPV, false, SYMV, XZ>), grid, block, lds, s, a); \
        else hipLaunchKernelGGL((k_jsweep_half<NPV, true, SYMV, XZ>), grid, block, lds, s, a);      \
    } while (0)
#define MGMC_JS_LAUNCH(NPV, SYMV)                                 \
    do {                                                          \
        if (!xzero) MGMC_JS_LAUNCH_XZ(NPV, SYMV, 0);              \
        else if (h == 0) MGMC_JS_LAUNCH_XZ(NPV, SYMV, 1);         \
        else MGMC_JS_LAUNCH_XZ(NPV, SYMV, 2);                     \
    } while (0)
        if (np == 256) {  // FEM prior's 27-point fine level at 512^3 (not symmetric bit for bit)
            MGMC_JS_LAUNCH(256, false);
        } else if (lv.sym) {  // the cubic FD hierarchies' 255^3 level: 8 distinct coefficients
            MGMC_JS_LAUNCH(128, true);
        } else {
            MGMC_JS_LAUNCH(128, false);
        }
#undef MGMC_JS_LAUNCH
#undef MGMC_JS_LAUNCH_XZ
    }
}

// zb: the sweep's Box-Muller pairs, drawn by an earlier launch (Op::pnz, plan_drawn_noise; 3D quad-pass
// levels, one chain; with xzero forward sweeps only)
void launch_quads(const Level& lv, const double* xin, double* xout, const double* f, const GibbsArg& g, int direction,
                  hipStream_t s, int nch = 1, bool xzero = false, const double2* zb = nullptr) {
    if (lv.jsweep) {
        launch_jsweep(lv, xin, xout, f, g, direction, s, nch, xzero);
        return;
    }
    QuadPassArgs a;
    a.zb = zb;
    a.cs = lv.L.nstore;
    a.L = lv.L;
    a.x0 = xin;
    a.xout = xout;
    a.f = f;
    a.S = lv.S;
    a.G = g;
    const int dim = lv.spec.dim;
    const int npair = lv.L.nx / 2;
    // T+1 thread rows of npair threads
    // (threads per workgroup, mgmc_tuning.hpp: 2D config 2 at 1024^2: 512 10,623, 256 10,775, 128 10,883
    // samples/s; 127^3 rows 256 threads 58.3 us per 512^3 cycle against 61.6 at 512; 63^3 / 31^3 rows 128
    // threads, 512^3 launches 7.3-7.8 -> 5.6-6.3 us against 512)
    a.T = std::max(1, (dim == 3 ? (npair > 32 ? tune::QUADS_NT_WIDE : tune::QUADS_NT3) : tune::QUADS_NT) / npair - 1);
    a.nblk_y = (lv.L.ny - 1 + 2 * a.T - 1) / (2 * a.T);
    const int nt = npair * (a.T + 1);
    const size_t lds = (size_t)(2 * a.T + 1) * (lv.L.nx + 2) * sizeof(double);
    const bool fwd = direction == MGMC_FORWARD;
    const bool lanes = dim == 3 && 64 % npair == 0 && tune::QUADS_LANES != 0;
    a.jp1 = fwd ? 0 : 1;  // first pair: colours (0,1) / (4,5) forward, (7,6) / (3,2) backward
    const int nhalf = dim == 3 ? 2 : 1;
    for (int h = 0; h < nhalf; ++h) {
        a.kp = fwd ? h : 1 - h;
        a.xz = h == 0 ? xin : xout;  // the second half reads the first half's new planes
        const int first = 2 - a.kp;
        const int nk = dim == 3 ? (first > lv.L.nz - 1 ? 0 : (lv.L.nz - 1 - first) / 2 + 1) : 1;
        if (nk == 0) continue;
        const dim3 grid(a.nblk_y * nk, 1, nch);
        if (dim == 3) {
            // xzero (3D): the first half takes every x row as 0.0, the second its own planes' rows
            // rows of npair dividing 64 (127^3 / 63^3 / 31^3 ...): whole rows per wavefront, the window's
            // outer columns by lane shifts (k_sweep_quads LANES)
#define MGMC_QD_LAUNCH(SYMV, XZ)                                                                            \
    do {                                                                                                    \
        if (lanes) {                                                                                        \
            if (fwd) hipLaunchKernelGGL((k_sweep_quads<3, false, SYMV, XZ, true>), grid, dim3(nt), lds, s, a); \
            else hipLaunchKernelGGL((k_sweep_quads<3, true, SYMV, XZ, true>), grid, dim3(nt), lds, s, a);      \
        } else if (fwd) hipLaunchKernelGGL((k_sweep_quads<3, false, SYMV, XZ>), grid, dim3(nt), lds, s, a);  \
        else hipLaunchKernelGGL((k_sweep_quads<3, true, SYMV, XZ>), grid, dim3(nt), lds, s, a);             \
    } while (0)
// (drawn noise with a known-zero input: forward sweeps only, plan_drawn_noise)
#define MGMC_QD_PZ(SYMV, LANESV)                                                                                   \
    do {                                                                                                           \
        if (xzero && h == 0) hipLaunchKernelGGL((k_sweep_quads<3, false, SYMV, 1, LANESV, true>), grid, dim3(nt), lds, s, a); \
        else if (xzero) hipLaunchKernelGGL((k_sweep_quads<3, false, SYMV, 2, LANESV, true>), grid, dim3(nt), lds, s, a);      \
        else if (fwd) hipLaunchKernelGGL((k_sweep_quads<3, false, SYMV, 0, LANESV, true>), grid, dim3(nt), lds, s, a);       \
        else hipLaunchKernelGGL((k_sweep_quads<3, true, SYMV, 0, LANESV, true>), grid, dim3(nt), lds, s, a);                  \
    } while (0)
#define MGMC_QD_XZ(SYMV)                              \
    do {                                              \
        if (zb && lanes) MGMC_QD_PZ(SYMV, true);      \
        else if (zb) MGMC_QD_PZ(SYMV, false);         \
        else if (!xzero) MGMC_QD_LAUNCH(SYMV, 0);     \
        else if (h == 0) MGMC_QD_LAUNCH(SYMV, 1);     \
        else MGMC_QD_LAUNCH(SYMV, 2);                 \
    } while (0)
            if (lv.sym) MGMC_QD_XZ(true);
            else MGMC_QD_XZ(false);
#undef MGMC_QD_XZ
#undef MGMC_QD_PZ
#undef MGMC_QD_LAUNCH
        } else {
            if (fwd) hipLaunchKernelGGL((k_sweep_quads<2, false>), grid, dim3(nt), lds, s, a);
            else hipLaunchKernelGGL((k_sweep_quads<2, true>), grid, dim3(nt), lds, s, a);
        }
    }
}

void launch_pairs(const Level& lv, double* x, const double* f, const GibbsArg& g, int direction, hipStream_t s,
                  int nch = 1) {
    PairPassArgs a;
    a.cs = lv.L.nstore;
    a.L = lv.L;
    a.x = x;
    a.f = f;
    a.S = lv.S;
    a.G = g;
    const int dim = lv.spec.dim;
    const int npair = lv.L.nx / 2;
    a.rows_per_block = 256 / npair;
    const int npass = dim == 3 ? 4 : 2;
    auto count = [](int n, int parity) {  // coordinates 2 - parity + 2t in [1, n-1]
        const int first = 2 - parity;
        return first > n - 1 ? 0 : (n - 1 - first) / 2 + 1;
    };
    for (int ps = 0; ps < npass; ++ps) {
        const int c = direction == MGMC_FORWARD ? 2 * ps : 2 * (npass - 1 - ps) + 1;  // first colour
        a.jp = (c >> 1) & 1;
        a.kp = (c >> 2) & 1;
        a.nrows_j = count(lv.L.ny, a.jp);
        a.nrows = a.nrows_j * (dim == 3 ? count(lv.L.nz, a.kp) : 1);
        if (a.nrows == 0) continue;
        const dim3 grid((a.nrows + a.rows_per_block - 1) / a.rows_per_block, 1, nch);
        const int nt = a.rows_per_block * npair;
        const bool odd = c & 1;
        if (dim == 3) {
            if (lv.sym) {
                if (odd) hipLaunchKernelGGL((k_sweep_pairs<3, true, true>), grid, dim3(nt), 0, s, a);
                else hipLaunchKernelGGL((k_sweep_pairs<3, false, true>), grid, dim3(nt), 0, s, a);
            } else {
                if (odd) hipLaunchKernelGGL((k_sweep_pairs<3, true>), grid, dim3(nt), 0, s, a);
                else hipLaunchKernelGGL((k_sweep_pairs<3, false>), grid, dim3(nt), 0, s, a);
            }
        } else {
            if (odd) hipLaunchKernelGGL((k_sweep_pairs<2, true>), grid, dim3(nt), 0, s, a);
            else hipLaunchKernelGGL((k_sweep_pairs<2, false>), grid, dim3(nt), 0, s, a);
        }
    }
}

// the coarse SSOR sampler's right-hand sides are precomputed when they fit next to x and f
bool coarse_precompute(const Level& lv, int nsweeps) {
    const long long ndof = (long long)(lv.L.nx - 1) * (lv.L.ny - 1) * (lv.spec.dim == 3 ? lv.L.nz - 1 : 1);
    return lv.lds_bytes + (size_t)nsweeps * ndof * sizeof(double) <= 150 * 1024;
}

// zb: its Box-Muller pairs drawn by the launch before (nullptr: drawn here)
void launch_coarse_lds(const Level& lv, const GibbsArg& g, int nsweeps, hipStream_t s, int nch = 1,
                       const double2* zb = nullptr, long long zs = 0) {
    const int dim = lv.spec.dim, np = lv.spec.npoints, nc = lv.spec.ncolours;
    dim3 block(1024), grid(1, 1, nch);
    const long long chs = lv.L.nstore;
    const long long ndof = (long long)(lv.L.nx - 1) * (lv.L.ny - 1) * (dim == 3 ? lv.L.nz - 1 : 1);
    const size_t lds_pre = lv.lds_bytes + (size_t)nsweeps * ndof * sizeof(double);
    const int pre = coarse_precompute(lv, nsweeps);
    const size_t lds = pre ? lds_pre : lv.lds_bytes;
#define MGMC_COARSE_LAUNCH(D, P)                                                                                 \
    do {                                                                                                           \
        if (pre && zb)                                                                                             \
            hipLaunchKernelGGL((k_coarse_ssor_lds<D, P, true, true>), grid, block, lds, s, lv.L, lv.x, lv.f, lv.S, \
                               g, nsweeps, nc, chs, zb, zs);                                                       \
        else if (pre)                                                                                              \
            hipLaunchKernelGGL((k_coarse_ssor_lds<D, P, true>), grid, block, lds, s, lv.L, lv.x, lv.f, lv.S, g,   \
                               nsweeps, nc, chs, nullptr, 0);                                                      \
        else                                                                                                       \
            hipLaunchKernelGGL((k_coarse_ssor_lds<D, P, false>), grid, block, lds, s, lv.L, lv.x, lv.f, lv.S, g,  \
                               nsweeps, nc, chs, nullptr, 0);                                                      \
    } while (0)
    if (dim == 3 && np == 27) MGMC_COARSE_LAUNCH(3, 27);
    else if (dim == 3 && np == 7) MGMC_COARSE_LAUNCH(3, 7);
    else if (dim == 2 && np == 9) MGMC_COARSE_LAUNCH(2, 9);
    else MGMC_COARSE_LAUNCH(2, 5);
#undef MGMC_COARSE_LAUNCH
}


template <int NPTS, int CX, int CY, int NT, bool SYM = false, bool LRF = false>
void launch_zresrestrict_t(const Level& lf, const Level& lc, const double* x, const double* f, double* fc, double* xc,
                           hipStream_t s, int nch, const TailNoiseLaunch* tn = nullptr, const LRRhsArg* lr = nullptr,
                           const PreNoiseLaunch* pn = nullptr) {
    ZRestrictArgs a;
    memset(&a, 0, sizeof(a));
    if (LRF) a.lr = *lr;
    if (pn) {  // (one chain: nch == 1)
        a.pn = pn->job;
        a.key = pn->key;
        a.sample = pn->sample;
    }
    a.csf = lf.L.nstore;
    a.csc = lc.L.nstore;
    a.Lf = lf.L;
    a.Lc = lc.L;
    a.x = x;
    a.f = f;
    a.fc = fc;
    a.xc = xc;
    a.S = lf.S;
    a.ntx = (lc.L.nx - 1 + CX - 1) / CX;
    a.nty = (lc.L.ny - 1 + CY - 1) / CY;
    // 8 coarse planes per workgroup, fewer on small levels so the grid still fills the chip
    // (512^3 level 1 -> 2: kz 4, 103 us against 116 / 146 us with 2 / 8)
    const long long work = (long long)a.ntx * a.nty * (lc.L.nz - 1);
    a.kz = work >= 8 * 1024 ? 8 : (work >= 4 * 1024 ? 4 : (work >= 512 ? 2 : 1));
    if (NPTS == 7 && work >= 16 * 1024) {
        // fine 7-point level: the deepest chunks that still give two full rounds of workgroups (every
        // chunk re-reads 2 x planes and 1 f plane below / above it: 512^3 with 64 x 4 tiles kz 8 -> 43
        // (6 chunks, 1536 tiles on 256 CUs x 3 workgroups): 561 -> 451 us; with 64 x 8 tiles kz 32)
        const long long slots = (NT >= 512 ? 2LL : 3LL) * lf.num_cu;  // workgroups per CU (LDS, VGPRs)
        const long long per_chunk = (long long)a.ntx * a.nty;
        const long long nchunk = std::max(1LL, (2 * slots + per_chunk - 1) / per_chunk);
        a.kz = std::max(8, (int)((lc.L.nz - 1 + nchunk - 1) / nchunk));
    }
    // (the same depth rule for the 7-point 64 x 4 instance: 256^3 fine level kz 4 -> 11, 2,048 -> 768
    // workgroups = one round, 64.4 -> 57.7 us)
    if ((NPTS == 27 || (NPTS == 7 && NT == 256)) && CX >= 48 && work >= 4 * 1024) {
        // 27-point levels with enough tiles for several rounds (512^3 level 1): the chunk depth that
        // minimises rounds of resident workgroups x planes staged per chunk (2 kz + 2); 512^3 level 1:
        // kz 11 = 768 tiles, one round of 3 x 256 slots: 108 -> 101 us (round 4, kernel traces)
        // workgroups per CU: LDS-bound, and at most 3 for the 27-point instances (> 128 VGPRs)
        const long long per_cu = std::min<long long>(160 * 1024 / zrestrict_lds_bytes(CX, CY),
                                                     NPTS == 27 ? std::max(3, tune::ZR27_MINW) : 4);
        const long long slots = per_cu * lf.num_cu;
        const long long per_chunk = (long long)a.ntx * a.nty;
        long long best = -1;
        for (int kz = 2; kz <= 16; ++kz) {
            const long long tiles = per_chunk * ((lc.L.nz - 1 + kz - 1) / kz);
            const long long cost = ((tiles + slots - 1) / slots) * (2 * kz + 2);
            if (best < 0 || cost < best) {
                best = cost;
                a.kz = kz;
            }
        }
    }
    a.ntz = (lc.L.nz - 1 + a.kz - 1) / a.kz;
    const int nt = a.ntx * a.nty * a.ntz;
    const int nb = (nt + 7) / 8 * 8;
    if (tn && !LRF) {
        a.nblk_main = nb;
        a.jobs = tn->jobs;
        a.njobs = tn->njobs;
        a.zb = tn->zb;
        a.zbs = tn->zbs;
        a.key = tn->key;
        a.chain0 = tn->chain0;
        a.seed_hi = tn->seed_hi;
        a.sample = tn->sample;
        const int nextra = (int)std::min<long long>((tn->zbs + NT - 1) / NT, 64);
        hipLaunchKernelGGL((k_zresrestrict<NPTS, CX, CY, NT, true, SYM>), dim3(nb + nextra, 1, nch), dim3(NT),
                           zrestrict_lds_bytes(CX, CY), s, a);
        return;
    }
    hipLaunchKernelGGL((k_zresrestrict<NPTS, CX, CY, NT, false, SYM, LRF>), dim3(nb, 1, nch), dim3(NT),
                       zrestrict_lds_bytes(CX, CY), s, a);
}

// tn: the small z-marching kernel also draws a tail's noise (zr_small_path; ignored elsewhere)
// skip_xc: the z-marching kernel leaves x_c alone (Op::xzero: the coarse level's first sweep takes it as
// zeros without loading it)
// the levels whose residual + restriction runs a k_zresrestrict instance with an LRF variant (the
// 7-point z-marching kernels of the non-small coarse levels: launch_residual_restrict below)
bool zres_lrf_capable(const Level& lf, const Level& lc) {
    return lf.spec.dim == 3 && lf.spec.npoints == 7 && !lf.field && !(lf.paths & PATH_NO_ZRESTRICT) &&
           lc.L.nx >= 8 && lc.L.nx >= tune::ZR_SMALL_NX;
}

// lr (non-null): the level's right-hand side is read in place (LRRhsArg; zres_lrf_capable levels only)
// the z-marching 27-point residual + restriction of a non-small coarse level: launch_residual_restrict's path
// for zero_xc = 1 that can also draw the coarse level's first pre-sweep's noise (pn)
bool zres_draws_noise(const Level& lf, const Level& lc) {
    return lf.spec.dim == 3 && lf.spec.npoints == 27 && !lf.field && !(lf.paths & PATH_NO_ZRESTRICT) &&
           lc.L.nx >= tune::ZR_SMALL_NX;
}

void launch_residual_restrict(const Level& lf, const Level& lc, const double* x, const double* f, double* fc,
                              double* xc, int zero_xc, hipStream_t s, int nch, const TailNoiseLaunch* tn,
                              bool skip_xc, const LRRhsArg* lr, const PreNoiseLaunch* pn) {
    const bool zr = lf.spec.dim == 3 && zero_xc && !lf.field && !(lf.paths & PATH_NO_ZRESTRICT) && lc.L.nx >= 8;
    if (nch > 1 && !zr) {  // batched chains on the generic kernels: one launch per chain
        for (int c = 0; c < nch; ++c)
            launch_residual_restrict(lf, lc, chain_ptr(x, lf, c), chain_ptr(f, lf, c), chain_ptr(fc, lc, c),
                                     chain_ptr(xc, lc, c), zero_xc, s, 1);
        return;
    }
    if (lf.field) {  // r = f - A x into the level's scratch, then fc = R r (and x_c = 0)
        dim3 block(64, 4, 1);
        dim3 grid = grid3(lf.L.nx - 1, lf.L.ny - 1, lf.spec.dim == 3 ? lf.L.nz - 1 : 1, block);
        dim3 gc = grid3(lc.L.nx - 1, lc.L.ny - 1, lf.spec.dim == 3 ? lc.L.nz - 1 : 1, block);
        if (lf.spec.dim == 3) {
            hipLaunchKernelGGL((k_fresidual<3>), grid, block, 0, s, lf.L, x, f, lf.F, lf.rbuf);
            hipLaunchKernelGGL((k_restrict<3>), gc, block, 0, s, lf.L, lc.L, (const double*)lf.rbuf, fc);
        } else {
            hipLaunchKernelGGL((k_fresidual<2>), grid, block, 0, s, lf.L, x, f, lf.F, lf.rbuf);
            hipLaunchKernelGGL((k_restrict<2>), gc, block, 0, s, lf.L, lc.L, (const double*)lf.rbuf, fc);
        }
        if (zero_xc) hipMemsetAsync(xc, 0, lc.L.nstore * sizeof(double), s);
        return;
    }
    // z-marching kernel on every 3D level with coarse n >= 8: 64 x 4 coarse points per workgroup from
    // coarse n = ZR_SMALL_NX up, 16 x 4 points (one wavefront) below, where the wide tiles would leave
    // most of the chip idle (the 27-point gather kernel took 24 us per launch on the 15^3 / 7^3 levels)
    if (lf.spec.dim == 3 && zero_xc && !(lf.paths & PATH_NO_ZRESTRICT) && lc.L.nx >= 8) {
        const bool small = lc.L.nx < tune::ZR_SMALL_NX;
        if (skip_xc) xc = nullptr;
        if (lr) {  // (zres_lrf_capable)
            if ((long long)((lc.L.nx + 62) / 64) * ((lc.L.ny + 6) / 8) * (lc.L.nz - 1) >= tune::ZR7_WIDE_MIN_TILES)
                launch_zresrestrict_t<7, 64, 8, 512, false, true>(lf, lc, x, f, fc, xc, s, nch, nullptr, lr);
            else launch_zresrestrict_t<7, 64, 4, 256, false, true>(lf, lc, x, f, fc, xc, s, nch, nullptr, lr);
        } else if (lf.spec.npoints == 7) {
            if (small) launch_zresrestrict_t<7, 16, 4, 64>(lf, lc, x, f, fc, xc, s, nch, tn);
            // 64 x 8 coarse points, 512 threads, 80 KB of LDS (2 workgroups per CU): half the y halo
            // of 64 x 4 (19 x planes rows per 16 fine rows instead of 11 per 8); 512^3 with kz 32:
            // 505-525 -> 488-502 us (interleaved A/B); at 256^3 too few tiles (73 against 66 us)
            else if ((long long)((lc.L.nx + 62) / 64) * ((lc.L.ny + 6) / 8) * (lc.L.nz - 1) >= tune::ZR7_WIDE_MIN_TILES)
                launch_zresrestrict_t<7, 64, 8, 512>(lf, lc, x, f, fc, xc, s, nch);
            else launch_zresrestrict_t<7, 64, 4, 256>(lf, lc, x, f, fc, xc, s, nch);
        } else {
            // (fold levels: the SYM instances, whose residual is fold27's)
            if (small && lf.fold) launch_zresrestrict_t<27, 16, 4, 64, true>(lf, lc, x, f, fc, xc, s, nch, tn);
            else if (small) launch_zresrestrict_t<27, 16, 4, 64>(lf, lc, x, f, fc, xc, s, nch, tn);
            else if (lf.fold)
                launch_zresrestrict_t<27, tune::ZR27_CX, tune::ZR27_CY, 256, true>(lf, lc, x, f, fc, xc, s, nch, nullptr,
                                                                                   nullptr, pn);
            else launch_zresrestrict_t<27, 64, 4, 256>(lf, lc, x, f, fc, xc, s, nch, nullptr, nullptr, pn);
        }
        return;
    }
    dim3 block(64, 4, 1);
    dim3 grid = grid3(lc.L.nx - 1, lc.L.ny - 1, lf.spec.dim == 3 ? lc.L.nz - 1 : 1, block);
    const int dim = lf.spec.dim, np = lf.spec.npoints;
    if (dim == 3 && np == 7)
        hipLaunchKernelGGL((k_residual_restrict<3, 7>), grid, block, 0, s, lf.L, lc.L, x, f, fc, xc, lf.S, zero_xc);
    else if (dim == 3 && lf.fold)
        hipLaunchKernelGGL((k_residual_restrict<3, 27, true>), grid, block, 0, s, lf.L, lc.L, x, f, fc, xc, lf.S, zero_xc);
    else if (dim == 3)
        hipLaunchKernelGGL((k_residual_restrict<3, 27>), grid, block, 0, s, lf.L, lc.L, x, f, fc, xc, lf.S, zero_xc);
    else if (np == 5)
        hipLaunchKernelGGL((k_residual_restrict<2, 5>), grid, block, 0, s, lf.L, lc.L, x, f, fc, xc, lf.S, zero_xc);
    else
        hipLaunchKernelGGL((k_residual_restrict<2, 9>), grid, block, 0, s, lf.L, lc.L, x, f, fc, xc, lf.S, zero_xc);
}

// 2D Galerkin level: its last pre-sweep and the residual + restriction onto lc in one launch
// (mgmc_qrestrict.hpp).  One pair item per thread per colour phase: NT >= (CJ + 3) nx / 2 with CJ
// coarse rows per workgroup, CJ as small as the thread count allows (the most workgroups: these levels
// are launch-bound, the recomputed edge rows cost little)
int qrestrict_threads(int npair) {
    const int nt = 4 * npair <= 256 ? 256 : (4 * npair <= 512 ? 512 : 1024);
    return 4 * npair <= nt ? nt : 0;
}

bool qrestrict_ok(const mgmc_handle* h, int level);


// zc != nullptr: spare workgroups also draw the coarsest level's SSOR-sampler noise (nsweeps sweeps from
// tag zc_tag) into zc, zcs items per chain
void launch_qrestrict(const Level& lv, const Level& lc, const double* xin, double* xout, const double* f, double* fc,
                      double* xc, const GibbsArg& g, int direction, hipStream_t s, int nch = 1, double2* zc = nullptr,
                      int zc_nsweeps = 0, uint32_t zc_tag = 0, long long zcs = 0) {
    QRestrictArgs a;
    a.zc = zc;
    a.zc_nsweeps = zc_nsweeps;
    a.zc_tag = zc_tag;
    a.zcs = zcs;
    a.L = lv.L;
    a.Lc = lc.L;
    a.xin = xin;
    a.xout = xout;
    a.f = f;
    a.fc = fc;
    a.xc = xc;
    a.S = lv.S;
    a.G = g;
    a.cs = lv.L.nstore;
    a.csc = lc.L.nstore;
    const int npair = lv.L.nx / 2;
    const int nt = qrestrict_threads(npair);
    a.CJ = nt / npair - 3;
    a.nblk_main = (lc.L.ny - 1 + a.CJ - 1) / a.CJ;
    const int nextra = zc ? (int)std::min<long long>((zcs + nt - 1) / nt, 64) : 0;
    const dim3 grid(a.nblk_main + nextra, 1, nch);
    const size_t lds = qrestrict_lds_bytes(lv.L.nx, a.CJ);
    const bool fwd = direction == MGMC_FORWARD;
#define MGMC_QR_LAUNCH(NT)                                                                               \
    do {                                                                                                   \
        if (fwd) hipLaunchKernelGGL((k_quads_restrict2d<NT, false>), grid, dim3(NT), lds, s, a);           \
        else hipLaunchKernelGGL((k_quads_restrict2d<NT, true>), grid, dim3(NT), lds, s, a);                \
    } while (0)
    if (nt == 256) MGMC_QR_LAUNCH(256);
    else if (nt == 512) MGMC_QR_LAUNCH(512);
    else MGMC_QR_LAUNCH(1024);
#undef MGMC_QR_LAUNCH
}

void launch_prolongate(const Level& lf, const Level& lc, double* x, const double* xc, double alpha, hipStream_t s,
                       int nch) {
    dim3 block(64, 4, 1);
    const int zper = lf.spec.dim == 3 ? lf.L.nz - 1 : 1;  // batched chains: blockIdx.z = chain * zper + plane
    dim3 grid = grid3(lf.L.nx / 2, lf.L.ny - 1, zper * nch, block);
    const long long csf = lf.L.nstore, csc = lc.L.nstore;
    // z-marching prolongation on big 3D levels (fine planes per thread: mgmc_tuning.hpp)
    if (lf.spec.dim == 3 && (long long)(lf.L.nx / 2) * (lf.L.ny - 1) * (lf.L.nz - 1) >= (1LL << 16) &&
        !(lf.paths & PATH_NO_PROLONG_Z)) {
        constexpr int TZ = tune::PROLONG_Z;
        // fewer planes per thread below 2^21 fine pair items: twice the threads on the 127^3 / 63^3
        // levels (512^3: 10.7 / 8.9 -> 9.2 / 6.3 us; 2 planes: 9.7 / 6.0 us)
        constexpr int TZS = tune::PROLONG_Z_SMALL;
        if (TZS != TZ && (long long)(lf.L.nx / 2) * (lf.L.ny - 1) * (lf.L.nz - 1) < (1LL << 21)) {
            const int nzc = (lf.L.nz - 1 + TZS - 1) / TZS;
            const dim3 gz = grid3(lf.L.nx / 2, lf.L.ny - 1, nzc * nch, block);
            hipLaunchKernelGGL((k_prolongate_z<TZS>), gz, block, 0, s, lf.L, lc.L, x, xc, alpha, nzc, csf, csc);
            return;
        }
        const int nzc = (lf.L.nz - 1 + TZ - 1) / TZ;
        const dim3 gz = grid3(lf.L.nx / 2, lf.L.ny - 1, nzc * nch, block);
        hipLaunchKernelGGL((k_prolongate_z<TZ>), gz, block, 0, s, lf.L, lc.L, x, xc, alpha, nzc, csf, csc);
        return;
    }
    if (lf.spec.dim == 3)
        hipLaunchKernelGGL((k_prolongate_pairs<3>), grid, block, 0, s, lf.L, lc.L, x, xc, alpha, zper, csf, csc);
    else
        hipLaunchKernelGGL((k_prolongate_pairs<2>), grid, block, 0, s, lf.L, lc.L, x, xc, alpha, zper, csf, csc);
}

void launch_pack(const Level& lv, const double* lex, double* pad, bool pack, hipStream_t s) {
    dim3 block(64, 4, 1);
    dim3 grid = grid3(lv.L.nx - 1, lv.L.ny - 1, lv.spec.dim == 3 ? lv.L.nz - 1 : 1, block);
    if (lv.spec.dim == 3) {
        if (pack)
            hipLaunchKernelGGL((k_pack<3>), grid, block, 0, s, lv.L, lex, pad);
        else
            hipLaunchKernelGGL((k_unpack<3>), grid, block, 0, s, lv.L, (const double*)pad, (double*)lex);
    } else {
        if (pack)
            hipLaunchKernelGGL((k_pack<2>), grid, block, 0, s, lv.L, lex, pad);
        else
            hipLaunchKernelGGL((k_unpack<2>), grid, block, 0, s, lv.L, (const double*)pad, (double*)lex);
    }
}

// ---- low-rank part (mgmc_lowrank.hpp) ----
// w = (sc_k B_k)^T v for all columns
// (batched chains: v cs apart; the partials nblk and w m apart per chain)
void lr_dots(const Level& lv, const double* v, LRScale scale, hipStream_t s, int nch) {
    const LowRankDev& r = lv.lr;
    const int sel = (int)scale;
    // few wavefronts (coarse levels): the staged kernel (the loads of a block in flight at once);
    // many: one wavefront per block, column values read once per group of chains
    const long long waves = (long long)r.nblk * ((nch + LRP_CH - 1) / LRP_CH);
    if (r.nblk > 0 && waves < tune::LR_STAGED_MAX_WAVES)
        hipLaunchKernelGGL(k_lr_partials_staged, dim3(r.nblk, nch), dim3(LRS_NT), 0, s, lv.L, (const LRBlock*)r.blk, sel,
                           (const long long*)r.ent_off, (const double*)r.ent_val, (const double*)r.dense_val, v,
                           r.part, (long long)lv.L.nstore, r.nblk);
    else if (r.nblk > 0)
        hipLaunchKernelGGL(k_lr_partials, dim3(r.nblk, (nch + LRP_CH - 1) / LRP_CH), dim3(64), 0, s, lv.L,
                           (const LRBlock*)r.blk, sel, (const long long*)r.ent_off,
                           (const double*)r.ent_val, (const double*)r.dense_val, v, r.part,
                           (long long)lv.L.nstore, r.nblk, nch);
    hipLaunchKernelGGL(k_lr_totals, dim3(r.m, 1, nch), dim3(64), 0, s, (const LRColMeta*)r.meta, (const double*)r.part,
                       r.w, r.nblk, r.m);
}

// patch y on the rows of B (LR_PATCH_NOISE: y += B Sigma^{-1/2} xi'; RESIDUAL: y -= B w; APPLY: y += B w)
void lr_patch(const mgmc_handle* h, const Level& lv, int mode, double* y, uint32_t tag, const uint64_t* sample,
              hipStream_t s, int nch = 1, double* eout = nullptr) {
    const LowRankDev& r = lv.lr;
    if (r.nrows == 0 && !eout) return;
    LRPatchArgs a;
    a.m = r.m;
    a.nrows = r.nrows;
    a.off = r.rows_off;
    a.coef = r.rows_coef;
    a.mask = r.rows_mask;
    a.t = r.w;
    a.sq = r.sq;
    a.key = h->key;
    a.tag = tag;
    a.sample = sample;
    a.y = y;
    a.save = r.save;
    a.mode = mode;
    a.cs = lv.L.nstore;
    a.chain0 = (uint32_t)h->chain;
    a.seed_hi = (uint32_t)(h->seed >> 32);
    a.split_g = mode == LR_PATCH_APPLY ? -1 : r.split_g;
    a.eout = eout;  // (a level read in place: LRRhsArg)
    a.bgc = r.dense_cval;
    hipLaunchKernelGGL(k_lr_patch, dim3(std::max((r.nrows + 255) / 256, 1), 1, nch), dim3(256), 0, s, a);
}

// the right-hand side a low-rank level's sweep (LR_PATCH_NOISE: f + B Sigma^{-1/2} xi') or
// residual (LR_PATCH_RESIDUAL: f - B t, t = r.w) reads; returns the vector to read.  Dense-column
// path: written to r.fe, f untouched; otherwise f is patched in place (saved for lr_restore).
// LR_PATCH_APPLY: f += B t in place on either path.
// post_tag >= 0 (dense-column path, LR_PATCH_RESIDUAL): the same launch also writes r.fe2 =
// f + B Sigma^{-1/2} xi' of the level's first post-sweep (tag post_tag), which then reads r.fe2
// inplace (non-null, a level with lr.rhs_inplace, LR_PATCH_NOISE / RESIDUAL): f is patched in place on
// the local rows and the chains' dense-only patch goes to lr.rhs_e; *inplace tells the consumer
// kernel how to read f (returned; post_tag unused: the first post-sweep's patch is lr_restore_patch's)
double* lr_rhs(const mgmc_handle* h, const Level& lv, int mode, double* f, uint32_t tag, const uint64_t* sample,
               hipStream_t s, int nch, int64_t post_tag, LRRhsArg* inplace) {
    const LowRankDev& r = lv.lr;
    if (!r.dense_path) {
        lr_patch(h, lv, mode, f, tag, sample, s, nch);
        return f;
    }
    if (inplace && r.rhs_inplace && mode != LR_PATCH_APPLY) {
        lr_patch(h, lv, mode, f, tag, sample, s, nch, r.rhs_e);
        *inplace = LRRhsArg{r.rhs_e};
        return f;
    }
    LRDenseArgs a;
    a.m = r.m;
    a.g = r.dense_g;
    a.mode = mode;
    a.nch = nch;
    a.cs = lv.L.nstore;
    a.chain0 = (uint32_t)h->chain;
    a.seed_hi = (uint32_t)(h->seed >> 32);
    a.key = h->key;
    a.tag = tag;
    a.sample = sample;
    a.sq = r.sq;
    a.t = r.w;
    a.f = f;
    a.out = mode == LR_PATCH_APPLY ? f : r.fe;
    a.out2 = post_tag >= 0 ? r.fe2 : nullptr;
    a.tag2 = post_tag >= 0 ? (uint32_t)post_tag : 0u;
    a.nrows = r.nrows;
    a.nbs = (r.nrows + LRD_NT - 1) / LRD_NT;
    a.off = r.rows_off;
    a.coef = r.rows_coef;
    a.mask = r.rows_mask;
    a.n = lv.L.nstore;
    a.skip = r.skip_b;
    a.bg = r.dense_val + (size_t)r.dense_slot * lv.L.nstore;  // the only dense column
    a.bgc = r.dense_cval;
    if (r.dense_const) a.bg = nullptr;  // B_g is one number: not streamed
    a.split_g = mode == LR_PATCH_APPLY ? -1 : r.split_g;
    const long long nbd = (a.n + LRD_ELEMS - 1) / LRD_ELEMS;
    hipLaunchKernelGGL(k_lr_dense_rhs, dim3((unsigned)(a.nbs + nbd)), dim3(LRD_NT), 0, s, a);
    return a.out;
}

// after a sweep in `direction`: x -= B_bar (B^T x) (sor_smoother.cc:47-51); restores f_restore
// on the rows of B when the sweep ran on a noise-patched f (not on the dense-column path, whose
// sweeps read r.fe)
void lr_fix(const Level& lv, double* x, int direction, double* f_restore, hipStream_t s, int nch) {
    const LowRankDev& r = lv.lr;
    lr_dots(lv, x, LR_SCALE_ONE, s, nch);
    const int d = direction == MGMC_FORWARD ? 0 : 1;
    if (r.dense_path) {
        LRDenseUpdateArgs a;
        a.m = r.m;
        a.g = r.dense_g;
        a.nch = nch;
        a.cs = lv.L.nstore;
        a.w = r.w;
        a.x = x;
        a.nbar = r.nbar[d];
        a.nbs = (r.nbar[d] + LRD_NT - 1) / LRD_NT;
        a.bar_off = r.bar_off[d];
        a.bar_val = r.bar_val[d];
        a.n = lv.L.nstore;
        a.skip = r.skip_y[d];
        a.yg = r.yg[d];
        a.ykey = r.ytab[d] ? r.ykey : nullptr;
        a.ytab = r.ytab[d];
        a.minv_g = r.minv_g[d];
        a.nrest = f_restore ? r.nrows : 0;  // (a right-hand side patched in place: rhs_inplace)
        a.rest_off = r.rows_off;
        a.rest_val = r.save;
        a.f = f_restore;
        a.nbs = (std::max(a.nbar, a.nrest) + LRD_NT - 1) / LRD_NT;
        const long long nbd = (a.n + LRD_ELEMS - 1) / LRD_ELEMS;
        hipLaunchKernelGGL(k_lr_dense_update, dim3((unsigned)(a.nbs + nbd)), dim3(LRD_NT), 0, s, a);
        return;
    }
    const int nrest = f_restore ? r.nrows : 0;
    const int n = std::max(r.nbar[d], nrest);
    if (n == 0) return;
    hipLaunchKernelGGL(k_lr_update, dim3((n + 255) / 256), dim3(256), 0, s, r.m, r.nbar[d],
                       (const long long*)r.bar_off[d], (const double*)r.bar_val[d], (const double*)r.w, x, nrest,
                       (const long long*)r.rows_off, (const double*)r.save, f_restore, nch, (long long)lv.L.nstore);
}

// the fused between-sweeps kernel (k_lr_small): fix x, restore f, patch f for the next op
void lr_small(const mgmc_handle* h, const Level& lv, double* x, int direction, int next, uint32_t next_tag,
              const uint64_t* sample, hipStream_t s, int nch = 1) {
    const LowRankDev& r = lv.lr;
    const int d = direction == MGMC_FORWARD ? 0 : 1;
    LRSmallArgs a;
    a.m = r.m;
    a.meta = r.meta;
    a.ent_off = r.ent_off;
    a.ent_val = r.ent_val;
    a.sc_one = r.sc_one;
    a.sc_inv = r.sc_inv;
    a.sq = r.sq;
    a.x = x;
    a.nbar = r.nbar[d];
    a.bar_off = r.bar_off[d];
    a.bar_val = r.bar_val[d];
    a.nrows = r.nrows;
    a.rows_off = r.rows_off;
    a.coef = r.rows_coef;
    a.mask = r.rows_mask;
    a.save = r.save;
    a.f = lv.f;
    a.restore = 1;
    a.next = next;
    a.key = h->key;
    a.tag = next_tag;
    a.sample = sample;
    a.cs = lv.L.nstore;  // batched chains: one workgroup per chain
    a.chain0 = (uint32_t)h->chain;
    a.seed_hi = (uint32_t)(h->seed >> 32);
    // k_lr_small_pf: one entry per lane, <= 8 columns, <= 2 rows of B_bar and of B per thread
    if (r.m <= 8 && r.max_col_n <= 64 && a.nbar <= 2048 && a.nrows <= 2048)
        hipLaunchKernelGGL((k_lr_small_pf<8, 2>), dim3(nch), dim3(1024), 0, s, a);
    else
        hipLaunchKernelGGL(k_lr_small, dim3(nch), dim3(1024), 0, s, a);
}

LRJob lr_job(const Level& lv, int restore, int noise, uint32_t tag) {
    const LowRankDev& r = lv.lr;
    LRJob j;
    j.m = r.m;
    j.nrows = r.nrows;
    j.off = r.rows_off;
    j.coef = r.rows_coef;
    j.mask = r.rows_mask;
    j.sq = r.sq;
    j.tag = tag;
    j.f = lv.f;
    j.save = r.save;
    j.restore = restore;
    j.noise = noise;
    j.split_g = r.split_g;
    j.eout = nullptr;
    j.bgc = r.dense_cval;
    return j;
}

// after a residual + restriction of a low-rank level: restore f (+ the patch of the first
// post-sweep) and the coarse level's first pre-sweep patch in one launch (k_lr_restore_patch)
void lr_restore_patch(const mgmc_handle* h, const Op& op, const Level& lv, const Level& lc, const uint64_t* sample,
                      hipStream_t s, int nch = 1) {
    LRRestorePatchArgs a;
    a.job[0] = lr_job(lv, 1, op.lr_post_patch, op.lr_post_tag);
    a.job[1] = op.lr_coarse_patch ? lr_job(lc, 0, 1, op.lr_coarse_tag) : lr_job(lc, 0, 0, 0);
    if (!op.lr_coarse_patch) a.job[1].nrows = 0;
    // (a level read in place: the first post-sweep's dense-only patch to rhs_e[nchains + c])
    if (lv.lr.rhs_inplace && op.lr_post_patch) a.job[0].eout = lv.lr.rhs_e + nch;
    a.nb0 = (a.job[0].nrows + 255) / 256;
    if (a.job[0].eout) a.nb0 = std::max(a.nb0, 1);
    const int nb = a.nb0 + (a.job[1].nrows + 255) / 256;
    a.key = h->key;
    a.sample = sample;
    a.cs[0] = lv.L.nstore;
    a.cs[1] = lc.L.nstore;
    a.chain0 = (uint32_t)h->chain;
    a.seed_hi = (uint32_t)(h->seed >> 32);
    if (nb > 0) hipLaunchKernelGGL(k_lr_restore_patch, dim3(nb, 1, nch), dim3(256), 0, s, a);
}

void lr_restore(const Level& lv, double* f, hipStream_t s, int nch, bool patched) {
    const LowRankDev& r = lv.lr;
    // dense-column path: f was never patched, unless read in place (patched)
    if (r.nrows == 0 || (r.dense_path && !patched)) return;
    hipLaunchKernelGGL(k_lr_restore, dim3((r.nrows + 255) / 256, 1, nch), dim3(256), 0, s, r.nrows,
                       (const long long*)r.rows_off, (const double*)r.save, f, (long long)lv.L.nstore);
}

// y = Q x on a level (LinearOperator::apply, linear_operator.hh:66-76)
void launch_operator_apply(const mgmc_handle* h, const Level& lv, const double* xs, double* ys, hipStream_t s) {
    dim3 block(64, 4, 1);
    dim3 grid = grid3(lv.L.nx - 1, lv.L.ny - 1, lv.spec.dim == 3 ? lv.L.nz - 1 : 1, block);
    const int dim = lv.spec.dim, np = lv.spec.npoints;
    if (lv.field && dim == 3)
        hipLaunchKernelGGL((k_fapply<3>), grid, block, 0, s, lv.L, xs, lv.F, ys);
    else if (lv.field)
        hipLaunchKernelGGL((k_fapply<2>), grid, block, 0, s, lv.L, xs, lv.F, ys);
    else if (dim == 3 && np == 7)
        hipLaunchKernelGGL((k_operator_apply<3, 7>), grid, block, 0, s, lv.L, xs, ys, lv.S);
    else if (dim == 3)
        hipLaunchKernelGGL((k_operator_apply<3, 27>), grid, block, 0, s, lv.L, xs, ys, lv.S);
    else if (np == 5)
        hipLaunchKernelGGL((k_operator_apply<2, 5>), grid, block, 0, s, lv.L, xs, ys, lv.S);
    else
        hipLaunchKernelGGL((k_operator_apply<2, 9>), grid, block, 0, s, lv.L, xs, ys, lv.S);
    if (lv.lr.m > 0) {  // y += B (Sigma^{-1} B^T x)  (linear_operator.hh:71-75)
        lr_dots(lv, xs, LR_SCALE_INV, s);
        lr_rhs(h, lv, LR_PATCH_APPLY, ys, 0, h->ctrl + 3, s);
    }
}

// coarsest level: x = G f (+ U xi) with the dense Cholesky factors, or the blocked banded solves
// (mgmc_cholesky.hpp)
void launch_coarse_chol(const mgmc_handle* h, const Level& lv, const double* f, double* x, bool noise, uint32_t tag,
                        const uint64_t* sample, hipStream_t s, int nch) {
    if (h->chol_B > 0) {
        CholBlockArgs b;
        b.L = lv.L;
        b.n = h->chol_n;
        b.B = h->chol_B;
        b.nb = h->chol_nb;
        const size_t blk = (size_t)h->chol_nb * h->chol_B * h->chol_B;
        b.Cf = h->chol_blk;
        b.Cb = h->chol_blk + blk;
        b.Df = h->chol_blk + 2 * blk;
        b.Db = h->chol_blk + 3 * blk;
        b.f = f;
        b.x = x;
        b.noise = noise ? 1 : 0;
        b.key = h->key;
        b.tag = tag;
        b.sample = sample;
        b.cs = lv.L.nstore;
        b.chain0 = (uint32_t)h->chain;
        b.seed_hi = (uint32_t)(h->seed >> 32);
        const dim3 grid(1, 1, nch), block((unsigned)std::min(1024, h->chol_B));
        const size_t lds = 2 * (size_t)h->chol_B * sizeof(double);
        if (lv.spec.dim == 3)
            hipLaunchKernelGGL(k_coarse_chol_blocked<3>, grid, block, lds, s, b);
        else
            hipLaunchKernelGGL(k_coarse_chol_blocked<2>, grid, block, lds, s, b);
        return;
    }
    CholArgs a;
    a.L = lv.L;
    a.n = h->chol_n;
    a.G = h->chol_G;
    a.Li = h->chol_Li;
    a.f = f;
    a.x = x;
    a.noise = noise ? 1 : 0;
    a.key = h->key;
    a.tag = tag;
    a.sample = sample;
    a.cs = lv.L.nstore;
    a.chain0 = (uint32_t)h->chain;
    a.seed_hi = (uint32_t)(h->seed >> 32);
    const dim3 grid((unsigned)((a.n + 255) / 256), 1, nch), block(256);
    const size_t lds = 2 * (size_t)a.n * sizeof(double);
    if (lv.spec.dim == 3)
        hipLaunchKernelGGL(k_coarse_chol<3>, grid, block, lds, s, a);
    else
        hipLaunchKernelGGL(k_coarse_chol<2>, grid, block, lds, s, a);
}

// ---- the op sequence of one sample (multigridmc_sampler.cc:103-138) ----
// cur[l] tracks which buffer holds x_l while the ops are generated (z-sweeps ping-pong).
void push_sweep(mgmc_handle* h, std::vector<int>& cur, int level, int direction, uint32_t& tag, int& pending_prolong) {
    Op op{OP_SWEEP, level, direction, tag++, 1};
    const Level& lv = h->levels[level];
    // fused prolongation on z-sweep levels (the 2D red-black kernel does not fold it: its staging
    // becomes a longer latency chain, 2D 1024^2 cycle 0.1292-0.1305 -> 0.1306-0.1316 ms against the
    // separate k_prolongate_pairs launch, measured in round 1)
    const bool fold = lv.zsweep && !(h->paths & PATH_NO_FUSE_PROLONG);
    if (lv.pingpong() && pending_prolong && !fold) {
        h->ops.push_back({OP_PROLONGATE, level, 0, 0, 0});
        h->ops.back().src = cur[level];
        pending_prolong = 0;
    }
    if (lv.pingpong()) {
        op.src = cur[level];
        op.prolong = pending_prolong;
        pending_prolong = 0;
        cur[level] = 1 - cur[level];
    } else if (pending_prolong) {
        h->ops.push_back({OP_PROLONGATE, level, 0, 0, 0});
        h->ops.back().src = cur[level];
        pending_prolong = 0;
    }
    h->ops.push_back(op);
}

void build_ops_level(mgmc_handle* h, int level, uint32_t& tag, std::vector<int>& cur) {
    const mgmc_config& c = h->cfg;
    const int nlevel = (int)h->levels.size();
    int none = 0;
    if (level == nlevel - 1) {
        // coarse sampler: SSORSampler(ncoarsesmooth) = ncoarsesmooth x (fwd SOR sampler, bwd SOR sampler)
        const Level& lv = h->levels[level];
        if (c.coarse_solver == MGMC_COARSE_CHOLESKY) {  // CholeskySampler (cholesky_sampler.hh:50-66)
            h->ops.push_back({OP_COARSE_CHOL, level, 0, tag++, 1});
        } else if (lv.lds_bytes > 0 && lv.lr.m == 0) {
            h->ops.push_back({OP_COARSE_LDS, level, MGMC_FORWARD, tag, 2 * c.ncoarsesmooth});
            tag += 2 * c.ncoarsesmooth;
        } else {
            for (int t = 0; t < c.ncoarsesmooth; ++t) {
                push_sweep(h, cur, level, MGMC_FORWARD, tag, none);
                push_sweep(h, cur, level, MGMC_BACKWARD, tag, none);
            }
        }
        return;
    }
    const int cycle_ = (level > 0) ? c.cycle : 1;
    for (int jc = 0; jc < cycle_; ++jc) {
        // presampler
        for (int t = 0; t < c.npresmooth; ++t) {
            push_sweep(h, cur, level, MGMC_FORWARD, tag, none);
            if (c.smoother == MGMC_SMOOTHER_SSOR) push_sweep(h, cur, level, MGMC_BACKWARD, tag, none);
        }
        if (level == 0) h->seg_end_pre = h->ops.size();
        Op rr{OP_RESIDUAL_RESTRICT, level, 0, 0, 0};
        rr.src = cur[level];
        h->ops.push_back(rr);
        cur[level + 1] = 0;  // residual_restrict zeroes x_{l+1} (buffer 0)
        build_ops_level(h, level + 1, tag, cur);
        if (cur[level + 1] != 0) {  // bring x_{l+1} back to its canonical buffer
            Op cp{OP_COPY, level + 1, 0, 0, 0};
            cp.src = cur[level + 1];
            h->ops.push_back(cp);
            cur[level + 1] = 0;
        }
        int pending_prolong = 1;
        if (level == 0) h->seg_begin_post = h->ops.size();
        for (int t = 0; t < c.npostsmooth; ++t) {
            if (c.smoother == MGMC_SMOOTHER_SOR) {
                push_sweep(h, cur, level, MGMC_BACKWARD, tag, pending_prolong);
            } else {
                push_sweep(h, cur, level, MGMC_FORWARD, tag, pending_prolong);
                push_sweep(h, cur, level, MGMC_BACKWARD, tag, pending_prolong);
            }
        }
        if (pending_prolong) {  // npostsmooth == 0
            h->ops.push_back({OP_PROLONGATE, level, 0, 0, 0});
            h->ops.back().src = cur[level];
        }
        if (level == 0) {
            h->seg_end_post = h->ops.size();
            // the timed fine segment starts at the first fine sweep: an unfused fine prolongation
            // stays in the coarse-correction segment, so fine_ms times Gibbs sweeps only
            while (h->seg_begin_post < h->seg_end_post &&
                   !(h->ops[h->seg_begin_post].kind == OP_SWEEP && h->ops[h->seg_begin_post].level == 0))
                ++h->seg_begin_post;
        }
    }
}

void build_ops(mgmc_handle* h) {
    h->ops.clear();
    h->seg_end_pre = h->seg_begin_post = h->seg_end_post = 0;
    uint32_t tag = 0;
    std::vector<int> cur(h->levels.size(), 0);
    build_ops_level(h, 0, tag, cur);
    if (cur[0] != 0) {
        Op cp{OP_COPY, 0, 0, 0, 0};
        cp.src = cur[0];
        h->ops.push_back(cp);
        h->seg_end_post = h->ops.size();
    }
    h->ops.push_back({OP_QOI, 0, 0, 0, 0});
    if (h->levels.size() == 1) h->seg_end_pre = h->seg_begin_post = h->seg_end_post = 0;
    // small low-rank levels: the kernel after a sweep also patches f for the level's next op
    for (size_t q = 0; q + 1 < h->ops.size(); ++q) {
        Op& op = h->ops[q];
        Op& nx = h->ops[q + 1];
        if (op.kind != OP_SWEEP || !h->levels[op.level].lr.small || nx.level != op.level) continue;
        if (nx.kind == OP_SWEEP) {
            op.lr_next = LR_NEXT_NOISE;
            op.lr_next_tag = nx.tag;
            nx.lr_skip_patch = 1;
        } else if (nx.kind == OP_RESIDUAL_RESTRICT) {
            op.lr_next = LR_NEXT_RESIDUAL;
            nx.lr_skip_patch = 1;
        }
    }
    // low-rank levels: the restore after a residual + restriction also patches f for the level's
    // first post-sweep (nothing writes f in between: the ops of coarser levels and this level's
    // prolongation touch only coarser f and this level's x) and for the coarse level's first
    // pre-sweep -- one launch instead of three
    if (!(h->paths & PATH_NO_LR_MERGE))
        for (size_t q = 0; q < h->ops.size(); ++q) {
            Op& op = h->ops[q];
            const int l = op.level;
            // (dense-column levels: f is never patched or restored; the residual's launch writes the
            // first post-sweep's right-hand side to lr.fe2, and the coarse patch stays separate)
            if (op.kind != OP_RESIDUAL_RESTRICT || h->levels[l].lr.m == 0) continue;
            if (q + 1 < h->ops.size() && !h->levels[l].lr.dense_path) {
                Op& nx = h->ops[q + 1];
                if (nx.kind == OP_SWEEP && nx.level == l + 1 && h->levels[l + 1].lr.m > 0 &&
                    !h->levels[l + 1].lr.dense_path && !nx.lr_skip_patch) {
                    op.lr_coarse_patch = 1;
                    op.lr_coarse_tag = nx.tag;
                    nx.lr_skip_patch = 1;
                }
            }
            for (size_t r = q + 1; r < h->ops.size(); ++r) {
                Op& o = h->ops[r];
                if (o.level > l || (o.kind == OP_PROLONGATE && o.level == l)) continue;
                if (o.kind == OP_SWEEP && o.level == l && !o.lr_skip_patch) {
                    op.lr_post_patch = 1;
                    op.lr_post_tag = o.tag;
                    o.lr_skip_patch = 1;
                }
                break;
            }
        }
}

// ---- the coarsest levels' sub-cycle in one workgroup (k_tail) ----
constexpr size_t TAIL_LDS_LIMIT = 150 * 1024;
// one 1024-thread workgroup (1024 / 512 / 256 threads: 256^3 cycle 0.529 / 0.538 / 0.570 ms, round 1)
constexpr int TAIL_NT = 1024;

// 3D plane stride padded to sp = 8 (mod 16) doubles: k_tail's colour passes give the two halves of a
// half-wave the planes k and k+2, whose ds_read_b64 bank pairs (d mod 32) then sit 16 apart, so the
// stride-2 class access is 2-way (the least a stride-2 access allows) instead of 4-way with sx odd
// and unpadded planes (MI355X_MICROARCH.md LDS banking)
long long tail_plane_stride(int nx, int ny) {
    const long long sp = (long long)(nx + 1) * (ny + 1);
    return sp + ((8 - sp % 16) + 16) % 16;
}

Layout tail_layout(const Layout& L) {
    Layout G = L;
    G.off = 0;
    G.sx = L.nx + 1;
    G.sp = L.dim == 3 ? tail_plane_stride(L.nx, L.ny) : G.sx * (L.ny + 1);
    G.nstore = L.dim == 3 ? G.sp * (L.nz + 1) : G.sp;
    return G;
}

// the same choice from the level shapes alone (at creation time, before any level is allocated)
int tail_start_by_size(const std::vector<LevelSpec>& specs, const mgmc_config& cfg, uint32_t paths, bool field) {
    if ((paths & PATH_NO_TAIL) || field || cfg.coarse_solver != MGMC_COARSE_SSOR) return -1;
    const int L = (int)specs.size();
    for (int lt = 1; lt + 1 < L; ++lt) {
        bool ok = true;
        size_t tot = 0, vmax = 0;
        for (int l = lt; l < L && ok; ++l) {
            const LevelSpec& sp = specs[l];
            ok = sp.npoints == (sp.dim == 3 ? 27 : 9);
            const size_t v = sp.dim == 3 ? (size_t)tail_plane_stride(sp.n[0], sp.n[1]) * (sp.n[2] + 1)
                                         : (size_t)(sp.n[0] + 1) * (sp.n[1] + 1);
            tot += 2 * v;
            vmax = std::max(vmax, v);
        }
        if (ok && (tot + vmax) * sizeof(double) <= TAIL_LDS_LIMIT) return lt;
    }
    return -1;
}

// smallest level lt >= 1 whose levels lt .. L-1 all fit one workgroup's LDS (x, f per level + one
// scratch of the largest + saved f on the rows of B): Galerkin levels, no low-rank part or a small
// one (k_lr_small's), ordinary (in-place) sweeps, SSOR coarse sampler; -1 if none or only the
// coarsest level fits (the coarse LDS kernel covers that)
int tail_level(const mgmc_handle* h) {
    if ((h->paths & PATH_NO_TAIL) || h->field_mode || h->cfg.coarse_solver != MGMC_COARSE_SSOR) return -1;
    const int L = (int)h->levels.size();
    for (int lt = 1; lt + 1 < L; ++lt) {
        bool ok = true;
        size_t tot = 0, vmax = 0;
        for (int l = lt; l < L && ok; ++l) {
            const Level& lv = h->levels[l];
            ok = (lv.lr.m == 0 || lv.lr.small) && !lv.pingpong() && lv.spec.npoints == (lv.spec.dim == 3 ? 27 : 9);
            const size_t v = (size_t)tail_layout(lv.L).nstore;
            tot += 2 * v + (size_t)lv.lr.nrows;
            vmax = std::max(vmax, v);
        }
        if (ok && (tot + vmax) * sizeof(double) <= TAIL_LDS_LIMIT) return lt;
    }
    return -1;
}

void free_tails(mgmc_handle* h) {
    for (auto p : h->tail_args)
        if (p) hipFree(p);
    for (auto p : h->tail_zb)
        if (p) hipFree(p);
    for (auto p : h->tail_jobs)
        if (p) hipFree(p);
    for (auto p : h->pn_bufs)
        if (p) hipFree(p);
    h->pn_bufs.clear();
    h->tail_pn_wg.clear();
    h->tail_args.clear();
    h->tail_lds.clear();
    h->tail_sym.clear();
    h->tail_zb.clear();
    h->tail_jobs.clear();
    h->tail_njobs.clear();
    h->tail_zn.clear();
}

// the residual + restriction from level lf onto lf + 1 runs as the small z-marching kernel
// (k_zresrestrict<., 16, 4, 64>): launch_residual_restrict's choice for zero_xc = 1
bool zr_small_path(const mgmc_handle* h, int lf) {
    const Level& f = h->levels[lf];
    const Level& c = h->levels[lf + 1];
    return f.spec.dim == 3 && !f.field && !(f.paths & PATH_NO_ZRESTRICT) && c.L.nx >= 8 && c.L.nx < 32;
}

// replace every maximal run of ops on levels >= lt (one call of build_ops_level(lt)) by one OP_TAIL
int build_tails_only(mgmc_handle* h) {
    free_tails(h);
    const int lt = tail_level(h);
    if (lt < 0) return MGMC_OK;
    const int L = (int)h->levels.size();
    std::vector<Op> out;
    size_t removed_before_pre = 0;
    const size_t pre_end = h->seg_end_pre;
    for (size_t q = 0; q < h->ops.size();) {
        if (h->ops[q].level < lt || h->ops[q].kind == OP_QOI) {
            out.push_back(h->ops[q++]);
            continue;
        }
        TailArgs A;
        memset(&A, 0, sizeof(A));
        size_t r = q;
        bool ok = true;
        for (; r < h->ops.size() && h->ops[r].level >= lt && h->ops[r].kind != OP_QOI; ++r) {
            const Op& op = h->ops[r];
            if (A.nops >= TAIL_MAX_OPS) { ok = false; break; }
            TailOp& t = A.ops[A.nops++];
            t.level = op.level - lt;
            t.dir = op.direction;
            t.tag = op.tag;
            t.nsweeps = op.nsweeps;
            switch (op.kind) {
                case OP_SWEEP: t.kind = TAIL_SWEEP; break;
                case OP_RESIDUAL_RESTRICT: t.kind = TAIL_RESTRICT; break;
                case OP_PROLONGATE: t.kind = TAIL_PROLONG; break;
                case OP_COARSE_LDS: t.kind = TAIL_COARSE; break;
                default: ok = false;
            }
        }
        if (!ok) {  // leave the ops as they are
            for (size_t u = q; u < r; ++u) out.push_back(h->ops[u]);
            q = r;
            continue;
        }
        A.nlev = L - lt;
        int off = 0;
        for (int l = lt; l < L; ++l) {
            TailLevel& tl = A.lv[l - lt];
            const Level& lv = h->levels[l];
            tl.G = tail_layout(lv.L);
            tl.ox = off;
            off += (int)tl.G.nstore;
            tl.of = off;
            off += (int)tl.G.nstore;
            tl.ncolours = lv.spec.ncolours;
            tl.fold = lv.fold ? 1 : 0;
            const GibbsArg g = make_gibbs(h, lv, 0, 0, h->ctrl);
            tl.sd = g.sd;
            tl.wd = g.wd;
            tl.S = lv.S;
            const LowRankDev& r = lv.lr;
            tl.m = r.m;
            if (r.m > 0) {
                tl.nrows = r.nrows;
                tl.meta = r.meta;
                tl.ent_off = r.t_ent_off;
                tl.ent_val = r.ent_val;
                tl.sc_one = r.sc_one;
                tl.sc_inv = r.sc_inv;
                tl.sq = r.sq;
                for (int d = 0; d < 2; ++d) {
                    tl.nbar[d] = r.nbar[d];
                    tl.bar_off[d] = r.t_bar_off[d];
                    tl.bar_val[d] = r.bar_val[d];
                }
                tl.rows_off = r.t_rows_off;
                tl.coef = r.rows_coef;
                tl.mask = r.rows_mask;
            }
        }
        int vmax = 0;
        for (int l = 0; l < A.nlev; ++l) vmax = std::max(vmax, (int)A.lv[l].G.nstore);
        A.oscr = off;
        off += vmax;
        for (int l = 0; l < A.nlev; ++l) {
            A.lv[l].osave = off;
            off += A.lv[l].m > 0 ? A.lv[l].nrows : 0;
        }
        A.lds_doubles = off;
        // the tail patches level lt's f itself: the restriction before it must not
        if (!out.empty() && out.back().kind == OP_RESIDUAL_RESTRICT) out.back().lr_coarse_patch = 0;
        // x_lt was just zeroed by that restriction (multigridmc_sampler.cc:122): not loaded
        A.x_zero = (lt > 0 && !out.empty() && out.back().kind == OP_RESIDUAL_RESTRICT && out.back().level == lt - 1 &&
                    !(h->paths & PATH_NO_XZERO)) ? 1 : 0;
        A.alpha = h->cfg.coarse_scaling;
        A.key = h->key;
        A.sample = h->ctrl;
        A.xg = h->levels[lt].x;
        A.fg = h->levels[lt].f;
        A.Lg = h->levels[lt].L;
        A.cs = h->levels[lt].L.nstore;  // batched chains: one workgroup per chain
        A.chain0 = (uint32_t)h->chain;
        A.seed_hi = (uint32_t)(h->seed >> 32);
        A.npn = 0;  // (post-sweep noise jobs: plan_drawn_noise)
#ifdef MGMC_TAIL_PROF
        if (h->tail_args.empty()) {
            if (!h->tail_prof) HIPCHK(h, hipMalloc(&h->tail_prof, 256 * sizeof(unsigned long long)));
            A.prof = h->tail_prof;
            h->tail_prof_ops.assign(A.ops, A.ops + A.nops);
        }
#endif
        // the sweeps' Box-Muller pairs: drawn by spare workgroups of the restriction before the tail when
        // that is the small z-marching kernel (3D; k_zresrestrict<..., ZN>), else here
        std::vector<TailNoiseJob> jobs;
        long long zn = 0;
        const bool pre_zr = !out.empty() && out.back().kind == OP_RESIDUAL_RESTRICT && out.back().level == lt - 1 &&
                            zr_small_path(h, lt - 1) && h->levels[lt - 1].lr.m == 0;
        for (int o = 0; o < A.nops; ++o) {
            TailOp& t = A.ops[o];
            t.zoff = -1;
            if (t.kind != TAIL_SWEEP && t.kind != TAIL_COARSE) continue;
            const Layout& G = A.lv[t.level].G;
            const long long items = (long long)(G.nx / 2) * (G.ny - 1) * (G.dim == 3 ? G.nz - 1 : 1);
            const int ns = t.kind == TAIL_SWEEP ? 1 : t.nsweeps;
            t.zoff = (int)zn;
            for (int sw = 0; sw < ns; ++sw) {
                jobs.push_back(TailNoiseJob{G.nx, G.ny, G.nz, t.tag + (uint32_t)sw, (int)zn});
                zn += items;
            }
        }
        double2* zb = nullptr;
        TailNoiseJob* dj = nullptr;
        if (pre_zr && !jobs.empty() && (int)jobs.size() <= TAIL_MAX_NOISE_JOBS && zn < (1LL << 30)) {
            std::vector<long long> zo, zi;  // the restriction's writes / the tail's reads stay in the buffer
            for (const TailNoiseJob& J : jobs) {
                zo.push_back(J.zoff);
                zi.push_back((long long)(J.nx / 2) * (J.ny - 1) * (J.nz - 1));
            }
            const std::string e = tail_noise_check(zo, zi, zn);
            if (!e.empty()) return fail(h, MGMC_E_INVALID, "internal layout check failed: " + e);
            HIPCHK(h, hipMalloc(&zb, (size_t)h->nchains * zn * sizeof(double2)));
            poison_fill(h, zb, (size_t)h->nchains * zn * sizeof(double2));
            HIPCHK(h, hipMalloc(&dj, jobs.size() * sizeof(TailNoiseJob)));
            HIPCHK(h, hipMemcpy(dj, jobs.data(), jobs.size() * sizeof(TailNoiseJob), hipMemcpyHostToDevice));
            A.zb = zb;
            A.zbs = zn;
            out.back().zpre = (int)h->tail_args.size() + 1;  // the restriction draws for tail #(zpre - 1)
        }
        h->tail_zb.push_back(zb);
        h->tail_jobs.push_back(dj);
        h->tail_njobs.push_back(zb ? (int)jobs.size() : 0);
        h->tail_zn.push_back(zb ? zn : 0);
        h->tail_pn_wg.push_back(0);
        TailArgs* d = nullptr;
        HIPCHK(h, hipMalloc(&d, sizeof(TailArgs)));
        HIPCHK(h, hipMemcpy(d, &A, sizeof(TailArgs), hipMemcpyHostToDevice));
        Op t{OP_TAIL, lt, 0, 0, 0};
        t.tail = (int)h->tail_args.size();
        h->tail_args.push_back(d);
        h->tail_lds.push_back((size_t)A.lds_doubles * sizeof(double));
        bool tsym = true;
        for (int l = lt; l < lt + A.nlev; ++l) tsym = tsym && h->levels[l].sym;
        h->tail_sym.push_back(tsym ? 1 : 0);
        out.push_back(t);
        if (r <= pre_end) removed_before_pre += r - q - 1;
        q = r;
    }
    const size_t removed = h->ops.size() - out.size();
    h->ops.swap(out);
    h->seg_end_pre -= removed_before_pre;
    h->seg_begin_post = h->seg_begin_post >= removed ? h->seg_begin_post - removed : 0;
    h->seg_end_post = h->seg_end_post >= removed ? h->seg_end_post - removed : 0;
    return MGMC_OK;
}

// a level whose last pre-sweep and residual + restriction can run as one k_quads_restrict2d launch:
// 2D 9-point Galerkin level swept by quad passes (out of place), no low-rank part, not the coarsest,
// rows of at most 256 pairs (one pair item per thread of a 1024-thread workgroup)
bool qrestrict_ok(const mgmc_handle* h, int level) {
    if (h->paths & PATH_NO_QRESTRICT) return false;
    if (level < 1 || level + 1 >= (int)h->levels.size()) return false;
    const Level& lv = h->levels[level];
    if (lv.spec.dim != 2 || lv.spec.npoints != 9 || !lv.quads || lv.jsweep || lv.field || lv.lr.m > 0 ||
        !lv.pingpong())
        return false;
    if (qrestrict_threads(lv.L.nx / 2) == 0) return false;
    const int CJ = qrestrict_threads(lv.L.nx / 2) / (lv.L.nx / 2) - 3;
    return qrestrict_lds_bytes(lv.L.nx, CJ) <= 150 * 1024;
}

// fuse every (sweep, residual + restriction) pair of ops on a qrestrict_ok level into one
// OP_SWEEP_RESTRICT (the restriction reads the buffer the sweep writes).  The fine level (level 0)
// keeps its ops, so the timed fine-sweep segments are unchanged.  (Measured and not kept, DESIGN.md
// section 3: the same fusion around the 2D fine level's k_rb2d, and the mirror image on the way up --
// prolongate-add + first post-sweep in one launch -- both bitwise, neither faster.)
void fuse_sweep_restrict(mgmc_handle* h) {
    std::vector<Op> out;
    std::vector<size_t> removed;  // original indices of the dropped restriction ops
    for (size_t q = 0; q < h->ops.size(); ++q) {
        const Op& op = h->ops[q];
        if (op.kind == OP_SWEEP && q + 1 < h->ops.size() && qrestrict_ok(h, op.level) && !op.prolong) {
            const Op& nx = h->ops[q + 1];
            if (nx.kind == OP_RESIDUAL_RESTRICT && nx.level == op.level && nx.src == 1 - op.src) {
                Op f = op;
                f.kind = OP_SWEEP_RESTRICT;
                out.push_back(f);
                removed.push_back(q + 1);
                ++q;
                continue;
            }
        }
        out.push_back(op);
    }
    auto shift = [&](size_t& seg) {
        size_t d = 0;
        for (size_t r : removed)
            if (r < seg) ++d;
        seg -= d;
    };
    shift(h->seg_end_pre);
    shift(h->seg_begin_post);
    shift(h->seg_end_post);
    h->ops.swap(out);
    // a fused restriction onto the coarsest level draws the coarse SSOR sampler's noise in spare
    // workgroups (QRestrictArgs::zc): the sampler's one workgroup then only reads it (4.5 of its ~19 us
    // were the draws at 2D 1024^2).  The pairs are adjacent ops, so one buffer serves every visit
    if (h->zbuf) hipFree(h->zbuf);
    h->zbuf = nullptr;
    h->zbuf_n = 0;
    for (size_t q = 0; q + 1 < h->ops.size(); ++q) {
        Op& op = h->ops[q];
        Op& co = h->ops[q + 1];
        if (op.kind != OP_SWEEP_RESTRICT || co.kind != OP_COARSE_LDS || co.level != op.level + 1 ||
            co.level + 1 != (int)h->levels.size() || !coarse_precompute(h->levels[co.level], co.nsweeps))
            continue;
        const Level& lc = h->levels[co.level];
        const long long n = (long long)co.nsweeps * (lc.L.ny - 1) * (lc.L.nx / 2);
        if (!h->zbuf) {
            if (hipMalloc(&h->zbuf, (size_t)h->nchains * n * sizeof(double2)) != hipSuccess) return;  // (draws stay in place)
            poison_fill(h, h->zbuf, (size_t)h->nchains * n * sizeof(double2));
            h->zbuf_n = n;
        }
        if (n != h->zbuf_n) continue;
        op.zpre = 1;
        co.zpre = 1;
    }
}

// A coarse level's first pre-sweep starts from x_{l+1} = 0 (multigridmc_sampler.cc:122, x_ell.setZero()
// before the recursive call).  Where that sweep is a j-marching level's out-of-place half-sweep pair and
// the restriction before it is the z-marching kernel, the sweep takes the zeros as constants instead of
// loading them (512^3 level 1: the first half moves 2 of its 4 streams, the second 3), and the
// restriction does not write them (142 MB of the fine residual + restriction's stores).  Nothing else
// reads that buffer before it is written whole: the sweep writes the other one, and the next sweep out
// of it (the post-sweep) overwrites every interior vertex; a copy back (OP_COPY) writes it whole too.
// Only the op right after the restriction is marked (W-cycles: the later visits start from the level's
// own result, not from zero).  Same values: the restriction's zero is +0.0, so is the constant.
void mark_zero_inputs(mgmc_handle* h) {
    for (Op& op : h->ops) op.xzero = 0;
    if (h->paths & PATH_NO_XZERO) return;
    for (size_t q = 0; q + 1 < h->ops.size(); ++q) {
        Op& rr = h->ops[q];
        Op& sw = h->ops[q + 1];
        if (rr.kind != OP_RESIDUAL_RESTRICT || sw.kind != OP_SWEEP || sw.level != rr.level + 1 || sw.src != 0 ||
            rr.zpre != 0)
            continue;
        const Level& lf = h->levels[rr.level];
        const Level& lc = h->levels[sw.level];
        const bool zr = lf.spec.dim == 3 && !lf.field && !(lf.paths & PATH_NO_ZRESTRICT) && lc.L.nx >= 8;
        // j-marching levels and 3D quad-pass levels: out of place, x read only as the half-sweeps' input
        const bool quads3 = lc.quads && lc.spec.dim == 3;
        // (low-rank levels too: the patches before a sweep change f only, the fix after it reads the
        // sweep's output, and the residual's dots read the fine level's x)
        if (!zr || !(lc.jsweep || quads3) || lc.field) continue;
        rr.xzero = 1;
        sw.xzero = 1;
    }
}

// A tail launch runs one workgroup on one CU (512^3: 40-43 us); the rest of the chip is idle meanwhile.
// Its spare workgroups draw the Box-Muller pairs of the sweeps that follow it instead: for every 3D
// Galerkin level swept by quad passes (not a field level; with or without a low-rank part), the first sweep on that
// level after the tail and before the next tail (in a V-cycle its post-sweep) whose input x is not known
// zero.  The pairs are those the sweep would draw (same Philox counter: pair id, the sweep's tag, the
// sample index at run time; same arithmetic), so the chain is bitwise unchanged.  512^3 (round 6): the
// 127^3 post quad passes 16.5 -> 13.9 us each, the tail launch +0.8 us with tune::TAIL_PN_WG = 32 spare
// workgroups (+4 us with one per CU).  Not the j-marching levels: their post half-sweeps,
// reading the pairs (16 B per pair) instead of drawing them, stayed at 72 us, and the 8.3 M pairs of
// the 255^3 level took the tail launch from 43 to 60 us.  One chain per handle (batched handles' tails
// run one workgroup per chain; their draws stay in the sweeps), and at most PN_MAX_PAIRS pairs per
// tail, well inside what the spare workgroups draw within the tail's own time.
constexpr long long PN_MAX_PAIRS = 2LL << 20;

//
// The same for the first pre-sweep of a 3D quad-pass level after a 27-point z-marching residual +
// restriction (zres_draws_noise): every workgroup of that launch draws its share of the coarse level's
// pairs after its own march (ZRestrictArgs::pn; the sweep then loads them, with xzero its known-zero
// x too).  One buffer per level serves both: the pre-sweep reads it before the tail rewrites it.
int plan_drawn_noise(mgmc_handle* h) {
    for (Op& op : h->ops) {
        op.pnz = nullptr;
        op.pn_dst = nullptr;
        op.pn_tag = 0;
    }
    if ((h->paths & PATH_NO_POST_NOISE) || h->nchains != 1) return MGMC_OK;
    std::vector<double2*> buf(h->levels.size(), nullptr);
    auto level_buf = [&](int l) -> double2* {
        if (!buf[l]) {
            const Level& lv = h->levels[l];
            const long long n = (long long)(lv.L.nx / 2) * (lv.L.ny - 1) * (lv.L.nz - 1);
            if (hipMalloc(&buf[l], (size_t)n * sizeof(double2)) != hipSuccess) {
                buf[l] = nullptr;
                (void)hipGetLastError();
                return nullptr;
            }
            poison_fill(h, buf[l], (size_t)n * sizeof(double2));
            h->pn_bufs.push_back(buf[l]);
        }
        return buf[l];
    };
    auto quad_consumer = [&](const Level& lv) {
        return lv.spec.dim == 3 && !lv.field && lv.quads && !lv.jsweep && lv.pingpong();
    };
    for (size_t q = 0; q + 1 < h->ops.size(); ++q) {  // pre-sweeps: drawn by the restriction before them
        Op& rr = h->ops[q];
        Op& sw = h->ops[q + 1];
        if (rr.kind != OP_RESIDUAL_RESTRICT || rr.zpre != 0 || sw.kind != OP_SWEEP || sw.level != rr.level + 1) continue;
        const Level& lf = h->levels[rr.level];
        const Level& lc = h->levels[sw.level];
        if (!zres_draws_noise(lf, lc) || !quad_consumer(lc) || (sw.xzero && sw.direction != MGMC_FORWARD)) continue;
        double2* b = level_buf(sw.level);
        if (!b) continue;
        rr.pn_dst = b;
        rr.pn_tag = sw.tag;
        sw.pnz = b;
    }
    for (size_t t = 0; t < h->ops.size(); ++t) {
        if (h->ops[t].kind != OP_TAIL) continue;
        const int ti = h->ops[t].tail;
        std::vector<PostNoiseJob> jobs;
        std::vector<char> used(h->levels.size(), 0);
        long long total = 0;
        for (size_t q = t + 1; q < h->ops.size() && h->ops[q].kind != OP_TAIL; ++q) {
            Op& op = h->ops[q];
            // (W-cycles: a restriction in the window that rewrites a level's buffer ends the tail's use of it)
            if (op.kind == OP_RESIDUAL_RESTRICT && op.pn_dst) used[op.level + 1] = 1;
            if (op.kind != OP_SWEEP || op.xzero || op.level < 1 || used[op.level]) continue;
            const Level& lv = h->levels[op.level];
            // (a low-rank level's sweep draws the same pairs: its patch of f and its fix are separate ops)
            if (!quad_consumer(lv) || op.pnz) continue;
            used[op.level] = 1;
            const long long n = (long long)(lv.L.nx / 2) * (lv.L.ny - 1) * (lv.L.nz - 1);
            if (total + n > PN_MAX_PAIRS || (int)jobs.size() >= TAIL_MAX_PN_JOBS) continue;
            double2* b = level_buf(op.level);
            if (!b) continue;  // (this sweep draws its own)
            total += n;
            jobs.push_back(PostNoiseJob{lv.L.nx, lv.L.ny, lv.L.nz, op.tag, b});
            op.pnz = b;
        }
        // (the spare workgroups keep the Box-Muller tables in the launch's LDS: 322 doubles)
        if (jobs.empty() || h->tail_lds[ti] < 322 * sizeof(double)) {
            for (size_t u = t + 1; u < h->ops.size() && h->ops[u].kind != OP_TAIL; ++u)
                if (h->ops[u].kind == OP_SWEEP && !(u > 0 && h->ops[u - 1].kind == OP_RESIDUAL_RESTRICT &&
                                                    h->ops[u - 1].pn_dst == h->ops[u].pnz))
                    h->ops[u].pnz = nullptr;  // (no jobs: the window's sweeps draw their own)
            continue;
        }
        TailArgs* d = h->tail_args[ti];
        const int npn = (int)jobs.size();
        HIPCHK(h, hipMemcpy(d->pn, jobs.data(), jobs.size() * sizeof(PostNoiseJob), hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(&d->npn, &npn, sizeof(int), hipMemcpyHostToDevice));
        // one workgroup per other CU (the tail's LDS admits one per CU), or tune::TAIL_PN_WG
        h->tail_pn_wg[ti] = tune::TAIL_PN_WG > 0 ? tune::TAIL_PN_WG : std::max(1, h->levels[0].num_cu - h->nchains);
    }
    return MGMC_OK;
}

int build_tails(mgmc_handle* h) {
    int rc = build_tails_only(h);
    if (rc == MGMC_OK) fuse_sweep_restrict(h);
    if (rc == MGMC_OK) mark_zero_inputs(h);
    if (rc == MGMC_OK) rc = plan_drawn_noise(h);
    return rc;
}

void enqueue_ops(mgmc_handle* h, size_t begin, size_t end, hipStream_t s) {
    const uint64_t* sample = h->ctrl;  // ctrl[0]
    const int nch = h->nchains;        // batched chains: every launch covers all of them
    for (size_t q = begin; q < end; ++q) {
        const Op& op = h->ops[q];
        Level& lv = h->levels[op.level];
        if (h->poison)  // (debug: poison_fill) the op's kernels start on NaN-filled LDS
            hipLaunchKernelGGL(k_lds_poison, dim3(8 * lv.num_cu), dim3(1024), LDS_POISON_DOUBLES * sizeof(double), s);
        switch (op.kind) {
            case OP_SWEEP: {
                GibbsArg g = make_gibbs(h, lv, op.tag, 0, sample);
                const bool lr = lv.lr.m > 0;
                double* fs = lv.f;  // the right-hand side the sweep reads
                // (rhs_inplace: f itself, patched by the sweep kernel as lrr says)
                LRRhsArg lrr{nullptr};
                const bool inplace = lr && lv.lr.rhs_inplace;  // (a z-sweep level)
                if (lr && !op.lr_skip_patch)
                    fs = lr_rhs(h, lv, LR_PATCH_NOISE, lv.f, op.tag, sample, s, nch, -1, inplace ? &lrr : nullptr);
                else if (inplace)  // patched (local rows, e) after the level's residual: lr_restore_patch
                    lrr = LRRhsArg{lv.lr.rhs_e + nch};
                else if (lr && lv.lr.dense_path)
                    fs = lv.lr.fe2;  // written with the level's residual
                double* xo = lv.x;
                if (lv.zsweep) {
                    const Level* lc = op.prolong ? &h->levels[op.level + 1] : nullptr;
                    xo = lv.buf(1 - op.src);
                    launch_zsweep(lv, lv.buf(op.src), xo, fs, g, op.direction, lc, lc ? lc->x : nullptr,
                                  h->cfg.coarse_scaling, s, nch, lrr.e ? &lrr : nullptr);
                } else if (lv.quads) {
                    xo = lv.buf(1 - op.src);
                    launch_quads(lv, lv.buf(op.src), xo, fs, g, op.direction, s, nch, op.xzero != 0, op.pnz);
                } else if (lv.rb2d) {
                    xo = lv.buf(1 - op.src);
                    launch_rb2d(lv, lv.buf(op.src), xo, fs, g, op.direction, true, s, nch);
                } else if (lv.pairs) {
                    launch_pairs(lv, lv.x, fs, g, op.direction, s, nch);
                } else {
                    launch_sweep(lv, lv.x, fs, g, op.direction, true, s, nch);
                }
                if (lr && lv.lr.small)
                    lr_small(h, lv, xo, op.direction, op.lr_next, op.lr_next_tag, sample, s, nch);
                else if (lr)
                    lr_fix(lv, xo, op.direction, lv.lr.dense_path && !inplace ? nullptr : lv.f, s, nch);
                break;
            }
            case OP_SWEEP_RESTRICT: {  // (2D Galerkin level, no low-rank part: qrestrict_ok)
                GibbsArg g = make_gibbs(h, lv, op.tag, 0, sample);
                Level& lc = h->levels[op.level + 1];
                if (op.zpre) {  // + the next op's (the coarse sampler's) noise
                    const Op& co = h->ops[q + 1];
                    launch_qrestrict(lv, lc, lv.buf(op.src), lv.buf(1 - op.src), lv.f, lc.f, lc.x, g, op.direction, s,
                                     nch, h->zbuf, co.nsweeps, co.tag, h->zbuf_n);
                } else {
                    launch_qrestrict(lv, lc, lv.buf(op.src), lv.buf(1 - op.src), lv.f, lc.f, lc.x, g, op.direction, s,
                                     nch);
                }
                break;
            }
            case OP_COARSE_CHOL: {
                launch_coarse_chol(h, lv, lv.f, lv.x, true, op.tag, sample, s, nch);
                break;
            }
            case OP_COARSE_LDS: {
                GibbsArg g = make_gibbs(h, lv, op.tag, 0, sample);
                if (op.zpre) launch_coarse_lds(lv, g, op.nsweeps, s, nch, h->zbuf, h->zbuf_n);
                else launch_coarse_lds(lv, g, op.nsweeps, s, nch);
                break;
            }
            case OP_RESIDUAL_RESTRICT: {
                Level& lc = h->levels[op.level + 1];
                const bool lr = lv.lr.m > 0;
                double* fr = lv.f;
                LRRhsArg lrr{nullptr};  // (rhs_inplace: f read in place, as lrr says)
                if (lr && !op.lr_skip_patch) {  // r = (f - B Sigma^{-1} B^T x) - A x
                    lr_dots(lv, lv.buf(op.src), LR_SCALE_INV, s, nch);
                    fr = lr_rhs(h, lv, LR_PATCH_RESIDUAL, lv.f, 0, sample, s, nch,
                                lv.lr.dense_path && op.lr_post_patch ? (int64_t)op.lr_post_tag : -1,
                                lv.lr.rhs_inplace && op.zpre == 0 ? &lrr : nullptr);
                }
                if (op.zpre > 0) {  // + the next op's (k_tail's) noise
                    const int ti = op.zpre - 1;
                    const TailNoiseLaunch tn{h->tail_jobs[ti], h->tail_njobs[ti], h->tail_zb[ti], h->tail_zn[ti],
                                             h->key, (uint32_t)h->chain, (uint32_t)(h->seed >> 32), sample};
                    launch_residual_restrict(lv, lc, lv.buf(op.src), fr, lc.f, lc.x, 1, s, nch, &tn);
                } else {
                    PreNoiseLaunch pnl;
                    if (op.pn_dst) {
                        pnl.job = PostNoiseJob{lc.L.nx, lc.L.ny, lc.L.nz, op.pn_tag, op.pn_dst};
                        pnl.key = h->key;
                        pnl.sample = sample;
                    }
                    launch_residual_restrict(lv, lc, lv.buf(op.src), fr, lc.f, lc.x, 1, s, nch, nullptr, op.xzero != 0,
                                             lrr.e ? &lrr : nullptr, op.pn_dst ? &pnl : nullptr);
                    if (op.xzero && h->poison)  // (debug) the skipped x_c write leaves stale values: make them NaN
                        for (int c = 0; c < nch; ++c)
                            hipLaunchKernelGGL(k_poison_interior, dim3((lc.L.nx - 1 + 255) / 256, lc.L.ny - 1,
                                                                       lc.spec.dim == 3 ? lc.L.nz - 1 : 1),
                                               dim3(256), 0, s, lc.L, chain_ptr(lc.x, lc, c));
                }
                if (lr && lv.lr.dense_path && !lrr.e)
                    ;  // f was never patched; the post-sweep's rhs went to lr.fe2 above
                else if (lr && (op.lr_post_patch || op.lr_coarse_patch))
                    lr_restore_patch(h, op, lv, lc, sample, s, nch);
                else if (lr)
                    lr_restore(lv, lv.f, s, nch, lrr.e != nullptr);
                break;
            }
            case OP_PROLONGATE: {
                Level& lc = h->levels[op.level + 1];
                launch_prolongate(lv, lc, lv.buf(op.src), lc.x, h->cfg.coarse_scaling, s, nch);
                break;
            }
            case OP_COPY: {  // the chains' copies are contiguous
                hipMemcpyAsync(lv.x, lv.buf(op.src), (size_t)nch * lv.L.nstore * sizeof(double),
                               hipMemcpyDeviceToDevice, s);
                break;
            }
            case OP_TAIL: {  // one workgroup per chain (+ spare workgroups drawing post-sweep noise)
                const size_t lds = h->tail_lds[op.tail];
                const dim3 grid(nch + h->tail_pn_wg[op.tail]);
                const TailArgs* ta = h->tail_args[op.tail];
                if (lv.spec.dim == 3 && h->tail_sym[op.tail])
                    hipLaunchKernelGGL((k_tail<3, true>), grid, dim3(TAIL_NT), lds, s, ta, nch);
                else if (lv.spec.dim == 3)
                    hipLaunchKernelGGL(k_tail<3>, grid, dim3(TAIL_NT), lds, s, ta, nch);
                else
                    hipLaunchKernelGGL(k_tail<2>, grid, dim3(TAIL_NT), lds, s, ta, nch);
                break;
            }
            case OP_QOI: {
                if (h->qv_n > 0) {  // a QoI vector is installed: its dot (skipped unless ctrl[2] = -2)
                    hipLaunchKernelGGL(k_qoi_dot, dim3(h->qv_nblk, nch), dim3(64), 0, s, (const double*)h->levels[0].x,
                                       (const long long*)h->qv_off, (const double*)h->qv_val, h->qv_n,
                                       (const uint64_t*)h->ctrl, h->qv_part, h->qv_nblk,
                                       (long long)h->levels[0].L.nstore);
                    hipLaunchKernelGGL(k_qoi_record_vec, dim3(1), dim3(64 * nch), 0, s, (const double*)h->levels[0].x,
                                       h->ctrl, h->series, h->series_cap, h->mom, nch, (long long)h->levels[0].L.nstore,
                                       (const double*)h->qv_part, h->qv_nblk);
                    break;
                }
                hipLaunchKernelGGL(k_qoi_record, dim3(1), dim3(64 * ((nch + 63) / 64)), 0, s,
                                   (const double*)h->levels[0].x, h->ctrl, h->series, h->series_cap, h->mom, nch,
                                   (long long)h->levels[0].L.nstore);
                break;
            }
        }
    }
}

int capture(mgmc_handle* h, size_t begin, size_t end, hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    enqueue_ops(h, begin, end, h->stream);
    HIPCHK(h, hipStreamEndCapture(h->stream, &g));
    HIPCHK(h, hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIPCHK(h, hipGraphDestroy(g));
    return MGMC_OK;
}

void destroy_graphs(mgmc_handle* h) {
    if (h->graph_all) hipGraphExecDestroy(h->graph_all);
    h->graph_all = nullptr;
    if (h->graph_unroll) hipGraphExecDestroy(h->graph_unroll);
    h->graph_unroll = nullptr;
    if (h->graph_timed) hipGraphExecDestroy(h->graph_timed);
    h->graph_timed = nullptr;
    if (h->graph_timed_src) hipGraphDestroy(h->graph_timed_src);
    h->graph_timed_src = nullptr;
}

// the timed cycle: the same ops in one graph with an external event-record node at each of the five
// segment boundaries (no extra graph launches; mgmc_sample_timed re-targets the nodes per step):
// fine pre-sampler | coarse-grid correction | fine post-sampler | QoI record
int capture_timed(mgmc_handle* h) {
    for (auto& e : h->timed_ev0)
        if (!e) HIPCHK(h, hipEventCreate(&e));
    const size_t b[5] = {0, h->seg_end_pre, h->seg_begin_post, h->seg_end_post, h->ops.size()};
    HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
    for (int q = 0; q < 5; ++q) {
        HIPCHK(h, hipEventRecordWithFlags(h->timed_ev0[q], h->stream, hipEventRecordExternal));
        if (q < 4) enqueue_ops(h, b[q], b[q + 1], h->stream);
    }
    HIPCHK(h, hipStreamEndCapture(h->stream, &h->graph_timed_src));
    size_t nn = 0;
    HIPCHK(h, hipGraphGetNodes(h->graph_timed_src, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn);
    HIPCHK(h, hipGraphGetNodes(h->graph_timed_src, nodes.data(), &nn));
    for (hipGraphNode_t nd : nodes) {
        hipGraphNodeType ty;
        HIPCHK(h, hipGraphNodeGetType(nd, &ty));
        if (ty != hipGraphNodeTypeEventRecord) continue;
        hipEvent_t e = nullptr;
        HIPCHK(h, hipGraphEventRecordNodeGetEvent(nd, &e));
        for (int q = 0; q < 5; ++q)
            if (e == h->timed_ev0[q]) h->timed_node[q] = nd;
    }
    for (int q = 0; q < 5; ++q)
        if (!h->timed_node[q]) return fail(h, MGMC_E_HIP, "timed graph: event-record node not captured");
    HIPCHK(h, hipGraphInstantiate(&h->graph_timed, h->graph_timed_src, nullptr, nullptr, 0));
    return MGMC_OK;
}

// (re)capture the graphs; they embed series/series_cap, so recapture when those change
int build_graphs(mgmc_handle* h) {
    destroy_graphs(h);
    int rc = capture(h, 0, h->ops.size(), &h->graph_all);
    if (rc) return rc;
    // small lattices: one hipGraphLaunch costs about as much host time as a 2D 1024^2 cycle takes on
    // the GPU, so the sample loops replay `unroll` cycles per launch (the sample index lives on the
    // device: the copies are identical)
    const uint64_t n0 = h->levels[0].spec.ndof;
    h->unroll = n0 <= (1u << 22) ? 8 : (n0 <= (1u << 25) ? 2 : 1);
    if (h->unroll_override > 0) h->unroll = h->unroll_override;
    if (h->unroll > 1) {
        hipGraph_t g = nullptr;
        HIPCHK(h, hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        for (int u = 0; u < h->unroll; ++u) enqueue_ops(h, 0, h->ops.size(), h->stream);
        HIPCHK(h, hipStreamEndCapture(h->stream, &g));
        HIPCHK(h, hipGraphInstantiate(&h->graph_unroll, g, nullptr, nullptr, 0));
        HIPCHK(h, hipGraphDestroy(g));
    }
    if (h->levels.size() > 1) {
        rc = capture_timed(h);
        if (rc) return rc;
    }
    return MGMC_OK;
}

int ensure_series(mgmc_handle* h, uint64_t needed) {
    if (needed <= h->series_cap) return MGMC_OK;
    uint64_t cap = std::max<uint64_t>(needed, 2 * h->series_cap);
    double* p = nullptr;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMalloc(&p, cap * h->nchains * sizeof(double)));  // chain c's series c * cap on
    poison_fill(h, p, cap * h->nchains * sizeof(double));
    if (h->series) HIPCHK(h, hipFree(h->series));
    h->series = p;
    h->series_cap = cap;
    return build_graphs(h);
}

int ensure_lex(mgmc_handle* h, size_t n) {
    if (n <= h->lex_cap) return MGMC_OK;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (h->lex_tmp) HIPCHK(h, hipFree(h->lex_tmp));
    HIPCHK(h, hipMalloc(&h->lex_tmp, n * sizeof(double)));
    poison_fill(h, h->lex_tmp, n * sizeof(double));
    h->lex_cap = n;
    return MGMC_OK;
}

int ensure_scratch(mgmc_handle* h, int level) {
    Level& lv = h->levels[level];
    for (auto& p : lv.scratch) {
        if (!p) {
            HIPCHK(h, hipMalloc(&p, lv.L.nstore * sizeof(double)));
            HIPCHK(h, hipMemsetAsync(p, 0, lv.L.nstore * sizeof(double), h->stream));
        }
    }
    return MGMC_OK;
}

// host (reference layout) -> padded device buffer
int upload(mgmc_handle* h, int level, const double* host, double* pad) {
    Level& lv = h->levels[level];
    int rc = ensure_lex(h, lv.spec.ndof);
    if (rc) return rc;
    HIPCHK(h, hipMemcpyAsync(h->lex_tmp, host, lv.spec.ndof * sizeof(double), hipMemcpyHostToDevice, h->stream));
    launch_pack(lv, h->lex_tmp, pad, true, h->stream);
    HIPCHK(h, hipGetLastError());
    return MGMC_OK;
}

int download(mgmc_handle* h, int level, const double* pad, double* host) {
    Level& lv = h->levels[level];
    int rc = ensure_lex(h, lv.spec.ndof);
    if (rc) return rc;
    launch_pack(lv, h->lex_tmp, const_cast<double*>(pad), false, h->stream);
    HIPCHK(h, hipGetLastError());
    HIPCHK(h, hipMemcpyAsync(host, h->lex_tmp, lv.spec.ndof * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

// a handle whose mgmc_set_lowrank rollback failed refuses every call that runs the cycle or
// needs the coarse factor: mgmc_apply, mgmc_sample*, mgmc_sample_timed*, mgmc_solve, and the per-level
// component calls (check_level); a later successful mgmc_set_lowrank clears it.  State, right-hand side,
// QoI and RCCL calls do not touch the factor and stay available, as does mgmc_destroy.
int refuse_unusable(mgmc_handle* h) {
    return fail(h, MGMC_E_INVALID, "handle unusable: a failed mgmc_set_lowrank could not restore the prior's coarse "
                                   "factor (mgmc_destroy it)");
}

int check_level(mgmc_handle* h, int level, bool need_coarser) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    if (h->unusable) return refuse_unusable(h);
    if (level < 0 || level >= (int)h->levels.size()) return fail(h, MGMC_E_INVALID, "level out of range");
    if (need_coarser && level + 1 >= (int)h->levels.size())
        return fail(h, MGMC_E_INVALID, "level has no coarser level");
    return MGMC_OK;
}

void fill_desc(const LevelSpec& s, mgmc_level_desc* d, bool varcoef = false) {
    memset(d, 0, sizeof(*d));
    d->varcoef = varcoef ? 1 : 0;
    d->nx = s.n[0];
    d->ny = s.n[1];
    d->nz = s.dim == 3 ? s.n[2] : 0;
    d->npoints = s.npoints;
    d->ncolours = s.ncolours;
    d->ndof = s.ndof;
    memcpy(d->stencil, s.st, sizeof(d->stencil));
}

// a level's coefficient field from its matrix (mgmc_field.hpp): the union of the rows' offsets in
// ascending column order, every row's entries at their offsets (zeros elsewhere); the colouring of
// the oracle's multicolour mode: red-black for a fine level of at most 2d+1 entries per row and reach
// 1, coordinates mod 3 for reach 2, parities otherwise
struct FieldHost {
    int np = 0, diag = -1, scheme = 0;
    int d[FIELD_MAXNP][3];
    std::vector<double> coef;
    double centre[27];
};

// the colouring of a matrix level (the oracle's init_colouring): 3^d classes (coordinates mod 3) for
// reach-2 couplings, red-black for a fine level whose couplings are all axis neighbours, 2^d
// coordinate parities otherwise
static int colour_scheme(int dim, int level, int reach, bool axis_only) {
    if (reach >= 2) return dim == 3 ? 27 : 9;
    return (level == 0 && axis_only) ? 2 : (1 << dim);
}

FieldHost make_field(const CsrHost& A, int dim, const int* n, int level) {
    FieldHost F;
    const int64_t nxi = n[0] - 1, nyi = n[1] - 1;
    auto euc = [&](int64_t e, int* idx) {
        idx[0] = (int)(e % nxi) + 1;
        idx[1] = (int)((e / nxi) % nyi) + 1;
        idx[2] = dim == 3 ? (int)(e / (nxi * nyi)) + 1 : 0;
    };
    auto key = [](int dx, int dy, int dz) { return (dz + 2) * 25 + (dy + 2) * 5 + (dx + 2); };
    bool present[125] = {false};
    int reach = 0;
    int64_t maxnnz = 0;
    for (int64_t r = 0; r < A.nrow; ++r) {
        int a[3], b[3];
        euc(r, a);
        maxnnz = std::max(maxnnz, A.rowptr[r + 1] - A.rowptr[r]);
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            euc(A.col[q], b);
            const int dx = b[0] - a[0], dy = b[1] - a[1], dz = b[2] - a[2];
            reach = std::max(reach, std::max(std::abs(dx), std::max(std::abs(dy), std::abs(dz))));
            present[key(dx, dy, dz)] = true;
        }
    }
    int slot[125];
    for (int k = 0; k < 125; ++k) {
        slot[k] = -1;
        if (!present[k]) continue;
        slot[k] = F.np;
        F.d[F.np][0] = k % 5 - 2;
        F.d[F.np][1] = (k / 5) % 5 - 2;
        F.d[F.np][2] = k / 25 - 2;
        if (k == key(0, 0, 0)) F.diag = F.np;
        ++F.np;
    }
    // red-black only when every coupling is an axis neighbour (the 5/7-point pattern): a row of at
    // most 2d+1 entries that couples diagonal neighbours ((+-1, +-1), edge neighbours in 3D) would
    // put coupled vertices into one colour
    bool axis_only = true;
    for (int k = 0; k < 125; ++k)
        if (present[k] && std::abs(k % 5 - 2) + std::abs((k / 5) % 5 - 2) + std::abs(k / 25 - 2) > 1) axis_only = false;
    (void)maxnnz;
    F.scheme = colour_scheme(dim, level, reach, axis_only);
    F.coef.assign((size_t)A.nrow * F.np, 0.0);
    for (int64_t r = 0; r < A.nrow; ++r) {
        int a[3], b[3];
        euc(r, a);
        for (int64_t q = A.rowptr[r]; q < A.rowptr[r + 1]; ++q) {
            euc(A.col[q], b);
            F.coef[(size_t)r * F.np + slot[key(b[0] - a[0], b[1] - a[1], b[2] - a[2])]] = A.val[q];
        }
    }
    // the row of the lattice's centre vertex, for mgmc_level_desc (3^d box)
    for (double& v : F.centre) v = 0.0;
    const int64_t rc = ((int64_t)(dim == 3 ? (n[2] / 2 - 1) : 0) * nyi + (n[1] / 2 - 1)) * nxi + (n[0] / 2 - 1);
    for (int p = 0; p < F.np; ++p) {
        const int* o = F.d[p];
        if (std::abs(o[0]) > 1 || std::abs(o[1]) > 1 || std::abs(o[2]) > 1) continue;
        const int k = dim == 3 ? (o[2] + 1) * 9 + (o[1] + 1) * 3 + (o[0] + 1) : (o[1] + 1) * 3 + (o[0] + 1);
        F.centre[k] = F.coef[(size_t)rc * F.np + p];
    }
    return F;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

int mgmc_abi_version(void) { return MGMC_ABI_VERSION; }

int mgmc_live_handles(void) { return g_live_handles.load(); }

const char* mgmc_last_error(const mgmc_handle* h) {
    if (h) return h->last_error.c_str();
    std::lock_guard<std::mutex> lock(g_err_mutex);
    static thread_local std::string copy;
    copy = g_last_error;
    return copy.c_str();
}

int mgmc_describe(const mgmc_config* cfg, mgmc_level_desc* out, int max_levels) {
    if (!cfg) return fail(nullptr, MGMC_E_INVALID, "null config");
    const std::string err = validate_config(*cfg);
    if (!err.empty()) return fail(nullptr, MGMC_E_INVALID, err);
    const std::vector<LevelSpec> lv = build_hierarchy(*cfg);
    if (out) {
        for (int l = 0; l < (int)lv.size() && l < max_levels; ++l) fill_desc(lv[l], &out[l]);
    }
    return (int)lv.size();
}

// the kernel families that address level l (the launch_* dispatch of this handle) and their check
static int zrestrict_cx_of(const mgmc_handle* h, int l) {  // launch_residual_restrict's tile width
    if (l + 1 >= (int)h->levels.size()) return 0;
    const Level& lf = h->levels[l];
    const Level& lc = h->levels[l + 1];
    if (lf.spec.dim != 3 || lf.field || (lf.paths & PATH_NO_ZRESTRICT) || lc.L.nx < 8) return 0;
    return lc.L.nx < 32 ? 16 : (lf.spec.npoints == 27 && lf.fold ? tune::ZR27_CX : 64);
}
// both directions and both halves of a j-marching level, with launch_jsweep's plan (short_grid: the plan
// with its last 8 workgroups dropped -- a negative control for the test, which the replay must reject)
static std::string jsweep_grid_check_level(const Layout& L, int num_cu, bool short_grid = false) {
    const size_t lds = jsweep_lds_bytes(L.nx / 2);
    for (int d = 0; d < 2; ++d)
        for (int half = 0; half < 2; ++half) {
            JSweepPlan p = jsweep_plan(L, d == 0, half, num_cu, lds, tune::JS_ROUNDS);
            if (short_grid && p.nb > 8) p.nb -= 8;
            const std::string e = jsweep_grid_check(L, p, JS_D);
            if (!e.empty()) return e;
        }
    return "";
}
static std::string check_level_layout_of(const mgmc_handle* h, int l) {
    const Level& lv = h->levels[l];
    unsigned fam = LF_POINT;
    if (lv.pairs || lv.quads) fam |= LF_PAIRS;
    if (lv.zsweep) fam |= LF_ZSWEEP;
    if (lv.rb2d) fam |= LF_RB2D;
    const int cx = zrestrict_cx_of(h, l);
    if (cx) fam |= LF_ZRESTRICT;
    if (l > 0 && h->levels[l - 1].zsweep) fam |= LF_ZSWEEP_C;
    if (lv.jsweep) fam |= LF_JSWEEP;
    if (qrestrict_ok(h, l)) fam |= LF_QRESTRICT;
    const int reach = lv.field && (lv.F.scheme == 9 || lv.F.scheme == 27) ? 2 : 1;
    std::string e = check_level_layout(lv.L, fam, reach, cx);
    if (e.empty() && lv.jsweep) e = jsweep_grid_check_level(lv.L, lv.num_cu);
    return e;
}

// mgmc_create / mgmc_create_csr: csr = the fine operator's matrix (null: the constant-coefficient
// hierarchy of cfg), every level then built from matrices
static int create_impl(const mgmc_config* cfg, const CsrHost* csr, int device, uint64_t seed, uint64_t chain_id,
                       int nchains, mgmc_handle** out, const double* fine_st = nullptr) {
    if (!cfg || !out) return fail(nullptr, MGMC_E_INVALID, "null argument");
    *out = nullptr;
    if (nchains < 1 || nchains > LR_MAX_CH)
        return fail(nullptr, MGMC_E_INVALID, "nchains must be in [1, " + std::to_string(LR_MAX_CH) + "]");
    const std::string err = validate_config(*cfg);
    if (!err.empty()) return fail(nullptr, MGMC_E_INVALID, err);
    std::vector<CsrHost> mats;  // per level (matrix path)
    if (csr) {
        const int n0[3] = {cfg->nx, cfg->ny, cfg->dim == 3 ? cfg->nz : 1};
        const std::string e = check_lattice_csr(cfg->dim, n0, *csr);
        if (!e.empty()) return fail(nullptr, MGMC_E_INVALID, "mgmc_create_csr: " + e);
        mats.push_back(*csr);
        int n[3] = {n0[0], n0[1], n0[2]};
        for (int l = 1; l < cfg->nlevel; ++l) {
            mats.push_back(galerkin_csr(mats.back(), cfg->dim, n));
            for (int d = 0; d < cfg->dim; ++d) n[d] /= 2;
        }
    }
    uint32_t paths = 0;
    std::string bad;
    if (!read_path_flags(&paths, &bad)) return fail(nullptr, MGMC_E_INVALID, "MGMC_DISABLE: unknown path '" + bad + "'");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(nullptr, MGMC_E_HIP, "no HIP device");
    if (device < 0 || device >= ndev) return fail(nullptr, MGMC_E_INVALID, "device index out of range");
    mgmc_handle* h = new mgmc_handle();
    h->paths = paths;
    if (const char* u = getenv("MGMC_GRAPH_UNROLL")) h->unroll_override = std::max(1, std::min(64, atoi(u)));
    if (const char* u = getenv("MGMC_POISON")) h->poison = atoi(u) != 0;
    h->cfg = *cfg;
    h->device = device;
    h->seed = seed;
    h->chain = chain_id;
    h->nchains = nchains;
    h->key = make_key(seed, chain_id);
    int ncu = 0;  // per handle: concurrent mgmc_create calls share no mutable state
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
    if (hipSetDevice(device) != hipSuccess) {
        delete h;
        return fail(nullptr, MGMC_E_HIP, "hipSetDevice failed");
    }
    int rc = MGMC_OK;
    auto bail = [&](int code) {
        set_global_error(h->last_error);
        mgmc_destroy(h);
        return code;
    };
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        h->last_error = "hipStreamCreate failed";
        return bail(MGMC_E_HIP);
    }
    std::vector<LevelSpec> specs = build_hierarchy(*cfg, fine_st);
    h->field_mode = csr != nullptr;
    std::vector<FieldHost> fields;
    for (size_t l = 0; l < mats.size(); ++l) {
        fields.push_back(make_field(mats[l], cfg->dim, specs[l].n, (int)l));
        specs[l].npoints = fields.back().np;
        specs[l].ncolours = fields.back().scheme;
        memcpy(specs[l].st, fields.back().centre, sizeof(specs[l].st));
    }
    if (!mats.empty()) h->coarse_csr = mats.back();
    const int tail0 = tail_start_by_size(specs, *cfg, h->paths, h->field_mode);  // levels k_tail can take (no quads there)
    size_t lds_limit = 150 * 1024;
    for (size_t l = 0; l < specs.size(); ++l) {
        Level lv;
        lv.num_cu = ncu;
        lv.spec = specs[l];
        lv.paths = h->paths;
        // reach-2 field levels (3^d colourings) read two vertices beyond every interior vertex
        lv.L = make_layout(cfg->dim, specs[l].n,
                           h->field_mode && (fields[l].scheme == 9 || fields[l].scheme == 27));
        memcpy(lv.S.a, specs[l].st, sizeof(lv.S.a));
        // (MGMC_DISABLE=fold keeps the reference's CSR summation order in the residuals of these levels;
        // sym stays: the Gibbs sweeps' arithmetic does not depend on it)
        const bool refl = !h->field_mode && lv.spec.dim == 3 && stencil_reflection_symmetric(lv.S.a, lv.spec.npoints);
        lv.fold = refl && !(h->paths & PATH_NO_FOLD);
        lv.sym = refl;
        const size_t bytes = lv.L.nstore * sizeof(double);
        const size_t cbytes = bytes * nchains;  // x, x2, f of every chain, L.nstore apart
        if (hipMalloc(&lv.x, cbytes) != hipSuccess || hipMalloc(&lv.f, cbytes) != hipSuccess) {
            h->levels.push_back(lv);
            h->last_error = "device allocation failed";
            return bail(MGMC_E_NOMEM);
        }
        hipMemsetAsync(lv.x, 0, cbytes, h->stream);
        hipMemsetAsync(lv.f, 0, cbytes, h->stream);
        if (h->field_mode) {  // per-vertex coefficients and a residual scratch
            const FieldHost& fh = fields[l];
            lv.field = true;
            memset(&lv.F, 0, sizeof(lv.F));
            lv.F.np = fh.np;
            lv.F.diag = fh.diag;
            lv.F.nxi = lv.L.nx - 1;
            lv.F.nyi = lv.L.ny - 1;
            lv.F.scheme = fh.scheme;
            lv.F.omega = cfg->omega;
            for (int q = 0; q < fh.np; ++q)
                lv.F.off[q] = (int)(fh.d[q][2] * lv.L.sp + fh.d[q][1] * lv.L.sx + fh.d[q][0]);
            double* coef = nullptr;
            if (hipMalloc(&coef, fh.coef.size() * sizeof(double)) != hipSuccess ||
                hipMalloc(&lv.rbuf, bytes) != hipSuccess) {
                lv.F.coef = coef;
                h->levels.push_back(lv);
                h->last_error = "device allocation failed (coefficient field)";
                return bail(MGMC_E_NOMEM);
            }
            lv.F.coef = coef;
            hipMemcpyAsync(coef, fh.coef.data(), fh.coef.size() * sizeof(double), hipMemcpyHostToDevice, h->stream);
            hipMemsetAsync(lv.rbuf, 0, bytes, h->stream);
        }
        // fused z-marching sweep: fine 3D 7-point levels whose row splits into 64-pair tiles
        const double* st = lv.spec.st;  // the z-sweep folds the symmetric FD stencil to 4 coefficients
        const bool symmetric = st[4] == st[22] && st[10] == st[16] && st[12] == st[14];
        lv.zsweep = !lv.field && cfg->dim == 3 && lv.spec.npoints == 7 && symmetric && l + 1 < specs.size() &&
                    (lv.L.nx % (2 * ZS_XP)) == 0 && !(h->paths & PATH_NO_ZSWEEP);
        lv.pairs = !lv.field && pairs_eligible(lv.spec, lv.L) && !(h->paths & PATH_NO_PAIRS);
        lv.rb2d = !lv.field && cfg->dim == 2 && lv.spec.npoints == 5 && l + 1 < specs.size() &&
                  !(h->paths & PATH_NO_RB2D);
        lv.jsweep = lv.pairs && jsweep_eligible(lv.spec, lv.L, h->paths) && (tail0 < 0 || (int)l < tail0);
        lv.quads = lv.jsweep || (lv.pairs && quads_eligible(lv.spec, lv.L, h->paths) && (tail0 < 0 || (int)l < tail0));
        if (lv.pingpong()) {
            if (hipMalloc(&lv.x2, cbytes) != hipSuccess) {
                h->levels.push_back(lv);
                h->last_error = "device allocation failed";
                return bail(MGMC_E_NOMEM);
            }
            hipMemsetAsync(lv.x2, 0, cbytes, h->stream);
        }
        if (!lv.field && l + 1 == specs.size() && 2 * bytes <= lds_limit) lv.lds_bytes = 2 * bytes;
        h->levels.push_back(lv);
    }
    if (hipMalloc(&h->ctrl, 8 * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&h->mom, 4 * sizeof(double) * nchains) != hipSuccess) {
        h->last_error = "device allocation failed";
        return bail(MGMC_E_NOMEM);
    }
    // ctrl[6]: the vertex the non-finite guard watches when no QoI is recorded (lattice centre)
    const Level& l0 = h->levels[0];
    const long long probe = l0.L.at(l0.L.nx / 2, l0.L.ny / 2, cfg->dim == 3 ? l0.L.nz / 2 : 0);
    uint64_t ctrl0[8] = {0, 0, (uint64_t)(int64_t)-1, 0, 0, 0, (uint64_t)probe, 0};
    hipMemcpyAsync(h->ctrl, ctrl0, sizeof(ctrl0), hipMemcpyHostToDevice, h->stream);
    hipMemsetAsync(h->mom, 0, 4 * sizeof(double) * nchains, h->stream);
    if (cfg->coarse_solver == MGMC_COARSE_CHOLESKY && (rc = build_coarse_chol(h, nullptr, nullptr, 0)) != MGMC_OK)
        return bail(rc);
    // every level's extreme addresses against its store (mgmc_layout_check.hpp)
    for (size_t l = 0; l < h->levels.size(); ++l) {
        const std::string e = check_level_layout_of(h, (int)l);
        if (!e.empty()) {
            h->last_error = "internal layout check failed: " + e;
            return bail(MGMC_E_INVALID);
        }
    }
    // op sequence of one sample
    build_ops(h);
    if ((rc = build_tails(h)) != MGMC_OK) return bail(rc);
    if ((rc = ensure_series(h, 1024)) != MGMC_OK) return bail(rc);
    if (hipStreamSynchronize(h->stream) != hipSuccess) {
        h->last_error = "stream sync failed after setup";
        return bail(MGMC_E_HIP);
    }
    if (cfg->verbose > 0) {
        printf("Setting up Multilevel MC sampler (HIP, device %d)\n", device);
        for (size_t l = 0; l < specs.size(); ++l)
            printf("  level %zu lattice : %dd lattice, %d x %d x %d cells, %llu unknowns, %d-point stencil\n", l,
                   cfg->dim, specs[l].n[0], specs[l].n[1], specs[l].n[2], (unsigned long long)specs[l].ndof,
                   specs[l].npoints);
    }
    *out = h;
    return MGMC_OK;
}

int mgmc_create(const mgmc_config* cfg, int device, uint64_t seed, uint64_t chain_id, mgmc_handle** out) {
    return create_impl(cfg, nullptr, device, seed, chain_id, 1, out);
}

int mgmc_create_batch(const mgmc_config* cfg, int device, uint64_t seed, uint64_t chain0, int nchains,
                      mgmc_handle** out) {
    return create_impl(cfg, nullptr, device, seed, chain0, nchains, out);
}

int mgmc_nchains(const mgmc_handle* h) { return h ? h->nchains : fail(nullptr, MGMC_E_INVALID, "null handle"); }

int mgmc_create_csr(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                    const double* val, int device, uint64_t seed, uint64_t chain_id, mgmc_handle** out) {
    return mgmc_create_csr_batch(cfg, nrow, rowptr, col, val, device, seed, chain_id, 1, out);
}

// the matrix's shape against cfg's lattice, before anything reads rowptr[nrow] or copies entries:
// nrow = the interior vertex count, rowptr non-decreasing from 0, at most 125 entries per row (the
// 5^d box of reach-2 couplings)
static std::string check_csr_shape(const mgmc_config& cfg_in, int64_t nrow, const int64_t* rowptr) {
    mgmc_config cfg = cfg_in;  // the matrix replaces kappa^2 and the fine-operator choice
    cfg.kappa_sq = 0.0;
    cfg.fine_operator = MGMC_OPERATOR_FD;
    const std::string err = validate_config(cfg);
    if (!err.empty()) return err;
    int64_t expect = (int64_t)(cfg.nx - 1) * (cfg.ny - 1);
    if (cfg.dim == 3) expect *= (cfg.nz - 1);
    if (nrow != expect)
        return "nrow " + std::to_string(nrow) + " != the lattice's " + std::to_string(expect) + " interior vertices";
    if (rowptr[0] != 0) return "rowptr[0] != 0";
    for (int64_t r = 0; r < nrow; ++r) {
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (len < 1 || len > 125) return "row " + std::to_string(r) + " has " + std::to_string(len) + " entries";
    }
    return "";
}

int mgmc_csr_colour_scheme(const mgmc_config* cfg, int level, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                           int* scheme) {
    if (!cfg || !rowptr || !col || !scheme || nrow < 1 || level < 0) return fail(nullptr, MGMC_E_INVALID, "null argument");
    mgmc_config c = *cfg;
    c.nlevel = 1;
    const std::string e0 = check_csr_shape(c, nrow, rowptr);
    if (!e0.empty()) return fail(nullptr, MGMC_E_INVALID, "mgmc_csr_colour_scheme: " + e0);
    CsrHost A;
    A.nrow = nrow;
    A.rowptr.assign(rowptr, rowptr + nrow + 1);
    A.col.assign(col, col + rowptr[nrow]);
    A.val.assign((size_t)rowptr[nrow], 1.0);
    const int n[3] = {cfg->nx, cfg->ny, cfg->dim == 3 ? cfg->nz : 1};
    const std::string e = check_lattice_csr(cfg->dim, n, A);
    if (!e.empty()) return fail(nullptr, MGMC_E_INVALID, "mgmc_csr_colour_scheme: " + e);
    *scheme = make_field(A, cfg->dim, n, level).scheme;
    return MGMC_OK;
}

int mgmc_create_csr_batch(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                          const double* val, int device, uint64_t seed, uint64_t chain0, int nchains,
                          mgmc_handle** out) {
    if (!cfg || !rowptr || !col || !val || !out || nrow < 1) return fail(nullptr, MGMC_E_INVALID, "null argument");
    const std::string e0 = check_csr_shape(*cfg, nrow, rowptr);
    if (!e0.empty()) return fail(nullptr, MGMC_E_INVALID, "mgmc_create_csr: " + e0);
    mgmc_config c = *cfg;  // the matrix replaces kappa^2 and the fine-operator choice
    c.kappa_sq = 0.0;
    c.fine_operator = MGMC_OPERATOR_FD;
    CsrHost A;
    A.nrow = nrow;
    A.rowptr.assign(rowptr, rowptr + nrow + 1);
    A.col.assign(col, col + rowptr[nrow]);
    A.val.assign(val, val + rowptr[nrow]);
    return create_impl(&c, &A, device, seed, chain0, nchains, out);
}

int mgmc_check_layout(int dim, const int* n, int reach, unsigned families, int zrestrict_cx, int legacy) {
    if (!n || (dim != 2 && dim != 3) || reach < 1 || reach > 2) return fail(nullptr, MGMC_E_INVALID, "invalid argument");
    // legacy bit 0: the round-2 layout without the reach-2 margin; bit 1: unclamped restriction columns
    const Layout L = make_layout(dim, n, reach == 2 && !(legacy & 1));
    std::string e = check_level_layout(L, families, reach, zrestrict_cx, (legacy & 2) != 0);
    if (e.empty() && (families & LF_JSWEEP)) e = jsweep_grid_check_level(L, 256, (legacy & 4) != 0);  // 256 CUs
    if (!e.empty()) return fail(nullptr, MGMC_E_INVALID, e);
    return MGMC_OK;
}

int mgmc_stencil_of_csr(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                        const double* val, double* stencil) {
    if (!cfg || !rowptr || !col || !val || !stencil || nrow < 1) return fail(nullptr, MGMC_E_INVALID, "null argument");
    mgmc_config c = *cfg;
    c.kappa_sq = 0.0;
    c.fine_operator = MGMC_OPERATOR_FD;
    const std::string e0 = check_csr_shape(c, nrow, rowptr);
    if (!e0.empty()) return fail(nullptr, MGMC_E_INVALID, "mgmc_stencil_of_csr: " + e0);
    const int dim = cfg->dim;
    const int64_t nxi = cfg->nx - 1, nyi = cfg->ny - 1, nzi = dim == 3 ? cfg->nz - 1 : 1;
    // the stencil of the lattice's centre row, then every row checked against its truncation
    double st[27] = {0};
    bool have[27] = {false};
    auto slot = [&](int64_t r, int32_t cidx, int* k) {
        const int64_t ri = r % nxi, rj = (r / nxi) % nyi, rk = r / (nxi * nyi);
        const int64_t ci = cidx % nxi, cj = (cidx / nxi) % nyi, ck = cidx / (nxi * nyi);
        const int64_t dx = ci - ri, dy = cj - rj, dz = ck - rk;
        if (dx < -1 || dx > 1 || dy < -1 || dy > 1 || dz < -1 || dz > 1) return false;
        *k = dim == 3 ? (int)((dz + 1) * 9 + (dy + 1) * 3 + (dx + 1)) : (int)((dy + 1) * 3 + (dx + 1));
        return true;
    };
    const int64_t rc = ((nzi / 2) * nyi + nyi / 2) * nxi + nxi / 2;
    for (int64_t q = rowptr[rc]; q < rowptr[rc + 1]; ++q) {
        int k;
        if (col[q] < 0 || col[q] >= nrow || !slot(rc, col[q], &k))
            return fail(nullptr, MGMC_E_UNSUPPORTED, "mgmc_stencil_of_csr: couplings beyond the 3^d box");
        st[k] = val[q];
        have[k] = true;
    }
    const int zr = dim == 3 ? 1 : 0;
    for (int64_t r = 0; r < nrow; ++r) {
        const int64_t ri = r % nxi + 1, rj = (r / nxi) % nyi + 1, rk = r / (nxi * nyi) + 1;
        int64_t q = rowptr[r];
        for (int dz = -zr; dz <= zr; ++dz)  // expected entries in ascending column order
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const int k = dim == 3 ? (dz + 1) * 9 + (dy + 1) * 3 + (dx + 1) : (dy + 1) * 3 + (dx + 1);
                    if (!have[k]) continue;
                    const int64_t i = ri + dx, j = rj + dy, kk = rk + dz;
                    if (i < 1 || i > nxi || j < 1 || j > nyi || (dim == 3 && (kk < 1 || kk > nzi))) continue;
                    const int64_t cexp = ((kk - 1) * nyi + (j - 1)) * nxi + (i - 1);
                    if (q >= rowptr[r + 1] || col[q] != cexp || val[q] != st[k])
                        return fail(nullptr, MGMC_E_UNSUPPORTED,
                                    "mgmc_stencil_of_csr: row " + std::to_string(r) + " is not the constant stencil");
                    ++q;
                }
        if (q != rowptr[r + 1])
            return fail(nullptr, MGMC_E_UNSUPPORTED,
                        "mgmc_stencil_of_csr: row " + std::to_string(r) + " has entries outside the stencil");
    }
    memcpy(stencil, st, sizeof(st));
    return MGMC_OK;
}

int mgmc_create_stencil_batch(const mgmc_config* cfg, const double* fine_stencil, int device, uint64_t seed,
                              uint64_t chain0, int nchains, mgmc_handle** out) {
    if (!cfg || !fine_stencil || !out) return fail(nullptr, MGMC_E_INVALID, "null argument");
    const int dim = cfg->dim;
    const double centre = fine_stencil[dim == 3 ? 13 : 4];
    if (!(centre > 0.0)) return fail(nullptr, MGMC_E_INVALID, "mgmc_create_stencil: non-positive centre coefficient");
    for (int k = 0; k < (dim == 3 ? 27 : 9); ++k)
        if (!std::isfinite(fine_stencil[k])) return fail(nullptr, MGMC_E_INVALID, "mgmc_create_stencil: non-finite coefficient");
    mgmc_config c = *cfg;  // the stencil replaces kappa^2 and the fine-operator choice
    c.kappa_sq = 0.0;
    c.fine_operator = MGMC_OPERATOR_FD;
    return create_impl(&c, nullptr, device, seed, chain0, nchains, out, fine_stencil);
}

int mgmc_operator_csr_size(const mgmc_operator_desc* d, int64_t* nrow, int64_t* nnz) {
    if (!d || !nrow || !nnz) return fail(nullptr, MGMC_E_INVALID, "null argument");
    const std::string e = validate_operator(*d);
    if (!e.empty()) return fail(nullptr, MGMC_E_INVALID, e);
    const CsrHost A = assemble_operator(*d);
    *nrow = A.nrow;
    *nnz = (int64_t)A.col.size();
    return MGMC_OK;
}

int mgmc_operator_csr(const mgmc_operator_desc* d, int64_t* rowptr, int32_t* col, double* val) {
    if (!d || !rowptr || !col || !val) return fail(nullptr, MGMC_E_INVALID, "null argument");
    const std::string e = validate_operator(*d);
    if (!e.empty()) return fail(nullptr, MGMC_E_INVALID, e);
    const CsrHost A = assemble_operator(*d);
    std::copy(A.rowptr.begin(), A.rowptr.end(), rowptr);
    std::copy(A.col.begin(), A.col.end(), col);
    std::copy(A.val.begin(), A.val.end(), val);
    return MGMC_OK;
}

int mgmc_destroy(mgmc_handle* h) {
    if (!h) return MGMC_OK;
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    destroy_graphs(h);
    for (auto e : h->timed_ev0)
        if (e) hipEventDestroy(e);
    free_tails(h);
    for (auto& lv : h->levels) {
        free_lowrank(lv.lr);
        if (lv.x) hipFree(lv.x);
        if (lv.x2) hipFree(lv.x2);
        if (lv.f) hipFree(lv.f);
        if (lv.F.coef && lv.field) hipFree((void*)lv.F.coef);
        if (lv.rbuf) hipFree(lv.rbuf);
        for (auto p : lv.scratch)
            if (p) hipFree(p);
    }
    for (auto p : h->sv)
        if (p) hipFree(p);
    if (h->chol_G) hipFree(h->chol_G);
    if (h->chol_Li) hipFree(h->chol_Li);
    if (h->chol_blk) hipFree(h->chol_blk);
    if (h->sv_scal) hipFree(h->sv_scal);
    if (h->sv_part) hipFree(h->sv_part);
    if (h->comm) ncclCommDestroy(h->comm);
    if (h->tail_prof) hipFree(h->tail_prof);
    if (h->comm_buf) hipFree(h->comm_buf);
    if (h->ctrl) hipFree(h->ctrl);
    if (h->mom) hipFree(h->mom);
    if (h->series) hipFree(h->series);
    if (h->qv_off) hipFree(h->qv_off);
    if (h->qv_val) hipFree(h->qv_val);
    if (h->qv_part) hipFree(h->qv_part);
    if (h->lex_tmp) hipFree(h->lex_tmp);
    if (h->zbuf) hipFree(h->zbuf);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
    return MGMC_OK;
}

int mgmc_level_desc_get(const mgmc_handle* h, int level, mgmc_level_desc* out) {
    if (!h || !out) return fail(nullptr, MGMC_E_INVALID, "null argument");
    if (level < 0 || level >= (int)h->levels.size()) return fail(nullptr, MGMC_E_INVALID, "level out of range");
    fill_desc(h->levels[level].spec, out, h->levels[level].field);
    return MGMC_OK;
}

int mgmc_level_kernels(const mgmc_handle* h, int level, char* out, size_t n) {
    if (!h || !out || n == 0) return fail(nullptr, MGMC_E_INVALID, "null argument");
    if (level < 0 || level >= (int)h->levels.size()) return fail(nullptr, MGMC_E_INVALID, "level out of range");
    const Level& lv = h->levels[level];
    const int dim = lv.spec.dim, np = lv.spec.npoints;
    const int tl = tail_level(h);
    const bool last = level + 1 == (int)h->levels.size();
    std::string sweep, post, res;
    if (tl >= 0 && level >= tl) {
        sweep = "k_tail<" + std::to_string(dim) + ">";
    } else if (last) {
        sweep = h->cfg.coarse_solver == MGMC_COARSE_CHOLESKY ? (h->chol_B > 0 ? "k_coarse_chol_blocked" : "k_coarse_chol") : "k_coarse_ssor_lds (or separate colour passes)";
    } else if (lv.field) {
        sweep = "k_fsweep<" + std::to_string(dim) + ">";
    } else if (lv.zsweep) {
        sweep = "k_zsweep_rb7<32," + std::to_string(zsweep_plain_rows(lv, h->nchains)) + ",...,0>";
        if (!(h->paths & PATH_NO_FUSE_PROLONG)) post = "k_zsweep_rb7<32," + std::to_string(tune::ZS_TYP) + ",...,PROLONG>";
    } else if (lv.jsweep) {
        sweep = "k_jsweep_half<" + std::to_string(lv.L.nx / 2) + (lv.sym && lv.L.nx == 256 ? ",sym" : "") + ">";
    } else if (lv.quads) {
        sweep = "k_sweep_quads<" + std::to_string(dim) + ">";
    } else if (lv.rb2d) {
        sweep = "k_rb2d";
    } else if (lv.pairs) {
        sweep = "k_sweep_pairs<" + std::to_string(dim) + ">";
    } else {
        sweep = (np == 2 * dim + 1 ? "k_sweep_rb<" : "k_sweep_mc<") + std::to_string(dim) + ">";
    }
    if (!last && !(tl >= 0 && level >= tl)) {
        const int cx = zrestrict_cx_of(h, level);
        if (lv.field) res = "k_fresidual + k_restrict";
        else if (cx) {
            const Level& lc = h->levels[level + 1];
            const bool wide = np == 7 && cx == 64 &&
                              (long long)((lc.L.nx + 62) / 64) * ((lc.L.ny + 6) / 8) * (lc.L.nz - 1) >= tune::ZR7_WIDE_MIN_TILES;
            res = "k_zresrestrict<" + std::to_string(np) + "," + std::to_string(cx) + "," + (wide ? "8" : "4") + ">";
        } else if (qrestrict_ok(h, level)) {
            sweep = "k_sweep_quads<2> (last pre-sweep: k_quads_restrict2d)";
            res = "k_quads_restrict2d";

        } else res = "k_residual_restrict<" + std::to_string(dim) + "," + std::to_string(np) + ">";
    }
    std::string text = "sweep=" + sweep;
    if (!post.empty()) text += ";post_sweep=" + post;
    // sweeps of this level read Box-Muller pairs drawn by an earlier launch (plan_drawn_noise): the
    // restriction before the first pre-sweep and / or a tail launch
    bool by_rr = false, by_tail = false;
    for (size_t q = 0; q < h->ops.size(); ++q) {
        const Op& op = h->ops[q];
        if (op.kind != OP_SWEEP || op.level != level || !op.pnz) continue;
        if (q > 0 && h->ops[q - 1].kind == OP_RESIDUAL_RESTRICT && h->ops[q - 1].pn_dst == op.pnz) by_rr = true;
        else by_tail = true;
    }
    if (by_rr || by_tail)
        text += std::string(";noise=") + (by_rr && by_tail ? "restriction+tail" : by_rr ? "restriction" : "tail");
    if (!res.empty()) text += ";residual_restrict=" + res;
    // the low-rank path of a posterior level (mgmc_lowrank.hpp; rhs_inplace: the sweeps and the
    // residual above run their LRF instances, f + e read in place)
    if (lv.lr.m > 0)
        text += std::string(";lowrank=") + (lv.lr.rhs_inplace ? "dense,rhs_inplace" : lv.lr.dense_path ? "dense"
                                             : lv.lr.small ? "small" : "rows");
    snprintf(out, n, "%s", text.c_str());
    return MGMC_OK;
}

// fine-level vector v of chain c (c < 0: every chain gets the upload of chain 0)
static int put_fine(mgmc_handle* h, double* v, int c, const double* host, size_t n, const char* what) {
    if (!h || !host) return fail(h, MGMC_E_INVALID, "null argument");
    if (n != h->levels[0].spec.ndof) return fail(h, MGMC_E_INVALID, std::string(what) + " size mismatch");
    if (c >= h->nchains) return fail(h, MGMC_E_INVALID, "chain index out of range");
    HIPCHK(h, hipSetDevice(h->device));
    const size_t ns = h->levels[0].L.nstore;
    int rc = upload(h, 0, host, v + (size_t)std::max(c, 0) * ns);
    if (rc) return rc;
    if (c < 0)
        for (int q = 1; q < h->nchains; ++q)
            HIPCHK(h, hipMemcpyAsync(v + q * ns, v, ns * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    return MGMC_OK;
}

int mgmc_set_rhs(mgmc_handle* h, const double* f, size_t n) {
    int rc = put_fine(h, h ? h->levels[0].f : nullptr, -1, f, n, "rhs");
    if (rc) return rc;
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

static int set_state_impl(mgmc_handle* h, int c, const double* x, size_t n) {
    int rc = put_fine(h, h ? h->levels[0].x : nullptr, c, x, n, "state");
    if (rc) return rc;
    HIPCHK(h, hipMemsetAsync(h->ctrl + 5, 0, sizeof(uint64_t), h->stream));  // a new state: guard cleared
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_set_state(mgmc_handle* h, const double* x, size_t n) { return set_state_impl(h, -1, x, n); }

int mgmc_set_state_chain(mgmc_handle* h, int chain, const double* x, size_t n) {
    if (chain < 0) return fail(h, MGMC_E_INVALID, "chain index out of range");
    return set_state_impl(h, chain, x, n);
}

int mgmc_get_state_chain(mgmc_handle* h, int chain, double* x, size_t n) {
    if (!h || !x) return fail(h, MGMC_E_INVALID, "null argument");
    if (n != h->levels[0].spec.ndof) return fail(h, MGMC_E_INVALID, "state size mismatch");
    if (chain < 0 || chain >= h->nchains) return fail(h, MGMC_E_INVALID, "chain index out of range");
    HIPCHK(h, hipSetDevice(h->device));
    return download(h, 0, h->levels[0].x + (size_t)chain * h->levels[0].L.nstore, x);
}

int mgmc_get_state(mgmc_handle* h, double* x, size_t n) { return mgmc_get_state_chain(h, 0, x, n); }

// the device-side non-finite guard (ctrl[5], set by k_qoi_record): MGMC_E_NONFINITE with the sample
// index and the watched vertex, instead of a chain that silently carries NaN / Inf
static int check_finite(mgmc_handle* h) {
    uint64_t flag = 0;
    HIPCHK(h, hipMemcpyAsync(&flag, h->ctrl + 5, sizeof(flag), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (flag == 0) return MGMC_OK;
    return fail(h, MGMC_E_NONFINITE,
                "non-finite chain state: the " +
                    std::string(h->qoi_store_index >= 0 ? "QoI vertex"
                                                        : (h->qoi_store_index == -2 ? "QoI vector's dot" : "lattice centre")) +
                    " became NaN / Inf in sample " + std::to_string(flag - 1) +
                    " (check the right-hand side, the low-rank Sigma and omega; mgmc_set_state clears the guard)");
}

static int set_qoi(mgmc_handle* h, int64_t qoi_index) {
    int64_t store = -1;
    if (qoi_index == MGMC_QOI_VECTOR) {
        if (h->qv_n == 0) return fail(h, MGMC_E_INVALID, "MGMC_QOI_VECTOR: no QoI vector installed (mgmc_set_qoi_vector)");
        store = -2;
    } else if (qoi_index < -1) {
        return fail(h, MGMC_E_INVALID, "qoi index out of range");
    } else if (qoi_index >= 0) {
        const Level& lv = h->levels[0];
        if ((uint64_t)qoi_index >= lv.spec.ndof) return fail(h, MGMC_E_INVALID, "qoi index out of range");
        const int nxi = lv.L.nx - 1, nyi = lv.L.ny - 1;
        const int i = (int)(qoi_index % nxi) + 1;
        const int j = (int)((qoi_index / nxi) % nyi) + 1;
        const int k = lv.spec.dim == 3 ? (int)(qoi_index / ((int64_t)nxi * nyi)) + 1 : 0;
        store = lv.L.at(i, j, k);
    }
    if (store != h->qoi_store_index) {
        HIPCHK(h, hipMemcpyAsync(h->ctrl + 2, &store, sizeof(int64_t), hipMemcpyHostToDevice, h->stream));
        HIPCHK(h, hipStreamSynchronize(h->stream));
        h->qoi_store_index = store;
    }
    return MGMC_OK;
}

int mgmc_apply(mgmc_handle* h, const double* f, double* x, size_t n) {
    if (!h || !f || !x) return fail(h, MGMC_E_INVALID, "null argument");
    if (h->unusable) return refuse_unusable(h);
    int rc = mgmc_set_rhs(h, f, n);
    if (rc) return rc;
    if ((rc = mgmc_set_state(h, x, n))) return rc;
    if ((rc = set_qoi(h, -1))) return rc;
    HIPCHK(h, hipGraphLaunch(h->graph_all, h->stream));
    if ((rc = mgmc_get_state(h, x, n))) return rc;
    return check_finite(h);
}

int mgmc_sample_async(mgmc_handle* h, int nsteps, int64_t qoi_index) {
    if (!h || nsteps < 0) return fail(h, MGMC_E_INVALID, "invalid argument");
    if (h->unusable) return refuse_unusable(h);
    HIPCHK(h, hipSetDevice(h->device));
    int rc = set_qoi(h, qoi_index);
    if (rc) return rc;
    // series restarts at 0 for each call
    HIPCHK(h, hipMemsetAsync(h->ctrl + 1, 0, sizeof(uint64_t), h->stream));
    if ((rc = ensure_series(h, (uint64_t)std::max(nsteps, 1)))) return rc;
    int s = 0;
    if (h->graph_unroll)
        for (; s + h->unroll <= nsteps; s += h->unroll) HIPCHK(h, hipGraphLaunch(h->graph_unroll, h->stream));
    for (; s < nsteps; ++s) HIPCHK(h, hipGraphLaunch(h->graph_all, h->stream));
    return MGMC_OK;
}

int mgmc_synchronize(mgmc_handle* h) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return check_finite(h);
}

int mgmc_sample(mgmc_handle* h, int nsteps, int64_t qoi_index, double* qoi_out) {
    int rc = mgmc_sample_async(h, nsteps, qoi_index);
    if (rc) return rc;
    if (qoi_out && nsteps > 0 && (qoi_index >= 0 || qoi_index == MGMC_QOI_VECTOR))
        HIPCHK(h, hipMemcpyAsync(qoi_out, h->series, nsteps * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return check_finite(h);
}

int mgmc_set_qoi_vector(mgmc_handle* h, int64_t nnz, const int64_t* rows, const double* vals) {
    if (!h || nnz < 0 || (nnz > 0 && (!rows || !vals))) return fail(h, MGMC_E_INVALID, "invalid argument");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    const Level& lv = h->levels[0];
    std::vector<long long> off((size_t)nnz);
    const int64_t nxi = lv.L.nx - 1, nyi = lv.L.ny - 1;
    for (int64_t e = 0; e < nnz; ++e) {
        if (rows[e] < 0 || (uint64_t)rows[e] >= lv.spec.ndof || (e > 0 && rows[e] <= rows[e - 1]))
            return fail(h, MGMC_E_INVALID, "QoI vector rows must be strictly ascending vertex indices");
        if (!std::isfinite(vals[e])) return fail(h, MGMC_E_INVALID, "non-finite QoI vector value");
        const int i = (int)(rows[e] % nxi) + 1, j = (int)((rows[e] / nxi) % nyi) + 1;
        const int k = lv.spec.dim == 3 ? (int)(rows[e] / (nxi * nyi)) + 1 : 0;
        off[(size_t)e] = lv.L.at(i, j, k);
    }
    if (h->qv_off) hipFree(h->qv_off);
    if (h->qv_val) hipFree(h->qv_val);
    if (h->qv_part) hipFree(h->qv_part);
    h->qv_off = nullptr;
    h->qv_val = nullptr;
    h->qv_part = nullptr;
    h->qv_n = 0;
    h->qv_nblk = 0;
    if (nnz > 0) {
        const int nblk = (int)((nnz + QV_BLK - 1) / QV_BLK);
        if (hipMalloc(&h->qv_off, nnz * sizeof(long long)) != hipSuccess ||
            hipMalloc(&h->qv_val, nnz * sizeof(double)) != hipSuccess ||
            hipMalloc(&h->qv_part, (size_t)nblk * h->nchains * sizeof(double)) != hipSuccess)
            return fail(h, MGMC_E_NOMEM, "device allocation failed (QoI vector)");
        HIPCHK(h, hipMemcpy(h->qv_off, off.data(), nnz * sizeof(long long), hipMemcpyHostToDevice));
        HIPCHK(h, hipMemcpy(h->qv_val, vals, nnz * sizeof(double), hipMemcpyHostToDevice));
        poison_fill(h, h->qv_part, (size_t)nblk * h->nchains * sizeof(double));
        h->qv_n = nnz;
        h->qv_nblk = nblk;
    }
    if (h->qoi_store_index == -2) {  // the vector mode ends with the vector
        int rc = set_qoi(h, -1);
        if (rc) return rc;
    }
    return build_graphs(h);
}

int mgmc_qoi_moments(mgmc_handle* h, double out[3]) { return mgmc_qoi_moments_chain(h, 0, out); }

int mgmc_qoi_moments_chain(mgmc_handle* h, int chain, double out[3]) {
    if (!h || !out) return fail(h, MGMC_E_INVALID, "null argument");
    if (chain < 0 || chain >= h->nchains) return fail(h, MGMC_E_INVALID, "chain index out of range");
    HIPCHK(h, hipSetDevice(h->device));
    double m[4];
    HIPCHK(h, hipMemcpyAsync(m, h->mom + 4 * chain, sizeof(m), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    out[0] = m[0];
    out[1] = m[1];
    out[2] = m[2];
    return MGMC_OK;
}

int mgmc_reset_moments(mgmc_handle* h) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemsetAsync(h->mom, 0, 4 * sizeof(double) * h->nchains, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_set_sample_index(mgmc_handle* h, uint64_t index) {
    if (!h) return fail(nullptr, MGMC_E_INVALID, "null handle");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemcpyAsync(h->ctrl, &index, sizeof(index), hipMemcpyHostToDevice, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_get_series(mgmc_handle* h, double* out, size_t n) { return mgmc_get_series_chain(h, 0, out, n); }

int mgmc_get_series_chain(mgmc_handle* h, int chain, double* out, size_t n) {
    if (!h || (!out && n > 0)) return fail(h, MGMC_E_INVALID, "null argument");
    if (n > h->series_cap) return fail(h, MGMC_E_INVALID, "more values than the series holds");
    if (chain < 0 || chain >= h->nchains) return fail(h, MGMC_E_INVALID, "chain index out of range");
    HIPCHK(h, hipSetDevice(h->device));
    if (n > 0)
        HIPCHK(h, hipMemcpyAsync(out, h->series + (size_t)chain * h->series_cap, n * sizeof(double),
                                 hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_get_sample_index(mgmc_handle* h, uint64_t* index) {
    if (!h || !index) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    HIPCHK(h, hipMemcpyAsync(index, h->ctrl, sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_get_stream(mgmc_handle* h, void** stream) {
    if (!h || !stream) return fail(h, MGMC_E_INVALID, "null argument");
    *stream = (void*)h->stream;
    return MGMC_OK;
}

// ---------------- component entry points ----------------

int mgmc_operator_apply(mgmc_handle* h, int level, const double* x, double* y) {
    int rc = check_level(h, level, false);
    if (rc) return rc;
    if (!x || !y) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level))) return rc;
    Level& lv = h->levels[level];
    if ((rc = upload(h, level, x, lv.scratch[0]))) return rc;
    launch_operator_apply(h, lv, lv.scratch[0], lv.scratch[1], h->stream);
    HIPCHK(h, hipGetLastError());
    return download(h, level, lv.scratch[1], y);
}

static int sweep_component(mgmc_handle* h, int level, int direction, int nsweeps, bool noise, uint32_t tag,
                           uint64_t sample, const double* b, double* x) {
    int rc = check_level(h, level, false);
    if (rc) return rc;
    if (!b || !x) return fail(h, MGMC_E_INVALID, "null argument");
    if (direction != MGMC_FORWARD && direction != MGMC_BACKWARD) return fail(h, MGMC_E_INVALID, "invalid direction");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level))) return rc;
    Level& lv = h->levels[level];
    if ((rc = upload(h, level, b, lv.scratch[0]))) return rc;
    if ((rc = upload(h, level, x, lv.scratch[1]))) return rc;
    HIPCHK(h, hipMemcpyAsync(h->ctrl + 3, &sample, sizeof(sample), hipMemcpyHostToDevice, h->stream));
    const bool lr = lv.lr.m > 0;
    int cur = 1;
    for (int s = 0; s < nsweeps; ++s) {
        GibbsArg g = make_gibbs(h, lv, tag + (uint32_t)s, 0, h->ctrl + 3);
        double* fb = lv.scratch[0];
        if (lr && noise) fb = lr_rhs(h, lv, LR_PATCH_NOISE, lv.scratch[0], tag + (uint32_t)s, h->ctrl + 3, h->stream);
        if (h->poison)  // (debug: as enqueue_ops) the sweep starts on NaN-filled LDS
            hipLaunchKernelGGL(k_lds_poison, dim3(8 * lv.num_cu), dim3(1024), LDS_POISON_DOUBLES * sizeof(double),
                               h->stream);
        if (noise && lv.zsweep) {  // the fused z-marching kernel of the V-cycle (out of place)
            launch_zsweep(lv, lv.scratch[cur], lv.scratch[3 - cur], fb, g, direction, nullptr, nullptr, 0.0, h->stream);
            cur = 3 - cur;
        } else if (noise && lv.quads) {  // two colour pairs per launch (out of place)
            launch_quads(lv, lv.scratch[cur], lv.scratch[3 - cur], fb, g, direction, h->stream);
            cur = 3 - cur;
        } else if (noise && lv.rb2d) {  // one-launch 2D red-black sweep (out of place)
            launch_rb2d(lv, lv.scratch[cur], lv.scratch[3 - cur], fb, g, direction, true, h->stream);
            cur = 3 - cur;
        } else if (noise && lv.pairs) {  // the colour-pair passes of the V-cycle (in place)
            launch_pairs(lv, lv.scratch[cur], fb, g, direction, h->stream);
        } else {
            launch_sweep(lv, lv.scratch[cur], fb, g, direction, noise, h->stream);
        }
        if (lr) lr_fix(lv, lv.scratch[cur], direction, noise && fb == lv.scratch[0] ? lv.scratch[0] : nullptr, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return download(h, level, lv.scratch[cur], x);
}

int mgmc_smoother_apply(mgmc_handle* h, int level, int direction, int nsweeps, const double* b, double* x) {
    return sweep_component(h, level, direction, nsweeps, false, 0, 0, b, x);
}

// noise-free sweeps on one level in a given order, the low-rank fix after the marked ones
// (the Smoother drop-ins below); x stays on the device between the sweeps
static int smoother_sequence(mgmc_handle* h, int level, const std::vector<std::pair<int, bool>>& seq,
                             const double* b, double* x) {
    int rc = check_level(h, level, false);
    if (rc) return rc;
    if (!b || !x) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level))) return rc;
    Level& lv = h->levels[level];
    if ((rc = upload(h, level, b, lv.scratch[0]))) return rc;
    if ((rc = upload(h, level, x, lv.scratch[1]))) return rc;
    for (const auto& st : seq) {
        GibbsArg g = make_gibbs(h, lv, 0, 0, h->ctrl + 3);
        launch_sweep(lv, lv.scratch[1], lv.scratch[0], g, st.first, false, h->stream);
        if (st.second && lv.lr.m > 0) lr_fix(lv, lv.scratch[1], st.first, nullptr, h->stream);
    }
    HIPCHK(h, hipGetLastError());
    return download(h, level, lv.scratch[1], x);
}

// nsmooth bound of the smoother drop-ins: SORSmoother::apply runs nsmooth^2 sweeps, so 1024 is a
// million sweeps; above it the sweep list (and nsmooth * nsmooth in int) would overflow
static constexpr int MAX_NSMOOTH = 1024;

int mgmc_sor_smoother_apply(mgmc_handle* h, int level, int direction, int nsmooth, const double* b, double* x) {
    if (direction != MGMC_FORWARD && direction != MGMC_BACKWARD) return fail(h, MGMC_E_INVALID, "invalid direction");
    if (nsmooth < 0 || nsmooth > MAX_NSMOOTH) return fail(h, MGMC_E_INVALID, "nsmooth must be in [0, 1024]");
    // SORSmoother::apply (sor_smoother.cc:41-53) over apply_sparse (:56-78): both loop nsmooth times
    std::vector<std::pair<int, bool>> seq;
    for (int k = 0; k < nsmooth; ++k)
        for (int j = 0; j < nsmooth; ++j) seq.push_back({direction, j == nsmooth - 1});
    return smoother_sequence(h, level, seq, b, x);
}

int mgmc_ssor_smoother_apply(mgmc_handle* h, int level, int nsmooth, const double* b, double* x) {
    if (nsmooth < 0 || nsmooth > MAX_NSMOOTH) return fail(h, MGMC_E_INVALID, "nsmooth must be in [0, 1024]");
    // SSORSmoother::apply (ssor_smoother.cc:9-15): its SORSmoothers have nsmooth 1 (ssor_smoother.hh:47-48)
    std::vector<std::pair<int, bool>> seq;
    for (int k = 0; k < nsmooth; ++k) {
        seq.push_back({MGMC_FORWARD, true});
        seq.push_back({MGMC_BACKWARD, true});
    }
    return smoother_sequence(h, level, seq, b, x);
}

int mgmc_sor_sampler_apply(mgmc_handle* h, int level, int direction, uint32_t sweep_tag, uint64_t sample_index,
                           const double* f, double* x) {
    return sweep_component(h, level, direction, 1, true, sweep_tag, sample_index, f, x);
}

int mgmc_restrict(mgmc_handle* h, int level, const double* r, double* rc_out) {
    int rc = check_level(h, level, true);
    if (rc) return rc;
    if (!r || !rc_out) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level)) || (rc = ensure_scratch(h, level + 1))) return rc;
    Level& lf = h->levels[level];
    Level& lc = h->levels[level + 1];
    if ((rc = upload(h, level, r, lf.scratch[0]))) return rc;
    dim3 block(64, 4, 1);
    dim3 grid = grid3(lc.L.nx - 1, lc.L.ny - 1, lf.spec.dim == 3 ? lc.L.nz - 1 : 1, block);
    if (lf.spec.dim == 3)
        hipLaunchKernelGGL((k_restrict<3>), grid, block, 0, h->stream, lf.L, lc.L, (const double*)lf.scratch[0],
                           lc.scratch[0]);
    else
        hipLaunchKernelGGL((k_restrict<2>), grid, block, 0, h->stream, lf.L, lc.L, (const double*)lf.scratch[0],
                           lc.scratch[0]);
    HIPCHK(h, hipGetLastError());
    return download(h, level + 1, lc.scratch[0], rc_out);
}

int mgmc_prolongate_add(mgmc_handle* h, int level, double alpha, const double* xc, double* x) {
    int rc = check_level(h, level, true);
    if (rc) return rc;
    if (!xc || !x) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level)) || (rc = ensure_scratch(h, level + 1))) return rc;
    Level& lf = h->levels[level];
    Level& lc = h->levels[level + 1];
    if ((rc = upload(h, level + 1, xc, lc.scratch[0]))) return rc;
    if ((rc = upload(h, level, x, lf.scratch[0]))) return rc;
    launch_prolongate(lf, lc, lf.scratch[0], lc.scratch[0], alpha, h->stream);
    HIPCHK(h, hipGetLastError());
    return download(h, level, lf.scratch[0], x);
}

int mgmc_residual_restrict(mgmc_handle* h, int level, const double* f, const double* x, double* fc) {
    int rc = check_level(h, level, true);
    if (rc) return rc;
    if (!f || !x || !fc) return fail(h, MGMC_E_INVALID, "null argument");
    HIPCHK(h, hipSetDevice(h->device));
    if ((rc = ensure_scratch(h, level)) || (rc = ensure_scratch(h, level + 1))) return rc;
    Level& lf = h->levels[level];
    Level& lc = h->levels[level + 1];
    if ((rc = upload(h, level, f, lf.scratch[0]))) return rc;
    if ((rc = upload(h, level, x, lf.scratch[1]))) return rc;
    double* fr = lf.scratch[0];
    if (lf.lr.m > 0) {  // f - B Sigma^{-1} B^T x, then the residual kernel
        lr_dots(lf, lf.scratch[1], LR_SCALE_INV, h->stream);
        fr = lr_rhs(h, lf, LR_PATCH_RESIDUAL, lf.scratch[0], 0, h->ctrl + 3, h->stream);
    }
    launch_residual_restrict(lf, lc, lf.scratch[1], fr, lc.scratch[0], lc.scratch[1], 1, h->stream);
    HIPCHK(h, hipGetLastError());
    return download(h, level + 1, lc.scratch[0], fc);
}

int mgmc_normals(mgmc_handle* h, uint64_t pair0, size_t n, uint32_t sweep_tag, uint64_t sample_index, double* out) {
    if (!h || !out) return fail(h, MGMC_E_INVALID, "null argument");
    if (n % 2) return fail(h, MGMC_E_INVALID, "n must be even");
    HIPCHK(h, hipSetDevice(h->device));
    int rc = ensure_lex(h, std::max<size_t>(n, 1));
    if (rc) return rc;
    const uint64_t npairs = n / 2;
    if (npairs) {
        hipLaunchKernelGGL(k_normals, dim3((unsigned)((npairs + 255) / 256)), dim3(256), 0, h->stream, h->key, pair0,
                           npairs, sweep_tag, sample_index, h->lex_tmp);
        HIPCHK(h, hipGetLastError());
        HIPCHK(h, hipMemcpyAsync(out, h->lex_tmp, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

int mgmc_time_fine_sweeps(mgmc_handle* h, int nsweeps, float* ms) {
    if (!h || !ms || nsweeps < 1) return fail(h, MGMC_E_INVALID, "invalid argument");
    HIPCHK(h, hipSetDevice(h->device));
    // the V-cycle's fine-level sweep dispatch, on scratch ping-pong copies of the state
    int rc = ensure_scratch(h, 0);
    if (rc) return rc;
    Level& lv = h->levels[0];
    HIPCHK(h, hipMemcpyAsync(lv.scratch[1], lv.x, lv.L.nstore * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    hipEvent_t e0, e1;
    HIPCHK(h, hipEventCreate(&e0));
    HIPCHK(h, hipEventCreate(&e1));
    HIPCHK(h, hipEventRecord(e0, h->stream));
    int cur = 1;
    for (int s = 0; s < nsweeps; ++s) {
        GibbsArg g = make_gibbs(h, lv, 0x80000000u + (uint32_t)s, 0, h->ctrl);
        const int dir = (s & 1) ? MGMC_BACKWARD : MGMC_FORWARD;
        if (lv.zsweep) {
            launch_zsweep(lv, lv.scratch[cur], lv.scratch[3 - cur], lv.f, g, dir, nullptr, nullptr, 0.0, h->stream);
            cur = 3 - cur;
        } else if (lv.rb2d) {
            launch_rb2d(lv, lv.scratch[cur], lv.scratch[3 - cur], lv.f, g, dir, true, h->stream);
            cur = 3 - cur;
        } else {
            launch_sweep(lv, lv.scratch[cur], lv.f, g, dir, true, h->stream);
        }
    }
    HIPCHK(h, hipEventRecord(e1, h->stream));
    HIPCHK(h, hipEventSynchronize(e1));
    HIPCHK(h, hipEventElapsedTime(ms, e0, e1));
    HIPCHK(h, hipGetLastError());
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return MGMC_OK;
}

int mgmc_sample_timed(mgmc_handle* h, int nsteps, int64_t qoi_index, double* total_ms, double* pre_ms, int* npre,
                      double* post_ms, int* npost) {
    return mgmc_sample_timed_stride(h, nsteps, 1, qoi_index, total_ms, pre_ms, npre, post_ms, npost);
}

#ifdef MGMC_TAIL_PROF
// timing builds only: the phase stamps of the last run of the first k_tail (wall clock, rate in kHz):
// out[0] start, out[1] after the LDS fill from HBM, out[2 + 2 o] after op o's right-hand sides (sweeps),
// out[3 + 2 o] after op o, out[2 + 2 nops] after the store; kinds[o] = 16 * level + TailKind
extern "C" int mgmc_debug_tail_profile(mgmc_handle* h, unsigned long long* out, int n, int* kinds, int* nops,
                                       int* rate_khz) {
    if (!h || !h->tail_prof) return fail(h, MGMC_E_UNSUPPORTED, "no tail profile");
    HIPCHK(h, hipStreamSynchronize(h->stream));
    HIPCHK(h, hipMemcpy(out, h->tail_prof, std::min(n, 256) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    *nops = (int)h->tail_prof_ops.size();
    for (int o = 0; o < *nops; ++o) kinds[o] = 16 * h->tail_prof_ops[o].level + h->tail_prof_ops[o].kind;
    HIPCHK(h, hipDeviceGetAttribute(rate_khz, hipDeviceAttributeWallClockRate, h->device));
    return MGMC_OK;
}
#endif

int mgmc_sample_timed_stride(mgmc_handle* h, int nsteps, int stride, int64_t qoi_index, double* total_ms,
                             double* pre_ms, int* npre, double* post_ms, int* npost) {
    if (!h || nsteps < 1 || stride < 1 || !total_ms || !pre_ms || !npre || !post_ms || !npost)
        return fail(h, MGMC_E_INVALID, "invalid argument");
    if (h->unusable) return refuse_unusable(h);
    if (h->levels.size() < 2) return fail(h, MGMC_E_UNSUPPORTED, "timed sampling needs nlevel >= 2");
    HIPCHK(h, hipSetDevice(h->device));
    int rc = set_qoi(h, qoi_index);
    if (rc) return rc;
    HIPCHK(h, hipMemsetAsync(h->ctrl + 1, 0, sizeof(uint64_t), h->stream));
    if ((rc = ensure_series(h, (uint64_t)nsteps))) return rc;
    // one graph launch per cycle; its five event-record nodes are re-targeted at this step's events
    // before the launch (boundaries: fine pre-sampler | coarse-grid correction | fine post-sampler |
    // QoI record)
    // every stride-th cycle runs the timed graph (the first and the last always), the others the plain
    // cycle graph: the event-record nodes cost ~5 us each, so sparse sampling of the segments keeps the
    // timed loop within ~0.5% of the plain one
    constexpr int NSEG = 5;
    std::vector<int> timed_steps;
    for (int s = 0; s < nsteps; ++s)
        if (s % stride == 0 || s == nsteps - 1) timed_steps.push_back(s);
    const int nt = (int)timed_steps.size();
    std::vector<hipEvent_t> ev(NSEG * (size_t)nt);
    for (auto& e : ev) HIPCHK(h, hipEventCreate(&e));
    // (runs of untimed cycles replay the unrolled graph where there is one, as the plain sample loop
    // does: one graph launch per cycle costs host time comparable to a small lattice's cycle)
    for (int s = 0, ti = 0; s < nsteps;) {
        if (ti < nt && timed_steps[ti] == s) {
            for (int q = 0; q < NSEG; ++q)
                HIPCHK(h, hipGraphExecEventRecordNodeSetEvent(h->graph_timed, h->timed_node[q], ev[NSEG * ti + q]));
            HIPCHK(h, hipGraphLaunch(h->graph_timed, h->stream));
            ++ti;
            ++s;
        } else if (h->graph_unroll && s + h->unroll <= (ti < nt ? timed_steps[ti] : nsteps)) {
            HIPCHK(h, hipGraphLaunch(h->graph_unroll, h->stream));
            s += h->unroll;
        } else {
            HIPCHK(h, hipGraphLaunch(h->graph_all, h->stream));
            ++s;
        }
    }
    HIPCHK(h, hipEventSynchronize(ev[NSEG * nt - 1]));
    float t = 0.f;
    double pre = 0.0, post = 0.0;
    for (int q = 0; q < nt; ++q) {
        HIPCHK(h, hipEventElapsedTime(&t, ev[NSEG * q], ev[NSEG * q + 1]));
        pre += t;
        HIPCHK(h, hipEventElapsedTime(&t, ev[NSEG * q + 2], ev[NSEG * q + 3]));
        post += t;
    }
    HIPCHK(h, hipEventElapsedTime(&t, ev[0], ev[NSEG * nt - 1]));
    *total_ms = t;  // from the first cycle's first event to the last cycle's last
    *pre_ms = pre;
    *post_ms = post;
    int cpre = 0, cpost = 0;
    for (size_t q = 0; q < h->ops.size(); ++q)
        if ((h->ops[q].kind == OP_SWEEP || h->ops[q].kind == OP_SWEEP_RESTRICT) &&
            h->ops[q].level == 0) {
            if (q < h->seg_end_pre) ++cpre;
            else if (q >= h->seg_begin_post && q < h->seg_end_post) ++cpost;
        }
    *npre = cpre * nt;
    *npost = cpost * nt;
    for (auto& e : ev) hipEventDestroy(e);
    return check_finite(h);
}

}  // extern "C"
