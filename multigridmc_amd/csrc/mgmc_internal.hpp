// mgmc_internal.hpp -- host-side state shared by the library's translation units: the handle
// (mgmc_handle: levels, op list, graphs, low-rank / Cholesky / solver / RCCL state), its per-level
// Level and LowRankDev, the kernel-path switches (MGMC_DISABLE), error helpers, and the launch /
// orchestration helpers one unit defines and another calls.
//   mgmc_capi.hip          launchers, the cycle's op list and graphs, create / destroy, the Sampler
//                          and component entry points
//   mgmc_chol_setup.hip    the coarsest level's Cholesky factors (build_coarse_chol)
//   mgmc_solve.hip         the exact-statistics engine (mgmc_solve)
//   mgmc_lowrank_setup.hip the low-rank posterior part (mgmc_set_lowrank)
//   mgmc_comm.hip          the RCCL communicator (mgmc_comm_*)
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mgmc.h"
#include "mgmc_hierarchy.hpp"
#include "mgmc_kernels.hpp"
#include "mgmc_zsweep.hpp"
#include "mgmc_tuning.hpp"
#include "mgmc_layout_check.hpp"
static_assert(MGMC_LAYOUT_POINT == mgmc::LF_POINT && MGMC_LAYOUT_PAIRS == mgmc::LF_PAIRS &&
                  MGMC_LAYOUT_ZSWEEP == mgmc::LF_ZSWEEP && MGMC_LAYOUT_ZSWEEP_COARSE == mgmc::LF_ZSWEEP_C &&
                  MGMC_LAYOUT_ZRESTRICT == mgmc::LF_ZRESTRICT && MGMC_LAYOUT_RB2D == mgmc::LF_RB2D &&
                  MGMC_LAYOUT_JSWEEP == mgmc::LF_JSWEEP && MGMC_LAYOUT_QRESTRICT == mgmc::LF_QRESTRICT,
              "layout family bits");
#include "mgmc_zrestrict.hpp"
#include "mgmc_tail.hpp"
#include "mgmc_gsweep.hpp"
#include "mgmc_qrestrict.hpp"
#include "mgmc_jsweep.hpp"
#include "mgmc_rb2d.hpp"
#include "mgmc_lowrank.hpp"
#include "mgmc_solver.hpp"
#include "mgmc_cholesky.hpp"
#include "mgmc_field.hpp"
#include "mgmc_operators.hpp"

using namespace mgmc;

namespace mgmc_host {

// the last error of any call (mgmc_last_error(nullptr)); defined in mgmc_capi.hip
void set_global_error(const std::string& s);

enum OpKind {
    OP_SWEEP = 0,
    OP_RESIDUAL_RESTRICT = 1,
    OP_PROLONGATE = 2,
    OP_COARSE_LDS = 3,
    OP_QOI = 4,
    OP_COPY = 5,
    OP_COARSE_CHOL = 6,
    OP_TAIL = 7,     // the sub-cycle of the coarsest levels in one workgroup (mgmc_tail.hpp)
    OP_SWEEP_RESTRICT = 8   // 2D Galerkin level: last pre-sweep + residual + restriction (mgmc_qrestrict.hpp)
};

struct Op {
    OpKind kind;
    int level;
    int direction;  // MGMC_FORWARD / MGMC_BACKWARD for sweeps
    uint32_t tag;   // first sweep tag
    int nsweeps;    // OP_COARSE_LDS
    int src = 0;    // buffer index read (x[src]); z-sweeps write x[1-src]
    int prolong = 0;  // z-sweep with fused prolongate-add of the coarser level's x
    int lr_next = 0;       // sweep on a small low-rank level: the patch of the next op, fused (LR_NEXT_*)
    uint32_t lr_next_tag = 0;
    int lr_skip_patch = 0;  // this op's low-rank patch was done by an earlier op's kernel
    int lr_post_patch = 0;  // OP_RESIDUAL_RESTRICT: the restore of f also patches the level's first post-sweep
    uint32_t lr_post_tag = 0;
    int lr_coarse_patch = 0;  // OP_RESIDUAL_RESTRICT: ... and the coarse level's first pre-sweep
    uint32_t lr_coarse_tag = 0;
    int tail = -1;           // OP_TAIL: index into mgmc_handle::tail_args
    int xzero = 0;           // OP_SWEEP: its input x is known zero (the restriction before it zeroed the level, nothing
                             // wrote it since): the kernel takes zeros instead of loading it (mark_zero_inputs);
                             // OP_RESIDUAL_RESTRICT: so the coarse x is not written at all
    int zpre = 0;            // OP_SWEEP_RESTRICT: also draws the next OP_COARSE_LDS's noise into mgmc_handle::zbuf;
                             // OP_COARSE_LDS: reads it from there; OP_RESIDUAL_RESTRICT: 1 + the index of
                             // the OP_TAIL after it whose noise its spare workgroups draw
    const double2* pnz = nullptr;  // OP_SWEEP: its Box-Muller pairs, drawn by an earlier launch (plan_drawn_noise)
    double2* pn_dst = nullptr;     // OP_RESIDUAL_RESTRICT: also draws the next op's (the coarse level's first
    uint32_t pn_tag = 0;           // pre-sweep's) pairs, tag pn_tag, into pn_dst
};


// Kernel-path switches.  Every default fast path has a general fallback (the same arithmetic, bitwise
// equal); MGMC_DISABLE=<comma list> turns fast paths off at mgmc_create so the variant tests
// (tests/test_gpu_parity.py test_variant_cycles_bitwise, test_gpu_lowrank.py) can run the fallbacks
// on shapes where the fast path would be taken.  Read once per handle; unknown tokens are an error.
enum PathFlag : uint32_t {
    PATH_NO_TAIL = 1u << 0,               // coarsest levels as separate launches instead of k_tail
    PATH_NO_FUSE_PROLONG = 1u << 1,       // separate prolongate-add pass before the first post-sweep
    PATH_NO_QUADS = 1u << 2,              // colour-pair passes instead of two pairs per launch
    PATH_NO_RB2D = 1u << 3,               // 2D fine level: colour passes instead of k_rb2d
    PATH_NO_ZSWEEP = 1u << 4,             // 3D fine level: colour passes instead of k_zsweep_rb7
    PATH_NO_PAIRS = 1u << 5,              // Galerkin levels: per-colour passes instead of pair passes
    PATH_NO_ZRESTRICT = 1u << 6,          // residual + restriction: per-point gather kernel
    PATH_NO_LR_SMALL = 1u << 7,           // low-rank fix: generic multi-launch path instead of k_lr_small
    PATH_NO_LR_MERGE = 1u << 8,           // low-rank: separate restore / patch launches around restriction
    PATH_NO_LR_DENSE = 1u << 9,           // dense low-rank column: the row lists over every vertex
    PATH_NO_CHOL_DENSE = 1u << 10,        // coarse Cholesky: the blocked banded solves at any size
    PATH_NO_JSWEEP = 1u << 11,            // 3D Galerkin levels of 64 / 128 pairs: colour-pair passes, not j-marching halves
    PATH_NO_QRESTRICT = 1u << 12,         // 2D Galerkin levels: last pre-sweep and residual + restriction as two launches
    PATH_NO_PROLONG_Z = 1u << 13,         // big 3D levels: the per-point prolongation instead of the z-marching one
    PATH_NO_XZERO = 1u << 14,             // the restriction zeroes x_{l+1} and its first pre-sweep loads it
    PATH_NO_FOLD = 1u << 15,              // 3D fold levels: residuals in the reference's CSR order, not fold27's
    PATH_NO_POST_NOISE = 1u << 16,        // every sweep draws its own noise (none drawn by a restriction / tail launch)
};

struct PathToken {
    const char* name;
    uint32_t flag;
};
constexpr PathToken kPathTokens[] = {
    {"tail", PATH_NO_TAIL},           {"fuse_prolong", PATH_NO_FUSE_PROLONG},
    {"quads", PATH_NO_QUADS},         {"rb2d", PATH_NO_RB2D},
    {"zsweep", PATH_NO_ZSWEEP},       {"pairs", PATH_NO_PAIRS},
    {"zrestrict", PATH_NO_ZRESTRICT}, {"lr_small", PATH_NO_LR_SMALL},
    {"lr_merge", PATH_NO_LR_MERGE},   {"lr_dense", PATH_NO_LR_DENSE},
    {"chol_dense", PATH_NO_CHOL_DENSE}, {"jsweep", PATH_NO_JSWEEP},
    {"qrestrict", PATH_NO_QRESTRICT}, {"prolong_z", PATH_NO_PROLONG_Z},
    {"xzero", PATH_NO_XZERO},         {"fold", PATH_NO_FOLD},
    {"post_noise", PATH_NO_POST_NOISE},
};

// parse MGMC_DISABLE; returns false (and the offending token in *bad) for an unknown token
inline bool read_path_flags(uint32_t* flags, std::string* bad) {
    *flags = 0;
    const char* e = getenv("MGMC_DISABLE");
    if (!e) return true;
    std::string list(e);
    size_t pos = 0;
    while (pos <= list.size()) {
        size_t end = list.find(',', pos);
        if (end == std::string::npos) end = list.size();
        const std::string tok = list.substr(pos, end - pos);
        if (!tok.empty()) {
            bool found = false;
            for (const PathToken& t : kPathTokens)
                if (tok == t.name) {
                    *flags |= t.flag;
                    found = true;
                }
            if (!found) {
                *bad = tok;
                return false;
            }
        }
        pos = end + 1;
    }
    return true;
}

// z-marching sweep tile shape (mgmc_zsweep.hpp): 32 x-pairs x TY rows, TY/2 core waves + 2 halo
// waves rounded up to a multiple of four (768 threads for TY 16); two workgroups per CU need <= 80
// VGPRs (6 waves per SIMD).  Values in mgmc_tuning.hpp, tuning history in DESIGN.md.
constexpr int ZS_XP = 32, ZS_TY = tune::ZS_TY, ZS_NT = zs_threads(ZS_TY), ZS_MINW = tune::ZS_MINW,
              ZS_TZ = tune::ZS_TZ, ZS_TYP = tune::ZS_TYP, ZS_NTP = zs_threads(ZS_TYP),
              ZS_MINWP = tune::ZS_MINWP, ZS_TZP = tune::ZS_TZP;

// device copy of a level's low-rank part (mgmc_lowrank.hpp); one allocation list, freed together
struct LowRankDev {
    int m = 0;
    int nblk = 0;                 // dot-product blocks over all columns
    LRColMeta* meta = nullptr;
    int* blk_col = nullptr;
    LRBlock* blk = nullptr;        // per dot-product block: column, range, value source, scales
    long long* ent_off = nullptr;  // sparse column entries: padded offsets, values
    double* ent_val = nullptr;
    double* dense_val = nullptr;   // dense columns: padded value arrays, L.nstore apart
    int nrows = 0;                 // rows of B: padded offsets, m coefficients, column masks, saved f
    long long* rows_off = nullptr;
    double* rows_coef = nullptr;
    uint64_t* rows_mask = nullptr;
    double* save = nullptr;
    int nbar[2] = {0, 0};          // B_bar rows, [0] forward [1] backward
    long long* bar_off[2] = {nullptr, nullptr};
    double* bar_val[2] = {nullptr, nullptr};
    double* sc_one = nullptr;      // dot scales: 1 (B^T x), 1/Sigma_k (Sigma^{-1} B^T x)
    double* sc_inv = nullptr;
    double* sq = nullptr;          // sqrt(1/Sigma_k)
    double* part = nullptr;        // block partials
    double* w = nullptr;           // m-vector of dots
    bool small = false;            // k_lr_small path (sparse columns, one block each, few rows)
    long long max_col_n = 0;       // most entries of one column
    int* t_ent_off = nullptr;      // the same offsets in k_tail's LDS layout (small levels)
    int* t_rows_off = nullptr;
    int* t_bar_off[2] = {nullptr, nullptr};
    // dense-column path (one dense column g, mgmc_lowrank.hpp k_lr_dense_*): the row lists above
    // hold only the local rows; the dense-only rows stream B_g / Y_g, and the patched right-hand
    // side goes to fe (nchains x L.nstore) instead of f
    bool dense_path = false;
    bool dense_const = false;     // ... its dense column is one number (LRColMeta::cflag): dense_cval
    double dense_cval = 0.0;
    int dense_slot = 0;           // ... its value array in dense_val
    int dense_g = -1;
    uint32_t* skip_b = nullptr;                 // bit p: not a dense-only row of the patch
    uint32_t* skip_y[2] = {nullptr, nullptr};   // bit p: not a dense-only row of B_bar (per direction)
    double* yg[2] = {nullptr, nullptr};         // column g of Y (padded, per direction)
    // ... or, when B_g is one number on a 5 / 7-point level, Y_g as a table: Y_g of a dense-only vertex
    // is a function of its colour and of which of its 2d neighbours exist (the solve from zero of a
    // constant right-hand side), so the update reads a 1-byte key per vertex and ytab[d][key]
    uint8_t* ykey = nullptr;
    double* ytab[2] = {nullptr, nullptr};
    double* minv_g[2] = {nullptr, nullptr};     // row g of Minv (per direction)
    double* fe = nullptr;
    double* fe2 = nullptr;                      // ... of the first post-sweep, written with the residual's
    // ... or, on a z-sweep level with B_g one number, read in place (LRRhsArg): f is patched in place
    // on the local rows (saved, restored: the row-list path's k_lr_patch / k_lr_restore_patch), and
    // the sweep / residual kernels add the dense-only patch e to f on the other rows (e per chain in
    // rhs_e: [c] the sweep's / residual's, [nchains + c] the first post-sweep's); fe, fe2 unused
    bool rhs_inplace = false;
    double* rhs_e = nullptr;
    // the split column of the row patches (mgmc_lowrank.hpp lr_row_patch): the level's one dense
    // column when every value of it is one number (dense_const), else -1
    int split_g = -1;
    long long nbar_all[2] = {0, 0};             // B_bar rows in total (local + dense-only with Y_g != 0)
    std::vector<void*> allocs;
};

struct Level {
    LevelSpec spec;
    Layout L;
    StencilArg S;
    double* x = nullptr;      // canonical state buffer
    double* x2 = nullptr;     // ping-pong partner (z-sweep levels only)
    double* f = nullptr;
    double* scratch[3] = {nullptr, nullptr, nullptr};
    size_t lds_bytes = 0;  // >0 if the whole-level LDS kernel can hold x and f
    int num_cu = 256;      // compute units of the handle's device (grid sizing; MI355X: 256)
    uint32_t paths = 0;    // PathFlag bits of the handle (MGMC_DISABLE)
    bool zsweep = false;   // fused z-marching red-black sweep available
    bool pairs = false;    // Galerkin level swept in colour-pair passes (mgmc_gsweep.hpp)
    bool quads = false;    // ... two pairs per launch, out of place (k_sweep_quads, or k_jsweep_half:)
    bool jsweep = false;   // ... j-marching half-sweeps (mgmc_jsweep.hpp)
    bool rb2d = false;     // 2D 5-point level: one-launch red-black sweep, out of place (k_rb2d)
    bool field = false;    // per-vertex coefficients (mgmc_create_csr, mgmc_field.hpp)
    bool sym = false;      // 27-point stencil bitwise reflection-symmetric: kernels fold it (stencil_coef<true>)
    bool fold = false;     // ... and its residuals take the class-folded sum (fold27; MGMC_DISABLE=fold: CSR order)
    FieldArg F;            // ... their device field, pattern and colouring
    double* rbuf = nullptr;  // ... residual scratch (padded layout, zero boundary)
    bool pingpong() const { return zsweep || quads || rb2d; }  // out-of-place sweeps: x <-> x2
    double* buf(int i) const { return i == 0 ? x : x2; }
    LowRankDev lr;
};

inline void free_lowrank(LowRankDev& lr) {
    for (void* p : lr.allocs) hipFree(p);
    lr = LowRankDev();
}

// handles alive in this process (mgmc_live_handles): every mgmc_handle counts itself (mgmc_capi.hip)
extern std::atomic<int> g_live_handles;
struct LiveHandleCount {
    LiveHandleCount() { g_live_handles.fetch_add(1); }
    ~LiveHandleCount() { g_live_handles.fetch_sub(1); }
    LiveHandleCount(const LiveHandleCount&) = delete;
    LiveHandleCount& operator=(const LiveHandleCount&) = delete;
};

}  // namespace mgmc_host

using namespace mgmc_host;

struct mgmc_handle {
    LiveHandleCount live;
    mgmc_config cfg;
    int device = 0;
    uint64_t seed = 0, chain = 0;   // chain = the first chain of a batch (mgmc_create_batch)
    int nchains = 1;                // chains of the batch: level vectors, QoI series and moments
                                    // are nchains copies, L.nstore / capacity / 4 doubles apart
    RngKey key;
    std::vector<Level> levels;
    hipStream_t stream = nullptr;
    uint64_t* ctrl = nullptr;       // [0] sample index [1] series length [2] qoi index [3] scratch sample
    double* mom = nullptr;          // running (n, mean, M2, pad) per chain
    double* series = nullptr;
    uint64_t series_cap = 0;
    double* lex_tmp = nullptr;      // staging buffer in reference layout (device)
    size_t lex_cap = 0;
    std::vector<Op> ops;            // one sample
    size_t seg_end_pre = 0, seg_begin_post = 0, seg_end_post = 0;  // fine-sweep segments
    hipGraphExec_t graph_all = nullptr;
    hipGraphExec_t graph_unroll = nullptr;  // unroll copies of the cycle in one graph (sample loops)
    // the cycle with four event-record nodes (before the fine pre-sampler, after it, before the fine
    // post-sampler, after the QoI record): mgmc_sample_timed points them at per-step events
    hipGraph_t graph_timed_src = nullptr;
    hipGraphExec_t graph_timed = nullptr;
    hipGraphNode_t timed_node[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipEvent_t timed_ev0[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    int unroll = 1;
    int64_t qoi_store_index = -1;   // padded offset of the QoI vertex, -1 none, -2 the QoI vector
    // QoI vector b (mgmc_set_qoi_vector): padded offsets, values, block partials [nchains][nblk]
    long long* qv_off = nullptr;
    double* qv_val = nullptr;
    double* qv_part = nullptr;
    long long qv_n = 0;
    int qv_nblk = 0;
    std::string last_error;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    double* comm_buf = nullptr;  // device scratch for collectives
    uint32_t paths = 0;          // PathFlag bits (MGMC_DISABLE)
    int unroll_override = 0;     // MGMC_GRAPH_UNROLL (cycles per sample-loop graph launch; 0 = by size)
    double2* zbuf = nullptr;           // the coarse SSOR sampler's pre-drawn Box-Muller pairs [chain][item]
    long long zbuf_n = 0;              // items per chain
    std::vector<TailArgs*> tail_args;  // device copies, one per OP_TAIL
    std::vector<size_t> tail_lds;      // dynamic LDS bytes per OP_TAIL
    std::vector<char> tail_sym;        // ... every level of it has a symmetric 27-point stencil (k_tail<3, true>)
    // per OP_TAIL: its sweeps' Box-Muller pairs, drawn by spare workgroups of the restriction launch
    // before it (nullptr: the tail draws them); the jobs (device) and items per chain
    std::vector<double2*> tail_zb;
    std::vector<TailNoiseJob*> tail_jobs;
    std::vector<int> tail_njobs;
    std::vector<long long> tail_zn;
    // per OP_TAIL: spare workgroups of its launch drawing the post-sweep noise jobs (plan_drawn_noise), and
    // the noise buffers of those jobs (one per level, freed with the tails)
    std::vector<int> tail_pn_wg;
    std::vector<double2*> pn_bufs;
    double* sv[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // solver: b x r z p q (level 0)
    double* sv_scal = nullptr;   // solver scalars
    double* sv_part = nullptr;   // reduction partials
    std::vector<LRColumn> lr_cols;  // low-rank columns of the coarsest level, and Sigma (for the factors)
    std::vector<double> lr_sigma;
    bool field_mode = false;     // hierarchy built from a matrix (mgmc_create_csr)
    CsrHost coarse_csr;          // ... and its coarsest level (dense Cholesky factors)
    int chol_n = 0;              // Cholesky factors of the coarsest level (mgmc_cholesky.hpp)
    double* chol_G = nullptr;    // dense: G and L^{-1}
    double* chol_Li = nullptr;
    int chol_B = 0, chol_nb = 0; // blocked banded (chol_B > 0): Cf, Cb, Df, Db in one allocation
    double* chol_blk = nullptr;
    bool unusable = false;       // a failed mgmc_set_lowrank could not restore the prior's coarse factor
    int debug_fail_chol = 0;     // testing hook (mgmc_debug_fail_coarse_factor): coarse-factor builds left to fail
    bool poison = false;         // MGMC_POISON=1: NaN-filled scratch allocations and LDS (debug, poison_fill)
    unsigned long long* tail_prof = nullptr;  // (timing builds, MGMC_TAIL_PROF: the first tail's phase stamps)
    std::vector<TailOp> tail_prof_ops;
};

#define HIPCHK(h, call)                                                                            \
    do {                                                                                             \
        hipError_t e_ = (call);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            std::string m_ = std::string("HIP error ") + hipGetErrorString(e_) + " at " #call;       \
            if (h) (h)->last_error = m_;                                                             \
            set_global_error(m_);                                                                    \
            return MGMC_E_HIP;                                                                       \
        }                                                                                            \
    } while (0)

inline int fail(mgmc_handle* h, int code, const std::string& msg) {
    if (h) h->last_error = msg;
    set_global_error(msg);
    return code;
}

// Debug poison (MGMC_POISON=1, read at mgmc_create*): every device buffer the library does not zero
// or fill completely at allocation (noise buffers, the QoI series, dot partials, staging, solver
// scratch) is filled with 0xFF bytes (a NaN pattern), and every op of a captured cycle graph is
// preceded by k_lds_poison, which fills the LDS of every CU with NaN.  A kernel that reads device
// memory or LDS that no kernel of the cycle wrote -- recycled allocations, the previous kernel's LDS
// -- then carries a NaN into the chain and the non-finite guard reports it (MGMC_E_NONFINITE).
inline void poison_fill(const mgmc_handle* h, void* p, size_t bytes) {
    if (h && h->poison && p && bytes) (void)hipMemsetAsync(p, 0xFF, bytes, h->stream);
}


// ---- helpers defined in mgmc_capi.hip and used by the other units ----
struct TailNoiseLaunch {  // spare workgroups of the launch draw a tail's noise (ZRestrictArgs)
    const TailNoiseJob* jobs;
    int njobs;
    double2* zb;
    long long zbs;
    RngKey key;
    uint32_t chain0, seed_hi;
    const uint64_t* sample;
};
// the workgroups of a 27-point residual + restriction also draw the coarse level's first pre-sweep's
// Box-Muller pairs (ZRestrictArgs::pn; plan_drawn_noise)
struct PreNoiseLaunch {
    PostNoiseJob job;
    RngKey key;
    const uint64_t* sample;
};
// the scale of the low-rank dots: LR_SCALE_ONE (B^T v) or LR_SCALE_INV (Sigma^{-1} B^T v) -- LRBlock::sc[sel]
enum LRScale { LR_SCALE_ONE = 0, LR_SCALE_INV = 1 };

namespace mgmc_host {
dim3 grid3(int nthreads_x, int nrows_y, int nz_blocks, dim3 block);
GibbsArg make_gibbs(const mgmc_handle* h, const Level& lv, uint32_t tag, int colour, const uint64_t* sample);
void launch_sweep(const Level& lv, double* x, const double* f, const GibbsArg& g0, int direction, bool noise,
                  hipStream_t s, int nch = 1);
bool zres_lrf_capable(const Level& lf, const Level& lc);
void launch_residual_restrict(const Level& lf, const Level& lc, const double* x, const double* f, double* fc,
                              double* xc, int zero_xc, hipStream_t s, int nch = 1, const TailNoiseLaunch* tn = nullptr,
                              bool skip_xc = false, const LRRhsArg* lr = nullptr, const PreNoiseLaunch* pn = nullptr);
bool zres_draws_noise(const Level& lf, const Level& lc);
void launch_prolongate(const Level& lf, const Level& lc, double* x, const double* xc, double alpha, hipStream_t s,
                       int nch = 1);
void lr_dots(const Level& lv, const double* v, LRScale scale, hipStream_t s, int nch = 1);
double* lr_rhs(const mgmc_handle* h, const Level& lv, int mode, double* f, uint32_t tag, const uint64_t* sample,
               hipStream_t s, int nch = 1, int64_t post_tag = -1, LRRhsArg* inplace = nullptr);
void lr_fix(const Level& lv, double* x, int direction, double* f_restore, hipStream_t s, int nch = 1);
void lr_restore(const Level& lv, double* f, hipStream_t s, int nch = 1, bool patched = false);
void launch_operator_apply(const mgmc_handle* h, const Level& lv, const double* xs, double* ys, hipStream_t s);
void launch_coarse_chol(const mgmc_handle* h, const Level& lv, const double* f, double* x, bool noise, uint32_t tag,
                        const uint64_t* sample, hipStream_t s, int nch = 1);
Layout tail_layout(const Layout& L);
void build_ops(mgmc_handle* h);
int build_tails(mgmc_handle* h);
int build_graphs(mgmc_handle* h);
void destroy_graphs(mgmc_handle* h);
int ensure_scratch(mgmc_handle* h, int level);
int upload(mgmc_handle* h, int level, const double* host, double* pad);
int download(mgmc_handle* h, int level, const double* pad, double* host);
int refuse_unusable(mgmc_handle* h);
int check_level(mgmc_handle* h, int level, bool need_coarser);
// mgmc_chol_setup.hip
int build_coarse_chol(mgmc_handle* h, const std::vector<LRColumn>* cols, const double* sigma, int m);
}  // namespace mgmc_host
