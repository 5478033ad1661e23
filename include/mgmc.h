/*
 * mgmc.h -- C-ABI boundary of the MI355X-native Multigrid Monte Carlo (MGMC) sampler.
 *
 * This is the drop-in boundary for the reference's `driver_mgmc` hot path
 * (nilsfriess/MultigridMC, all citations relative to its src/ directory):
 *
 *   Sampler::apply(f, x)                     sampler/sampler.hh:41           -> mgmc_apply / mgmc_sample
 *   Sampler::fix_rhs(f)                      sampler/sampler.hh:56           -> mgmc_set_rhs
 *   MultigridMCSampler ctor                  sampler/multigridmc_sampler.cc:8-100 -> mgmc_create
 *   MultigridMCSampler::sample(level)        sampler/multigridmc_sampler.cc:103-130 (one V/W-cycle per sample)
 *   SORSampler::apply                        sampler/sor_sampler.cc:37-59    -> mgmc_sor_sampler_apply
 *   SORSmoother::apply_sparse                smoother/sor_smoother.cc:56-78  -> mgmc_smoother_apply
 *   LinearOperator::apply                    linear_operator/linear_operator.hh:66-76 -> mgmc_operator_apply
 *   IntergridOperator::restrict              intergrid/intergrid_operator.hh:74-88    -> mgmc_restrict
 *   IntergridOperator::prolongate_add        intergrid/intergrid_operator.hh:106-120  -> mgmc_prolongate_add
 *   LinearOperator::coarsen (Galerkin RAP)   linear_operator/linear_operator.cc:10-23 -> mgmc_describe (stencils)
 *   measure_sampling_time QoI loop           driver_mgmc.cc:66-94            -> mgmc_sample + mgmc_qoi_moments
 *
 * Every function returns MGMC_OK (0) or a negative MGMC_E* code; the text of the last
 * error is available from mgmc_last_error(handle) (or mgmc_last_error(NULL) for errors
 * raised before a handle exists).  The reference prints and exit(-1)s instead
 * (e.g. sampler/multigridmc_sampler.cc:47-49); the C++ wrapper in mgmc_sampler.hh restores
 * that behaviour at the driver level.
 *
 * Vectors crossing this boundary as host pointers use the reference's layout: one double per
 * interior lattice vertex, numbered lexicographically with x fastest
 * (lattice/lattice3d.hh:126-135, lattice/lattice2d.hh:95-103).  Device-resident state uses
 * a padded zero-halo layout ("Data layout in HBM") and never leaves HBM unless a
 * get/apply call asks for it.
 */
#ifndef MGMC_H
#define MGMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGMC_ABI_VERSION 5

/* error codes */
#define MGMC_OK 0
#define MGMC_E_INVALID -1   /* invalid argument / configuration           */
#define MGMC_E_HIP -2       /* HIP runtime error (incl. no device)        */
#define MGMC_E_NOMEM -3     /* device allocation failed                   */
#define MGMC_E_UNSUPPORTED -4 /* feature not (yet) on the device path     */
#define MGMC_E_NONFINITE -5 /* the chain state became NaN / Inf (guard on the QoI vertex, or the
                               lattice centre without a QoI, checked after every cycle); the flag
                               stays set until mgmc_set_state */

/* smoother kinds (parameters.hh:145-174 MultigridParameters::smoother) */
#define MGMC_SMOOTHER_SOR 0   /* forward SOR pre-sampler, backward SOR post-sampler */
#define MGMC_SMOOTHER_SSOR 1  /* SSOR (forward+backward) pre- and post-sampler      */

/* coarse solvers (MultigridParameters::coarse_solver) */
#define MGMC_COARSE_SSOR 0
#define MGMC_COARSE_CHOLESKY 1 /* Cholesky factors of the coarsest level (cholesky_sampler.cc:9-41): dense inverses up to
                                  8192 unknowns, blocked banded solves above (rows of at most 4096 unknowns) */

/* fine-level operators (driver_mgmc.cc:414-425, PriorParameters::pde_model) */
#define MGMC_OPERATOR_FD 0  /* ShiftedLaplaceFDOperator: 5/7-point (shiftedlaplace_fd_operator.cc:9-57) */
#define MGMC_OPERATOR_FEM 1 /* ShiftedLaplaceFEMOperator: Q1 elements, 9/27-point
                               (shiftedlaplace_fem_operator.cc:9-145) */
#define MGMC_OPERATOR_SQUARED_FD 2 /* SquaredShiftedLaplaceFDOperator, 2D 13-point
                                      (squared_shiftedlaplace_fd_operator.cc:9-96); CSR path only */

/* correlation-length models (linear_operator/correlationlength_model.hh:45-112) */
#define MGMC_KAPPA_CONSTANT 0 /* kappa^2 = 1 / Lambda^2 */
#define MGMC_KAPPA_PERIODIC 1 /* Lambda(x) = L1 + L2 prod_d cos(pi x_d), L1/2 = (Lambda_max +/- Lambda_min)/2 */
#define MGMC_KAPPA_GIVEN 2    /* constant kappa^2 given directly (mgmc_config.kappa_sq's convention) */

/* sweep directions (smoother/sor_smoother.hh:14-18) */
#define MGMC_FORWARD 1
#define MGMC_BACKWARD 2

/* Plain-old-data configuration; mirrors the MultigridParameters / LatticeParameters /
 * ConstantCorrelationLengthModelParameters / PriorParameters fields of auxilliary/parameters.hh
 * that reach the hot path.  The fine operator is ShiftedLaplaceFDOperator or
 * ShiftedLaplaceFEMOperator with constant kappa^2 = 1/Lambda^2
 * (linear_operator/shiftedlaplace_fd_operator.cc:9-57, shiftedlaplace_fem_operator.cc:9-145,
 * correlationlength_model.hh:45-66).  Zero-initialise and set the fields: 0 in fine_operator is
 * the FD operator. */
typedef struct mgmc_config {
    int dim;            /* 2 or 3 */
    int nx, ny, nz;     /* cells per direction (nz ignored for dim=2) */
    int nlevel;         /* number of multigrid levels (>=1) */
    int cycle;          /* 1 = V-cycle, 2 = W-cycle, ... (applies below level 0) */
    int npresmooth;
    int npostsmooth;
    int ncoarsesmooth;
    int smoother;       /* MGMC_SMOOTHER_* */
    int coarse_solver;  /* MGMC_COARSE_* */
    int verbose;
    double omega;          /* overrelaxation factor of the Gibbs samplers */
    double coarse_scaling; /* factor on the prolongated coarse correction */
    double kappa_sq;       /* 1/Lambda^2 */
    int fine_operator;     /* MGMC_OPERATOR_* (ABI 2) */
    int pad_;
} mgmc_config;

/* Host-side description of one multigrid level (no device needed). */
typedef struct mgmc_level_desc {
    int nx, ny, nz;       /* cells per direction on this level (nz = 0 for 2D) */
    int npoints;          /* stencil points: 5/7 (fine FD) or 9/27 (fine FEM, Galerkin) */
    int ncolours;         /* colours of the Gibbs sweep: 2 (5/7-point) or 2^dim (9/27-point) */
    int varcoef;          /* 1: per-vertex coefficients (mgmc_create_csr); stencil = the centre row */
    uint64_t ndof;        /* number of interior unknowns */
    /* stencil coefficients indexed by offset (dz+1)*9 + (dy+1)*3 + (dx+1) (3D) or
     * (dy+1)*3 + (dx+1) (2D); entries outside the stencil are 0 */
    double stencil[27];
} mgmc_level_desc;

typedef struct mgmc_handle mgmc_handle;

/* ---- host-only helpers (no GPU touched) ---- */
int mgmc_abi_version(void);
/* Handles created and not yet destroyed in this process (any mgmc_create* variant).  A host
 * integration checks with it that its owners release their device state (the reference's
 * shared_ptr ownership). */
int mgmc_live_handles(void);
/* Validate cfg and fill out[0..nlevel-1] with the level hierarchy and Galerkin stencils.
 * Returns the number of levels (> 0) or a negative MGMC_E* code. */
int mgmc_describe(const mgmc_config* cfg, mgmc_level_desc* out, int max_levels);
const char* mgmc_last_error(const mgmc_handle* h);

/* ---- fine operators as matrices (ABI 3; host only, no GPU touched) ----
 * The reference's LinearOperator subclasses with any correlation-length model
 * (ShiftedLaplaceFDOperator shiftedlaplace_fd_operator.cc:9-57, ShiftedLaplaceFEMOperator
 * shiftedlaplace_fem_operator.cc:9-145, SquaredShiftedLaplaceFDOperator
 * squared_shiftedlaplace_fd_operator.cc:9-96; PeriodicCorrelationLengthModel
 * correlationlength_model.hh:68-112) assembled as their A_sparse: CSR, rows = interior vertices in
 * the lattice order (x fastest), columns ascending, entries summed as the reference sums them. */
typedef struct mgmc_operator_desc {
    int dim, nx, ny, nz;       /* lattice (nz ignored for dim = 2) */
    int pde;                   /* MGMC_OPERATOR_FD / _FEM / _SQUARED_FD */
    int kappa_model;           /* MGMC_KAPPA_CONSTANT / _PERIODIC */
    double Lambda;             /* constant model */
    double Lambda_min, Lambda_max; /* periodic model */
    double kappa_sq;           /* MGMC_KAPPA_GIVEN */
} mgmc_operator_desc;
/* rows and stored entries of the assembled matrix */
int mgmc_operator_csr_size(const mgmc_operator_desc* d, int64_t* nrow, int64_t* nnz);
/* fill rowptr[nrow + 1], col[nnz], val[nnz] */
int mgmc_operator_csr(const mgmc_operator_desc* d, int64_t* rowptr, int32_t* col, double* val);

/* The colouring mgmc_create_csr gives a level with this matrix (ABI 5; host only): 2 (red-black, a
 * fine level whose couplings are all axis neighbours), 4 / 8 (coordinate parities, other reach-1
 * levels) or 9 / 27 (coordinates mod 3, reach-2 levels).  cfg gives the level's lattice; level 0 is
 * the fine level.  Same validation as mgmc_create_csr. */
int mgmc_csr_colour_scheme(const mgmc_config* cfg, int level, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                           int* scheme);

/* The constant stencil of a matrix (ABI 5; host only): MGMC_OK and stencil[27] (offset order of
 * mgmc_level_desc) if every row of the CSR is that 3^d stencil truncated at the lattice boundary, in
 * ascending column order with bitwise equal values -- the matrix of a constant-coefficient operator
 * such as ShiftedLaplaceFDOperator / ShiftedLaplaceFEMOperator with a constant correlation length;
 * MGMC_E_UNSUPPORTED otherwise (use mgmc_create_csr).  A reference-side adapter calls this on
 * LinearOperator::get_sparse() (linear_operator.hh:93) to pick the stencil fast path. */
int mgmc_stencil_of_csr(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                        const double* val, double* stencil);

/* Host-side bounds check of one level's padded layout (ABI 5; host only; mgmc_create runs it on
 * every level of every handle).  families: MGMC_LAYOUT_* bits of the kernels that address the level;
 * reach: 1 (3^d couplings) or 2 (the squared FD operator's levels); zrestrict_cx: coarse points per
 * tile of the z-marching residual + restriction on this level (0: none).  legacy: bit 0 builds the
 * round-2 reach-2 layout without its margin rows / planes, bit 1 the unclamped restriction columns,
 * bit 2 a j-sweep grid 8 workgroups short (all wrong: kept so the test shows the check catches them).  MGMC_OK, or MGMC_E_INVALID
 * with the offending offset range in mgmc_last_error(NULL). */
#define MGMC_LAYOUT_POINT 1u
#define MGMC_LAYOUT_PAIRS 2u
#define MGMC_LAYOUT_ZSWEEP 4u
#define MGMC_LAYOUT_ZSWEEP_COARSE 8u
#define MGMC_LAYOUT_ZRESTRICT 16u
#define MGMC_LAYOUT_RB2D 32u
#define MGMC_LAYOUT_JSWEEP 64u     /* + a replay of the j-marching half-sweeps' whole grid (256 CUs) */
#define MGMC_LAYOUT_QRESTRICT 128u /* 2D fused last pre-sweep + residual + restriction */
int mgmc_check_layout(int dim, const int* n, int reach, unsigned families, int zrestrict_cx, int legacy);

/* ---- lifetime ---- */
int mgmc_create(const mgmc_config* cfg, int device, uint64_t seed, uint64_t chain_id, mgmc_handle** out);
/* A sampler on a fine operator given as a matrix (LinearOperator::A_sparse, linear_operator.hh:187):
 * CSR on cfg's lattice (rows = interior vertices, columns strictly ascending, a positive diagonal,
 * couplings at most 2 vertices apart per direction).  Every coarse level is the Galerkin product
 * R A R^T (linear_operator.cc:10-23) formed on the host; every level is swept with its own per-vertex
 * coefficients (2 colours for a 5/7-point fine level, 2^d for reach-1 levels, 3^d for reach-2
 * levels such as the squared FD operator's).  cfg.kappa_sq and cfg.fine_operator are ignored. */
int mgmc_create_csr(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                    const double* val, int device, uint64_t seed, uint64_t chain_id, mgmc_handle** out);
/* Batched chains (ABI 4): nchains (1..16) independent chains chain0, chain0+1, ... in one handle.
 * They share the hierarchy, the stencils and the low-rank data (B, B_bar); each keeps its own state
 * and right-hand side in HBM and its own Philox key make_key(seed, chain0 + c), so chain c draws
 * exactly what a single-chain handle with chain_id = chain0 + c draws (bitwise).  Every kernel of
 * the cycle covers all chains in one launch; the low-rank fix reads B_bar once per row for all
 * chains (x -= B_bar W, W = B^T X: the (N x m)(m x C) product of the batch, sor_smoother.cc:47-51).
 * The entry points below without _chain act on every chain (set_rhs, set_state: the same vector)
 * or on chain 0 (get_state, get_series, qoi_moments).  Replaces running several
 * MultigridMCSampler objects (driver_mgmc.cc:188-314 measure_convergence's chains). */
int mgmc_create_batch(const mgmc_config* cfg, int device, uint64_t seed, uint64_t chain0, int nchains,
                      mgmc_handle** out);
int mgmc_create_csr_batch(const mgmc_config* cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                          const double* val, int device, uint64_t seed, uint64_t chain0, int nchains,
                          mgmc_handle** out);
/* A sampler whose fine level is the constant stencil fine_stencil[27] (ABI 5; e.g. from
 * mgmc_stencil_of_csr): the stencil hierarchy of mgmc_create (Galerkin levels by stencil RAP, the
 * fused z-marching / pair-pass kernels) without a kappa^2.  Couplings only to axis neighbours:
 * red-black fine sweeps; otherwise 2^d colours.  cfg.kappa_sq and cfg.fine_operator are ignored. */
int mgmc_create_stencil_batch(const mgmc_config* cfg, const double* fine_stencil, int device, uint64_t seed,
                              uint64_t chain0, int nchains, mgmc_handle** out);
int mgmc_nchains(const mgmc_handle* h);
int mgmc_destroy(mgmc_handle* h);
int mgmc_level_desc_get(const mgmc_handle* h, int level, mgmc_level_desc* out);
/* The kernels this handle runs on a level (ABI 5), as text "sweep=<kernel>[;post_sweep=<kernel>]
 * [;residual_restrict=<kernel>][;noise=<source>][;lowrank=<path>]" -- for labels (bench.py) and profiles;
 * <source>: restriction | tail | restriction+tail -- sweeps of the level read Box-Muller pairs drawn by the
 * restriction launch before the first pre-sweep and / or a tail launch's spare workgroups;
 * <path> on a posterior level: small | rows | dense | dense,rhs_inplace */
int mgmc_level_kernels(const mgmc_handle* h, int level, char* out, size_t n);

/* ---- posterior operator Q = A + B Sigma^{-1} B^T (MeasuredOperator) ----
 * Replaces MeasuredOperator's B / Sigma (linear_operator/measured_operator.cc:9-49,
 * LinearOperator::get_B / get_Sigma, linear_operator.hh:187-197).  B is N x m in CSC form:
 * column k holds rows[colptr[k] .. colptr[k+1]) (reference vertex indices, strictly ascending)
 * with values vals[...]; sigma[k] > 0 is the diagonal of Sigma.  A column listing all N rows is a
 * dense column (the global average measurement).  Coarse levels get B_c = R B, Sigma_c = Sigma
 * (linear_operator.cc:10-23); every SOR smoother sets up its B_bar (sor_smoother.cc:17-37) here,
 * so the call costs 2 m noise-free sweeps per level.  From then on every sweep applies the
 * low-rank fix and noise, and residuals / operator applications include B Sigma^{-1} B^T.
 * m = 0 restores the prior operator.  1 <= m <= 64.  Invalid arguments (MGMC_E_INVALID from the
 * checks of m, colptr, rows, vals, sigma) leave the handle unchanged; a failure after them (a coarse
 * band the blocked Cholesky cannot take, the host work limit, an allocation) leaves the prior operator
 * (no low-rank part on any level, the prior's coarse factors) and returns the error code. */
int mgmc_set_lowrank(mgmc_handle* h, int m, const int64_t* colptr, const int64_t* rows, const double* vals,
                     const double* sigma);
/* m of the current low-rank part (LinearOperator::get_m_lowrank); *nrows_bbar = rows stored for
 * B_bar of (level, direction) */
int mgmc_lowrank_info(const mgmc_handle* h, int level, int direction, int* m, int64_t* nrows_bbar);
/* testing hook: the handle's next n builds of the coarse Cholesky factor fail with MGMC_E_NOMEM, so
 * tests can drive mgmc_set_lowrank's rollback (a failed restore leaves the handle refusing the cycle
 * and solver calls until a later mgmc_set_lowrank succeeds).  n = 0 clears it. */
int mgmc_debug_fail_coarse_factor(mgmc_handle* h, int n);

/* ---- Sampler interface (host buffers, reference layout) ---- */
int mgmc_set_rhs(mgmc_handle* h, const double* f, size_t n);       /* fix_rhs: f stays in HBM */
int mgmc_set_state(mgmc_handle* h, const double* x, size_t n);
int mgmc_get_state(mgmc_handle* h, double* x, size_t n);
int mgmc_set_state_chain(mgmc_handle* h, int chain, const double* x, size_t n);
int mgmc_get_state_chain(mgmc_handle* h, int chain, double* x, size_t n);
/* Sampler::apply(f, x): upload f and x, run one MGMC cycle, download x (PCIe inclusive). */
int mgmc_apply(mgmc_handle* h, const double* f, double* x, size_t n);

/* ---- device-resident sampling loop (the hot path) ----
 * Run nsteps MGMC cycles on the device-resident state.  After every cycle the QoI
 * z = x[qoi_index] (reference index, radius-0 measurement vector,
 * linear_operator/measured_operator.cc:74-91) is appended to a device time series and folded
 * into device-side running moments.  If qoi_out != NULL the nsteps values are copied back. */
int mgmc_sample(mgmc_handle* h, int nsteps, int64_t qoi_index, double* qoi_out);
/* qoi_index = MGMC_QOI_VECTOR records z = b^T x with the vector b of mgmc_set_qoi_vector (ABI 5). */
#define MGMC_QOI_VECTOR (-2)
/* The QoI vector b for qoi_index = MGMC_QOI_VECTOR: the radius > 0 measurement vector of
 * MeasuredOperator::measurement_vector (linear_operator/measured_operator.cc:92-171) that
 * driver_mgmc.cc:58-59, :76 dots with every sample.  nnz entries, rows strictly ascending (reference
 * vertex indices), values; nnz = 0 removes it.  The dot runs in the cycle graph in a fixed order
 * (4096-entry blocks, lane-strided sums, xor butterflies -- the low-rank dots' order): the state
 * stays in HBM.  Rebuilds the handle's graphs. */
int mgmc_set_qoi_vector(mgmc_handle* h, int64_t nnz, const int64_t* rows, const double* vals);
/* Enqueue nsteps cycles on the handle's stream without synchronising or copying back. */
int mgmc_sample_async(mgmc_handle* h, int nsteps, int64_t qoi_index);
int mgmc_synchronize(mgmc_handle* h);
/* out[0] = n, out[1] = mean, out[2] = M2 (sum of squared deviations) of the recorded QoI */
int mgmc_qoi_moments(mgmc_handle* h, double out[3]);
int mgmc_qoi_moments_chain(mgmc_handle* h, int chain, double out[3]);
int mgmc_reset_moments(mgmc_handle* h);
int mgmc_set_sample_index(mgmc_handle* h, uint64_t index);
int mgmc_get_sample_index(mgmc_handle* h, uint64_t* index);
/* Copy the QoI series recorded by the last mgmc_sample / mgmc_sample_async call (n values; waits
 * for the handle's stream).  With mgmc_sample_async on several handles this collects the series of
 * chains that ran concurrently (measure_convergence's batched chains, driver_mgmc.cc:188-314). */
int mgmc_get_series(mgmc_handle* h, double* out, size_t n);
int mgmc_get_series_chain(mgmc_handle* h, int chain, double* out, size_t n);
/* HIP stream (hipStream_t) the handle enqueues on */
int mgmc_get_stream(mgmc_handle* h, void** stream);

/* ---- component entry points (host buffers, reference layout) used by the parity tests ---- */
/* y = Q_level x  (LinearOperator::apply; Q = A + B Sigma^{-1} B^T once mgmc_set_lowrank ran) */
int mgmc_operator_apply(mgmc_handle* h, int level, const double* x, double* y);
/* deterministic multicolour SOR sweeps (SORSmoother::apply, no noise; with the B_bar fix) */
int mgmc_smoother_apply(mgmc_handle* h, int level, int direction, int nsweeps,
                        const double* b, double* x);
/* The Smoother drop-ins (include/reference_adapter/hip_sor_smoother.hh), noise-free multicolour sweeps:
 * SORSmoother::apply exactly as the reference nests it -- nsmooth x (nsmooth sweeps of apply_sparse,
 * then the B_bar fix once), smoother/sor_smoother.cc:41-53 over :56-78 -- so nsmooth^2 sweeps;
 * 0 <= nsmooth <= 1024, else MGMC_E_INVALID ... */
int mgmc_sor_smoother_apply(mgmc_handle* h, int level, int direction, int nsmooth, const double* b, double* x);
/* ... and SSORSmoother::apply (smoother/ssor_smoother.cc:9-15): nsmooth x (forward sweep + fix,
 * backward sweep + fix) */
int mgmc_ssor_smoother_apply(mgmc_handle* h, int level, int nsmooth, const double* b, double* x);
/* one noisy multicolour SOR Gibbs sweep with explicit RNG counter (SORSampler::apply, nsmooth=1) */
int mgmc_sor_sampler_apply(mgmc_handle* h, int level, int direction, uint32_t sweep_tag,
                           uint64_t sample_index, const double* f, double* x);
/* coarse = R r  (restrict, level -> level+1) */
int mgmc_restrict(mgmc_handle* h, int level, const double* r, double* rc);
/* x += alpha * P xc  (prolongate_add, level+1 -> level) */
int mgmc_prolongate_add(mgmc_handle* h, int level, double alpha, const double* xc, double* x);
/* fc = R (f - Q x)  (fused residual + restriction of multigridmc_sampler.cc:118-120) */
int mgmc_residual_restrict(mgmc_handle* h, int level, const double* f, const double* x, double* fc);
/* ---- exact-statistics engine (linear_operator.hh:119-174 targets at any lattice size) ----
 * x = Q^{-1} b with the multigrid preconditioner of MultigridPreconditioner
 * (preconditioner/multigrid_preconditioner.cc:74-109): one deterministic cycle of the handle's
 * hierarchy from x = 0 (its smoothers without noise, with the B_bar fix).  The coarsest level is
 * solved exactly with its Cholesky factors, as the reference's CholeskySolver, when the handle has
 * them (coarse_solver Cholesky, or a coarsest level of at most 2048 unknowns); otherwise it takes
 * ncoarsesmooth SSOR sweeps.  method MGMC_SOLVER_LOOP is the
 * reference's LoopSolver (solver/loop_solver.cc:9-53, x -= M(Qx - b)); MGMC_SOLVER_CG wraps the
 * same (symmetric) cycle in conjugate gradients.  Stops when ||r||/||b|| < rtol and ||r|| < atol
 * (the reference's test) or after maxiter iterations; *iters and *rnorm report the outcome.
 * Host buffers, reference layout; the chain state is untouched. */
#define MGMC_SOLVER_LOOP 0
#define MGMC_SOLVER_CG 1
int mgmc_solve(mgmc_handle* h, int method, const double* b, double* x, double rtol, double atol, int maxiter,
               int* iters, double* rnorm);
/* n standard normals of pair ids [pair0, pair0+n/2) for (sweep_tag, sample_index):
 * out[2p] = cos branch, out[2p+1] = sin branch of the Box-Muller pair p */
int mgmc_normals(mgmc_handle* h, uint64_t pair0, size_t n, uint32_t sweep_tag, uint64_t sample_index,
                 double* out);

/* ---- timing hooks for the roofline measurement (bench.py) ----
 * Run `nsweeps` noisy fine-level (level 0) Gibbs sweeps on the device state, bracketed by
 * HIP events recorded on the handle's own stream; *ms = elapsed milliseconds. */
int mgmc_time_fine_sweeps(mgmc_handle* h, int nsweeps, float* ms);
/* Same as mgmc_sample_async + synchronize, but each cycle is replayed as three graph segments
 * [fine pre-sampler | coarse-grid correction | fine post-sampler + QoI record] with HIP events
 * recorded between them on the handle's stream.  *total_ms = first-to-last event time of the nsteps
 * cycles; *pre_ms / *post_ms = summed time of the fine-level (level 0) pre- / post-sampler segments
 * (the post segment holds the sweep with the fused prolongation and the ~4 us QoI record);
 * *npre / *npost = number of fine-level sweeps they contain. */
int mgmc_sample_timed(mgmc_handle* h, int nsteps, int64_t qoi_index, double* total_ms, double* pre_ms, int* npre,
                      double* post_ms, int* npost);
/* The same with the segments timed on every stride-th cycle only (and the last); the other cycles
 * replay the plain cycle graph (ABI 5).  *npre / *npost count the timed sweeps. */
int mgmc_sample_timed_stride(mgmc_handle* h, int nsteps, int stride, int64_t qoi_index, double* total_ms,
                             double* pre_ms, int* npre, double* post_ms, int* npost);

/* ---- multi-GPU: one chain per rank, RCCL over xGMI for the final QoI reduction ----
 * (the reference is single-process; this is the only collective of the path) */
#define MGMC_UNIQUE_ID_BYTES 128
/* rank 0 creates the id and ships it to the other ranks (any host channel) */
int mgmc_comm_unique_id(unsigned char out[MGMC_UNIQUE_ID_BYTES]);
int mgmc_comm_init(mgmc_handle* h, int nranks, int rank, const unsigned char id[MGMC_UNIQUE_ID_BYTES]);
/* all ranks: out[3*(r*nchains + c) .. +2] = (n, mean, M2) of chain c of rank r's handle (device-side
 * QoI moments; 3 * nranks * mgmc_nchains(h) doubles) */
int mgmc_comm_allgather_moments(mgmc_handle* h, double* out);
/* all ranks: *value <- max over ranks (used for the max-over-ranks benchmark time) */
int mgmc_comm_allreduce_max(mgmc_handle* h, double* value);
/* device-side barrier over the communicator, followed by a stream synchronisation */
int mgmc_comm_barrier(mgmc_handle* h);
int mgmc_comm_destroy(mgmc_handle* h);
/* what the communicator really spans: *rccl_ranks = ncclCommCount (0 without a communicator),
 * *rccl_rank = ncclCommUserRank (-1 without one), *pci_bus_id = PCI bus id of the handle's device
 * (ranks that report the same id share one GPU, where RCCL cannot run). */
int mgmc_comm_info(const mgmc_handle* h, int* rccl_ranks, int* rccl_rank, int* pci_bus_id);

#ifdef __cplusplus
}
#endif

#endif /* MGMC_H */
