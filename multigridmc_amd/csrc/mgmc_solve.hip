// mgmc_solve.hip -- the exact-statistics engine: multigrid-preconditioned LoopSolver / CG on the device
// (mgmc_solve; linear_operator.hh:119-174 targets, multigrid_preconditioner.cc:74-109, loop_solver.cc:9-53).
#include "mgmc_internal.hpp"

// ---------------- exact-statistics engine: multigrid-preconditioned solvers ----------------
namespace {

// x = M f: one deterministic multigrid cycle from x = 0 (MultigridPreconditioner::solve,
// multigrid_preconditioner.cc:74-101) with the hierarchy's noise-free smoothers (B_bar fix
// included) and ncoarsesmooth SSOR sweeps on the coarsest level.  Levels >= 1 work in their
// scratch buffers; x of level 0 must be zero on entry.
void mg_precond(mgmc_handle* h, int level, double* x, double* f, hipStream_t s) {
    const mgmc_config& c = h->cfg;
    Level& lv = h->levels[level];
    auto sweep = [&](int dir) {
        GibbsArg g = make_gibbs(h, lv, 0, 0, h->ctrl + 3);
        launch_sweep(lv, x, f, g, dir, false, s);
        if (lv.lr.m > 0) lr_fix(lv, x, dir, nullptr, s);
    };
    if (level == (int)h->levels.size() - 1) {
        if (h->chol_n > 0) {  // exact coarse solve, as the reference's CholeskySolver
            launch_coarse_chol(h, lv, f, x, false, 0, h->ctrl + 3, s);
            return;
        }
        for (int t = 0; t < c.ncoarsesmooth; ++t) {
            sweep(MGMC_FORWARD);
            sweep(MGMC_BACKWARD);
        }
        return;
    }
    Level& lc = h->levels[level + 1];
    const int cycle_ = level > 0 ? c.cycle : 1;
    for (int j = 0; j < cycle_; ++j) {
        for (int t = 0; t < c.npresmooth; ++t) {
            sweep(MGMC_FORWARD);
            if (c.smoother == MGMC_SMOOTHER_SSOR) sweep(MGMC_BACKWARD);
        }
        double* fr = f;
        if (lv.lr.m > 0) {
            lr_dots(lv, x, LR_SCALE_INV, s);
            fr = lr_rhs(h, lv, LR_PATCH_RESIDUAL, f, 0, h->ctrl + 3, s);
        }
        launch_residual_restrict(lv, lc, x, fr, lc.scratch[1], lc.scratch[0], 1, s);  // zeroes x_{l+1}
        if (lv.lr.m > 0) lr_restore(lv, f, s);
        mg_precond(h, level + 1, lc.scratch[0], lc.scratch[1], s);
        launch_prolongate(lv, lc, x, lc.scratch[0], c.coarse_scaling, s);
        for (int t = 0; t < c.npostsmooth; ++t) {
            if (c.smoother == MGMC_SMOOTHER_SSOR) sweep(MGMC_FORWARD);
            sweep(MGMC_BACKWARD);
        }
    }
}

void dev_dot(mgmc_handle* h, const double* a, const double* b, int slot) {
    const long long n = h->levels[0].L.nstore;
    hipLaunchKernelGGL(k_dot_partial, dim3(SOLVE_NB), dim3(256), 0, h->stream, n, a, b, h->sv_part);
    hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(256), 0, h->stream, (const double*)h->sv_part, SOLVE_NB, h->sv_scal,
                       slot);
}

int host_scalar(mgmc_handle* h, int slot, double* v) {
    HIPCHK(h, hipMemcpyAsync(v, h->sv_scal + slot, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    return MGMC_OK;
}

}  // namespace

extern "C" {

int mgmc_solve(mgmc_handle* h, int method, const double* b, double* x, double rtol, double atol, int maxiter,
               int* iters, double* rnorm) {
    if (!h || !b || !x || !iters || !rnorm) return fail(h, MGMC_E_INVALID, "null argument");
    if (method != MGMC_SOLVER_LOOP && method != MGMC_SOLVER_CG) return fail(h, MGMC_E_INVALID, "invalid solver method");
    if (maxiter < 0) return fail(h, MGMC_E_INVALID, "maxiter must be >= 0");
    if (h->unusable) return refuse_unusable(h);
    HIPCHK(h, hipSetDevice(h->device));
    int rc;
    for (size_t l = 1; l < h->levels.size(); ++l)
        if ((rc = ensure_scratch(h, (int)l))) return rc;
    Level& l0 = h->levels[0];
    const long long n = l0.L.nstore;
    const size_t bytes = (size_t)n * sizeof(double);
    for (auto& p : h->sv) {
        if (!p) {
            if (hipMalloc(&p, bytes) != hipSuccess) {
                p = nullptr;
                return fail(h, MGMC_E_NOMEM, "device allocation failed (solver vectors)");
            }
            HIPCHK(h, hipMemsetAsync(p, 0, bytes, h->stream));
        }
    }
    // MultigridPreconditioner always solves the coarsest level exactly (Cholesky,
    // multigrid_preconditioner.cc:41-45): build the dense factors if the level is small enough
    if (h->chol_n == 0 && h->levels.back().spec.ndof <= 2048) {
        if ((rc = build_coarse_chol(h, h->lr_cols.empty() ? nullptr : &h->lr_cols, h->lr_sigma.data(),
                                    (int)h->lr_cols.size())))
            return rc;
    }
    if (!h->sv_scal) {
        HIPCHK(h, hipMalloc(&h->sv_scal, 16 * sizeof(double)));
        poison_fill(h, h->sv_scal, 16 * sizeof(double));
    }
    if (!h->sv_part) {
        HIPCHK(h, hipMalloc(&h->sv_part, SOLVE_NB * sizeof(double)));
        poison_fill(h, h->sv_part, SOLVE_NB * sizeof(double));
    }
    double *vb = h->sv[0], *vx = h->sv[1], *vr = h->sv[2], *vz = h->sv[3], *vp = h->sv[4], *vq = h->sv[5];
    hipStream_t s = h->stream;
    const dim3 gv(4096), bv(256);
    if ((rc = upload(h, 0, b, vb))) return rc;
    HIPCHK(h, hipMemsetAsync(vx, 0, bytes, s));
    dev_dot(h, vb, vb, 4);
    double bb = 0.0;
    if ((rc = host_scalar(h, 4, &bb))) return rc;
    const double r0 = sqrt(bb);
    *iters = 0;
    *rnorm = r0;
    if (r0 == 0.0) return download(h, 0, vx, x);
    if (method == MGMC_SOLVER_LOOP) {  // LoopSolver::apply (loop_solver.cc:9-53): x -= M (A x - b)
        for (int k = 0; k < maxiter; ++k) {
            launch_operator_apply(h, l0, vx, vq, s);
            hipLaunchKernelGGL(k_sub, gv, bv, 0, s, n, (const double*)vq, (const double*)vb, vr);
            dev_dot(h, vr, vr, 2);
            double rr;
            if ((rc = host_scalar(h, 2, &rr))) return rc;
            *rnorm = sqrt(rr);
            *iters = k;
            if (*rnorm / r0 < rtol && *rnorm < atol) break;
            HIPCHK(h, hipMemsetAsync(vz, 0, bytes, s));
            mg_precond(h, 0, vz, vr, s);
            hipLaunchKernelGGL(k_sub, gv, bv, 0, s, n, (const double*)vx, (const double*)vz, vx);
            *iters = k + 1;
        }
    } else {  // conjugate gradients preconditioned by the same multigrid cycle
        HIPCHK(h, hipMemcpyAsync(vr, vb, bytes, hipMemcpyDeviceToDevice, s));
        HIPCHK(h, hipMemsetAsync(vz, 0, bytes, s));
        mg_precond(h, 0, vz, vr, s);
        HIPCHK(h, hipMemcpyAsync(vp, vz, bytes, hipMemcpyDeviceToDevice, s));
        dev_dot(h, vr, vz, 0);  // rz
        for (int k = 0; k < maxiter; ++k) {
            launch_operator_apply(h, l0, vp, vq, s);
            dev_dot(h, vp, vq, 1);  // pq
            hipLaunchKernelGGL(k_axpy_ratio, gv, bv, 0, s, n, (const double*)h->sv_scal, (const double*)(h->sv_scal + 1),
                               1.0, (const double*)vp, vx);
            hipLaunchKernelGGL(k_axpy_ratio, gv, bv, 0, s, n, (const double*)h->sv_scal, (const double*)(h->sv_scal + 1),
                               -1.0, (const double*)vq, vr);
            dev_dot(h, vr, vr, 2);
            double rr;
            if ((rc = host_scalar(h, 2, &rr))) return rc;
            *rnorm = sqrt(rr);
            *iters = k + 1;
            if (*rnorm / r0 < rtol && *rnorm < atol) break;
            HIPCHK(h, hipMemsetAsync(vz, 0, bytes, s));
            mg_precond(h, 0, vz, vr, s);
            dev_dot(h, vr, vz, 3);  // rz_new
            hipLaunchKernelGGL(k_xpby_ratio, gv, bv, 0, s, n, (const double*)vz, (const double*)(h->sv_scal + 3),
                               (const double*)h->sv_scal, vp);
            HIPCHK(h, hipMemcpyAsync(h->sv_scal, h->sv_scal + 3, sizeof(double), hipMemcpyDeviceToDevice, s));
        }
    }
    HIPCHK(h, hipGetLastError());
    return download(h, 0, vx, x);
}

}  // extern "C"
