// mgmc_sampler.hh -- header-only C++ host side over the C-ABI in mgmc.h.
//
// Mirrors the reference's Sampler plugin contract (nilsfriess/MultigridMC src/sampler/sampler.hh:23-72)
// with plain buffers instead of Eigen vectors, so that it compiles without Eigen:
//
//   Sampler::apply(f, x)          sampler/sampler.hh:41     -> HipMultigridMCSampler::apply
//   Sampler::fix_rhs / unfix_rhs  sampler/sampler.hh:56,63  -> fix_rhs / unfix_rhs
//   MultigridMCSampler ctor       sampler/multigridmc_sampler.cc:8-100 (MultigridParameters,
//                                 auxilliary/parameters.hh:145-174)
//   Smoother::apply(b, x)         smoother/smoother.hh:15-34 -> HipMulticolourSORSmoother::apply
//
// Error behaviour matches the reference at the driver level: every failing C-ABI call prints the
// library's message and calls exit(-1) (cf. sampler/multigridmc_sampler.cc:47-49).  The reference-side
// adapter `class HipMultigridMCSampler : public Sampler` that forwards Eigen vectors to this class is
// shown in INTEGRATION.md.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "mgmc.h"

namespace mgmc {

inline void check(int rc, const mgmc_handle* h, const char* what) {
    if (rc < 0) {  // mgmc_describe returns the level count, everything else MGMC_OK
        std::fprintf(stderr, "ERROR: %s failed (%d): %s\n", what, rc, mgmc_last_error(h));
        std::exit(-1);
    }
}

// Field-for-field the MultigridParameters of auxilliary/parameters.hh:145-174 (strings as enums).
struct MultigridParameters {
    int nlevel = 2;
    int smoother = MGMC_SMOOTHER_SOR;      // "SOR" / "SSOR"
    int coarse_solver = MGMC_COARSE_SSOR;  // "SSOR" / "Cholesky"
    int npresmooth = 1;
    int npostsmooth = 1;
    int ncoarsesmooth = 1;
    double omega = 1.0;
    int cycle = 1;
    double coarse_scaling = 1.0;
    int verbose = 0;
};

// fine_operator: MGMC_OPERATOR_FD (pdemodel "shiftedlaplace_fd") or MGMC_OPERATOR_FEM ("shiftedlaplace_fem")
inline mgmc_config make_config(int dim, int nx, int ny, int nz, double kappa_sq, const MultigridParameters& p,
                               int fine_operator = MGMC_OPERATOR_FD) {
    mgmc_config c{};
    c.fine_operator = fine_operator;
    c.dim = dim;
    c.nx = nx;
    c.ny = ny;
    c.nz = dim == 3 ? nz : 0;
    c.nlevel = p.nlevel;
    c.cycle = p.cycle;
    c.npresmooth = p.npresmooth;
    c.npostsmooth = p.npostsmooth;
    c.ncoarsesmooth = p.ncoarsesmooth;
    c.smoother = p.smoother;
    c.coarse_solver = p.coarse_solver;
    c.verbose = p.verbose;
    c.omega = p.omega;
    c.coarse_scaling = p.coarse_scaling;
    c.kappa_sq = kappa_sq;
    return c;
}

// One MGMC chain on one GPU.  apply(f, x) = one cycle = one sample, like the reference's
// MultigridMCSampler::apply (sampler/multigridmc_sampler.cc:132-138).
class HipMultigridMCSampler {
   public:
    // nchains > 1: a batch of chains chain_id .. chain_id + nchains - 1 in one handle
    // (mgmc_create_batch); apply / set_state act on every chain, the *_chain accessors on one
    HipMultigridMCSampler(const mgmc_config& cfg, int device, uint64_t seed, uint64_t chain_id = 0, int nchains = 1) {
        mgmc_handle* h = nullptr;
        check(mgmc_create_batch(&cfg, device, seed, chain_id, nchains, &h), nullptr, "mgmc_create");
        adopt(h);
    }
    // fine level given as a constant 3^d stencil (mgmc_create_stencil_batch, e.g. from mgmc_stencil_of_csr)
    HipMultigridMCSampler(const mgmc_config& cfg, const double* fine_stencil, int device, uint64_t seed,
                          uint64_t chain_id = 0, int nchains = 1) {
        mgmc_handle* h = nullptr;
        check(mgmc_create_stencil_batch(&cfg, fine_stencil, device, seed, chain_id, nchains, &h), nullptr,
              "mgmc_create_stencil");
        adopt(h);
    }
    // fine level given as a matrix, LinearOperator::A_sparse (mgmc_create_csr_batch)
    HipMultigridMCSampler(const mgmc_config& cfg, int64_t nrow, const int64_t* rowptr, const int32_t* col,
                          const double* val, int device, uint64_t seed, uint64_t chain_id = 0, int nchains = 1) {
        mgmc_handle* h = nullptr;
        check(mgmc_create_csr_batch(&cfg, nrow, rowptr, col, val, device, seed, chain_id, nchains, &h), nullptr,
              "mgmc_create_csr");
        adopt(h);
    }
    size_t get_ndof() const { return ndof_; }
    mgmc_handle* handle() const { return h_.get(); }

    // Sampler::apply(f, x): x in/out on the host (PCIe inclusive).  Without a fixed rhs, f is uploaded
    // and used.  After fix_rhs, f = nullptr or a vector equal to the fixed one skips the upload; any
    // other f is used, as the reference uses the f it is given (MultigridMCSampler keeps
    // Sampler::fix_rhs a no-op, sampler/sampler.hh:56), and becomes the resident fixed rhs.
    // multigridmc_amd/sampler.py MultigridMCSampler.apply behaves the same.
    void apply(const double* f, double* x) const {  // const like Sampler::apply (sampler.hh:41)
        if (rhs_fixed_ && f && std::memcmp(f, fixed_.data(), ndof_ * sizeof(double)) != 0) set_fixed(f);
        if (rhs_fixed_) {
            check(mgmc_set_state(h_.get(), x, ndof_), h_.get(), "mgmc_set_state");
            check(mgmc_sample(h_.get(), 1, -1, nullptr), h_.get(), "mgmc_sample");
            check(mgmc_get_state(h_.get(), x, ndof_), h_.get(), "mgmc_get_state");
        } else {
            check(mgmc_apply(h_.get(), f, x, ndof_), h_.get(), "mgmc_apply");
        }
    }
    void fix_rhs(const double* f) { set_fixed(f); }
    void unfix_rhs() {
        rhs_fixed_ = false;
        fixed_.clear();
    }
    // Posterior operator (MeasuredOperator, measured_operator.cc:9-49): B as CSC (m columns, rows
    // ascending), Sigma diagonal; m = 0 drops it.  Sets up every level's B_bar (sor_smoother.cc:17-37).
    void set_lowrank(int m, const int64_t* colptr, const int64_t* rows, const double* vals, const double* sigma) {
        check(mgmc_set_lowrank(h_.get(), m, colptr, rows, vals, sigma), h_.get(), "mgmc_set_lowrank");
    }

    // Device-resident sampling loop (driver_mgmc.cc:66-94): nsteps cycles, QoI x[qoi_index] recorded
    // after each; the state never leaves HBM.
    std::vector<double> sample(int nsteps, int64_t qoi_index) const {
        std::vector<double> q((size_t)nsteps);
        check(mgmc_sample(h_.get(), nsteps, qoi_index, q.data()), h_.get(), "mgmc_sample");
        return q;
    }
    void set_state(const double* x) { check(mgmc_set_state(h_.get(), x, ndof_), h_.get(), "mgmc_set_state"); }
    void get_state(double* x) const { check(mgmc_get_state(h_.get(), x, ndof_), h_.get(), "mgmc_get_state"); }
    // (n, mean, M2) of the recorded QoI
    void qoi_moments(double out[3]) const { check(mgmc_qoi_moments(h_.get(), out), h_.get(), "mgmc_qoi_moments"); }
    // one chain of a batch
    int nchains() const { return mgmc_nchains(h_.get()); }
    void get_state(int chain, double* x) const {
        check(mgmc_get_state_chain(h_.get(), chain, x, ndof_), h_.get(), "mgmc_get_state_chain");
    }
    void qoi_moments(int chain, double out[3]) const {
        check(mgmc_qoi_moments_chain(h_.get(), chain, out), h_.get(), "mgmc_qoi_moments_chain");
    }

   private:
    void adopt(mgmc_handle* h) {
        h_.reset(h);
        mgmc_level_desc d{};
        check(mgmc_level_desc_get(h_.get(), 0, &d), h_.get(), "mgmc_level_desc_get");
        ndof_ = (size_t)d.ndof;
    }
    struct Deleter {
        void operator()(mgmc_handle* h) const { mgmc_destroy(h); }
    };
    std::unique_ptr<mgmc_handle, Deleter> h_;
    size_t ndof_ = 0;
    // the fixed rhs: resident in HBM plus a host copy that apply compares its f with (mutable like the
    // reference sampler's scratch, sampler/multigridmc_sampler.hh:66-72)
    mutable bool rhs_fixed_ = false;
    mutable std::vector<double> fixed_;
    void set_fixed(const double* f) const {
        check(mgmc_set_rhs(h_.get(), f, ndof_), h_.get(), "mgmc_set_rhs");
        fixed_.assign(f, f + ndof_);
        rhs_fixed_ = true;
    }
};

// Deterministic multicolour SOR smoother on level `level` of a sampler's hierarchy
// (SORSmoother::apply, smoother/sor_smoother.cc:56-78; direction smoother/sor_smoother.hh:14-18).
class HipMulticolourSORSmoother {
   public:
    HipMulticolourSORSmoother(const HipMultigridMCSampler& s, int level, int direction, int nsweeps = 1)
        : h_(s.handle()), level_(level), direction_(direction), nsweeps_(nsweeps) {}
    void apply(const double* b, double* x) const {
        check(mgmc_smoother_apply(h_, level_, direction_, nsweeps_, b, x), h_, "mgmc_smoother_apply");
    }

   private:
    mgmc_handle* h_;
    int level_, direction_, nsweeps_;
};

}  // namespace mgmc
