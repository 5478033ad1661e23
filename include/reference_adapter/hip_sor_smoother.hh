// hip_sor_smoother.hh -- reference-side adapter: the MI355X multicolour SOR / SSOR smoothers as
// `Smoother`s of nilsfriess/MultigridMC.  A maintainer drops this file into the reference as
// src/smoother/hip_sor_smoother.hh next to hip_multigridmc_sampler.hh and
// links -lmgmc_hip.
//
// Written against the reference's own interfaces (citations relative to its src/):
//   Smoother / SmootherFactory   smoother/smoother.hh:15-44 (apply :29, get :43)
//   Direction                    smoother/sor_smoother.hh:14-18
//   SORSmoother(op, omega, nsmooth, direction)   smoother/sor_smoother.hh:53-60, sor_smoother.cc:9-78
//   SORSmootherFactory(omega, nsmooth, direction)   smoother/sor_smoother.hh:91-125
//   SSORSmoother(op, omega, nsmooth), SSORSmootherFactory   smoother/ssor_smoother.hh:31-100,
//                                                           ssor_smoother.cc:9-15
//
// Semantics kept from the reference:
//   * apply(b, x) is SORSmoother::apply exactly as the reference nests it: nsmooth x (apply_sparse =
//     nsmooth sweeps, then the low-rank update x -= B_bar (B^T x) once) -- nsmooth^2 sweeps in all
//     (sor_smoother.cc:41-53 loops nsmooth times over apply_sparse, which loops nsmooth times, :64);
//   * SSORSmoother::apply: nsmooth x (forward SORSmoother::apply, backward SORSmoother::apply), its
//     two SORSmoothers built with nsmooth 1 (ssor_smoother.hh:47-48);
//   * a MeasuredOperator's low-rank part (get_m_lowrank() > 0) gets its B_bar update after the
//     sweeps, B_bar set up once per direction at construction (sor_smoother.cc:17-37);
//   * errors print and exit(-1).
// Deliberate deviation: the sweeps are multicolour (red-black on 5/7-point
// levels, 2^d colours on 3^d-point ones; forward = colours ascending, backward = descending) instead
// of lexicographic, and B_bar is the one of the multicolour splitting.  Both leave the solution of
// A x = b invariant (smoother/test_smoother.hh:90-114), which tests/test_gpu_smoother.py checks.
//
// Each smoother owns a one-level device handle of its operator (the stencil or the matrix path, as
// HipMultigridMCSampler chooses it); apply moves b and x over PCIe like the reference's by-reference
// Eigen vectors.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <memory>

#include "hip_multigridmc_sampler.hh"
#include "smoother/smoother.hh"
#include "smoother/sor_smoother.hh"

namespace hip_smoother_detail {
// the operator as a one-level hierarchy: level 0 is the operator itself, its smoother is what apply runs
inline std::unique_ptr<mgmc::HipMultigridMCSampler> one_level(const LinearOperator& op, double omega, int device) {
    MultigridParameters p;
    p.nlevel = 1;
    p.smoother = "SOR";
    p.coarse_solver = "SSOR";
    p.npresmooth = 1;
    p.npostsmooth = 1;
    p.ncoarsesmooth = 1;
    p.omega = omega;
    p.cycle = 1;
    p.coarse_scaling = 1.0;
    p.verbose = 0;
    // (the seed only keys the noise of sampling, which a smoother never draws)
    return HipMultigridMCSampler::make_impl(op, p, device, HipMultigridMCSampler::default_seed, 0, 1);
}
inline void check_sizes(const char* who, const Eigen::VectorXd& b, const Eigen::VectorXd& x, size_t ndof) {
    if ((size_t)b.size() != ndof || (size_t)x.size() != ndof) {
        std::fprintf(stderr, "ERROR: %s::apply: vector size %td / %td, operator %zu\n", who, b.size(), x.size(), ndof);
        std::exit(-1);
    }
}
}  // namespace hip_smoother_detail

class HipSORSmoother : public Smoother {
   public:
    typedef Smoother Base;
    HipSORSmoother(const std::shared_ptr<LinearOperator> linear_operator_, const double omega_, const int nsmooth_,
                   const Direction direction_, int device = 0)
        : Base(linear_operator_), omega(omega_), nsmooth(nsmooth_), direction(direction_),
          impl(hip_smoother_detail::one_level(*linear_operator_, omega_, device)) {
        if (direction_ != forward && direction_ != backward) {
            std::fprintf(stderr, "ERROR: HipSORSmoother: invalid direction %d\n", (int)direction_);
            std::exit(-1);
        }
    }
    // SORSmoother::apply (sor_smoother.cc:41-53): b in, x in/out
    void apply(const Eigen::VectorXd& b, Eigen::VectorXd& x) const override {
        hip_smoother_detail::check_sizes("HipSORSmoother", b, x, impl->get_ndof());
        const int dir = direction == forward ? MGMC_FORWARD : MGMC_BACKWARD;
        mgmc::check(mgmc_sor_smoother_apply(impl->handle(), 0, dir, nsmooth, b.data(), x.data()), impl->handle(),
                    "mgmc_sor_smoother_apply");
    }
    mgmc_handle* handle() const { return impl->handle(); }

   protected:
    const double omega;
    const int nsmooth;
    const Direction direction;
    std::unique_ptr<mgmc::HipMultigridMCSampler> impl;
};

class HipSSORSmoother : public Smoother {
   public:
    typedef Smoother Base;
    HipSSORSmoother(const std::shared_ptr<LinearOperator> linear_operator_, const double omega_, const int nsmooth_,
                    int device = 0)
        : Base(linear_operator_), nsmooth(nsmooth_), impl(hip_smoother_detail::one_level(*linear_operator_, omega_, device)) {}
    // SSORSmoother::apply (ssor_smoother.cc:9-15)
    void apply(const Eigen::VectorXd& b, Eigen::VectorXd& x) const override {
        hip_smoother_detail::check_sizes("HipSSORSmoother", b, x, impl->get_ndof());
        mgmc::check(mgmc_ssor_smoother_apply(impl->handle(), 0, nsmooth, b.data(), x.data()), impl->handle(),
                    "mgmc_ssor_smoother_apply");
    }

   protected:
    const int nsmooth;
    std::unique_ptr<mgmc::HipMultigridMCSampler> impl;
};

// SORSmootherFactory (sor_smoother.hh:91-125) / SSORSmootherFactory (ssor_smoother.hh:70-100): what
// MultigridPreconditioner hands the levels (multigrid_preconditioner.cc:18-33)
class HipSORSmootherFactory : public SmootherFactory {
   public:
    HipSORSmootherFactory(const double omega_, const int nsmooth_, const Direction direction_, int device_ = 0)
        : omega(omega_), nsmooth(nsmooth_), direction(direction_), device(device_) {}
    virtual ~HipSORSmootherFactory() {}
    std::shared_ptr<Smoother> get(std::shared_ptr<LinearOperator> linear_operator) override {
        return std::make_shared<HipSORSmoother>(linear_operator, omega, nsmooth, direction, device);
    }

   private:
    const double omega;
    const int nsmooth;
    const Direction direction;
    const int device;
};

class HipSSORSmootherFactory : public SmootherFactory {
   public:
    HipSSORSmootherFactory(const double omega_, const int nsmooth_, int device_ = 0)
        : omega(omega_), nsmooth(nsmooth_), device(device_) {}
    virtual ~HipSSORSmootherFactory() {}
    std::shared_ptr<Smoother> get(std::shared_ptr<LinearOperator> linear_operator) override {
        return std::make_shared<HipSSORSmoother>(linear_operator, omega, nsmooth, device);
    }

   private:
    const double omega;
    const int nsmooth;
    const int device;
};
