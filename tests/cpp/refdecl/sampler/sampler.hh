// Test scaffolding (tests/cpp/refdecl/README.md): the Sampler plugin contract --
// sampler/sampler.hh:23-72 (ctor :31-34, apply :41, get_linear_operator :44-47, fix_rhs :56,
// unfix_rhs :63, protected members :67-71).  Like the reference's class it declares no destructor:
// a derived sampler must be owned as the reference owns its samplers, std::make_shared<Derived>
// (driver_mgmc.cc:450-457), whose deleter destroys the Derived object.
#pragma once
#include <memory>
#include <random>

#include <Eigen/Dense>
#include "linear_operator/linear_operator.hh"

class Sampler {
   public:
    Sampler(const std::shared_ptr<LinearOperator> linear_operator_, std::mt19937_64& rng_)
        : linear_operator(linear_operator_), rng(rng_), normal_dist(0.0, 1.0) {}
    virtual void apply(const Eigen::VectorXd& f, Eigen::VectorXd& x) const = 0;
    std::shared_ptr<LinearOperator> get_linear_operator() const { return linear_operator; }
    virtual void fix_rhs(const Eigen::VectorXd& f) { (void)f; }
    virtual void unfix_rhs() {}

   protected:
    const std::shared_ptr<LinearOperator> linear_operator;
    std::mt19937_64& rng;
    mutable std::normal_distribution<double> normal_dist;
};
