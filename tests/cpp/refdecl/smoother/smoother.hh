// Test scaffolding (tests/cpp/refdecl/README.md): the Smoother plugin contract --
// smoother/smoother.hh:15-44 (ctor :22, apply :29, protected linear_operator :33, SmootherFactory::get
// :43).  A virtual destructor is added, as in sampler.hh.
#pragma once
#include <memory>

#include <Eigen/Dense>
#include "linear_operator/linear_operator.hh"

class Smoother {
   public:
    Smoother(const std::shared_ptr<LinearOperator> linear_operator_) : linear_operator(linear_operator_) {}
    virtual ~Smoother() = default;
    virtual void apply(const Eigen::VectorXd& b, Eigen::VectorXd& x) const = 0;

   protected:
    const std::shared_ptr<LinearOperator> linear_operator;
};

class SmootherFactory {
   public:
    virtual ~SmootherFactory() = default;
    virtual std::shared_ptr<Smoother> get(std::shared_ptr<LinearOperator> linear_operator) = 0;
};
