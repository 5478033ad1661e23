// Test scaffolding (tests/cpp/refdecl/README.md): the Smoother plugin contract --
// smoother/smoother.hh:15-44 (ctor :22, apply :29, protected linear_operator :33, SmootherFactory::get
// :43).  No destructor is declared, as in the reference: smoothers are owned through
// std::make_shared<Derived> (multigrid_preconditioner.cc:18-33).
#pragma once
#include <memory>

#include <Eigen/Dense>
#include "linear_operator/linear_operator.hh"

class Smoother {
   public:
    Smoother(const std::shared_ptr<LinearOperator> linear_operator_) : linear_operator(linear_operator_) {}
    virtual void apply(const Eigen::VectorXd& b, Eigen::VectorXd& x) const = 0;

   protected:
    const std::shared_ptr<LinearOperator> linear_operator;
};

class SmootherFactory {
   public:
    virtual std::shared_ptr<Smoother> get(std::shared_ptr<LinearOperator> linear_operator) = 0;
};
