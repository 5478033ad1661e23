// Test scaffolding (tests/cpp/refdecl/README.md): LinearOperator as the adapter sees it --
// linear_operator/linear_operator.hh:28-198: ctor :40-48, get_lattice :54, get_ndof :79,
// get_m_lowrank :82, get_sparse :93, get_B :96, get_Sigma :99, protected data :186-197.
#pragma once
#include <memory>

#include <Eigen/Dense>
#include <Eigen/Sparse>
#include "lattice/lattice.hh"

class LinearOperator {
   public:
    typedef Eigen::SparseMatrix<double> SparseMatrixType;
    typedef Eigen::MatrixXd DenseMatrixType;
    LinearOperator(const std::shared_ptr<Lattice> lattice_, const unsigned int m_lowrank_ = 0)
        : lattice(lattice_), m_lowrank(m_lowrank_), A_sparse(lattice_->Nvertex, lattice_->Nvertex),
          B(lattice_->Nvertex, m_lowrank_), Sigma_inv_BT(m_lowrank_, lattice_->Nvertex), Sigma_diag(m_lowrank_) {}
    virtual ~LinearOperator() = default;
    std::shared_ptr<Lattice> get_lattice() const { return lattice; }
    const unsigned int get_ndof() const { return (unsigned int)A_sparse.rows(); }
    const unsigned int get_m_lowrank() const { return m_lowrank; }
    const SparseMatrixType& get_sparse() const { return A_sparse; }
    const SparseMatrixType& get_B() const { return B; }
    const Eigen::DiagonalMatrix<double, Eigen::Dynamic> get_Sigma() const { return Sigma_diag; }

   protected:
    const std::shared_ptr<Lattice> lattice;
    const unsigned int m_lowrank;
    SparseMatrixType A_sparse;
    SparseMatrixType B;
    SparseMatrixType Sigma_inv_BT;
    Eigen::DiagonalMatrix<double, Eigen::Dynamic> Sigma_diag;
};
