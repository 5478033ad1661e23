// Test scaffolding (tests/cpp/refdecl/README.md): the reference's lattice base class as the adapter
// sees it -- lattice/lattice.hh:18-129 (Ncell / Nvertex members :125-128, shape() :113, dim() :116).
#pragma once
#include <memory>
#include <string>

#include <Eigen/Dense>

class Lattice {
   public:
    Lattice(const unsigned int Ncell_, const unsigned int Nvertex_) : Ncell(Ncell_), Nvertex(Nvertex_) {}
    virtual Eigen::VectorXi shape() const = 0;
    virtual int dim() const { return (int)shape().size(); }
    virtual std::string get_info() const = 0;
    const unsigned int Ncell;
    const unsigned int Nvertex;
};
