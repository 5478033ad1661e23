// mgmc_hierarchy.hpp -- host-side construction of the multigrid hierarchy (no device code).
//
// Mirrors the setup half of MultigridMCSampler (sampler/multigridmc_sampler.cc:8-100):
//  * lattice coarsening n -> n/2 per direction, with the reference's validity checks
//    (lattice/lattice3d.hh:241-257, lattice/lattice2d.hh:198-213);
//  * the fine shifted-Laplace FD operator (linear_operator/shiftedlaplace_fd_operator.cc:9-57)
//    with a constant kappa^2 (linear_operator/correlationlength_model.hh:45-66);
//  * Galerkin coarsening A_c = R A R^T (linear_operator/linear_operator.cc:10-23) with the
//    linear-interpolation intergrid operator (intergrid/intergrid_operator_linear.cc:8-30).
// Because the fine operator has constant coefficients and P embeds coarse vertex i at fine
// vertex 2i with zero extension, every Galerkin level is a constant 3^d-point stencil
// truncated at the Dirichlet boundary; the Galerkin product is therefore evaluated on the
// stencil (27 numbers per level) instead of as a sparse matrix triple product.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mgmc.h"

namespace mgmc {

struct LevelSpec {
    int dim;
    int n[3];        // cells per direction (n[2] = 0 in 2D)
    int npoints;     // 5/7 for the fine FD level, 9/27 for Galerkin levels
    int ncolours;    // 2 or 2^dim
    uint64_t ndof;
    double st[27];   // stencil, index (dz+1)*9+(dy+1)*3+(dx+1) (3D) / (dy+1)*3+(dx+1) (2D)
    double diag() const { return dim == 3 ? st[13] : st[4]; }
};

// Returns "" on success, otherwise an error message.
std::string validate_config(const mgmc_config& cfg);

// Build all levels (cfg must be valid).  fine_st (27 doubles, may be null): the fine level's constant
// stencil instead of cfg's FD / FEM operator; a stencil whose couplings are all axis neighbours is
// swept red-black (5/7 points), any other 3^d stencil in 2^d colours.
std::vector<LevelSpec> build_hierarchy(const mgmc_config& cfg, const double* fine_st = nullptr);

// true if every nonzero of the 3^d stencil is the centre or an axis neighbour
bool stencil_axis_only(int dim, const double* st);

// Galerkin product of a 3^d stencil with the (1/2,1,1/2)^d linear interpolation.
void galerkin_stencil(int dim, const double* fine, double* coarse);

}  // namespace mgmc
