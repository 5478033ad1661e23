// mgmc_operators.hpp -- host-side assembly of the reference's fine operators as CSR and the Galerkin
// coarsening of a CSR operator (no device code).
//
// Variable coefficients (the periodic correlation-length model) and the squared FD operator have no
// constant 3^d-point stencil, so their hierarchy is built from matrices:
//  * assemble_operator: ShiftedLaplaceFDOperator (shiftedlaplace_fd_operator.cc:9-57),
//    ShiftedLaplaceFEMOperator (shiftedlaplace_fem_operator.cc:9-145) and
//    SquaredShiftedLaplaceFDOperator (squared_shiftedlaplace_fd_operator.cc:9-96, 2D) with the
//    constant or periodic kappa^2 model (correlationlength_model.hh:45-112), rows in the lattice's
//    vertex order, entries summed as setFromTriplets / coeffRef sum them, columns ascending;
//  * galerkin_csr: A_c = (R A) R^T (linear_operator.cc:10-23) as two Gustavson products with the
//    linear-interpolation restriction R (intergrid_operator_linear.cc:8-30, colidx of
//    intergrid_operator.cc:8-20): row by row, each product term added in the order of the left
//    factor's row entries, output columns ascending.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mgmc.h"

namespace mgmc {

struct CsrHost {
    int64_t nrow = 0;
    std::vector<int64_t> rowptr;
    std::vector<int32_t> col;
    std::vector<double> val;
};

// "" or the reason the descriptor is invalid
std::string validate_operator(const mgmc_operator_desc& d);

// kappa^2 of the descriptor's correlation-length model at the point x (dim coordinates)
double kappa_sq_at(const mgmc_operator_desc& d, const double* x);

CsrHost assemble_operator(const mgmc_operator_desc& d);

// A_c = R A R^T on the next-coarser lattice (n -> n/2 per direction)
CsrHost galerkin_csr(const CsrHost& A, int dim, const int* nfine);

// "" if A is an operator of the lattice the multicolour sweeps can run: nrow = interior vertices,
// columns ascending within each row, couplings at most 2 vertices apart per direction, a positive
// diagonal entry in every row
std::string check_lattice_csr(int dim, const int* n, const CsrHost& A);

// largest |offset| per direction over all entries (the coupling reach, 1 or 2)
int csr_reach(int dim, const int* n, const CsrHost& A);

}  // namespace mgmc
