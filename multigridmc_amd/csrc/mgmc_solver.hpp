// mgmc_solver.hpp -- vector kernels of the exact-statistics engine (multigrid-preconditioned CG
// and the reference's LoopSolver) on the padded level-0 layout.
//
// Reference: MultigridPreconditioner (preconditioner/multigrid_preconditioner.cc:74-109),
// LoopSolver (solver/loop_solver.cc:9-53); the exact targets they stand in for are
// LinearOperator::mean / observed_mean_and_variance (linear_operator.hh:119-174), which the
// reference computes with a sparse Cholesky factorisation -- infeasible for 3D lattices of 255^3
// and more.  Every vector here is a padded array whose halo is zero in all operands, so the
// kernels run over the whole storage (nstore) and the halo stays zero.
#pragma once
#include <hip/hip_runtime.h>

namespace mgmc {

constexpr int SOLVE_NB = 1024;  // reduction blocks (fixed: deterministic two-stage sums)

// partial[b] = sum over block b's grid-stride range of a_i * b_i  (fixed order per block)
static __global__ void __launch_bounds__(256) k_dot_partial(long long n, const double* __restrict__ a,
                                                      const double* __restrict__ b, double* __restrict__ partial) {
    __shared__ double red[256];
    double acc = 0.0;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        acc = fma(a[i], b[i], acc);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// out[slot] = sum of the partials (one workgroup, fixed tree)
static __global__ void __launch_bounds__(256) k_dot_final(const double* __restrict__ partial, int np, double* __restrict__ out,
                                                    int slot) {
    __shared__ double red[256];
    double acc = 0.0;
    for (int i = threadIdx.x; i < np; i += 256) acc = acc + partial[i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[slot] = red[0];
}

// y = a x + y  (alpha read from device scalars: alpha = num[0] / den[0] * sign)
static __global__ void __launch_bounds__(256) k_axpy_ratio(long long n, const double* __restrict__ num,
                                                     const double* __restrict__ den, double sign,
                                                     const double* __restrict__ x, double* __restrict__ y) {
    const double alpha = sign * (num[0] / den[0]);
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        y[i] = fma(alpha, x[i], y[i]);
}

// p = z + beta p, beta = num[0] / den[0]
static __global__ void __launch_bounds__(256) k_xpby_ratio(long long n, const double* __restrict__ z,
                                                     const double* __restrict__ num, const double* __restrict__ den,
                                                     double* __restrict__ p) {
    const double beta = num[0] / den[0];
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        p[i] = fma(beta, p[i], z[i]);
}

// y = a - b
static __global__ void __launch_bounds__(256) k_sub(long long n, const double* __restrict__ a, const double* __restrict__ b,
                                              double* __restrict__ y) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        y[i] = a[i] - b[i];
}

}  // namespace mgmc
