// hip_multigridmc_sampler.hh -- reference-side adapter: the MI355X MGMC sampler as a `Sampler` of
// nilsfriess/MultigridMC.  A maintainer drops this file into the reference as
// src/sampler/hip_multigridmc_sampler.hh and links -lmgmc_hip.
//
// It is written against the reference's own interfaces (citations relative to its src/):
//   Sampler                    sampler/sampler.hh:23-72 (ctor :31-34, apply :41, fix_rhs :56, unfix_rhs :63)
//   LinearOperator             linear_operator/linear_operator.hh:28-198 (get_lattice :54, get_ndof :79,
//                              get_m_lowrank :82, get_sparse :93, get_B :96, get_Sigma :99)
//   Lattice                    lattice/lattice.hh:18-129 (shape :113, dim :116)
//   MultigridParameters        auxilliary/parameters.hh:145-174
//   MultigridMCSampler         sampler/multigridmc_sampler.cc:8-138 (what this replaces)
//
// Every operator goes through its matrix: get_sparse() is the precision matrix A_sparse, an Eigen
// ColMajor SparseMatrix<double> with int indices.  Its compressed-column arrays are handed over as
// the rows of the matrix (column j of A is row j of A^T): that is exactly what the reference's SOR
// sweeps read (SORSmoother::apply_sparse, smoother/sor_smoother.cc:56-78, walks the ColMajor storage
// as rows), and it is A itself for the symmetric operators of the reference.
//   * mgmc_stencil_of_csr: if every row is one constant 3^d stencil truncated at the boundary
//     (ShiftedLaplaceFDOperator / ShiftedLaplaceFEMOperator with a constant correlation length), the
//     sampler takes the stencil fast path (mgmc_create_stencil_batch: stencil Galerkin hierarchy,
//     fused z-marching fine sweeps, no matrix in HBM).
//   * otherwise (periodic correlation length, SquaredShiftedLaplaceFDOperator, any user matrix) the
//     matrix path (mgmc_create_csr_batch: Galerkin products of the matrix, per-vertex coefficients).
// A MeasuredOperator's low-rank part (get_m_lowrank() > 0) is installed from get_B() (ColMajor =
// the CSC form mgmc_set_lowrank takes) and get_Sigma().diagonal().
//
// Noise: the reference's sampler draws from the shared std::mt19937_64; the device stream is
// counter-based (Philox keyed by seed and chain id).  By default the Philox seed
// is the next output of a COPY of the shared engine, so the samples follow the driver's seed
// (driver_mgmc.cc:448) while the engine itself is never advanced: the reference's
// MultigridMCSampler consumes none at construction (multigridmc_sampler.cc:8-100), so the SSOR /
// Cholesky samplers driver_mgmc builds after it (driver_mgmc.cc:450-501) see the engine state they
// see in an unmodified reference.  The reference's samplers sharing one engine draw different noise,
// so a second sampler built on the same (unadvanced) engine state in this process does not reuse the
// seed: every repeat of an engine state mixes a construction counter into it (the first sampler keeps
// the engine's output itself).  An explicit seed (the last constructor argument) is taken as given.
// Ownership: like the reference's Sampler, the base class has no virtual destructor, so a sampler is
// owned as driver_mgmc.cc:450-457 owns it, std::make_shared<HipMultigridMCSampler>(...) (the
// shared_ptr's deleter destroys the derived object and its device handle).  Errors print and
// exit(-1) like the reference (multigridmc_sampler.cc:47-49).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "auxilliary/parameters.hh"
#include "sampler/sampler.hh"
#include "mgmc_sampler.hh"  // this repo: include/mgmc_sampler.hh (over include/mgmc.h)

class HipMultigridMCSampler : public Sampler {
   public:
    enum class Path { stencil, matrix };
    static constexpr uint64_t default_seed = 5418513;  // driver_mgmc.cc:448 (seed of the noise-free smoother handles)

    // Philox seed by default: the next output of a copy of the shared engine (the engine is not
    // advanced); the k-th repeat of that output in this process (k >= 1) is mixed with k (splitmix64)
    static uint64_t engine_seed(const std::mt19937_64& rng_) {
        std::mt19937_64 copy = rng_;
        const uint64_t s = copy();
        static std::mutex mu;
        static std::map<uint64_t, uint64_t> uses;  // engine output -> samplers seeded from it so far
        uint64_t k;
        {
            std::lock_guard<std::mutex> lock(mu);
            k = uses[s]++;
        }
        if (k == 0) return s;
        uint64_t z = k + 0x9E3779B97F4A7C15ull;  // splitmix64(k)
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return s ^ (z ^ (z >> 31));
    }

    // The reference's MultigridMCSampler(linear_operator, rng, params, cholesky_params) plus where to
    // run: the HIP device and the chain id of the Philox key (one chain per rank, nchains per handle).
    // rng_ is kept as the Sampler base keeps it and is not drawn from.
    HipMultigridMCSampler(const std::shared_ptr<LinearOperator> linear_operator_, std::mt19937_64& rng_,
                          const MultigridParameters params_, int device = 0, uint64_t chain_id = 0, int nchains = 1)
        : HipMultigridMCSampler(linear_operator_, rng_, params_, device, chain_id, nchains, engine_seed(rng_)) {}

    // ... with an explicit Philox seed
    HipMultigridMCSampler(const std::shared_ptr<LinearOperator> linear_operator_, std::mt19937_64& rng_,
                          const MultigridParameters params_, int device, uint64_t chain_id, int nchains,
                          uint64_t seed_)
        : Sampler(linear_operator_, rng_), seed(seed_) {
        Path path = Path::matrix;
        impl = make_impl(*linear_operator_, params_, device, seed, chain_id, nchains, &path);
        path_ = path;
    }

    // sampler.hh:41 -- one call = one MGMC cycle (multigridmc_sampler.cc:132-138), x in/out on the host
    void apply(const Eigen::VectorXd& f, Eigen::VectorXd& x) const override {
        if ((size_t)x.size() != impl->get_ndof() || (size_t)f.size() != impl->get_ndof()) {
            std::fprintf(stderr, "ERROR: HipMultigridMCSampler::apply: vector size %td / %td, operator %zu\n", f.size(),
                         x.size(), impl->get_ndof());
            std::exit(-1);
        }
        impl->apply(f.data(), x.data());
    }
    void fix_rhs(const Eigen::VectorXd& f) override { impl->fix_rhs(f.data()); }  // sampler.hh:56
    void unfix_rhs() override { impl->unfix_rhs(); }                              // sampler.hh:63

    // The device-resident loop for measure_sampling_time (driver_mgmc.cc:66-80): nsamples cycles on
    // the fixed rhs, x stays in HBM, the QoI x[qoi_index] is recorded on the device.
    std::vector<double> sample(int nsamples, int64_t qoi_index) const { return impl->sample(nsamples, qoi_index); }
    // (n, mean, M2) of the recorded QoI (driver_mgmc.cc:86-94 statistics, Welford on the device)
    void qoi_moments(double out[3]) const { impl->qoi_moments(out); }
    void set_state(const Eigen::VectorXd& x) { impl->set_state(x.data()); }
    void get_state(Eigen::VectorXd& x) const { impl->get_state(x.data()); }

    Path path() const { return path_; }
    uint64_t get_seed() const { return seed; }
    mgmc_handle* handle() const { return impl->handle(); }

    // Host-only decision (no device touched): the config and the stencil or matrix a sampler for
    // this operator would be built from.
    struct Plan {
        Path path = Path::matrix;
        mgmc_config cfg{};
        double stencil[27] = {0};
        std::vector<int64_t> outer;  // row pointer (the ColMajor outer index, widened)
        const int32_t* inner = nullptr;
        const double* values = nullptr;
    };
    static Plan classify(const LinearOperator& op, const MultigridParameters& p) {
        Plan plan;
        const std::shared_ptr<Lattice> lat = op.get_lattice();
        const Eigen::VectorXi shape = lat->shape();
        const int dim = lat->dim();
        if (dim != 2 && dim != 3) {
            std::fprintf(stderr, "ERROR: HipMultigridMCSampler needs a 2D or 3D lattice, got %dD\n", dim);
            std::exit(-1);
        }
        plan.cfg = mgmc::make_config(dim, shape[0], shape[1], dim == 3 ? shape[2] : 0, 0.0, to_mgmc(p));
        const LinearOperator::SparseMatrixType& A = op.get_sparse();
        if (!A.isCompressed() || A.rows() != A.cols() || (int64_t)A.rows() != (int64_t)op.get_ndof()) {
            std::fprintf(stderr, "ERROR: HipMultigridMCSampler: A_sparse must be square and compressed\n");
            std::exit(-1);
        }
        const int64_t n = A.rows();
        static_assert(sizeof(LinearOperator::SparseMatrixType::StorageIndex) == sizeof(int32_t),
                      "Eigen's default int StorageIndex");
        plan.outer.assign(A.outerIndexPtr(), A.outerIndexPtr() + n + 1);
        plan.inner = reinterpret_cast<const int32_t*>(A.innerIndexPtr());
        plan.values = A.valuePtr();
        const int rc = mgmc_stencil_of_csr(&plan.cfg, n, plan.outer.data(), plan.inner, plan.values, plan.stencil);
        if (rc == MGMC_OK)
            plan.path = Path::stencil;
        else if (rc == MGMC_E_UNSUPPORTED)
            plan.path = Path::matrix;
        else
            mgmc::check(rc, nullptr, "mgmc_stencil_of_csr");
        return plan;
    }

    // A device sampler for the operator: the stencil or the matrix path (classify), with a
    // MeasuredOperator's low-rank part installed.  The Smoother drop-ins (hip_sor_smoother.hh) build
    // their one-level handle through it too.
    static std::unique_ptr<mgmc::HipMultigridMCSampler> make_impl(const LinearOperator& op, const MultigridParameters& p,
                                                                  int device, uint64_t seed, uint64_t chain_id,
                                                                  int nchains, Path* path = nullptr) {
        const Plan plan = classify(op, p);
        std::unique_ptr<mgmc::HipMultigridMCSampler> impl;
        if (plan.path == Path::stencil)
            impl.reset(new mgmc::HipMultigridMCSampler(plan.cfg, plan.stencil, device, seed, chain_id, nchains));
        else
            impl.reset(new mgmc::HipMultigridMCSampler(plan.cfg, (int64_t)plan.outer.size() - 1, plan.outer.data(),
                                                       plan.inner, plan.values, device, seed, chain_id, nchains));
        if (path) *path = plan.path;
        if (op.get_m_lowrank() > 0) install_lowrank(op, *impl);
        return impl;
    }

   private:
    static mgmc::MultigridParameters to_mgmc(const MultigridParameters& p) {
        mgmc::MultigridParameters q;
        q.nlevel = (int)p.nlevel;
        q.npresmooth = (int)p.npresmooth;
        q.npostsmooth = (int)p.npostsmooth;
        q.ncoarsesmooth = (int)p.ncoarsesmooth;
        q.omega = p.omega;
        q.cycle = (int)p.cycle;
        q.coarse_scaling = p.coarse_scaling;
        q.verbose = p.verbose;
        // the reference accepts exactly these names (multigridmc_sampler.cc:34-49, :52-73)
        if (p.smoother == "SOR")
            q.smoother = MGMC_SMOOTHER_SOR;
        else if (p.smoother == "SSOR")
            q.smoother = MGMC_SMOOTHER_SSOR;
        else {
            std::fprintf(stderr, "ERROR: invalid sampler \'%s\'\n", p.smoother.c_str());
            std::exit(-1);
        }
        if (p.coarse_solver == "SSOR")
            q.coarse_solver = MGMC_COARSE_SSOR;
        else if (p.coarse_solver == "Cholesky")
            q.coarse_solver = MGMC_COARSE_CHOLESKY;
        else {
            std::fprintf(stderr, "ERROR: multigrid coarse sampler \'%s\'\n", p.coarse_solver.c_str());
            std::exit(-1);
        }
        return q;
    }

    // MeasuredOperator (measured_operator.cc:9-49): B (ColMajor: colptr / row index / values, the CSC
    // form of mgmc_set_lowrank) and Sigma's diagonal
    static void install_lowrank(const LinearOperator& op, mgmc::HipMultigridMCSampler& impl) {
        const LinearOperator::SparseMatrixType& B = op.get_B();
        const int m = (int)B.cols();
        std::vector<int64_t> colptr(B.outerIndexPtr(), B.outerIndexPtr() + m + 1);
        std::vector<int64_t> rows(B.innerIndexPtr(), B.innerIndexPtr() + B.nonZeros());
        const Eigen::VectorXd sigma = op.get_Sigma().diagonal();
        impl.set_lowrank(m, colptr.data(), rows.data(), B.valuePtr(), sigma.data());
    }

    const uint64_t seed;
    Path path_ = Path::matrix;
    std::unique_ptr<mgmc::HipMultigridMCSampler> impl;
};
