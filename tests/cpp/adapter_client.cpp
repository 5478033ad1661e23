// Test driver for include/reference_adapter/hip_multigridmc_sampler.hh (tests/test_adapter.py,
// tests/test_gpu_adapter.py): the adapter used the way driver_mgmc.cc uses a Sampler, on operators
// whose A_sparse is filled from the library's own assembly of the reference operators
// (mgmc_operator_csr).  Built against tests/cpp/refdecl (declaration scaffolding).
//
//   adapter_client describe                  which path each operator takes (host only)
//   adapter_client sample <n> <fd|fem|periodic>   seed, path, then n QoI values of apply() cycles
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "hip_multigridmc_sampler.hh"

namespace {

class TestLattice : public Lattice {
   public:
    explicit TestLattice(std::vector<int> n) : Lattice(ncell(n), nvertex(n)), n_(std::move(n)) {}
    Eigen::VectorXi shape() const override {
        Eigen::VectorXi s((std::ptrdiff_t)n_.size());
        for (size_t d = 0; d < n_.size(); ++d) s[(std::ptrdiff_t)d] = n_[d];
        return s;
    }
    std::string get_info() const override { return "test lattice"; }

   private:
    static unsigned ncell(const std::vector<int>& n) {
        unsigned c = 1;
        for (int v : n) c *= (unsigned)v;
        return c;
    }
    static unsigned nvertex(const std::vector<int>& n) {
        unsigned c = 1;
        for (int v : n) c *= (unsigned)(v - 1);
        return c;
    }
    std::vector<int> n_;
};

// A LinearOperator whose A_sparse is the reference operator as the library assembles it (symmetric:
// its CSR arrays are its ColMajor arrays)
class AssembledOperator : public LinearOperator {
   public:
    AssembledOperator(std::shared_ptr<Lattice> lat, int pde, bool periodic) : LinearOperator(lat, 0) {
        const Eigen::VectorXi s = lat->shape();
        mgmc_operator_desc d{};
        d.dim = lat->dim();
        d.nx = s[0];
        d.ny = s[1];
        d.nz = d.dim == 3 ? s[2] : 0;
        d.pde = pde;
        d.kappa_model = periodic ? MGMC_KAPPA_PERIODIC : MGMC_KAPPA_CONSTANT;
        d.Lambda = 0.2;
        d.Lambda_min = 0.2;
        d.Lambda_max = 0.4;
        int64_t nrow = 0, nnz = 0;
        mgmc::check(mgmc_operator_csr_size(&d, &nrow, &nnz), nullptr, "mgmc_operator_csr_size");
        std::vector<int64_t> rowptr((size_t)nrow + 1);
        std::vector<int32_t> col((size_t)nnz);
        std::vector<double> val((size_t)nnz);
        mgmc::check(mgmc_operator_csr(&d, rowptr.data(), col.data(), val.data()), nullptr, "mgmc_operator_csr");
        A_sparse.assign_compressed(std::vector<int>(rowptr.begin(), rowptr.end()), std::vector<int>(col.begin(), col.end()),
                                   std::move(val));
    }
};

MultigridParameters params(unsigned nlevel) {
    MultigridParameters p;
    p.nlevel = nlevel;
    p.smoother = "SOR";
    p.coarse_solver = "SSOR";
    p.npresmooth = 1;
    p.npostsmooth = 1;
    p.ncoarsesmooth = 1;
    p.omega = 1.0;
    p.cycle = 1;
    p.coarse_scaling = 1.0;
    p.verbose = 0;
    return p;
}

std::shared_ptr<LinearOperator> make_op(const std::string& kind) {
    if (kind == "fd") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{16, 16, 16}), MGMC_OPERATOR_FD, false);
    if (kind == "fem") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{16, 16, 16}), MGMC_OPERATOR_FEM, false);
    if (kind == "periodic") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{32, 32}), MGMC_OPERATOR_FD, true);
    std::fprintf(stderr, "unknown operator %s\n", kind.c_str());
    std::exit(2);
}

const char* name(HipMultigridMCSampler::Path p) { return p == HipMultigridMCSampler::Path::stencil ? "stencil" : "matrix"; }

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "describe";
    if (mode == "describe") {
        for (const char* k : {"fd", "fem", "periodic"}) {
            const auto plan = HipMultigridMCSampler::classify(*make_op(k), params(3));
            std::printf("%s path %s\n", k, name(plan.path));
        }
        return 0;
    }
    if (mode == "sample" && argc > 3) {
        const int n = std::atoi(argv[2]);
        const std::shared_ptr<LinearOperator> op = make_op(argv[3]);
        std::mt19937_64 rng(5418513);  // driver_mgmc.cc:448
        HipMultigridMCSampler sampler(op, rng, params(3), /*device=*/0, /*chain_id=*/0);
        std::printf("seed %llu\npath %s\n", (unsigned long long)sampler.get_seed(), name(sampler.path()));
        const std::ptrdiff_t ndof = (std::ptrdiff_t)op->get_ndof();
        Eigen::VectorXd f(ndof), x(ndof);
        f.setZero();
        x.setZero();
        sampler.fix_rhs(f);
        const std::ptrdiff_t q = ndof / 2;  // the lattice centre
        for (int k = 0; k < n; ++k) {
            sampler.apply(f, x);  // measure_sampling_time's loop body (driver_mgmc.cc:72-76)
            std::printf("%.17g\n", x[q]);
        }
        return 0;
    }
    std::fprintf(stderr, "usage: adapter_client describe | sample <n> <fd|fem|periodic>\n");
    return 2;
}
