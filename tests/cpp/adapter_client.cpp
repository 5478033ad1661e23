// Test driver for include/reference_adapter/hip_multigridmc_sampler.hh (tests/test_adapter.py,
// tests/test_gpu_adapter.py): the adapter used the way driver_mgmc.cc uses a Sampler, on operators
// whose A_sparse is filled from the library's own assembly of the reference operators
// (mgmc_operator_csr).  Built against tests/cpp/refdecl (declaration scaffolding).
//
//   adapter_client describe                  which path each operator takes (host only)
//   adapter_client sample <n> <fd|fem|periodic>   seed, path, then n QoI values of apply() cycles
//   adapter_client rngcheck                  constructs a sampler on the driver's shared engine and
//                                            reports (also from an atexit handler, so a failed device
//                                            call's exit(-1) reports too) whether the engine moved
//   adapter_client seedrepeat                three default seeds drawn from the unadvanced shared engine
//                                            (no device): the engine's own output first, then distinct ones
//   adapter_client smoother <fd|fem|periodic> <sor|ssor> <nsmooth> <fwd|bwd> [lowrank]
//                                            b, x and x after one Smoother::apply(b, x) of the Smoother
//                                            drop-in (b, x from a fixed mt19937_64 stream); "lowrank" adds two
//                                            point measurements (MeasuredOperator-like B, Sigma)
//   adapter_client ownership <rounds>        samplers and smoothers owned the reference's way
//                                            (std::make_shared<Derived> held as shared_ptr<Base>,
//                                            driver_mgmc.cc:450-457, multigrid_preconditioner.cc:18-33),
//                                            used and released; prints mgmc_live_handles() after each
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "hip_multigridmc_sampler.hh"
#include "hip_sor_smoother.hh"

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
    AssembledOperator(std::shared_ptr<Lattice> lat, int pde, bool periodic, bool lowrank = false)
        : LinearOperator(lat, lowrank ? 2 : 0) {
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
        if (lowrank) {  // two point measurements (rows N/3, 2N/3), Sigma = diag(1e-3, 2e-3)
            const int n = (int)nrow;
            B.assign_compressed({0, 1, 2}, {n / 3, 2 * n / 3}, {1.0, 1.0});
            Sigma_diag.diagonal()[0] = 1e-3;
            Sigma_diag.diagonal()[1] = 2e-3;
        }
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

std::shared_ptr<LinearOperator> make_op(const std::string& kind, bool lowrank = false) {
    if (kind == "fd") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{16, 16, 16}), MGMC_OPERATOR_FD, false, lowrank);
    if (kind == "fem") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{16, 16, 16}), MGMC_OPERATOR_FEM, false, lowrank);
    if (kind == "periodic") return std::make_shared<AssembledOperator>(std::make_shared<TestLattice>(std::vector<int>{32, 32}), MGMC_OPERATOR_FD, true, lowrank);
    std::fprintf(stderr, "unknown operator %s\n", kind.c_str());
    std::exit(2);
}

const char* name(HipMultigridMCSampler::Path p) { return p == HipMultigridMCSampler::Path::stencil ? "stencil" : "matrix"; }

// rngcheck: the driver's engine and a copy of its state at construction time
std::mt19937_64 g_rng(5418513);  // driver_mgmc.cc:448-449
std::mt19937_64 g_rng_before;
void report_engine() { std::printf("engine %s\n", g_rng == g_rng_before ? "unchanged" : "CHANGED"); std::fflush(stdout); }

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
    if (mode == "rngcheck") {
        g_rng_before = g_rng;
        std::atexit(report_engine);  // runs on the exit(-1) of a failed device call too
        HipMultigridMCSampler sampler(make_op("fd"), g_rng, params(3), /*device=*/0, /*chain_id=*/0);
        std::printf("seed %llu\n", (unsigned long long)sampler.get_seed());
        std::mt19937_64 fresh(5418513);
        std::printf("engine_first %llu\n", (unsigned long long)fresh());
        return 0;
    }
    if (mode == "seedrepeat") {
        g_rng_before = g_rng;
        for (int q = 0; q < 3; ++q)
            std::printf("seed%d %llu\n", q, (unsigned long long)HipMultigridMCSampler::engine_seed(g_rng));
        std::mt19937_64 fresh(5418513);
        std::printf("engine_first %llu\n", (unsigned long long)fresh());
        report_engine();
        return 0;
    }
    if (mode == "ownership" && argc > 2) {
        const int rounds = std::atoi(argv[2]);
        std::printf("live %d\n", mgmc_live_handles());
        for (int r = 0; r < rounds; ++r) {
            const std::shared_ptr<LinearOperator> op = make_op(r % 2 ? "periodic" : "fd");
            std::shared_ptr<Sampler> sampler = std::make_shared<HipMultigridMCSampler>(op, g_rng, params(3), 0, (uint64_t)r);
            std::shared_ptr<SmootherFactory> sor = std::make_shared<HipSORSmootherFactory>(1.0, 1, forward);
            std::shared_ptr<SmootherFactory> ssor = std::make_shared<HipSSORSmootherFactory>(1.0, 1);
            std::vector<std::shared_ptr<Smoother>> smoothers{sor->get(op), ssor->get(op)};
            const std::ptrdiff_t ndof = (std::ptrdiff_t)op->get_ndof();
            Eigen::VectorXd f(ndof), x(ndof);
            f.setZero();
            x.setZero();
            sampler->fix_rhs(f);
            sampler->apply(f, x);
            for (const auto& sm : smoothers) sm->apply(f, x);
            int finite = 1;
            for (std::ptrdiff_t i = 0; i < ndof; ++i) finite &= std::isfinite(x[i]) ? 1 : 0;
            const int held = mgmc_live_handles();
            sampler.reset();  // through the base pointer: the make_shared deleter destroys the derived object
            smoothers.clear();
            sor.reset();
            ssor.reset();
            std::printf("round %d held %d live %d x %d\n", r, held, mgmc_live_handles(), finite);
        }
        return 0;
    }
    if (mode == "smoother" && argc > 5) {
        const bool lowrank = argc > 6 && std::string(argv[6]) == "lowrank";
        const std::shared_ptr<LinearOperator> op = make_op(argv[2], lowrank);
        const std::string kind = argv[3];
        const int nsmooth = std::atoi(argv[4]);
        const Direction dir = std::string(argv[5]) == "bwd" ? backward : forward;
        std::shared_ptr<SmootherFactory> factory;
        if (kind == "sor")
            factory = std::make_shared<HipSORSmootherFactory>(1.0, nsmooth, dir);
        else
            factory = std::make_shared<HipSSORSmootherFactory>(1.0, nsmooth);
        const std::shared_ptr<Smoother> smoother = factory->get(op);  // multigrid_preconditioner.cc:18-33
        const std::ptrdiff_t ndof = (std::ptrdiff_t)op->get_ndof();
        Eigen::VectorXd b(ndof), x(ndof);
        std::mt19937_64 r(7);
        std::uniform_real_distribution<double> u(-1.0, 1.0);
        for (std::ptrdiff_t i = 0; i < ndof; ++i) b[i] = u(r);
        for (std::ptrdiff_t i = 0; i < ndof; ++i) x[i] = u(r);
        for (std::ptrdiff_t i = 0; i < ndof; ++i) std::printf("%.17g\n", b[i]);
        for (std::ptrdiff_t i = 0; i < ndof; ++i) std::printf("%.17g\n", x[i]);
        smoother->apply(b, x);
        for (std::ptrdiff_t i = 0; i < ndof; ++i) std::printf("%.17g\n", x[i]);
        return 0;
    }
    std::fprintf(stderr, "usage: adapter_client describe | sample <n> <fd|fem|periodic> | rngcheck | "
                         "smoother <fd|fem|periodic> <sor|ssor> <nsmooth> <fwd|bwd> [lowrank] | ownership <rounds>\n");
    return 2;
}
