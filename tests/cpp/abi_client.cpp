// C++ client of include/mgmc_sampler.hh (the host side a reference maintainer would call from
// driver_mgmc).  Modes:
//   abi_client describe            host only: print the level hierarchy of the 3D 64^3 4-level config
//   abi_client sample NSTEPS       create a 3D 16^3 3-level sampler (seed 5418513) and print the QoI series
// On a host without a GPU `sample` must print the library's error and exit(-1) (reference convention).
#include <cstdio>
#include <cstring>

#include "mgmc_sampler.hh"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    mgmc::MultigridParameters p;
    if (!std::strcmp(argv[1], "describe")) {
        p.nlevel = 4;
        const mgmc_config c = mgmc::make_config(3, 64, 64, 64, 25.0, p);
        mgmc_level_desc d[4];
        mgmc::check(mgmc_describe(&c, d, 4), nullptr, "mgmc_describe");
        std::printf("abi %d\n", mgmc_abi_version());
        for (int l = 0; l < 4; ++l)
            std::printf("level %d n %d ndof %llu npoints %d ncolours %d centre %.17g\n", l, d[l].nx,
                        (unsigned long long)d[l].ndof, d[l].npoints, d[l].ncolours, d[l].stencil[13]);
        return 0;
    }
    if (!std::strcmp(argv[1], "sample")) {
        const int nsteps = argc > 2 ? std::atoi(argv[2]) : 4;
        p.nlevel = 3;
        const mgmc_config c = mgmc::make_config(3, 16, 16, 16, 25.0, p);
        mgmc::HipMultigridMCSampler s(c, 0, 5418513ull, 0);
        const int64_t qoi = 7 * 15 * 15 + 7 * 15 + 7;  // vertex (8,8,8)
        const auto q = s.sample(nsteps, qoi);
        for (double v : q) std::printf("%.17g\n", v);
        return 0;
    }
    return 2;
}
