// Test scaffolding (tests/cpp/refdecl/README.md): MultigridParameters' fields --
// auxilliary/parameters.hh:145-174 (libconfig parsing left out).
#pragma once
#include <string>

class MultigridParameters {
   public:
    unsigned int nlevel;
    std::string smoother;
    std::string coarse_solver;
    unsigned int npresmooth;
    unsigned int npostsmooth;
    unsigned int ncoarsesmooth;
    double omega;
    unsigned int cycle;
    double coarse_scaling;
    int verbose;
};
