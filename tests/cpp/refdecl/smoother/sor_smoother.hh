// Test scaffolding (tests/cpp/refdecl/README.md): the sweep direction of smoother/sor_smoother.hh:14-18
// (the reference's SORSmoother class itself is what include/reference_adapter/hip_sor_smoother.hh
// stands in for, so it is not restated).
#pragma once
#include "smoother.hh"

enum Direction { forward = 1, backward = 2 };
