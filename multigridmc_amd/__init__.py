"""multigridmc_amd -- MI355X-native Multigrid Monte Carlo sampler (HIP / gfx950).

The hot path (one MGMC cycle: multicolour Gibbs sweeps with fused Philox noise, fused
residual+restriction, prolongate-add, single-workgroup coarse SSOR sampler) lives in
csrc/*.hip behind the C-ABI of include/mgmc.h; this package is the host-side mirror of the
reference's Sampler / LinearOperator interfaces.
"""
from ._native import QOI_VECTOR, MgmcError, load_library  # noqa: F401
from .measured import LowRankUpdate, MeasuredOperator, measurement_vector, synthetic_posterior  # noqa: F401
from .parameters import MultigridParameters, read_config  # noqa: F401
from .sampler import (  # noqa: F401
    BACKWARD,
    FORWARD,
    HipMulticolourSORSmoother,
    Lattice,
    Lattice2d,
    Lattice3d,
    MultigridMCSampler,
    ShiftedLaplaceFDOperator,
    ShiftedLaplaceFEMOperator,
    SquaredShiftedLaplaceFDOperator,
    SparseMatrixOperator,
    SORSmoother,
    SORSmootherFactory,
    SSORSmoother,
    SSORSmootherFactory,
    ConstantCorrelationLengthModel,
    PeriodicCorrelationLengthModel,
    comm_unique_id,
    csr_colour_scheme,
    describe,
    make_config,
    measurement_vector_index,
    sampler_csr_matrix,
)

__version__ = "0.1.0"
