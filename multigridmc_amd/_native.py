"""ctypes binding of the C-ABI in include/mgmc.h (libmgmc_hip.so, built in-tree for gfx950).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, importing the
device path raises.  The CPU oracle under oracle/ is test infrastructure and is never used here.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmgmc_hip.so")

MGMC_OK = 0
MGMC_E_INVALID = -1
MGMC_E_HIP = -2
MGMC_E_NOMEM = -3
MGMC_E_UNSUPPORTED = -4
MGMC_E_NONFINITE = -5
QOI_VECTOR = -2  # mgmc_sample's qoi_index for the vector of mgmc_set_qoi_vector

SMOOTHER_SOR = 0
SMOOTHER_SSOR = 1
COARSE_SSOR = 0
COARSE_CHOLESKY = 1
OPERATOR_FD = 0
OPERATOR_FEM = 1
OPERATOR_SQUARED_FD = 2
KAPPA_CONSTANT = 0
KAPPA_PERIODIC = 1
KAPPA_GIVEN = 2
ABI_VERSION = 5
SOLVER_LOOP = 0
SOLVER_CG = 1
FORWARD = 1
BACKWARD = 2


class MgmcConfig(ctypes.Structure):
    _fields_ = [
        ("dim", c_int), ("nx", c_int), ("ny", c_int), ("nz", c_int),
        ("nlevel", c_int), ("cycle", c_int),
        ("npresmooth", c_int), ("npostsmooth", c_int), ("ncoarsesmooth", c_int),
        ("smoother", c_int), ("coarse_solver", c_int), ("verbose", c_int),
        ("omega", c_double), ("coarse_scaling", c_double), ("kappa_sq", c_double),
        ("fine_operator", c_int), ("pad_", c_int),
    ]


class MgmcLevelDesc(ctypes.Structure):
    _fields_ = [
        ("nx", c_int), ("ny", c_int), ("nz", c_int),
        ("npoints", c_int), ("ncolours", c_int), ("varcoef", c_int),
        ("ndof", c_uint64),
        ("stencil", c_double * 27),
    ]


class MgmcOperatorDesc(ctypes.Structure):
    _fields_ = [
        ("dim", c_int), ("nx", c_int), ("ny", c_int), ("nz", c_int),
        ("pde", c_int), ("kappa_model", c_int),
        ("Lambda", c_double), ("Lambda_min", c_double), ("Lambda_max", c_double), ("kappa_sq", c_double),
    ]


class MgmcError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"mgmc error {code}: {message}")
        self.code = code


# (name, restype, argtypes) -- every symbol declared in include/mgmc.h
_DP = POINTER(c_double)
_H = c_void_p
SIGNATURES = [
    ("mgmc_abi_version", c_int, []),
    ("mgmc_live_handles", c_int, []),
    ("mgmc_describe", c_int, [POINTER(MgmcConfig), POINTER(MgmcLevelDesc), c_int]),
    ("mgmc_last_error", c_char_p, [_H]),
    ("mgmc_create", c_int, [POINTER(MgmcConfig), c_int, c_uint64, c_uint64, POINTER(c_void_p)]),
    ("mgmc_create_csr", c_int, [POINTER(MgmcConfig), c_int64, POINTER(c_int64), POINTER(ctypes.c_int32), _DP, c_int,
                                c_uint64, c_uint64, POINTER(c_void_p)]),
    ("mgmc_operator_csr_size", c_int, [POINTER(MgmcOperatorDesc), POINTER(c_int64), POINTER(c_int64)]),
    ("mgmc_operator_csr", c_int, [POINTER(MgmcOperatorDesc), POINTER(c_int64), POINTER(ctypes.c_int32), _DP]),
    ("mgmc_csr_colour_scheme", c_int, [POINTER(MgmcConfig), c_int, c_int64, POINTER(c_int64), POINTER(ctypes.c_int32),
                                       POINTER(c_int)]),
    ("mgmc_check_layout", c_int, [c_int, POINTER(c_int), c_int, ctypes.c_uint, c_int, c_int]),
    ("mgmc_stencil_of_csr", c_int, [POINTER(MgmcConfig), c_int64, POINTER(c_int64), POINTER(ctypes.c_int32), _DP,
                                    _DP]),
    ("mgmc_create_stencil_batch", c_int, [POINTER(MgmcConfig), _DP, c_int, c_uint64, c_uint64, c_int,
                                          POINTER(c_void_p)]),
    ("mgmc_create_batch", c_int, [POINTER(MgmcConfig), c_int, c_uint64, c_uint64, c_int, POINTER(c_void_p)]),
    ("mgmc_create_csr_batch", c_int, [POINTER(MgmcConfig), c_int64, POINTER(c_int64), POINTER(ctypes.c_int32), _DP,
                                      c_int, c_uint64, c_uint64, c_int, POINTER(c_void_p)]),
    ("mgmc_nchains", c_int, [_H]),
    ("mgmc_destroy", c_int, [_H]),
    ("mgmc_level_desc_get", c_int, [_H, c_int, POINTER(MgmcLevelDesc)]),
    ("mgmc_level_kernels", c_int, [_H, c_int, ctypes.c_char_p, c_size_t]),
    ("mgmc_set_lowrank", c_int, [_H, c_int, POINTER(c_int64), POINTER(c_int64), _DP, _DP]),
    ("mgmc_lowrank_info", c_int, [_H, c_int, c_int, POINTER(c_int), POINTER(c_int64)]),
    ("mgmc_debug_fail_coarse_factor", c_int, [_H, c_int]),
    ("mgmc_set_rhs", c_int, [_H, _DP, c_size_t]),
    ("mgmc_set_state", c_int, [_H, _DP, c_size_t]),
    ("mgmc_get_state", c_int, [_H, _DP, c_size_t]),
    ("mgmc_set_state_chain", c_int, [_H, c_int, _DP, c_size_t]),
    ("mgmc_get_state_chain", c_int, [_H, c_int, _DP, c_size_t]),
    ("mgmc_apply", c_int, [_H, _DP, _DP, c_size_t]),
    ("mgmc_sample", c_int, [_H, c_int, c_int64, _DP]),
    ("mgmc_set_qoi_vector", c_int, [_H, c_int64, POINTER(c_int64), _DP]),
    ("mgmc_sample_async", c_int, [_H, c_int, c_int64]),
    ("mgmc_synchronize", c_int, [_H]),
    ("mgmc_qoi_moments", c_int, [_H, _DP]),
    ("mgmc_qoi_moments_chain", c_int, [_H, c_int, _DP]),
    ("mgmc_reset_moments", c_int, [_H]),
    ("mgmc_set_sample_index", c_int, [_H, c_uint64]),
    ("mgmc_get_sample_index", c_int, [_H, POINTER(c_uint64)]),
    ("mgmc_get_series", c_int, [_H, POINTER(c_double), c_size_t]),
    ("mgmc_get_series_chain", c_int, [_H, c_int, POINTER(c_double), c_size_t]),
    ("mgmc_get_stream", c_int, [_H, POINTER(c_void_p)]),
    ("mgmc_operator_apply", c_int, [_H, c_int, _DP, _DP]),
    ("mgmc_smoother_apply", c_int, [_H, c_int, c_int, c_int, _DP, _DP]),
    ("mgmc_sor_smoother_apply", c_int, [_H, c_int, c_int, c_int, _DP, _DP]),
    ("mgmc_ssor_smoother_apply", c_int, [_H, c_int, c_int, _DP, _DP]),
    ("mgmc_sor_sampler_apply", c_int, [_H, c_int, c_int, c_uint32, c_uint64, _DP, _DP]),
    ("mgmc_restrict", c_int, [_H, c_int, _DP, _DP]),
    ("mgmc_prolongate_add", c_int, [_H, c_int, c_double, _DP, _DP]),
    ("mgmc_residual_restrict", c_int, [_H, c_int, _DP, _DP, _DP]),
    ("mgmc_normals", c_int, [_H, c_uint64, c_size_t, c_uint32, c_uint64, _DP]),
    ("mgmc_solve", c_int, [_H, c_int, _DP, _DP, c_double, c_double, c_int, POINTER(c_int), _DP]),
    ("mgmc_time_fine_sweeps", c_int, [_H, c_int, POINTER(c_float)]),
    ("mgmc_sample_timed", c_int, [_H, c_int, c_int64, _DP, _DP, POINTER(c_int), _DP, POINTER(c_int)]),
    ("mgmc_sample_timed_stride", c_int, [_H, c_int, c_int, c_int64, _DP, _DP, POINTER(c_int), _DP, POINTER(c_int)]),
    ("mgmc_comm_unique_id", c_int, [ctypes.c_char_p]),
    ("mgmc_comm_init", c_int, [_H, c_int, c_int, ctypes.c_char_p]),
    ("mgmc_comm_allgather_moments", c_int, [_H, _DP]),
    ("mgmc_comm_allreduce_max", c_int, [_H, _DP]),
    ("mgmc_comm_barrier", c_int, [_H]),
    ("mgmc_comm_destroy", c_int, [_H]),
    ("mgmc_comm_info", c_int, [_H, ctypes.POINTER(c_int), ctypes.POINTER(c_int), ctypes.POINTER(c_int)]),
]

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libmgmc_hip.so and bind every C-ABI symbol; raises if the library is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("MGMC_LIBRARY") or LIB_PATH  # MGMC_LIBRARY: experiment builds (build/)
    if not os.path.exists(p):
        raise ImportError(
            f"{p} not found: the HIP extension is not built (run `python -c 'import __graft_entry__ as g; g.build()'`)")
    lib = ctypes.CDLL(p)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.mgmc_abi_version() != ABI_VERSION:  # the config struct layout changes with the ABI
        raise ImportError(f"{p}: ABI {lib.mgmc_abi_version()}, this package needs {ABI_VERSION} (rebuild)")
    if path is None:
        _lib = lib
    return lib


def last_error(handle=None) -> str:
    msg = load_library().mgmc_last_error(handle)
    return msg.decode() if msg else ""


def check(code: int, handle=None) -> int:
    if code < 0:
        raise MgmcError(code, last_error(handle))
    return code
