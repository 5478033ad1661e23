"""Host-side bounds check of the padded level layouts (mgmc_layout_check.hpp, CPU only).

Every kernel addresses a level as L.at(i, j, k) + chain * nstore with unconditional loads, so the
extreme coordinates of each kernel family must stay inside [0, nstore) of each chain's copy (the
batched chains are nstore apart, so the per-chain range is the whole condition).  mgmc_create runs
the check on every level; here it runs over many lattice shapes with the union of all families
(a superset of what any level uses), and it is shown to catch the two layouts that were out of
bounds: round 2's reach-2 layout without margin rows / planes (the fault fixed in 185bd2c) and the
residual + restriction's unclamped last-tile columns (lattices with n/2 - 1 = 1 mod 64, e.g. 132)."""
import ctypes

import pytest

import multigridmc_amd as mg
from multigridmc_amd import _native

ALL2 = 1 | 2 | 32 | 128     # point, pairs, rb2d, fused last pre-sweep + residual + restriction
ALL3 = 1 | 2 | 4 | 8 | 16   # point, pairs, zsweep (+ coarse side), z-marching residual + restriction
JSWEEP = 64                 # j-marching half-sweeps (levels with nx = 256 / 512): box + whole-grid replay


def check(shape, reach=1, families=None, cx=None, legacy=0):
    dim = len(shape)
    n = (ctypes.c_int * 3)(*(list(shape) + [0] * (3 - dim)))
    if families is None:
        families = ALL3 if dim == 3 else ALL2
        if dim == 3 and shape[0] in (256, 512):
            families |= JSWEEP
    if cx is None:
        cx = 0 if dim == 2 else (16 if shape[0] // 2 < 32 else 64)
    return mg.load_library().mgmc_check_layout(dim, n, reach, families, cx, legacy)


def hierarchy(shape, nlevel=12):
    out = [tuple(shape)]
    while len(out) < nlevel and all(v % 2 == 0 and v // 2 > 1 for v in out[-1]):
        out.append(tuple(v // 2 for v in out[-1]))
    return out


SHAPES = ([(n, n) for n in range(4, 1030, 6)] + [(n, 2 * n + 4) for n in range(4, 300, 10)] +
          [(n, n, n) for n in range(4, 300, 4)] + [(132, 36, 20), (260, 68, 8), (512, 16, 24), (68, 132, 260)])


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_every_level_inside_its_store(shape):
    for lv in hierarchy(shape):
        assert check(lv) == _native.MGMC_OK, mg.load_library().mgmc_last_error(None)


@pytest.mark.parametrize("shape", [(16, 16), (32, 64), (64, 32), (130, 66), (1024, 1024)])
def test_reach2_levels_need_the_margin(shape):
    """Squared FD (2D) levels read rows / columns two apart: inside with the margin, and the round-2
    layout without it starts before the allocation (the GPU fault of round 2)."""
    for lv in hierarchy(shape):
        assert check(lv, reach=2) == _native.MGMC_OK
    rc = check(shape, reach=2, legacy=1)
    assert rc == _native.MGMC_E_INVALID
    assert b"leave the level store [0," in mg.load_library().mgmc_last_error(None)


@pytest.mark.parametrize("n", [132, 260, 388])
def test_restriction_last_tile_columns_clamped(n):
    """n/2 - 1 = 1 (mod 64): the last 64-wide tile of the residual + restriction ran 2 CX - 2
    columns past the row; on the last row of the last plane that is past the store.  The clamp keeps
    it inside; the unclamped form is flagged."""
    shape = (n, 16, 16)
    assert check(shape) == _native.MGMC_OK
    assert check(shape, legacy=2) == _native.MGMC_E_INVALID
    assert b"residual + restriction" in mg.load_library().mgmc_last_error(None)
    assert check((512, 16, 16), legacy=2) == _native.MGMC_OK  # powers of two never reached it


@pytest.mark.parametrize("shape", [(256, 256, 256), (512, 512, 512), (256, 24, 20), (512, 24, 20), (256, 2, 2),
                                   (256, 4, 6), (512, 130, 66), (256, 256, 6)],
                         ids=lambda s: "x".join(map(str, s)))
def test_jsweep_grid_replay(shape):
    """k_jsweep_half (round 3): the host replay of its whole grid -- XCD tile order, chunk steps
    s0-1 .. s1, the idle steps of the unrolled loop, loads JS_D steps ahead, f loads, stores -- with
    launch_jsweep's own plan (both directions, both k-parity halves) stays inside rows [0, ny] and
    planes [0, nz], stores only interior rows, and covers every (plane, chunk) tile exactly once."""
    assert check(shape, families=JSWEEP) == _native.MGMC_OK, mg.load_library().mgmc_last_error(None)


def test_jsweep_grid_replay_rejects_a_short_grid():
    """Negative control: the same replay with the plan's last 8 workgroups dropped reports the
    (plane, chunk) tiles nobody sweeps."""
    assert check((512, 512, 512), families=JSWEEP, legacy=4) == _native.MGMC_E_INVALID
    assert b"not covered by the grid" in mg.load_library().mgmc_last_error(None)
