"""Phase times of k_tail (timing build MGMC_TAIL_PROF: CXXDEFS=-DMGMC_TAIL_PROF VARIANTS="tprof=-" bash
scripts/build_exp.sh; MGMC_LIBRARY=build/libmgmc_tprof.so python scripts/tail_prof.py [n] [nlevel] [npoints]).
Runs a few prior V-cycles and prints the wall-clock time of every phase of the first tail: the LDS
fill from HBM, each op's right-hand sides (sweeps) and the rest of the op, the store."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multigridmc_amd as mg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
nl = int(sys.argv[2]) if len(sys.argv) > 2 else 7
npost = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # > 0: config 5's posterior with that many points
lat = mg.Lattice3d(n, n, n)
op = mg.ShiftedLaplaceFDOperator(lat, 25.0)
if npost > 0:
    op = mg.synthetic_posterior(op, npost, 0.0, False)
s = mg.MultigridMCSampler(op, 1, mg.MultigridParameters(nlevel=nl))
lib = mg.load_library()
f = lib.mgmc_debug_tail_profile
f.restype = ctypes.c_int
KIND = {0: "sweep", 1: "restrict", 2: "prolong", 3: "coarse"}
for rep in range(3):
    s.sample(5)
    out = (ctypes.c_ulonglong * 256)()
    kinds = (ctypes.c_int * 96)()
    nops, rate = ctypes.c_int(), ctypes.c_int()
    rc = f(s.handle, out, 256, kinds, ctypes.byref(nops), ctypes.byref(rate))
    assert rc == 0, rc
    us = 1e3 / rate.value  # microseconds per tick
    t = list(out)
    print(f"rep {rep}: total {(t[2 + 2 * nops.value] - t[0]) * us:.1f} us, load {(t[1] - t[0]) * us:.1f} us")
    prev = t[1]
    for o in range(nops.value):
        k, lv = kinds[o] % 16, kinds[o] // 16
        if k in (0, 3):
            print(f"  op {o:2d} {KIND[k]:8s} level {lv}: rhs {(t[2 + 2 * o] - prev) * us:6.2f} us, "
                  f"passes {(t[3 + 2 * o] - t[2 + 2 * o]) * us:6.2f} us")
        else:
            print(f"  op {o:2d} {KIND[k]:8s} level {lv}: {(t[3 + 2 * o] - prev) * us:6.2f} us")
        prev = t[3 + 2 * o]
    print(f"  store {(t[2 + 2 * nops.value] - prev) * us:.2f} us", flush=True)
s.close()
