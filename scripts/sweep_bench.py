"""Micro-benchmark of the fine-level sweep and of the whole V-cycle (GPU box), default paths and with
fast paths switched off (MGMC_DISABLE).  Usage: python scripts/sweep_bench.py [n] [nlevel]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r'''
import sys, json, os
sys.path.insert(0, %r)
import multigridmc_amd as mg
n, nlevel = %d, %d
lat = mg.Lattice3d(n, n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=nlevel))
s.time_fine_sweeps(2)
ms = min(s.time_fine_sweeps(10) / 10 for _ in range(3))
s.sample(3)
_t = s.sample_timed(10); tot, fine, nfine = _t["total_ms"], _t["pre_ms"], _t["npre"]
print(json.dumps({"sweep_ms": ms, "GBps": 24 * lat.Nvertex / ms / 1e6, "vcycle_ms": tot / 10,
                  "fine_in_cycle_ms": fine / nfine}))
'''

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
nlevel = int(sys.argv[2]) if len(sys.argv) > 2 else 7
variants = [("default", {}), ("no-fuse-prolong", {"MGMC_DISABLE": "fuse_prolong"})]
for name, env in variants:
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, n, nlevel)], env=e, capture_output=True, text=True,
                       timeout=300)
    if r.returncode != 0:
        print(name, "FAILED rc", r.returncode, r.stderr[-500:], flush=True)
        if r.returncode not in (0, 1):
            sys.exit(r.returncode)
        continue
    print(name, r.stdout.strip().splitlines()[-1], flush=True)
