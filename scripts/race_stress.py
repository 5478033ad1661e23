#!/usr/bin/env python3
"""LDS-race stress of the standalone fine sweep: for each library (product or build/libmgmc_<name>.so), a
child process with MGMC_POISON=1 (the LDS of every CU is filled with NaN before each sweep) runs REPS
level-0 noisy sweeps (mgmc_sor_sampler_apply, 256^3, both directions) on one input and counts the
results that are not bitwise equal to the first one, and the non-finite ones.  A kernel that reads LDS
no wave of its own workgroup wrote shows up as a NaN or a changed bit.
usage: race_stress.py [lib ...] (0 = product)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json
sys.path.insert(0, %r)
import numpy as np
import multigridmc_amd as mg
n, reps = 256, int(sys.argv[1])
lat = mg.Lattice3d(n, n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=6))
m = s.level_desc(0)["ndof"]
rng = np.random.default_rng(400)
f, x = rng.standard_normal(m), rng.standard_normal(m)
out = {}
for d, name in ((mg.BACKWARD, "backward"), (mg.FORWARD, "forward")):
    ref = s.sor_sampler_apply(0, d, 5, 17, f, x)
    diff = nonfinite = 0
    for _ in range(reps):
        r = s.sor_sampler_apply(0, d, 5, 17, f, x)
        nonfinite += int(not np.isfinite(r).all())
        diff += int(not np.array_equal(r, ref))
    out[name] = {"reps": reps, "differ": diff, "nonfinite": nonfinite, "ref_finite": bool(np.isfinite(ref).all())}
print(json.dumps(out))
''' % ROOT

for ent in sys.argv[1:] or ["0"]:
    env = dict(os.environ, MGMC_POISON="1")
    env["MGMC_LIBRARY"] = "" if ent == "0" else os.path.join(ROOT, "build", f"libmgmc_{ent}.so")
    r = subprocess.run([sys.executable, "-c", CHILD, os.environ.get("REPS", "40")], env=env, capture_output=True,
                       text=True, timeout=600)
    line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else r.stderr[-600:]
    print(ent, line, flush=True)
