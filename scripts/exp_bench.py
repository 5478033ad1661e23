"""Fine-sweep timing of experiment builds (build/libmgmc_<N>.so, see scripts/build_exp.sh) against the
product library.  python scripts/exp_bench.py [exps, 0 = product]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, os
sys.path.insert(0, %r)
import multigridmc_amd as mg
lat = mg.Lattice3d(512, 512, 512)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=7))
s.time_fine_sweeps(2)
print(min(s.time_fine_sweeps(10) / 10 for _ in range(3)))
'''
exps = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0", "1", "2", "3", "4"]
names = {"0": "product", "1": "no-BoxMuller", "2": "no-halo", "3": "no-Philox", "4": "no-stencil", "5": "skeleton", "6": "no-barriers", "7": "nt-store", "8": "nt-f", "9": "nt-store+f"}
for x in exps:
    env = dict(os.environ)
    if x != "0":
        env["MGMC_LIBRARY"] = os.path.join(ROOT, "build", f"libmgmc_{x}.so")  # x = N or s<shape>
    r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f"FAILED {r.stderr[-300:]}"
    print(f"{names.get(x, x):14s} {out}", flush=True)
