"""In-cycle timing of library builds: for each library (product or build/libmgmc_<name>.so; "<lib>+VAR=value"
adds an environment switch, e.g. 0+MGMC_DISABLE=sym), K timed
N^3 (default 512^3, NLEVEL 7; env N / NLEVEL) V-cycles (mgmc_sample_timed: fine pre / post sweep segments) in a fresh child process, and the
plain single-graph replay of the same K cycles.  python scripts/lib_cycle_bench.py [exps, 0 = product]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, time
sys.path.insert(0, %r)
import multigridmc_amd as mg
import os
n, nl = int(os.environ.get("N", "512")), int(os.environ.get("NLEVEL", "7"))
lat = mg.Lattice3d(n, n, n)
s = mg.MultigridMCSampler(mg.ShiftedLaplaceFDOperator(lat, 25.0), 1, mg.MultigridParameters(nlevel=nl))
s.sample(5)
import hashlib
digest = hashlib.sha1(s.get_state().tobytes()).hexdigest()[:12]  # same bits in every correct build
best = None
for _ in range(3):
    t = s.sample_timed(30)
    s.synchronize(); t0 = time.perf_counter(); s.sample_async(30); s.synchronize(); plain = (time.perf_counter() - t0) / 30 * 1e3
    r = {"pre_ms": t["pre_ms"] / t["npre"], "post_ms": t["post_ms"] / t["npost"], "timed_cycle_ms": t["total_ms"] / 30,
         "plain_cycle_ms": plain}
    best = r if best is None or r["timed_cycle_ms"] < best["timed_cycle_ms"] else best
best["state_sha1"] = digest
print(json.dumps(best))
'''
libs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["0"]
for x in [x for _ in range(int(os.environ.get("REPS", "1"))) for x in libs]:  # interleaved repetitions
    env = dict(os.environ)
    lib, _, extra = x.partition("+")  # "<lib>+VAR=value": the library with an environment switch
    if extra:
        k, _, v = extra.partition("=")
        env[k] = v
    if lib != "0":
        env["MGMC_LIBRARY"] = os.path.join(ROOT, "build", f"libmgmc_{lib}.so")
    r = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=300)
    print(x, r.stdout.strip().splitlines()[-1] if r.returncode == 0 else f"FAILED {r.stderr[-400:]}", flush=True)
