"""Interleaved A/B of bench.py V-cycle time over env configurations (repeated runs, GPU box).
python scripts/ab_bench.py reps 'name:VAR=val,VAR2=val' ..."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
reps = int(sys.argv[1])
cfgs = []
for spec in sys.argv[2:]:
    name, _, envs = spec.partition(":")
    env = dict(kv.split("=", 1) for kv in envs.split(",") if kv)
    cfgs.append((name, env))
res = {n: [] for n, _ in cfgs}
for r in range(reps):
    for name, env in cfgs:
        e = dict(os.environ, **env)
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "200", "--warmup", "10",
                              "--no-cpu-baseline"], env=e, capture_output=True, text=True, timeout=600)
        if out.returncode != 0:
            print(name, "FAILED", out.stderr[-400:], flush=True)
            sys.exit(out.returncode)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[name].append(d["ms_per_step"])
        print(name, r, d["ms_per_step"], d["roofline"]["avg_launch_ms"], flush=True)
for name, v in res.items():
    print(f"{name:24s} median {statistics.median(v):.4f} ms  min {min(v):.4f}  max {max(v):.4f}")
