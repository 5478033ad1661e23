"""HBM traffic per fine-sweep launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of
scripts/vcycle_once.py (V-cycles at n^3), for both level-0 sweeps of the cycle: the plain pre-sweep
(k_zsweep_rb7<..., PROLONG = 0, ...>) and the post-sweep with the fused prolongation (PROLONG > 0).
Corrected as MI355X_MICROARCH.md (HBM section) prescribes: counters are in KiB, and on gfx950
FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads (the z-sweep's loads are all 16-B
double2 loads) -> FETCH x 2; WRITE_SIZE is exact for 16-B stores.

  python scripts/pmc_traffic.py gpurun_out/round profiles/pmc_traffic.json [n] [head]
"""
import csv
import datetime
import json
import re
import subprocess
import sys

# <XP, TY, NT, PROLONG, MINW[, LRF]>: the prior's instances (LRF = false, the low-rank posterior's in-place
# right-hand side: not part of the bench)
KERNEL = re.compile(r"k_zsweep_rb7<\s*(\d+),\s*(\d+),\s*(\d+),\s*(\d+),\s*(\d+)\s*(?:,\s*false\s*)?>")


def per_launch(path, post):
    vals, name = [], None
    for r in csv.DictReader(open(path)):
        m = KERNEL.search(r["Kernel_Name"])
        if m and (int(m.group(4)) > 0) == post:
            vals.append(float(r["Counter_Value"]))
            name = m.group(0)
    return sum(vals) / len(vals), len(vals), name


def main():
    src, dst = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    head = sys.argv[4] if len(sys.argv) > 4 else subprocess.run(
        ["git", "rev-parse", "--short=12", "HEAD"], capture_output=True, text=True).stdout.strip()
    n0 = (n - 1) ** 3
    n1 = (n // 2 - 1) ** 3
    out = {"n": n, "head": head, "date": datetime.date.today().isoformat(),
           "source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes) of scripts/vcycle_once.py",
           "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane reads), KiB -> bytes x1024 (MI355X_MICROARCH.md HBM section)"}
    for key, post, algo in (("pre_sweep", False, 24.0 * n0), ("post_sweep", True, 24.0 * n0 + 8.0 * n1)):
        fetch_kib, nf, name = per_launch(f"{src}/pmc_FETCH_SIZE/pmc_counter_collection.csv", post)
        write_kib, nw, _ = per_launch(f"{src}/pmc_WRITE_SIZE/pmc_counter_collection.csv", post)
        fetch = 2.0 * fetch_kib * 1024.0
        write = write_kib * 1024.0
        out[key] = {"kernel": name, "launches": [nf, nw], "fetch_size_kib_raw": fetch_kib,
                    "write_size_kib_raw": write_kib, "fetch_bytes_corrected": fetch, "write_bytes": write,
                    "hbm_bytes_per_launch": fetch + write, "algorithmic_bytes_per_launch": algo,
                    "traffic_over_algorithmic": (fetch + write) / algo}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
