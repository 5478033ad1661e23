#!/usr/bin/env python3
"""HBM traffic per launch of every kernel of a V-cycle, from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE) of scripts/vcycle_once.py, grouped by kernel instance and grid.  Corrected as
MI355X_MICROARCH.md's HBM section prescribes (KiB counters, FETCH_SIZE x 2 on gfx950 for the 16-byte
per lane loads these kernels issue; WRITE_SIZE exact).  Algorithmic bytes per launch are given for
the kernels SURVEY.md section 8(d) prices (n = fine cells):
  fine sweeps 24 B x N0 (+ 8 B x N1 with the fused prolongation), fine residual + restriction
  16 B x N0 + 16 B x N1, level-1 half-sweep 12 B x N1 (half of a 24 B sweep), level-1 residual +
  restriction 16 B x N1 + 16 B x N2, level-2 -> 1 prolongation 16 B x N1 + 8 B x N2.

usage: pmc_by_kernel.py <dir>/pmc_FETCH_SIZE <dir>/pmc_WRITE_SIZE [n]
"""
import collections
import csv
import glob
import re
import sys


def load(d):
    out = collections.defaultdict(list)
    for f in glob.glob(f"{d}/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"^void ", "", r["Kernel_Name"]).replace("mgmc::", "")
            name = re.sub(r"\(.*$", "", name)
            out[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def main():
    fetch, write = load(sys.argv[1]), load(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 512
    N = [(n // 2 ** l - 1) ** 3 for l in range(4)]
    rows = []
    for key in fetch:
        fb = 2.0 * 1024.0 * sum(fetch[key]) / len(fetch[key])
        wb = 1024.0 * sum(write.get(key, [0.0])) / max(1, len(write.get(key, [1])))
        name, grid = key
        algo = None
        if name.startswith("k_zsweep_rb7"):
            prolong = name.split(",")[3].strip() != "0"
            algo = 24.0 * N[0] + (8.0 * N[1] if prolong else 0.0)
        elif name.startswith("k_zresrestrict<7"):
            algo = 16.0 * N[0] + 16.0 * N[1]
        elif name.startswith("k_jsweep_half<128"):
            algo = 12.0 * N[1]
        elif name.startswith("k_zresrestrict<27, 64") and fb > 0.2 * 16.0 * N[1]:
            algo = 16.0 * N[1] + 16.0 * N[2]
        elif name.startswith("k_prolongate_pairs") and fb + wb > 0.5 * 16.0 * N[1]:
            algo = 16.0 * N[1] + 8.0 * N[2]
        rows.append((fb + wb, name, grid, len(fetch[key]), fb, wb, algo))
    print(f"# FETCH_SIZE x2 + WRITE_SIZE (KiB x 1024) per launch, {n}^3 V-cycles; traffic / algorithmic where priced")
    print(f"{'kernel':60s} {'grid':>9s} {'launches':>8s} {'fetch_MB':>9s} {'write_MB':>9s} {'total_MB':>9s} {'x alg':>6s}")
    for tot, name, grid, nl, fb, wb, algo in sorted(rows, reverse=True)[:24]:
        ratio = f"{tot / algo:6.3f}" if algo else "     -"
        print(f"{name[:60]:60s} {grid:9d} {nl:8d} {fb / 1e6:9.1f} {wb / 1e6:9.1f} {tot / 1e6:9.1f} {ratio}")


if __name__ == "__main__":
    main()
