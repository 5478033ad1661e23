#!/usr/bin/env python3
"""Where the waves' cycles go, per kernel instance: one rocprofv3 --pmc pass of SQ counters over V-cycles
(scripts/gpu_r6_final2.sh: SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU).  Columns in % of SQ_WAVE_CYCLES: wait = parked on
s_waitcnt / barrier, instwait = issue stalls, active = issuing (the three are disjoint), ldswait, valu,
lds; then VALU instructions per launch.

usage: sq_table.py <dir with *counter_collection.csv> [rows]
"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
nrows = int(sys.argv[2]) if len(sys.argv) > 2 else 16
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"^void ", "", r["Kernel_Name"]).replace("mgmc::", "")
        name = re.sub(r"\(.*$", "", name)[:46]
        vals[(name, int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))


def avg(d, c):
    v = d.get(c)
    return sum(v) / len(v) if v else float("nan")


print("# SQ wave-cycle split per kernel (% of SQ_WAVE_CYCLES), 512^3 V-cycles")
print(f"{'kernel':46s} {'grid':>9s} {'wave_cyc':>9s} {'wait%':>6s} {'instw%':>6s} {'active%':>7s} {'ldsw%':>6s} "
      f"{'valu%':>6s} {'lds%':>5s} {'insts_valu':>10s}")
rows = sorted(vals.items(), key=lambda kv: -avg(kv[1], "SQ_WAVE_CYCLES"))
for (name, grid), c in rows[:nrows]:
    w = avg(c, "SQ_WAVE_CYCLES")
    pct = lambda k: 100.0 * avg(c, k) / w if w > 0 else float("nan")  # noqa: E731
    print(f"{name:46s} {grid:9d} {w:9.3g} {pct('SQ_WAIT_ANY'):6.1f} {pct('SQ_WAIT_INST_ANY'):6.1f} "
          f"{pct('SQ_ACTIVE_INST_ANY'):7.1f} {pct('SQ_WAIT_INST_LDS'):6.1f} {pct('SQ_ACTIVE_INST_VALU'):6.1f} "
          f"{pct('SQ_ACTIVE_INST_LDS'):5.1f} {avg(c, 'SQ_INSTS_VALU'):10.3g}")
