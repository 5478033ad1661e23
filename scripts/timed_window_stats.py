#!/usr/bin/env python3
"""Per-kernel statistics of a rocprofv3 kernel trace restricted to the bench's timed window.

rocprofv3 --stats averages every launch of the process, including the warm-up cycles (the first
launches of a fresh process run slower: caches, clocks).  bench.py times only its last K cycles.  This
script finds the cycle boundaries from the fine pre-sweep launches (one per cycle), keeps the launches
of the last K cycles, and prints per-kernel count / average / min / max, plus, given the bench's JSON
line, the relative difference between the trace's fine-sweep averages and the line's
roofline.per_kernel avg_launch_ms.

usage: timed_window_stats.py kernel_trace.csv K [bench.json] > summary.csv
"""
import csv
import json
import sys
from collections import defaultdict


def kernel_key(name):
    base = name.split("(")[0]
    # the two fine sweeps are instances of one template: keep the template arguments
    if "k_zsweep_rb7" in name:
        return "k_zsweep_rb7<" + name.split("k_zsweep_rb7<")[1].split(">")[0] + ">"
    if "k_zresrestrict" in name:
        return "k_zresrestrict<" + name.split("k_zresrestrict<")[1].split(">")[0] + ">"
    if "k_jsweep_half" in name:
        return "k_jsweep_half<" + name.split("k_jsweep_half<")[1].split(">")[0] + ">"
    return base[:60]


def is_pre_sweep(name):
    # k_zsweep_rb7<32, TY, NT, PROLONG = 0, MINW>
    if "k_zsweep_rb7" not in name:
        return False
    args = name.split("k_zsweep_rb7<")[1].split(">")[0].split(",")
    return len(args) >= 4 and args[3].strip() == "0"


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    K = int(sys.argv[2])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pre = [r for r in rows if is_pre_sweep(r["Kernel_Name"])]
    if len(pre) < K:
        sys.exit(f"only {len(pre)} fine pre-sweep launches in the trace, K = {K}")
    t0 = int(pre[len(pre) - K]["Start_Timestamp"])
    win = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
    d = defaultdict(list)
    for r in win:
        d[kernel_key(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in d.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalNs", "Percentage", "PerCycleUs"])
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([k, len(v), round(sum(v) / len(v), 1), min(v), max(v), sum(v), round(100.0 * sum(v) / tot, 2),
                    round(sum(v) / K / 1000.0, 2)])
    print(f"# timed window: last {K} of {len(pre)} cycles (warm-up launches dropped), {len(win)} launches, "
          f"kernel time per cycle {tot / K / 1000.0:.1f} us", file=sys.stderr)
    if len(sys.argv) > 3:
        line = None
        for ln in open(sys.argv[3]):
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
        if line and line.get("roofline"):
            for seg, r in line["roofline"]["per_kernel"].items():
                prolong = seg == "post_sweep"
                keys = [k for k in d if k.startswith("k_zsweep_rb7<") and (k.split(",")[3].strip() != "0") == prolong]
                if not keys:
                    continue
                v = d[keys[0]]
                avg_ms = sum(v) / len(v) / 1e6
                print(f"# {seg}: trace {avg_ms:.4f} ms over {len(v)} launches, bench line {r['avg_launch_ms']:.4f} ms "
                      f"(frac {r['frac']}): {100.0 * (avg_ms / r['avg_launch_ms'] - 1.0):+.2f}%", file=sys.stderr)


if __name__ == "__main__":
    main()
