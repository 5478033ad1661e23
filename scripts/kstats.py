"""Per-kernel summary (grouped by kernel + grid) of a rocprofv3 kernel-trace CSV."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ncyc = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
d = collections.defaultdict(list)
for r in rows:
    key = (r["Kernel_Name"].split("(")[0][:48], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:24]:
    print(f"{k[0]:48s} {k[1]:>8s}x{k[2]:>5s}x{k[3]:>4s} n={len(v):5d} avg={sum(v)/len(v)/1000:9.1f}us "
          f"per-cycle={sum(v)/ncyc/1000:8.1f}us {100*sum(v)/tot:5.1f}%")
print(f"total kernel time per cycle {tot/ncyc/1000:.1f} us")
