"""One V-cycle's kernel sequence from a rocprofv3 kernel trace (the 6th cycle): name, grid, duration.
python scripts/cycle_seq.py trace.csv [min_us]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].split("(")[0].replace("void mgmc::", "")[:40] for r in rows]
first = [i for i, n in enumerate(names) if n.startswith("k_zsweep_rb7") and ", 0, " in n]
a, b = first[5], first[6]
tot = 0.0
lo = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
for i in range(a, b):
    r = rows[i]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    if names[i].startswith("__amd"):
        continue
    tot += d
    if d >= lo:
        print(f"{names[i]:42s} grid={r['Grid_Size_X']:>8s}x{r['Grid_Size_Y']:>4s}x{r['Grid_Size_Z']:>4s} {d:8.1f}us")
print(f"kernel sum per cycle {tot:.1f} us")
