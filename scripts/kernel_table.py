"""Per-(kernel, grid) average durations from a rocprofv3 --kernel-trace run (results.db or
kernel_trace.csv): python scripts/kernel_table.py <file> [top] [compare_file]"""
import collections
import csv
import sqlite3
import sys


def load(path):
    agg = collections.defaultdict(list)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, gx, d in c.execute("select name, grid_x, duration from kernels"):
            agg[(name[:90], int(gx))].append(d / 1e3)
    else:
        for r in csv.DictReader(open(path)):
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[(r["Kernel_Name"][:90], int(r["Grid_Size_X"]))].append(d)
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main():
    a = load(sys.argv[1])
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    b = load(sys.argv[3]) if len(sys.argv) > 3 else {}
    rows = sorted(a.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:top]
    for (name, g), (avg, n) in rows:
        other = f"{b[(name, g)][0]:8.1f} x{b[(name, g)][1]:<5d}" if (name, g) in b else " " * 15
        print(f"{avg:8.1f} x{n:<5d} {other} {g:>9} {name}")
    if b:
        print("only in the second:")
        for (name, g), (avg, n) in sorted(b.items(), key=lambda kv: -kv[1][0] * kv[1][1])[:top]:
            if (name, g) not in a:
                print(f"{'':16} {avg:8.1f} x{n:<5d} {g:>9} {name}")


if __name__ == "__main__":
    main()
