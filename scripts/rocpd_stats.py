#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (results.db): name, grid, launches, average and
total microseconds, sorted by total time.  usage: rocpd_stats.py results.db [top]"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = con.execute("select name, grid_x, grid_z, workgroup_x, count(*), avg(duration) / 1000.0, sum(duration) / 1000.0 "
                   "from kernels group by name, grid_x, grid_z order by sum(duration) desc limit ?", (top,)).fetchall()
print(f"{'kernel':70s} {'grid_x':>8s} {'z':>3s} {'wg':>5s} {'calls':>6s} {'avg_us':>9s} {'total_us':>10s}")
for name, gx, gz, wx, n, avg, tot in rows:
    print(f"{name[:70]:70s} {gx:8d} {gz:3d} {wx:5d} {n:6d} {avg:9.1f} {tot:10.0f}")
