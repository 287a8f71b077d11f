#!/usr/bin/env python3
"""Per-kernel summary (calls, total/avg/min/max ns, % of kernel time) of a rocprofv3
--kernel-trace run, from its rocpd SQLite output (ROCm 7.2 writes .db by default).
Usage: python tools/prof/db_stats.py run_results.db > profiles/rNN/<name>_kernel_stats.csv"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                 "from kernels group by name order by sum(end-start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage")
for name, n, s, a, mn, mx in rows:
    short = name.split("(")[0].replace(",", ";")
    print("%s,%d,%d,%.1f,%d,%d,%.2f" % (short, n, s, a, mn, mx, 100.0 * s / tot))
