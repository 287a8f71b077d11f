#!/usr/bin/env python3
"""How the coalescer merged: from a rocprofv3 --kernel-trace rocpd .db, every k_h2c_field
dispatch (one per verify submission) with its set count (grid_x; one lane per message), its
start, and the gap to the previous submission's k_final_verdict; then the histogram.
Usage: python tools/prof/merge_sizes.py run_results.db"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, grid_x, queue_id from kernels order by start").fetchall()
subs = [(r[1], r[3], r[4]) for r in rows if "k_h2c_field" in r[0]]
fins = [(r[1], r[2]) for r in rows if "k_final_verdict" in r[0]]
if not subs:
    sys.exit("no k_h2c_field dispatches")
t0 = subs[0][0]
hist = collections.Counter()
for s, n, q in subs:
    hist[n] += 1
span = (fins[-1][1] - t0) / 1e9 if fins else 0
print("submissions %d, sets %d, span %.3f s" % (len(subs), sum(n for _, n, _ in subs), span))
print("sets per submission:", sorted(hist.items()))
busy = collections.Counter()
for r in rows:
    nm = r[0].split("(")[0].replace("void ", "").replace("gbls::", "").split("<")[0]
    busy[nm] += (r[2] - r[1]) / 1e6
print("kernel ms (sum over dispatches):", ", ".join("%s %.1f" % kv for kv in busy.most_common(14)))
for s, n, q in subs[:40]:
    print("  t=%8.3f ms n=%4d q=%s" % ((s - t0) / 1e6, n, q))
