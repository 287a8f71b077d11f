#!/usr/bin/env python3
"""Does the signature-side stream (the MSM, the extra pairs' lines) or the key-side stream ever
delay the Miller product's start?  From a rocprofv3 --kernel-trace rocpd .db of bench.py: for
every submission's join (its k_ml_pcols dispatch on the main stream X, the first kernel after
the side streams are waited on), the end of the main chain's last kernel before it and the end
of the last kernel on the context's side streams (X + 1: keys, X + 2: signatures -- the
engine creates each context's streams in that order) since the previous join on X.
delay = max(0, side_end - main_end): the time the join waited for a side stream.
Usage: python tools/prof/join_wait.py run_results.db [min_grid]"""
import sqlite3
import sys

db = sys.argv[1]
min_grid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
c = sqlite3.connect(db)
rows = c.execute("select name, stream_id, start, end, grid_x from kernels order by start").fetchall()
short = lambda n: n.split("(")[0].replace("void ", "").replace("gbls::", "")
joins = [r for r in rows if short(r[0]).startswith("k_ml_pcols") and r[4] >= min_grid]
prev = {}
out = []
for name, x, t0, t1, grid in joins:
    lo = prev.get(x, 0)
    main = [r for r in rows if r[1] == x and r[2] < t0 and r[2] >= lo and not short(r[0]).startswith("k_ml_pcols")]
    side = {s: [r for r in rows if r[1] == s and r[3] <= t0 + 50_000 and r[2] >= lo] for s in (x + 1, x + 2)}
    if not main:
        prev[x] = t0
        continue
    main_end = max(r[3] for r in main)
    ends = {s: max((r[3] for r in v), default=0) for s, v in side.items()}
    side_end = max(ends.values())
    last = {s: short(max(v, key=lambda r: r[3])[0]) if v else "-" for s, v in side.items()}
    out.append((x, (t0 - main_end) / 1e6, max(0, side_end - main_end) / 1e6, (main_end - side_end) / 1e6,
                last[x + 1], last[x + 2]))
    prev[x] = t0
print("%6s %12s %12s %14s  %-24s %-24s" % ("stream", "join_gap_ms", "delay_ms", "side_slack_ms", "last key-side", "last sig-side"))
for x, gap, d, slack, k1, k2 in out:
    print("%6d %12.3f %12.3f %14.3f  %-24s %-24s" % (x, gap, d, slack, k1[:24], k2[:24]))
if out:
    ds = [o[2] for o in out]
    print("joins %d, delayed %d, max delay %.3f ms, mean delay %.3f ms" %
          (len(ds), sum(1 for d in ds if d > 0.01), max(ds), sum(ds) / len(ds)))
