#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 --kernel-trace rocpd .db: the union of kernel intervals over the
last part of the run (from the K-th dispatch of an anchor kernel on), its busy fraction, and the
longest gaps with the kernels on either side.
Usage: python tools/prof/gaps.py run_results.db [anchor] [k]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_h2c_field"
k = int(sys.argv[3]) if len(sys.argv) > 3 else -10
rows = c.execute("select name, start, end, queue_id from kernels order by start").fetchall()
nm = lambda r: r[0].split("(")[0].replace("void ", "").replace("gbls::", "")
idx = [i for i, r in enumerate(rows) if anchor in r[0]]
rows = rows[idx[k]:]
t0 = rows[0][1]
span_end = max(r[2] for r in rows)
busy, cur_s, cur_e, gaps, last = 0, rows[0][1], rows[0][2], [], rows[0]
for r in rows[1:]:
    if r[1] > cur_e:
        busy += cur_e - cur_s
        gaps.append((r[1] - cur_e, (cur_e - t0) / 1e6, nm(last), nm(r)))
        cur_s, cur_e = r[1], r[2]
    else:
        cur_e = max(cur_e, r[2])
    if r[2] >= cur_e:
        last = r
busy += cur_e - cur_s
span = span_end - t0
print("span %.3f ms, busy %.3f ms (%.1f %%), %d gaps, idle %.3f ms" % (span / 1e6, busy / 1e6, 100 * busy / span,
                                                                   len(gaps), sum(g[0] for g in gaps) / 1e6))
for g in sorted(gaps, reverse=True)[:15]:
    print("  gap %.3f ms at %.3f ms: after %s, before %s" % (g[0] / 1e6, g[1], g[2][:30], g[3][:30]))
