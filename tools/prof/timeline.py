#!/usr/bin/env python3
"""Per-dispatch timeline of one bench step from a rocprofv3 --kernel-trace rocpd .db:
start/end/duration (ms, relative to the step's first dispatch) and the HW queue of every
kernel between the K-th and (K+1)-th dispatch of an anchor kernel (default k_h2c_field,
the first kernel of a step).
Usage: python tools/prof/timeline.py run_results.db [step_index] [anchor]"""
import sqlite3
import sys

db = sys.argv[1]
step = int(sys.argv[2]) if len(sys.argv) > 2 else -2
anchor = sys.argv[3] if len(sys.argv) > 3 else "k_h2c_field"
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
qcol = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
sel = "select name, start, end%s from kernels order by start" % ((", " + qcol) if qcol else "")
rows = c.execute(sel).fetchall()
starts = [i for i, r in enumerate(rows) if r[0].split("(")[0].split("<")[0].endswith(anchor)]
if len(starts) < 2:
    sys.exit("anchor %s found %d times" % (anchor, len(starts)))
i0 = starts[step]
i1 = starts[step + 1] if step + 1 < len(starts) and step != -1 else len(rows)
t0 = rows[i0][1]
print("%-28s %8s %8s %8s %s" % ("kernel", "start", "end", "dur", "queue"))
for r in rows[i0:i1]:
    name = r[0].split("(")[0]
    name = name.replace("void ", "").replace("gbls::", "")
    q = r[3] if qcol else ""
    print("%-28s %8.3f %8.3f %8.3f %s" % (name[:28], (r[1] - t0) / 1e6, (r[2] - t0) / 1e6,
                                         (r[2] - r[1]) / 1e6, q))
