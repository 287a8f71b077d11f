#!/usr/bin/env python3
"""Which HW queue each stream's kernels ran on (rocprofv3 --kernel-trace rocpd .db): per
(queue_id, stream_id) the dispatch count and the most frequent kernels.  HIP maps streams onto a
few hardware queues per priority (GPU_MAX_HW_QUEUES); two streams on one queue serialise.
Usage: python tools/prof/queues.py run_results.db"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select queue_id, stream_id, name from kernels").fetchall()
by = collections.defaultdict(collections.Counter)
for q, s, name in rows:
    short = name.split("(")[0].replace("void ", "").replace("gbls::", "")[:30]
    by[(q, s)][short] += 1
for (q, s), cnt in sorted(by.items()):
    top = ", ".join("%s x%d" % kv for kv in cnt.most_common(4))
    print("queue %3s stream %3s  %6d  %s" % (q, s, sum(cnt.values()), top))
