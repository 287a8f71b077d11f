#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (rocpd
SQLite output).  FETCH_SIZE / WRITE_SIZE are in KiB, summed over counter instances per
dispatch.  Per MI355X_MICROARCH.md, gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so the
"fetch_bytes_corrected" column doubles it.
Usage: python tools/prof/pmc_bytes.py [--largest] fetch.db write.db > profiles/rNN/<name>_pmc_bytes.csv
  --largest: only each kernel's largest-grid launches (the bench's 16-batch C2 submissions, not
  its single-batch leg)"""
import sqlite3
import sys


def per_kernel(path, counter, largest=False):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select kernel_name, dispatch_id, sum(value), max(grid_size) from counters_collection where counter_name=? "
        "group by dispatch_id", (counter,)).fetchall()
    top = {}
    for name, _, _, gs in rows:
        top[name] = max(top.get(name, 0), gs)
    acc = {}
    for name, _, v, gs in rows:
        if largest and gs != top[name]:
            continue
        short = name.split("(")[0].replace(",", ";")
        acc.setdefault(short, []).append(v * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


args = [a for a in sys.argv[1:] if a != "--largest"]
big = "--largest" in sys.argv
fetch = per_kernel(args[0], "FETCH_SIZE", big)
write = per_kernel(args[1], "WRITE_SIZE", big)
print("Kernel,FetchBytesRaw,FetchBytesCorrected,WriteBytes,TrafficBytesPerLaunch")
for k in sorted(set(fetch) | set(write), key=lambda k: -(2 * fetch.get(k, 0) + write.get(k, 0))):
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    print("%s,%.0f,%.0f,%.0f,%.0f" % (k, f, 2 * f, w, 2 * f + w))
