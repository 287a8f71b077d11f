#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (rocpd
SQLite output).  FETCH_SIZE / WRITE_SIZE are in KiB, summed over counter instances per
dispatch.  Per MI355X_MICROARCH.md, gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so the
"fetch_bytes_corrected" column doubles it.
Usage: python tools/prof/pmc_bytes.py fetch.db write.db > profiles/rNN/<name>_pmc_bytes.csv"""
import sqlite3
import sys


def per_kernel(path, counter):
    c = sqlite3.connect(path)
    rows = c.execute(
        "select kernel_name, dispatch_id, sum(value) from counters_collection where counter_name=? "
        "group by dispatch_id", (counter,)).fetchall()
    acc = {}
    for name, _, v in rows:
        short = name.split("(")[0].replace(",", ";")
        acc.setdefault(short, []).append(v * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
write = per_kernel(sys.argv[2], "WRITE_SIZE")
print("Kernel,FetchBytesRaw,FetchBytesCorrected,WriteBytes,TrafficBytesPerLaunch")
for k in sorted(set(fetch) | set(write), key=lambda k: -(2 * fetch.get(k, 0) + write.get(k, 0))):
    f, w = fetch.get(k, 0.0), write.get(k, 0.0)
    print("%s,%.0f,%.0f,%.0f,%.0f" % (k, f, 2 * f, w, 2 * f + w))
