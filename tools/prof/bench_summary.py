#!/usr/bin/env python3
"""One line per bench JSON file: value, ms/step, single-batch value, dominant kernel and
its fraction, whole-path fraction, and the per-stage ms of a step.
Usage: python tools/prof/bench_summary.py gpurun_out/<run>/bench_*.txt"""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable:", e)
        continue
    r = d.get("roofline") or {}
    print("%-40s %12s %9s  single=%s  dom=%s frac=%s path=%s" % (
        path, d.get("value"), d.get("ms_per_step"), (d.get("single_batch") or {}).get("value"),
        r.get("kernel"), r.get("frac"), (r.get("path") or {}).get("frac")))
    print("    ", {k: v for k, v in (r.get("stage_ms_per_step") or {}).items()})
