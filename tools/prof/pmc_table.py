#!/usr/bin/env python3
"""Per-kernel, per-launch averages of rocprofv3 --pmc counters from one or more runs
(rocpd SQLite output, one counter pass per run), summed over counter instances
(XCDs / SEs) per dispatch.  Derived columns:
  valu_busy   = SQ_ACTIVE_INST_VALU * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                (SQ_ACTIVE_* count quad-cycles; GRBM_GUI_ACTIVE sums the 8 XCDs)
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  fetch_bytes = 2 * FETCH_SIZE KiB * 1024 (gfx950 correction, MI355X_MICROARCH.md)
  fill        = SQ_WAVE_CYCLES * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8): resident waves per SIMD
Usage: python tools/prof/pmc_table.py [--largest] out.csv run1.db [run2.db ...]
  --largest: only each kernel's largest-grid launches (a run mixing batch sizes, e.g. the
  bench's C2 submissions and its single-batch leg, otherwise averages unlike launches)"""
import sqlite3
import sys


def load(path, largest=False):
    c = sqlite3.connect(path)
    rows = c.execute("select kernel_name, dispatch_id, counter_name, sum(value), max(grid_size) "
                     "from counters_collection group by dispatch_id, counter_name").fetchall()
    top = {}
    for name, did, cn, v, gs in rows:
        top[name] = max(top.get(name, 0), gs)
    acc = {}
    for name, did, cn, v, gs in rows:
        if largest and gs != top[name]:
            continue
        short = name.split("(")[0].split("::")[-1].replace(",", ";")
        acc.setdefault(short, {}).setdefault(cn, {})[did] = v
    return acc


def main():
    args = sys.argv[1:]
    largest = "--largest" in args
    args = [a for a in args if a != "--largest"]
    out = args[0]
    table = {}
    for path in args[1:]:
        for k, cnts in load(path, largest).items():
            for cn, per in cnts.items():
                table.setdefault(k, {})[cn] = (sum(per.values()) / len(per), len(per))
    cols = sorted({cn for v in table.values() for cn in v})
    derived = ["valu_busy", "fill", "lds_bank_conflict_frac", "fetch_bytes", "write_bytes"]
    with open(out, "w") as fh:
        fh.write("kernel,launches," + ",".join(cols + derived) + "\n")
        for k in sorted(table, key=lambda k: -table[k].get("GRBM_GUI_ACTIVE", (0, 0))[0]):
            v = {cn: table[k][cn][0] for cn in table[k]}
            n = max(x[1] for x in table[k].values())
            gui = v.get("GRBM_GUI_ACTIVE")
            busy = v["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * gui / 8) if gui and "SQ_ACTIVE_INST_VALU" in v else ""
            fill = (v["SQ_WAVE_CYCLES"] * 4 / (1024 * gui / 8)
                    if gui and "SQ_WAVE_CYCLES" in v else "")
            bc = (v["SQ_LDS_BANK_CONFLICT"] / v["SQ_LDS_IDX_ACTIVE"]
                  if v.get("SQ_LDS_IDX_ACTIVE") else "")
            fb = 2 * v["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in v else ""
            wb = v["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in v else ""
            row = [k, str(n)] + ["%.6g" % v[c] if c in v else "" for c in cols]
            row += ["%.4f" % x if isinstance(x, float) else str(x) for x in (busy, fill, bc, fb, wb)]
            fh.write(",".join(row) + "\n")


if __name__ == "__main__":
    main()
