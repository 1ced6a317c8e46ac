#!/usr/bin/env python3
"""Per-kernel medians of a rocprofv3 --pmc counter_collection.csv (SQ / GRBM
passes), one entry per (kernel, grid size), with the derived figures the
reduce-vs-pure-read comparison uses:

  clock_GHz      GRBM_GUI_ACTIVE / 8 XCDs / kernel wall time
  wait_frac      SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / barrier)
  issue_frac     SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (ready, waiting to issue)
  active_frac    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  waves_per_cu   SQ_WAVE_CYCLES / (GRBM_GUI_ACTIVE / 8 * 4 quad-cycles) / 256 CUs
                 (the average resident waves per CU)

    python tools/sq_summary.py RUN_counter_collection.csv [--match k_reduce_il,k_read_probe]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import statistics


def summarize(path, match=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if match and not any(m in name for m in match):
            continue
        short = name.replace("(anonymous namespace)::", "").replace("void ", "")
        key = (short.split("(")[0], r["Grid_Size"])
        d = (key, r["Dispatch_Id"])
        agg[d][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["VGPR_Count"],
                   r["LDS_Block_Size"])
    per = collections.defaultdict(list)
    for (key, disp), c in agg.items():
        per[key].append((c, meta[(key, disp)]))
    out = {}
    for (kname, grid), lst in per.items():
        med = {n: statistics.median(c[n] for c, _ in lst) for n in lst[0][0]}
        ns = statistics.median(m[0] for _, m in lst)
        e = {"dispatches": len(lst), "grid": int(grid), "vgpr": lst[0][1][1],
             "lds": lst[0][1][2], "wall_us": round(ns / 1e3, 2),
             "counters": {k: v for k, v in sorted(med.items())}}
        wc = med.get("SQ_WAVE_CYCLES")
        ga = med.get("GRBM_GUI_ACTIVE")
        if ga and ns:
            e["clock_GHz"] = round(ga / 8 / ns, 3)
        if wc:
            for k, n in (("wait_frac", "SQ_WAIT_ANY"), ("issue_frac", "SQ_WAIT_INST_ANY"),
                         ("active_frac", "SQ_ACTIVE_INST_ANY")):
                if n in med:
                    e[k] = round(med[n] / wc, 4)
            if ga:
                e["waves_per_cu"] = round(wc / (ga / 8 / 4) / 256, 2)
        out[f"{kname} grid={grid}"] = e
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--match", default="k_reduce_il,k_read_probe")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    s = summarize(a.csv, a.match.split(",") if a.match else None)
    for k, e in s.items():
        print(k, {x: e.get(x) for x in ("dispatches", "wall_us", "clock_GHz", "waves_per_cu",
                                         "wait_frac", "issue_frac", "active_frac", "vgpr")})
    if a.json:
        with open(a.json, "w") as f:
            json.dump(s, f, indent=1)
