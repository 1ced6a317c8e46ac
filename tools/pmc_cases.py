#!/usr/bin/env python3
"""Attribute rocprofv3 --pmc counter CSVs to the cases of tools/t1_probe.py
--pmc (dispatch order) and summarise them per case.

    python tools/pmc_cases.py CASES.json OUT.json PASS1.csv [PASS2.csv ...]

Every reduce dispatch (kernel name containing "k_reduce") is taken in
Dispatch_Id order; case k owns dispatches [k*calls, (k+1)*calls).  Per case and
counter the median over its dispatches is reported, plus:
  hbm_read_bytes   = 2 * FETCH_SIZE * 1024   (gfx950 half-count of 16 B/lane
                     streaming reads, MI355X_MICROARCH.md §HBM)
  hbm_write_bytes  = WRITE_SIZE * 1024       (exact for 16 B/lane stores; the
                     narrower stores are what TCC_EA0_WRREQ / _64B show)
  wr_req_32B       = TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B (write requests that
                     carry 32 bytes or less)
  frac_*           = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over
                     SQ_WAVE_CYCLES
  clock_GHz        = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration under the profiler
"""
from __future__ import annotations

import csv
import json
import re
import statistics
import sys


def load(paths):
    disp = {}  # dispatch id -> {"name", "dur_ns", counters...}
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                if "k_reduce" not in row["Kernel_Name"]:
                    continue
                key = (p, int(row["Dispatch_Id"]))
                d = disp.setdefault(key, {"name": row["Kernel_Name"],
                                          "dur_ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
                d[row["Counter_Name"]] = float(row["Counter_Value"])
    by_pass = {}
    for (p, did), d in disp.items():
        by_pass.setdefault(p, []).append((did, d))
    return [[d for _, d in sorted(v, key=lambda x: x[0])] for v in by_pass.values()]


def main():
    cases = json.load(open(sys.argv[1]))["dispatch_order"]
    out_path = sys.argv[2]
    passes = load(sys.argv[3:])
    res = {}
    for pi, seq in enumerate(passes):
        need = sum(c["calls"] for c in cases)
        if len(seq) != need:
            raise SystemExit(f"pass {sys.argv[3 + pi]}: {len(seq)} reduce dispatches, expected {need}")
        i = 0
        for c in cases:
            part = seq[i:i + c["calls"]]
            i += c["calls"]
            m = re.search(r"(k_\w+(<[^>]*>)?)", part[0]["name"])
            r = res.setdefault(c["label"], {"kernel": m.group(1) if m else part[0]["name"],
                                            "bytes_algorithmic": c["bytes"], "plan": c["plan"]})
            for k in part[0]:
                if k in ("name",):
                    continue
                v = statistics.median(p[k] for p in part)
                if k == "dur_ns":
                    r.setdefault("dur_ns_by_pass", []).append(v)
                else:
                    r[k] = v
    for label, r in res.items():
        if "FETCH_SIZE" in r:
            r["hbm_read_bytes"] = 2 * r["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in r:
            r["hbm_write_bytes"] = r["WRITE_SIZE"] * 1024
        if "hbm_read_bytes" in r and "hbm_write_bytes" in r:
            r["traffic_over_algorithmic"] = round(
                (r["hbm_read_bytes"] + r["hbm_write_bytes"]) / r["bytes_algorithmic"], 4)
        if "TCC_EA0_WRREQ_sum" in r and "TCC_EA0_WRREQ_64B_sum" in r:
            r["wr_req_32B"] = r["TCC_EA0_WRREQ_sum"] - r["TCC_EA0_WRREQ_64B_sum"]
        if "SQ_WAVE_CYCLES" in r:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if k in r:
                    r["frac_" + k[3:].lower()] = round(r[k] / r["SQ_WAVE_CYCLES"], 3)
        if "GRBM_GUI_ACTIVE" in r and r.get("dur_ns_by_pass"):
            r["clock_GHz"] = round(r["GRBM_GUI_ACTIVE"] / 8 / statistics.median(r["dur_ns_by_pass"]), 3)
        print(label, json.dumps({k: v for k, v in r.items() if k != "plan"}))
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
