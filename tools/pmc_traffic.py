#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs as
MI355X_MICROARCH.md §rocprofv3 PMC slots requires) into per-launch HBM bytes
of the reduce kernel, and record them in profiles/pmc_traffic.json for bench.py
(keyed by config, then by banks per launch: 8 at N=1, 8/N for one rank of an
N-GPU run, profiled with bench.py --local-banks).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) reports half
the bytes of a wide (16 B/lane) coalesced streaming read -> x2; WRITE_SIZE is
exact for 16 B/lane stores (the reduce kernel's output writes are 4 B and tiny;
taken as reported).

    python tools/pmc_traffic.py CONFIG BANKS_PER_LAUNCH FETCH.csv WRITE.csv
    python tools/pmc_traffic.py --kurt CONFIG BANKS FETCH.csv WRITE.csv   (getkurtosis call:
        every kernel of the call (k_kurt_regs / mid / leaf and the tree merge),
        FETCH x2 (coalesced streams: 128-B requests tallied at 64 B), summed
        per call; key "kurt_CONFIG")
"""
from __future__ import annotations

import csv
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_dispatch(path, counter, kernel_substr="k_reduce"):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_substr in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel_substr} in {path}")
    return vals


def kurt_call(fpath, wpath):
    """Per-call HBM bytes of the streamed-leaf kurtosis: every kernel of the
    call, medians per kernel, FETCH of the 16 B/lane leaf stream x2."""
    kern, hbm = {}, 0.0
    for name in ("k_kurt_regs", "k_kurt_mid", "k_kurt_leaf", "k_kurt_tree", "k_kurt_final"):
        try:
            f = statistics.median(per_dispatch(fpath, "FETCH_SIZE", name))
            w = statistics.median(per_dispatch(wpath, "WRITE_SIZE", name))
        except SystemExit:
            continue
        # every one of these is a coalesced stream whose 128-B requests gfx950
        # tallies at 64 B (4, 8 and 16 B per lane alike: k_kurt_mid's FETCH is
        # exactly half its 4 B/lane window, the tree's half its partials)
        mult = 2
        kern[name] = {"fetch_size_kib_median": f, "write_size_kib_median": w,
                      "hbm_bytes": int(mult * f * 1024 + w * 1024)}
        hbm += mult * f * 1024 + w * 1024
    return kern, hbm


def main():
    if sys.argv[1] == "--kurt":
        cfg, nbank, fpath, wpath = "kurt_" + sys.argv[2], int(sys.argv[3]), sys.argv[4], sys.argv[5]
        kern, hbm = kurt_call(fpath, wpath)
        fetch = write = [0]
        f_kib = sum(k["fetch_size_kib_median"] for k in kern.values())
        w_kib = sum(k["write_size_kib_median"] for k in kern.values())
    else:
        cfg, nbank, fpath, wpath = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
        kern = None
        fetch = per_dispatch(fpath, "FETCH_SIZE")
        write = per_dispatch(wpath, "WRITE_SIZE")
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        hbm = 2 * f_kib * 1024 + w_kib * 1024
    out = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(out) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    d.setdefault(cfg, {})
    if "banks_per_launch" in d[cfg]:  # older flat layout: one entry per config
        d[cfg] = {str(d[cfg]["banks_per_launch"]): d[cfg]}
    d[cfg][str(nbank)] = {"banks_per_launch": nbank, "hbm_bytes_per_launch": int(hbm),
              "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib,
              "dispatches": [len(fetch), len(write)],
              "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 half-count "
                            "of 16B/lane streaming reads)",
              "source": [os.path.relpath(fpath, REPO), os.path.relpath(wpath, REPO)]}
    if kern:
        d[cfg][str(nbank)]["kernels"] = kern
        d[cfg][str(nbank)]["dispatches"] = None
        d[cfg][str(nbank)]["correction"] = ("per call, every kernel: 2*FETCH_SIZE*1024 + "
                                            "WRITE_SIZE*1024 (gfx950 half-count of coalesced "
                                            "streaming reads)")
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d[cfg][str(nbank)]))


if __name__ == "__main__":
    main()
