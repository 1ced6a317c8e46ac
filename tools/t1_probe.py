#!/usr/bin/env python3
"""The reference's own fqav (no time integration, tavby = 1) on the shapes
VERDICT r02 lists, timed through the C ABI; also the driver for rocprofv3
--pmc passes over the same launches.

    python tools/t1_probe.py [--iters 20] [--rounds 5] [--json out.json]
    rocprofv3 --pmc FETCH_SIZE ... -- python tools/t1_probe.py --pmc --json cases.json

With --pmc every case runs exactly --pmc-calls times back to back (no
warm-up outside them) and the JSON lists the cases in dispatch order, so
tools/pmc_cases.py can attribute the reduce dispatches of the counter CSV.

Shapes (reference: src/gbtworkerfunctions.jl:16-20, 188):
  0000 band   8 x (2^26, 1, 16), F = 2
  0002 band   8 x (65536, 1, 279), F = 2, 3 (65535-channel window),
              8, 12 (65532-channel window), 64, 256
  0002 file   1 x (65536, 1, 279), F = 64 (exactly getdata(f; fqavby=64))
  0001 band   8 x (512, 1, 880000), F = 1, 2, 3, 4, 8, 12, 16, 64, 512 (--which 0001)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def build_cases(pkg, which="all"):
    eng = pkg.engine
    cases = []

    def band_case(label, banks, F, T, nc=None):
        nchan, nif, ntime = banks[0].shape
        nc = nc or nchan
        win = [0, nc, 1, 0, 1, 1, 0, ntime, 1]
        out = eng.fb_empty(len(banks) * (nc // F), nif, ntime // T)
        ptrs = (ctypes.c_void_p * len(banks))(*[b.data_ptr() for b in banks])
        keep, wp = pkg._lib.win_arg(win)
        nbytes = len(banks) * 4 * (nc * nif * ntime + (nc // F) * nif * (ntime // T))
        plan = eng.plan(banks[0], F, T, "sum", win)

        def go(L, sp):
            rc = L.bldp_band_reduce_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), nchan,
                                        nif, ntime, wp, F, T, 0, out.data_ptr(), sp)
            assert rc == 0, rc
        cases.append({"label": label, "go": go, "bytes": nbytes, "out": out, "keep": (keep, ptrs),
                      "plan": plan, "banks": banks})

    if which in ("all", "0000"):
        b3 = [eng.synth(1 << 26, 1, 16, 1 << 20, seed=10 * b, kind=0, out=o)
              for b, o in enumerate(eng.band_empty(8, 1 << 26, 1, 16))]
        band_case("0000 band F2 T1", b3, 2, 1)
    if which in ("all", "0002"):
        b2 = [eng.synth(65536, 1, 279, 1024, seed=10 * b + 2, kind=0, out=o)
              for b, o in enumerate(eng.band_empty(8, 65536, 1, 279))]
        for F, nc in ((2, 65536), (3, 65535), (8, 65536), (12, 65532), (64, 65536), (256, 65536)):
            band_case(f"0002 band F{F} T1", b2, F, 1, nc)
        band_case("0002 file F64 T1", b2[:1], 64, 1)
    if which == "0001":  # 8 x (512, 1, 880000): VERDICT r03 next #5
        b4 = [eng.synth(512, 1, 880000, 8, seed=10 * b + 1, kind=0, out=o)
              for b, o in enumerate(eng.band_empty(8, 512, 1, 880000))]
        for F in (1, 2, 3, 4, 8, 12, 16, 64, 512):
            band_case(f"0001 band F{F} T1", b4, F, 1, 512 // F * F)
    return cases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pmc", action="store_true")
    ap.add_argument("--pmc-calls", type=int, default=5)
    ap.add_argument("--which", default="all", choices=["all", "0000", "0002", "0001"])
    ap.add_argument("--lib", default=None, help="a variant libbldp .so (tools/ab_variants.py)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()

    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    L = pkg._lib.lib()
    if a.lib:
        L = ctypes.CDLL(a.lib)
        for name, (args, res) in pkg._lib.SIGNATURES.items():
            if hasattr(L, name):  # (variants of earlier revisions lack newer entry points)
                getattr(L, name).argtypes = args
                getattr(L, name).restype = res
    stream = torch.cuda.current_stream()
    sp = int(stream.cuda_stream)
    cases = build_cases(pkg, a.which)
    torch.cuda.synchronize()
    res = {}
    if a.pmc:
        for c in cases:
            for _ in range(a.pmc_calls):
                c["go"](L, sp)
            torch.cuda.synchronize()
        res = {"dispatch_order": [{"label": c["label"], "calls": a.pmc_calls, "bytes": c["bytes"],
                                   "plan": c["plan"]} for c in cases]}
    else:
        times = {c["label"]: [] for c in cases}
        for r in range(a.rounds):
            for c in cases:
                c["go"](L, sp)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(a.iters):
                    c["go"](L, sp)
                e1.record(stream)
                e1.synchronize()
                times[c["label"]].append(e0.elapsed_time(e1) / a.iters)
        for c in cases:
            ts = sorted(times[c["label"]])
            med = ts[len(ts) // 2]
            res[c["label"]] = {"median_ms": round(med, 5), "min_ms": round(ts[0], 5),
                               "bytes": c["bytes"], "GBps_median": round(c["bytes"] / med / 1e6, 1),
                               "plan": c["plan"]}
            print(c["label"], json.dumps(res[c["label"]]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
