#!/usr/bin/env python3
"""Time the three reduce paths on 0002-band-sized data (8 banks x 65540 ch x
1 IF x 272 spectra, F=64-ish, T=16): an aligned window (vector path), a
window starting one channel in (misaligned -> scalar path), and odd F.
Prints GB/s per case (HIP events, median of 9)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng = pkg.engine
    if "--big" in sys.argv:  # cfg3 scale: 8 banks x 2^26 channels x 16 spectra
        n = 1 << 26
        banks = [eng.synth(n + 4, 1, 16, 1024, seed=b, kind=0) for b in range(8)]
        cases = {
            "cfg3 aligned F1024": ([0, n, 1, 0, 1, 1, 0, 16, 1], 1024, 16),
            "cfg3 misaligned F1024 (c0=1)": ([1, n, 1, 0, 1, 1, 0, 16, 1], 1024, 16),
            "cfg3 misaligned F64 (c0=3)": ([3, n, 1, 0, 1, 1, 0, 16, 1], 64, 16),
            "cfg3 F3": ([0, n - 1, 1, 0, 1, 1, 0, 16, 1], 3, 16),
            "cfg3 misaligned F1 (c0=1)": ([1, n, 1, 0, 1, 1, 0, 16, 1], 1, 16),
        }
        nt = 16
    else:
        banks = [eng.synth(65540, 1, 272, 1024, seed=b, kind=0) for b in range(8)]
        nt = 272
    cases = cases if "--big" in sys.argv else {
        "aligned F64": ([0, 65536, 1, 0, 1, 1, 0, 272, 1], 64, 16),
        "misaligned F64 (c0=1)": ([1, 65536, 1, 0, 1, 1, 0, 272, 1], 64, 16),
        "aligned F3": ([0, 65538, 1, 0, 1, 1, 0, 272, 1], 3, 16),
        "aligned F1": ([0, 65536, 1, 0, 1, 1, 0, 272, 1], 1, 16),
        "misaligned F1 (c0=1)": ([1, 65536, 1, 0, 1, 1, 0, 272, 1], 1, 16),
        "strided cs=2 F32": ([0, 32768, 2, 0, 1, 1, 0, 272, 1], 32, 16),
    }
    res = {}
    for name, (w, F, T) in cases.items():
        plan = eng.plan(banks[0], F, T, "sum", w)
        nb = 8 * 4 * (w[1] * nt + (w[1] // F) * (nt // T))
        for _ in range(3):
            eng.band_reduce(banks, F, T, "sum", w)
        ts = []
        for _ in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.band_reduce(banks, F, T, "sum", w)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[4]
        res[name] = {"path": plan["path"], "ms": round(ms, 4), "GBps": round(nb / ms / 1e6, 1)}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
