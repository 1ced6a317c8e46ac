#!/usr/bin/env python3
"""MEASUREMENT TOOL (not product code): the pure-read rate of this GPU for a
buffer of a given size, through build/libbldp_probe.so (tools/hbm_probe.hip,
built by __graft_entry__.build()).  bench.py sets each reduce's bandwidth
beside it (roofline.box_read_probe): HBM rates differ box to box by several
percent, so a reduce is also compared with what a kernel that only reads
reaches on the same GPU.  It is a reference, not a ceiling: a reduce can beat
a probe form that under-reads some shapes.

    python tools/hbm_probe.py [MiB ...] [--cold]   (prints one JSON line per size)
"""
from __future__ import annotations

import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(REPO, "build", "libbldp_probe.so")

# nt loads, 16 or 8 in flight, contiguous or slab-spread: the forms that led
# some size of tools/read_probe_sweep.py (profiles/r04/read_probe_sweep_r04probe_b.json)
PROBE_FORMS = (0, 3, 513, 514, 520, 1537, 1544)

_lib = None


def lib():
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (one HIP runtime in the process, torch's)

        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built; run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        L.bldp_probe_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.bldp_probe_read.restype = ctypes.c_int
        _lib = L
    return _lib


def read_probe(nbytes, launches=20, forms=PROBE_FORMS, buf=None, stream=None, every=False,
               pkg=None, copies=1) -> dict:
    """``launches`` back-to-back launches per form (form: workgroups per CU |
    plain loads << 8 | 8 loads in flight << 9 | slabs << 10), each timed by
    events carried on its dispatch; the best form's median.  ``copies`` > 1:
    launch i reads copy i % copies of the buffer (a cold-cache figure for a
    buffer the 256 MB Infinity Cache would otherwise keep between launches,
    as bench.py --cache cold rotates the workload)."""
    import torch

    if pkg is None:
        sys.path.insert(0, REPO)
        import __graft_entry__ as entry

        pkg = entry.load_package()
    L = lib()
    nbytes = int(nbytes) // 16 * 16
    copies = max(1, int(copies))
    pitch = (nbytes + 255) // 256 * 256
    if buf is None:
        buf = torch.zeros(max(copies * pitch // 4, 4), dtype=torch.float32, device="cuda")
    elif buf.numel() * buf.element_size() < (copies - 1) * pitch + nbytes:
        raise ValueError("probe buffer smaller than copies x nbytes")
    base = buf.data_ptr()
    sp = pkg._lib.stream_ptr(stream)
    HipEvent = pkg._lib.HipEvent
    evs = [(HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False))
           for _ in range(launches)]
    best, seen = None, []
    for g in forms:
        for i in range(3):
            if L.bldp_probe_read(base + (i % copies) * pitch, nbytes, g, sp, None, None):
                raise RuntimeError(f"bldp_probe_read form {g} failed")
        for i, (e0, e1) in enumerate(evs):
            if L.bldp_probe_read(base + ((i + 3) % copies) * pitch, nbytes, g, sp, e0.ev, e1.ev):
                raise RuntimeError(f"bldp_probe_read form {g} failed")
        torch.cuda.synchronize()
        ms = statistics.median(e0.elapsed_time(e1) for e0, e1 in evs)
        r = {"GBps": round(nbytes / (ms * 1e-3) / 1e9, 1), "ms": round(ms, 5),
             "form": g, "wg_per_cu": g & 255, "loads": "plain" if g & 256 else "nt",
             "in_flight": 8 if g & 512 else 16, "slabs": bool(g & 1024), "bytes": nbytes,
             "copies": copies}
        seen.append(r)
        if best is None or r["GBps"] > best["GBps"]:
            best = r
    return dict(best, forms=seen) if every else best


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("mib", nargs="*", type=float, default=[64, 4096])
    ap.add_argument("--cold", action="store_true",
                    help="rotate over copies totalling >= 1 GiB (bench.py --cache cold)")
    a = ap.parse_args()
    for mb in a.mib:
        n = int(mb * (1 << 20))
        k = max(2, -(-(1 << 30) // n)) if a.cold and n < (1 << 30) else 1
        print(json.dumps(read_probe(n, every=True, copies=k)), flush=True)
