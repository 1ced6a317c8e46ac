#!/usr/bin/env python3
"""Probe: a page-cache-resident file straight to HBM without the bounce copy.

The raw-run reader (bldp_runs_to_device) preads the file into pinned slots and
copies those to the device: host memory sees every byte three times (page cache
read, slot write, DMA read).  Here the file is mmap'ed read-only and the mapped
page-cache pages are registered with HIP (hipHostRegister, ReadOnly), so the
copy engine reads them in place: host memory sees every byte once.  Timed:

  native   filestream.read_runs_to_device (the current reader)
  whole    register the whole mapping, one H2D copy, unregister
  chunked  C MiB windows: register window k+1 while window k is copied,
           unregister behind the copies
Every rep maps the file afresh, so registration starts cold each time (the
round-2 first version reused one mapping and reported the warm cost).

    python tools/mmap_register_probe.py [--gib 2] [--chunk-mib 64] [--reps 3]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PROT_READ, MAP_SHARED = 1, 1
H2D = 1
REG_READONLY = 0x08


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=2.0)
    ap.add_argument("--chunk-mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    libc = ctypes.CDLL(None, use_errno=True)
    libc.mmap.restype = ctypes.c_void_p
    libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                          ctypes.c_int, ctypes.c_long]
    libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]

    size = int(a.gib * (1 << 30))
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bldp_mmap_probe.bin")
    rng = np.random.default_rng(1)
    with open(path, "wb") as f:
        for _ in range(size >> 26):
            f.write(rng.integers(0, 255, 1 << 26, dtype=np.uint8).tobytes())
    want = np.fromfile(path, np.uint8)  # also warms the page cache
    dev = torch.device("cuda", 0)
    out = torch.empty(size, dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)
    res = {"bytes": size, "chunk_mib": a.chunk_mib}

    def check(t):
        return bool(np.array_equal(t.cpu().numpy()[:: 1 << 20], want[:: 1 << 20]) and
                    np.array_equal(t[-4096:].cpu().numpy(), want[-4096:]))

    # the current reader
    runs = np.array([[0, size]], np.int64)
    pkg.filestream.read_runs_to_device(path, runs, dev)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        o = pkg.filestream.read_runs_to_device(path, runs, dev)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    res["native"] = {"GBps": round(size / min(ts) / 1e9, 2), "ok": check(o)}
    del o
    print(json.dumps(res), flush=True)

    fd = os.open(path, os.O_RDONLY)

    def fresh_map():  # a new mapping every rep: registration starts cold
        b = libc.mmap(None, size, PROT_READ, MAP_SHARED, fd, 0)
        if b in (None, ctypes.c_void_p(-1).value):
            raise OSError(ctypes.get_errno(), "mmap")
        return b

    try:
        # whole mapping at once
        rows = []
        for _ in range(a.reps):
            base = fresh_map()
            out.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = hip.hipHostRegister(base, size, REG_READONLY)
            t1 = time.perf_counter()
            if rc:
                res["whole"] = {"hipHostRegister_rc": rc}
                break
            rc2 = hip.hipMemcpyAsync(out.data_ptr(), base, size, H2D, sp)
            hip.hipStreamSynchronize(sp)
            t2 = time.perf_counter()
            hip.hipHostUnregister(base)
            t3 = time.perf_counter()
            libc.munmap(base, size)
            rows.append((t1 - t0, t2 - t1, t3 - t2, rc2))
        if rows:
            best = min(rows, key=lambda r: sum(r[:3]))
            res["whole"] = {"register_ms": round(best[0] * 1e3, 2),
                            "copy_ms": round(best[1] * 1e3, 2),
                            "unregister_ms": round(best[2] * 1e3, 2), "copy_rc": best[3],
                            "GBps_total": round(size / sum(best[:3]) / 1e9, 2),
                            "GBps_copy": round(size / best[1] / 1e9, 2), "ok": check(out)}
        print(json.dumps(res), flush=True)
        # chunked: register ahead, copy, unregister behind
        C = a.chunk_mib << 20
        ts = []
        for _ in range(a.reps):
            base = fresh_map()
            out.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            evs, regd, bad = [], [], 0
            for off in range(0, size, C):
                n = min(C, size - off)
                rc = hip.hipHostRegister(base + off, n, REG_READONLY)
                if rc:
                    bad = rc
                    break
                regd.append((off, n))
                hip.hipMemcpyAsync(out.data_ptr() + off, base + off, n, H2D, sp)
                ev = torch.cuda.Event()
                ev.record(s)
                evs.append(ev)
                if len(evs) > 2:  # unregister the window two copies behind
                    evs.pop(0).synchronize()
                    o0, _ = regd.pop(0)
                    hip.hipHostUnregister(base + o0)
            hip.hipStreamSynchronize(sp)
            for o0, _ in regd:
                hip.hipHostUnregister(base + o0)
            ts.append(time.perf_counter() - t0)
            libc.munmap(base, size)
            if bad:
                res["chunked"] = {"hipHostRegister_rc": bad}
                break
        else:
            res["chunked"] = {"GBps": round(size / min(ts) / 1e9, 2), "ok": check(out)}
    finally:
        os.close(fd)
        os.remove(path)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
