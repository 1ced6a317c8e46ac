#!/usr/bin/env python3
"""Probe: is the raw band's end-to-end read bound by the
host's memory?  One box, one process, the 0002 band as 8 uncompressed FBH5
files in the page cache (585 MB of Float32), each figure the median of --reps:

  getband      GBT.getband(workers on GPU 0, fqavby=64): the whole call
  read_call    the band read alone (filestream.files_to_device: reader threads
               pread every file into the library's pinned slot ring, each slot
               copied to HBM as it lands)
  pread_only   the same preads (16 threads, os.preadv) into one pinned host
               buffer, no copy to the GPU: the page cache -> pinned memcpy
  h2d_only     one pinned 585 MB buffer -> HBM (the copy engine), no reads
  memcpy       host memory -> host memory, torch's threads (16): what the
               socket's memory gives one process
  pread_with_h2d  pread_only while a second pinned buffer is copied to HBM in
               a loop: the two halves of read_call sharing host memory

Every byte of read_call crosses host memory three times (page-cache read,
slot write, DMA read), so the call cannot beat the rate at which host memory
serves ~3x its bytes; pread_with_h2d measures that sharing directly.

    python tools/host_bound_probe.py [--reps 5] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import threading
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def med(ts):
    ts = sorted(ts)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()

    import numpy as np
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng, G, fs = pkg.engine, pkg.GBT, pkg.filestream
    torch.set_num_threads(a.threads)
    nchan, ntime = 65536, 279
    d = tempfile.mkdtemp(prefix="bldp_hostbound_")
    names = []
    for b in range(8):
        p = os.path.join(d, f"blc0{b}_guppi_59000_12345_X_0011.rawspec.0002.h5")
        x = eng.synth(nchan, 1, ntime, 1024, seed=10 * b + 2, kind=1)
        pkg.fbh5.write(p, dict(fch1=8400.0 - 187.5 * b, foff=-187.5 / nchan, nchans=nchan,
                               nifs=1, tsamp=1.07, nfpc=1024), eng.fb_to_numpy(x))
        names.append(p)
    torch.cuda.synchronize()
    per = 4 * nchan * ntime
    nbytes = 8 * per
    offs = [pkg.fbh5.raw_layout(p)[0] for p in names]
    gbps = lambda ms: round(nbytes / ms / 1e6, 2)  # noqa: E731
    res = {"bytes": nbytes, "threads": a.threads}

    # the whole call and the read alone
    C = pkg.COLON
    w = [0] * 8
    G.getband(w, names, (C, C, C), fqavby=64)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        G.getband(w, names, (C, C, C), fqavby=64)
        ts.append((time.perf_counter() - t0) * 1e3)
    res["getband_ms"] = round(med(ts), 3)
    geo = [G._bank_geometry(p) for p in names]
    runs0, dshape, _ = fs.plan_window((nchan, 1, ntime), [0, nchan, 1, 0, 1, 1, 0, ntime, 1], 0)
    fs.files_to_device(names, [g[2] for g in geo], runs0, dshape, "cuda:0")
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vs = fs.files_to_device(names, [g[2] for g in geo], runs0, dshape, "cuda:0")
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        del vs
    res["read_call_ms"] = round(med(ts), 3)

    # the halves alone
    pin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pv = pin.numpy()
    fds = [os.open(p, os.O_RDONLY) for p in names]
    piece = 4 << 20
    jobs = [(b, o) for b in range(8) for o in range(0, per, piece)]

    def read_one(job):
        b, o = job
        n = min(piece, per - o)
        mv = memoryview(pv[b * per + o:b * per + o + n])
        got = os.preadv(fds[b], [mv], offs[b] + o)
        assert got == n

    def pread_all(ex):
        list(ex.map(read_one, jobs))

    with ThreadPoolExecutor(max_workers=a.threads) as ex:
        pread_all(ex)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            pread_all(ex)
            ts.append((time.perf_counter() - t0) * 1e3)
        res["pread_only_ms"] = round(med(ts), 3)

        dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        s = torch.cuda.Stream()
        ts = []
        for _ in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.cuda.stream(s):
                dev.copy_(pin, non_blocking=True)
            s.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        res["h2d_only_ms"] = round(med(ts[1:]), 3)

        src = torch.empty(nbytes, dtype=torch.uint8)
        src.fill_(1)
        dst = torch.empty(nbytes, dtype=torch.uint8)
        dst.copy_(src)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            dst.copy_(src)
            ts.append((time.perf_counter() - t0) * 1e3)
        res["memcpy_ms"] = round(med(ts), 3)

        pin2 = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        pin2.fill_(2)
        stop = threading.Event()
        copied = [0]

        def h2d_loop():
            with torch.cuda.stream(s):
                while not stop.is_set():
                    dev.copy_(pin2, non_blocking=True)
                    s.synchronize()
                    copied[0] += nbytes

        th = threading.Thread(target=h2d_loop)
        th.start()
        time.sleep(0.05)
        ts = []
        c0, t00 = copied[0], time.perf_counter()
        for _ in range(a.reps):
            t0 = time.perf_counter()
            pread_all(ex)
            ts.append((time.perf_counter() - t0) * 1e3)
        h2d_rate = (copied[0] - c0) / (time.perf_counter() - t00) / 1e9
        stop.set()
        th.join()
        res["pread_with_h2d_ms"] = round(med(ts), 3)
        res["h2d_GBps_during_preads"] = round(h2d_rate, 2)
    for f in fds:
        os.close(f)
    for p in names:
        os.remove(p)
    os.rmdir(d)
    for k in ("getband", "read_call", "pread_only", "h2d_only", "memcpy", "pread_with_h2d"):
        res[k + "_GBps"] = gbps(res[k + "_ms"])
    res["host_traffic_GBps_at_read_call"] = round(3 * res["read_call_GBps"], 1)
    res["what"] = ("the 0002 band as 8 uncompressed FBH5 files (585 MB) in the page cache, "
                   "GPU 0; medians of %d reps; read_call's bytes cross host memory 3x "
                   "(page-cache read, slot write, DMA read)" % a.reps)
    print(json.dumps(res), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
