#!/usr/bin/env python3
"""GBT.getband end to end, device stitch against the host concatenation
(VERDICT r02 next-2): one 0002-shaped band of 8 files (65536 ch x 1 IF x 279
spectra, integer-valued Float32, uncompressed FBH5 in the page cache), all
workers on GPU 0; each mode timed over --reps calls after one warm call, and
checked bit for bit against the other.

    python tools/getband_probe.py [--reps 5] [--json out.json] [--compressed]

--compressed: the 8 files are rawspec-style compressed FBH5 (HDF5 filter
32008, chunks (16, 1, 4096) produced by the bitshuffle library: the committed
fixture chunk tests/golden/bslz4_v1.npz replicated), 272 spectra; the device
stitch then takes the bank-by-bank branch (chunks decoded on the GPU, each
bank's reduce writing its slot).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--nchan", type=int, default=65536)
    ap.add_argument("--ntime", type=int, default=279)
    ap.add_argument("--compressed", action="store_true")
    ap.add_argument("--threads", type=int, default=0,
                    help="reader threads (BLDP_READ_THREADS; 0: the library's default, 16)")
    ap.add_argument("--batch-mb", type=int, default=0,
                    help="pinned slot size (BLDP_NATIVE_BATCH_MB; 0: the default, 32)")
    ap.add_argument("--ring-mb", type=int, default=0,
                    help="pinned ring total (BLDP_NATIVE_RING_MB; 0: the default, 256)")
    ap.add_argument("--cases", default="",
                    help="comma-separated case labels to run (default: all)")
    a = ap.parse_args()
    if a.threads:
        os.environ["BLDP_READ_THREADS"] = str(a.threads)
    if a.batch_mb:
        os.environ["BLDP_NATIVE_BATCH_MB"] = str(a.batch_mb)
    if a.ring_mb:
        os.environ["BLDP_NATIVE_RING_MB"] = str(a.ring_mb)
    if a.compressed:
        a.ntime -= a.ntime % 16

    import numpy as np
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng, G = pkg.engine, pkg.GBT
    d = tempfile.mkdtemp(prefix="bldp_band_")
    names = []
    if a.compressed:
        z = np.load(os.path.join(REPO, "tests", "golden", "bslz4_v1.npz"), allow_pickle=False)
        chunk = z["chunk_gamma_chunk_b2048"].tobytes()
        nchunk = (a.nchan // 4096) * (a.ntime // 16)
    for b in range(8):
        p = os.path.join(d, f"blc0{b}_guppi_59000_12345_X_0011.rawspec.0002.h5")
        attrs = dict(fch1=8400.0 - 187.5 * b, foff=-187.5 / a.nchan, nchans=a.nchan, nifs=1,
                     tsamp=1.07, nfpc=1024)
        if a.compressed:
            pkg.fbh5.write_bslz4_chunks(p, attrs, (a.nchan, 1, a.ntime), (16, 1, 4096),
                                        (chunk for _ in range(nchunk)))
        else:
            x = eng.synth(a.nchan, 1, a.ntime, 1024, seed=10 * b + 2, kind=1)  # integers 0..255
            pkg.fbh5.write(p, attrs, eng.fb_to_numpy(x))
        names.append(p)
    torch.cuda.synchronize()
    workers = [0] * 8
    C = pkg.COLON
    cases = [("F64 T1", dict(fqavby=64)), ("F64 T1 despike", dict(fqavby=64, despike_nfpc=16)),
             ("F1 T1 despike", dict(despike_nfpc=1024)), ("F64 T9", dict(fqavby=64, tavby=9)) if not a.compressed else
             ("F64 T8", dict(fqavby=64, tavby=8)),
             ("F64 T16 (cfg2 window 1:272)", dict(fqavby=64, tavby=16, idxs=(C, C, pkg.JRange(1, 272))))]
    if a.cases:
        want = set(a.cases.split(","))
        cases = [c for c in cases if c[0] in want]
    res = {"reader_threads": a.threads or "default", "batch_mb": a.batch_mb or "default",
           "ring_mb": a.ring_mb or "default"}
    for label, kw in cases:
        out = {}
        kw = dict(kw)
        idxs = kw.pop("idxs", (C, C, C))
        for mode in ("host", "device"):
            G.getband(workers, names, idxs, stitch=mode, **kw)  # warm (page cache, plans)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                band = G.getband(workers, names, idxs, stitch=mode, **kw)
                ts.append((time.perf_counter() - t0) * 1e3)
            ts.sort()
            out[mode] = {"median_ms": round(ts[len(ts) // 2], 3), "min_ms": round(ts[0], 3),
                         "shape": list(band.shape)}
            out[mode + "_band"] = band
        same = bool(np.array_equal(out["host_band"].view(np.uint32),
                                   out["device_band"].view(np.uint32)))
        # the device path's host timeline of one more call (ms per stage)
        tm = {}
        G._band_on_device(workers, names, idxs, kw.get("fqavby", 1), "sum", kw.get("tavby", 1),
                          kw.get("despike_nfpc"), timings=tm)
        nbytes = 8 * 4 * a.nchan * a.ntime
        res[label] = {"host": out["host"], "device": out["device"], "bit_identical": same,
                      "speedup": round(out["host"]["median_ms"] / out["device"]["median_ms"], 3),
                      "device_GBps_of_files": round(nbytes / out["device"]["median_ms"] / 1e6, 2),
                      "device_timeline_ms": tm}
        print(label, json.dumps(res[label]), flush=True)
        assert same, label
    for p in names:
        os.remove(p)
    os.rmdir(d)
    res["what"] = ("GBT.getband on 8 %s FBH5 files of (%d ch x 1 IF x %d spectra) "
                   "Float32, every worker on GPU 0, files in the page cache; 'host' = each bank "
                   "reduced on the GPU, copied to the host and concatenated there (round 2), "
                   "despike H2D + kernel + D2H; 'device' = each bank reduced into its slot of the "
                   "band on the GPU, despike in place, one D2H" %
                   ("compressed (filter 32008)" if a.compressed else "uncompressed", a.nchan,
                    a.ntime))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
