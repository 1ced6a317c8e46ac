#!/usr/bin/env python3
"""Where does a compressed FBH5 getdata spend its time?  The bench_file file
(1 GiB decoded, 4096 bitshuffle/LZ4 chunks of (16,1,4096), page cache warm):
stage times of the device read, and each stage's ceiling alone: chunk index
parse, parallel preads into pinned memory, H2D of the compressed bytes,
GPU decode of device-resident chunks."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import __graft_entry__ as entry  # noqa: E402


def main():
    import torch

    pkg = entry.load_package()
    fb, fs = pkg.fbh5, pkg.filestream
    z = np.load(os.path.join(REPO, "tests", "golden", "bslz4_v1.npz"), allow_pickle=False)
    chunk = z["chunk_gamma_chunk_b2048"].tobytes()
    nrep = 4096
    jshape = (4096, 1, 16 * nrep)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bldp_file_probe.h5")
    fb.write_bslz4_chunks(path, dict(foff=-187.5 / 65536, nfpc=1024), jshape, (16, 1, 4096),
                          (chunk for _ in range(nrep)))
    C = pkg.COLON
    W = pkg.WorkerFunctions
    nbytes = 4 * int(np.prod(jshape))
    for _ in range(2):
        W.getdata(path, (C, C, C), fqavby=64, tavby=16)
    res = {}
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        W.getdata(path, (C, C, C), fqavby=64, tavby=16)
        ts.append(time.perf_counter() - t0)
    res["getdata_ms"] = round(1e3 * sorted(ts)[2], 2)
    res["getdata_GBps"] = round(nbytes / sorted(ts)[2] / 1e9, 2)
    tm = {}
    for _ in range(3):
        tm = {}
        x = fb._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm)
        del x
    res["device_read_stages"] = {k: (round(v * 1e3, 2) if isinstance(v, float) else v)
                                 for k, v in tm.items()}
    os.environ["BLDP_TRACE_READ"] = "1"
    tm = {}
    x = fb._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm)
    del x
    os.environ.pop("BLDP_TRACE_READ")
    res["trace (batch, queued ms host, copy start ms gpu, copy end ms gpu, bytes)"] = tm.get("trace")
    os.environ["BLDP_TRACE_READ"] = "1"
    ts, tr = [], None
    for _ in range(5):
        tm = {}
        x = fb._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm)
        del x
        ts.append(tm["total_s"])
        tr = tm.get("trace")
    os.environ.pop("BLDP_TRACE_READ")
    res["pipeline_total_ms"] = round(1e3 * sorted(ts)[2], 2)
    res["pipeline_copy_span_ms"] = round(tr[-1][3] - tr[0][2], 3) if tr else None
    # batch schedule x gather sweep (device read total, ms, median of 7, interleaved)
    # (native: bldp_chunks_to_device; python: the reader pool in fbh5.py)
    sweep = [(64, 16, False, True, "python"), (64, 16, True, False, "python"),
             (64, 16, True, False, "native"), (64, 8, True, False, "native"),
             (32, 8, True, False, "native"), (128, 16, True, False, "native"),
             (64, 16, True, True, "native")]
    tsw = {k: [] for k in sweep}
    stages = {}
    for _ in range(7):
        for key in sweep:
            bb, fbb, ramp, dense, impl = key
            os.environ["BLDP_NATIVE_READ"] = "1" if impl == "native" else "0"
            tm = {}
            x = fb._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm,
                                          batch_bytes=bb << 20, first_batch_bytes=fbb << 20,
                                          ramp=ramp, dense=dense)
            del x
            tsw[key].append(tm["total_s"])
            stages[key] = tm
    os.environ.pop("BLDP_NATIVE_READ")
    for key, ts in tsw.items():
        bb, fbb, ramp, dense, impl = key
        res[f"{impl}_batch_{bb}MiB_first_{fbb}MiB_{'ramp' if ramp else 'flat'}_"
            f"{'gather' if dense else 'view'}_total_ms"] = round(1e3 * sorted(ts)[3], 2)
    res["native_stages_ms"] = {k: (round(v * 1e3, 3) if isinstance(v, float) else v)
                               for k, v in stages[(64, 16, True, False, "native")].items()}
    os.environ["BLDP_TRACE_READ"] = "1"
    os.environ["BLDP_NATIVE_READ"] = "0"  # (the trace is the python reader's)
    tm = {}
    x = fb._read_window_bslz4_dev(path, (C, C, C), "cuda:0", timings=tm, dense=False)
    del x
    os.environ.pop("BLDP_TRACE_READ")
    os.environ.pop("BLDP_NATIVE_READ")
    res["trace_ramp_view"] = tm.get("trace")
    res["trace_batch0_host_ms (task start, end; stage0 start)"] = tm.get("trace_batch0_host_ms")
    res["trace_stages_ms"] = {k: (round(v * 1e3, 3) if isinstance(v, float) else v)
                              for k, v in tm.items() if not k.startswith("trace")}
    # ceilings
    H = fb.h5().L
    f = H.H5Fopen(path.encode(), 0, 0)
    d = H.H5Dopen2(f, b"data", 0)
    t0 = time.perf_counter()
    tab = pkg.h5chunks.chunk_table(path, H, d)
    res["chunk_table_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
    H.H5Dclose(d)
    H.H5Fclose(f)
    ents = [tab["index"][k] for k in sorted(tab["index"])]
    base = min(e[0] for e in ents)
    span = max(e[0] + e[1] for e in ents) - base  # the chunks' bytes in the file
    total = span
    pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    mv = memoryview(pinned.numpy())
    fd = os.open(path, os.O_RDONLY)
    pool = fs._ring("cuda:0").pool
    for piece in (4 << 20, 16 << 20):
        tasks = [(o, o - base, min(piece, base + total - o)) for o in range(base, base + total, piece)]
        for _ in range(2):
            t0 = time.perf_counter()
            list(pool.map(lambda t: fs._pread_into(fd, mv[t[1]:t[1] + t[2]], t[0]), tasks))
            el = time.perf_counter() - t0
        res[f"pread_pool_{piece >> 20}MiB_GBps"] = round(total / el / 1e9, 2)
    os.close(fd)
    # O_DIRECT (page cache bypassed: the device's own rate), aligned pieces
    try:
        fdd = os.open(path, os.O_RDONLY | os.O_DIRECT)
        al = 4096
        lo = base - base % al
        hi = -(-(base + total) // al) * al
        dbuf = torch.empty(hi - lo + al, dtype=torch.uint8, pin_memory=True)
        a0 = (-dbuf.data_ptr()) % al
        dmv = memoryview(dbuf.numpy())[a0:a0 + hi - lo]
        piece = 4 << 20
        tasks = [(o, o - lo, min(piece, hi - o)) for o in range(lo, hi, piece)]
        for _ in range(2):
            t0 = time.perf_counter()
            list(pool.map(lambda t: os.preadv(fdd, [dmv[t[1]:t[1] + t[2]]], t[0]), tasks))
            el = time.perf_counter() - t0
        res["odirect_pool_4MiB_GBps"] = round((hi - lo) / el / 1e9, 2)
        os.close(fdd)
    except OSError as e:
        res["odirect_error"] = str(e)
    # preads concurrent with a running H2D stream (host memory contention)
    fd = os.open(path, os.O_RDONLY)
    dv2 = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    s2 = torch.cuda.Stream()
    tasks = [(o, o - base, min(4 << 20, base + total - o)) for o in range(base, base + total, 4 << 20)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(s2):
        for _ in range(3):
            dv2.copy_(pinned, non_blocking=True)
    list(pool.map(lambda t: fs._pread_into(fd, mv[t[1]:t[1] + t[2]], t[0]), tasks))
    t_rd = time.perf_counter() - t0
    s2.synchronize()
    t_all = time.perf_counter() - t0
    res["concurrent_pread_GBps"] = round(total / t_rd / 1e9, 2)
    res["concurrent_h2d_GBps"] = round(3 * total / t_all / 1e9, 2)
    os.close(fd)
    dv = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    for _ in range(2):
        t0 = time.perf_counter()
        dv.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    res["h2d_pinned_GBps"] = round(total / el / 1e9, 2)
    # copies alone: one big copy vs 64 MiB pieces, one vs two streams
    dvx = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    for label, nstreams, piece in (("one_copy", 1, total), ("pieces_1stream", 1, 64 << 20),
                                   ("pieces_2streams", 2, 64 << 20)):
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for j, o in enumerate(range(0, total, piece)):
                with torch.cuda.stream((sA, sB)[j % nstreams]):
                    dvx[o:o + piece].copy_(pinned[o:o + piece], non_blocking=True)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        res[f"h2d_{label}_GBps"] = round(total / el / 1e9, 2)
    # decode alone: all chunks device-resident, one async call + error check
    L = pkg._lib.lib()
    host = pinned.numpy()
    offs = np.array([e[0] - base for e in ents], np.uint64)
    lens = np.array([e[1] for e in ents], np.uint64)
    cvol = 16 * 4096
    ooff = np.arange(len(ents), dtype=np.uint64) * (4 * cvol)
    olen = np.full(len(ents), 4 * cvol, np.uint64)
    out = torch.empty(len(ents) * cvol, dtype=torch.float32, device="cuda:0")
    err = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    sp = pkg._lib.stream_ptr()
    for _ in range(3):
        t0 = time.perf_counter()
        pkg._lib.check(L.bldp_bslz4_decode_dev_async(len(ents), host.ctypes.data, dv.data_ptr(),
                                                     offs.ctypes.data, lens.ctypes.data, 4,
                                                     out.data_ptr(), ooff.ctypes.data,
                                                     olen.ctypes.data, err.data_ptr(), sp))
        t1 = time.perf_counter()
        pkg._lib.check(L.bldp_bslz4_error(err.data_ptr(), sp))
        el = time.perf_counter() - t0
    res["decode_host_queue_ms"] = round(1e3 * (t1 - t0), 2)
    res["decode_total_ms"] = round(1e3 * el, 2)
    res["compressed_bytes"] = int(lens.sum())
    res["file_span_bytes"] = total
    res["cpus"] = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}
    os.remove(path)
    import json
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
