"""Raw filterbank bytes from a file straight into HBM: parallel positional
reads into a ring of pinned host buffers, each batch copied to the device
asynchronously while the next one is read.

This is the read half of ``WorkerFunctions.getdata`` for data stored without
a filter: an uncompressed contiguous FBH5 ``data`` dataset (file offset from
``H5Dget_offset``; src/gbtworkerfunctions.jl:179-189) and the data block of a
32-bit SIGPROC ``.fil`` file (after the header; :171-177).  The reference
reads these with one thread through libhdf5 / mmap and reduces on the CPU.
Here only the rows and channel spans the window touches are read, by several
threads at once, and the window itself is applied by the reduction kernels
(no gather copy): :func:`plan_window` returns the byte runs to read and the
window relative to the dense device block they form.

Layout on disk (both formats): C order ``[nsamps][nifs][nchans]`` of
little-endian float32, i.e. Julia's ``(nchans, nifs, nsamps)``.
"""
from __future__ import annotations

import os
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from ._lib import BoundsError

# A window's channel span is read on its own (one run per (time, IF) row)
# only when it is a small part of a wide row; otherwise whole rows are read.
SUBSPAN_MIN_BYTES = 256 << 10
SUBSPAN_MAX_FRACTION = 0.5
PIECE_BYTES = 4 << 20    # largest single pread
BATCH_BYTES = 64 << 20   # one pinned slot = one H2D copy
NSLOTS = 4               # up to NSLOTS - 1 batches being read while one is copied
# the native reader's ring (bldp_runs_to_device / bldp_file_runs_to_device):
# the same 256 MiB of pinned slots as 8 x 32 MiB, so the first H2D copy
# starts after 32 MiB of reads and the last one is half as long
# (BLDP_NATIVE_BATCH_MB / BLDP_NATIVE_RING_MB override the slot size and the
# ring's total, for probes)
NATIVE_BATCH_BYTES = int(os.environ.get("BLDP_NATIVE_BATCH_MB", "32")) << 20
NATIVE_RING_BYTES = int(os.environ.get("BLDP_NATIVE_RING_MB", "256")) << 20
NATIVE_NSLOTS = max(2, min(16, NATIVE_RING_BYTES // NATIVE_BATCH_BYTES))


def _check(win, jshape):
    for ax in range(3):
        st, ct, sp = win[3 * ax: 3 * ax + 3]
        if ct > 0:
            last = st + (ct - 1) * sp
            if min(st, last) < 0 or max(st, last) >= jshape[ax]:
                raise BoundsError(-6, f"BoundsError: axis {ax + 1} window {st + 1}:{sp}:"
                                      f"{last + 1} of {jshape[ax]}")


def _ascending(st, ct, sp):
    """Lowest index, |step|, and the relative (start, step) that walks the
    ascending dense copy in window order."""
    if ct <= 1:
        return st, 1, 0, 1
    lo = min(st, st + (ct - 1) * sp)
    return lo, abs(sp), (ct - 1 if sp < 0 else 0), (-1 if sp < 0 else 1)


def plan_window(jshape, win, base=0, esize=4):
    """Byte runs of a window of a raw (nchan, nif, ntime) array stored C-order
    at file offset ``base``.

    Returns ``(runs, dshape, rwin)``: ``runs`` an (n, 2) int64 array of
    (file offset, bytes) read back to back into a dense device block of Julia
    shape ``dshape``; ``rwin`` the 9-int window of the original request
    relative to that block."""
    nchan, nif, ntime = (int(x) for x in jshape)
    c0, nc, cs, i0, ni, is_, t0, nt, ts = (int(x) for x in win)
    _check(win, (nchan, nif, ntime))
    if nc * ni * nt == 0:
        return np.zeros((0, 2), np.int64), (0, 0, 0), [0, nc, cs, 0, ni, is_, 0, nt, ts]
    t_lo, t_step, rt0, rts = _ascending(t0, nt, ts)
    c_lo = min(c0, c0 + (nc - 1) * cs)
    c_hi = max(c0, c0 + (nc - 1) * cs)
    span = c_hi - c_lo + 1
    row = nchan * nif * esize
    t_rows = t_lo + t_step * np.arange(nt, dtype=np.int64)
    if span * esize >= SUBSPAN_MIN_BYTES and span < SUBSPAN_MAX_FRACTION * nchan:
        # one run per (time, IF) pair: the channel span only
        i_lo, i_step, ri0, ris = _ascending(i0, ni, is_)
        i_rows = i_lo + i_step * np.arange(ni, dtype=np.int64)
        off = base + ((t_rows[:, None] * nif + i_rows[None, :]) * nchan + c_lo) * esize
        off = off.ravel()
        size = span * esize
        dshape = (span, ni, nt)
        rwin = [c0 - c_lo, nc, cs, ri0, ni, ris, rt0, nt, rts]
    else:
        # whole rows (every IF, every channel) of the selected spectra
        off = base + t_rows * row
        size = row
        dshape = (nchan, nif, nt)
        rwin = [c0, nc, cs, i0, ni, is_, rt0, nt, rts]
    # merge runs that continue each other in the file
    brk = np.flatnonzero(np.diff(off) != size) + 1
    starts = np.concatenate(([0], brk))
    ends = np.concatenate((brk, [len(off)]))
    runs = np.stack([off[starts], (ends - starts) * size], axis=1).astype(np.int64)
    return runs, dshape, rwin


def _pieces(runs):
    """Split runs into preads of at most PIECE_BYTES: (file offset, block
    offset, bytes), block offsets consecutive."""
    out = []
    pos = 0
    cap = min(PIECE_BYTES, BATCH_BYTES)  # a piece always fits one pinned slot
    for off, n in runs.tolist():
        k = 0
        while k < n:
            m = min(cap, n - k)
            out.append((off + k, pos + k, m))
            k += m
        pos += n
    return out


def _pread_into(fd, mv, off):
    got = 0
    n = len(mv)
    while got < n:
        r = os.preadv(fd, [mv[got:]], off + got)
        if r <= 0:
            raise OSError(f"short read at offset {off + got}")
        got += r


def read_runs_host(path, runs):
    """The same runs into one numpy uint8 buffer (host path; tests)."""
    total = int(runs[:, 1].sum()) if len(runs) else 0
    buf = np.empty(total, np.uint8)
    fd = os.open(path, os.O_RDONLY)
    try:
        mv = memoryview(buf)
        for f_off, b_off, n in _pieces(runs):
            _pread_into(fd, mv[b_off:b_off + n], f_off)
    finally:
        os.close(fd)
    return buf


class _Ring:
    """NSLOTS pinned host buffers of BATCH_BYTES, one copy stream and one
    event per slot, per device; plus the reader threads."""

    def __init__(self, device, threads):
        import torch

        self.device = device
        self.slot_bytes = BATCH_BYTES
        self.slots = [torch.empty(BATCH_BYTES, dtype=torch.uint8, pin_memory=True)
                      for _ in range(NSLOTS)]
        self.views = [memoryview(s.numpy()) for s in self.slots]
        with torch.cuda.device(device):
            self.stream = torch.cuda.Stream(device)
        self.events = [None] * NSLOTS
        self.pool = ThreadPoolExecutor(max_workers=threads, thread_name_prefix="bldp-read")
        self.lock = threading.Lock()  # one streaming call at a time per device


_rings: dict = {}
_rings_lock = threading.Lock()


def _ring(device):
    import torch

    dev = torch.device(device)
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    with _rings_lock:
        r = _rings.get(key)
        if r is not None and r.slot_bytes < BATCH_BYTES:  # batch size raised since
            with r.lock:
                r.pool.shutdown()
            r = None
        if r is None:
            threads = int(os.environ.get("BLDP_READ_THREADS", "0")) or min(
                16, max(2, (os.cpu_count() or 8)))
            r = _rings[key] = _Ring(torch.device("cuda", key), threads)
    return r


def read_runs_to_device(path, runs, device, timings=None):
    """Read ``runs`` of ``path`` into a new dense uint8 device tensor.

    Batches of BATCH_BYTES are read by the ring's threads into pinned slots
    (several preads per batch, up to NSLOTS - 1 batches in flight) and each
    is copied to the device on the ring's copy stream as soon as its reads
    land, while later batches are still being read.  The caller's current
    stream waits for the last copy."""
    import time

    import torch

    total = int(runs[:, 1].sum()) if len(runs) else 0
    if os.environ.get("BLDP_NATIVE_READ", "1") != "0":
        return _runs_native(path, runs, device, total, timings)
    ring = _ring(device)
    dev = ring.device
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    if total == 0:
        return out
    pieces = _pieces(runs)
    # batches: consecutive pieces within one slot
    batches, cur, lo = [], [], 0
    for p in pieces:
        if cur and p[1] + p[2] - lo > BATCH_BYTES:
            batches.append((lo, cur))
            cur, lo = [], p[1]
        if not cur:
            lo = p[1]
        cur.append(p)
    batches.append((lo, cur))
    t0 = time.perf_counter()
    t_read = 0.0
    fd = os.open(path, os.O_RDONLY)
    try:
        with ring.lock:
            reading = []  # (slot, preads, block lo, block hi) in batch order

            def land():  # oldest batch: wait for its preads, queue its H2D copy
                nonlocal t_read
                s, futs, blo, hi = reading.pop(0)
                tr = time.perf_counter()
                for f in futs:
                    f.result()
                t_read += time.perf_counter() - tr
                with torch.cuda.device(dev), torch.cuda.stream(ring.stream):
                    out[blo:hi].copy_(ring.slots[s][:hi - blo], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(ring.stream)
                ring.events[s] = ev

            for k, (blo, bp) in enumerate(batches):
                s = k % NSLOTS
                if ring.events[s] is not None:
                    ring.events[s].synchronize()  # the slot's previous copy is done
                mv = ring.views[s]
                futs = [ring.pool.submit(_pread_into, fd, mv[b - blo:b - blo + n], f)
                        for f, b, n in bp]
                reading.append((s, futs, blo, bp[-1][1] + bp[-1][2]))
                if len(reading) >= NSLOTS - 1:
                    land()
            while reading:
                land()
            with torch.cuda.device(dev):
                torch.cuda.current_stream(dev).wait_stream(ring.stream)
                out.record_stream(ring.stream)
    finally:
        os.close(fd)
    if timings is not None:
        torch.cuda.synchronize(dev)
        timings.update(total_s=time.perf_counter() - t0, read_s=t_read, bytes=total,
                       batches=len(batches), runs=len(runs), threads=ring.pool._max_workers)
    return out


_native_streams: dict = {}


def _runs_native(path, runs, device, total, timings):
    """read_runs_to_device through bldp_runs_to_device: the library's reader
    threads and pinned slot ring (no Python thread on the read path)."""
    import ctypes
    import time

    import torch

    from . import _lib

    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    if total == 0:
        return out
    cs = _native_streams.get(dev.index)
    if cs is None:
        cs = _native_streams[dev.index] = torch.cuda.Stream(dev, priority=-1)
    r = np.ascontiguousarray(runs, np.int64)
    fo, ln = np.ascontiguousarray(r[:, 0]), np.ascontiguousarray(r[:, 1])
    stats = (ctypes.c_double * 4)()
    t0 = time.perf_counter()
    fd = os.open(path, os.O_RDONLY)
    try:
        with torch.cuda.device(dev):
            rc = _lib.lib().bldp_runs_to_device(fd, len(ln), fo.ctypes.data, ln.ctypes.data,
                                                out.data_ptr(), out.numel(),
                                                NATIVE_BATCH_BYTES, NATIVE_NSLOTS,
                                                cs.cuda_stream, _lib.stream_ptr(), stats)
    finally:
        os.close(fd)
    _lib.check(rc, "bldp_runs_to_device")
    if timings is not None:
        torch.cuda.synchronize(dev)
        timings.update(total_s=time.perf_counter() - t0, first_copy_s=stats[0] / 1e3,
                       reads_s=stats[1] / 1e3, bytes=total, batches=-(-total // BATCH_BYTES),
                       runs=len(runs), pieces=int(stats[2]), threads=int(stats[3]), native=True)
    return out


def window_to_device(path, base, jshape, win, device, timings=None):
    """The window of a raw array at ``base`` in ``path`` as a Julia-order
    device tensor (the dense block) plus the window relative to it."""
    runs, dshape, rwin = plan_window(jshape, win, base)
    if not len(runs):
        return None, dshape, rwin
    buf = read_runs_to_device(path, runs, device, timings)
    x = buf.view(dtype=__import__("torch").float32).view(dshape[2], dshape[1], dshape[0])
    return x.permute(2, 1, 0), dshape, rwin


def files_to_device(paths, bases, runs0, dshape, device, timings=None):
    """The same window of several raw files (a band's banks: identical
    geometry, data block at ``bases[k]`` of ``paths[k]``) as one stream of
    batches into one device buffer (bldp_file_runs_to_device): bank k's dense
    block (``runs0`` of :func:`plan_window` relative to base 0, Julia shape
    ``dshape``) at byte k * block.  Returns the banks' Julia-order Float32
    views, in order.  The caller's current stream waits for the last copy."""
    import ctypes
    import time

    import torch

    from . import _lib

    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    runs0 = np.ascontiguousarray(runs0, np.int64)
    per = int(runs0[:, 1].sum()) if len(runs0) else 0
    n = len(paths)
    out = torch.empty(n * per, dtype=torch.uint8, device=dev)
    if per:
        cs = _native_streams.get(dev.index)
        if cs is None:
            cs = _native_streams[dev.index] = torch.cuda.Stream(dev, priority=-1)
        fds = []
        try:
            for pth in paths:
                fds.append(os.open(pth, os.O_RDONLY))
            nr = len(runs0)
            fo = np.concatenate([runs0[:, 0] + int(b) for b in bases])
            ln = np.tile(runs0[:, 1], n)
            fd = np.repeat(np.asarray(fds, np.int32), nr)
            stats = (ctypes.c_double * 4)()
            t0 = time.perf_counter()
            with torch.cuda.device(dev):
                rc = _lib.lib().bldp_file_runs_to_device(
                    len(ln), fd.ctypes.data, fo.ctypes.data, ln.ctypes.data, out.data_ptr(),
                    out.numel(), NATIVE_BATCH_BYTES, NATIVE_NSLOTS, cs.cuda_stream,
                    _lib.stream_ptr(), stats)
        finally:
            for f in fds:
                os.close(f)
        _lib.check(rc, "bldp_file_runs_to_device")
        if timings is not None:
            timings.update(read_call_ms=(time.perf_counter() - t0) * 1e3,
                           first_copy_ms=stats[0], reads_ms=stats[1], bytes=n * per,
                           pieces=int(stats[2]), threads=int(stats[3]))
    nc, ni, nt = dshape
    return [out[k * per:(k + 1) * per].view(torch.float32).view(nt, ni, nc).permute(2, 1, 0)
            for k in range(n)]
