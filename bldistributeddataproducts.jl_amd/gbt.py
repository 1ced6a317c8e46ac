"""Mirror of module ``GBT`` (src/gbt.jl) on one MI355X node.

In the reference a *worker* is a Julia process on a ``blcXY`` host reached
over ssh (src/gbt.jl:12-46).  Here a worker is a GPU of this node: worker
``w`` runs its bank's read + reduce on device ``w``.  The fan-out/gather shape
of every call is unchanged: one call per ``(worker, fname)`` pair, results in
an array of the same size (src/gbt.jl:73-78).  ``getband`` is the additive
stitched-product call.
"""
from __future__ import annotations

import warnings
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import readers, worker as W
from .idxs import COLON

__all__ = ["datahosts", "setupworkers", "getinventories", "getheaders", "getdata",
           "getkurtosis", "getband", "bandaxis", "fqav"]

fqav = W.fqav  # `using .WorkerFunctions` re-exports fqav (src/gbt.jl:6)

_workers: list[int] = []


def datahosts(prefix: str = "") -> list[str]:
    """["blc00", ..., "blc77"] (src/gbt.jl:8-10)."""
    return [f"{prefix}blc{i}{j}" for i in range(8) for j in range(8)]


def setupworkers(hosts=(), **kwargs) -> list[int]:
    """Bind one worker per host to the GPUs of this node, round-robin
    (src/gbt.jl:12-46).  Warns and returns [] when workers already exist
    (:20-23)."""
    global _workers
    if _workers:
        warnings.warn("workers already added, not adding more")
        return []
    import torch

    ndev = torch.cuda.device_count()
    if ndev == 0:
        raise RuntimeError("no GPU visible: workers run on MI355X devices")
    hosts = list(hosts) or datahosts(kwargs.get("prefix", ""))
    _workers = [k % ndev for k in range(len(hosts))]
    from . import engine

    engine.init(sorted(set(_workers)))  # streams, staging pipelines, peer access
    return list(_workers)


def _fanout(workers, fnames, fn):
    workers, fnames = np.asarray(workers, dtype=object), np.asarray(fnames, dtype=object)
    assert workers.shape == fnames.shape, "workers and fnames must have the same size"
    flat = list(zip(workers.ravel(), fnames.ravel()))
    with ThreadPoolExecutor(max_workers=max(1, len(flat))) as ex:  # @spawnat per pair
        res = list(ex.map(lambda wf: fn(*wf), flat))  # fetch.(futures)
    out = np.empty(len(res), dtype=object)
    out[:] = res
    return out.reshape(workers.shape)


def getinventories(workers, filere=r"0002.h5$", root="/datax/dibas",
                   sessionre=readers.DEFAULT_SESSIONRE, extra="GUPPI",
                   playerre=readers.DEFAULT_PLAYERRE):
    """src/gbt.jl:48-58."""
    return [readers.getinventory(filere, root=root, sessionre=sessionre, extra=extra,
                                 playerre=playerre, worker=w) for w in workers]


def getheaders(workers, fnames):
    """src/gbt.jl:60-67."""
    return _fanout(workers, fnames, lambda w, f: readers.getheader(f))


def getdata(workers, fnames, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1):
    """src/gbt.jl:69-79 (+ tavby): an array of per-bank (nchan/fqavby, nif,
    ntime/tavby) Float32 arrays, the same size as workers/fnames."""
    return _fanout(workers, fnames,
                   lambda w, f: W.getdata(f, idxs, fqavby, fqavfunc, tavby, device=int(w)))


def getkurtosis(workers, fnames, idxs=(COLON, COLON, COLON)):
    """src/gbt.jl:81-88."""
    return _fanout(workers, fnames, lambda w, f: W.getkurtosis(f, idxs, device=int(w)))


def _chan_window(idxs, nchans):
    """(start0, count, step) of the channel index (idxs[0]) over nchans."""
    from .idxs import JRange, is_colon, sanitizeidxs

    if len(idxs) != 3:  # @assert length(idxs) == 3 (src/gbtworkerfunctions.jl:172,180)
        raise AssertionError("idxs must have exactly three indices")
    c = sanitizeidxs(idxs)[0]
    if is_colon(c):
        return 0, int(nchans), 1
    if isinstance(c, JRange):
        if len(c) and not (1 <= c.first <= nchans and 1 <= c.first + (len(c) - 1) * c.step <= nchans):
            raise IndexError(f"BoundsError: channel index {c!r} outside 1:{nchans}")
        return c.first - 1, len(c), c.step
    raise TypeError(f"unsupported channel index {c!r}")


def bandaxis(headers, idxs=(COLON, COLON, COLON), fqavby=1):
    """Frequency axis (MHz) of the stitched band product that ``getband``
    returns for the same ``idxs``/``fqavby``.

    Bank b's window is ``range(fch1_b + foff_b*c0; step=foff_b*cs, length=nc)``
    (headers from getheaders, src/gbtworkerfunctions.jl:131-159), decimated
    by ``fqav(r, fqavby)`` (:27-33) and concatenated in bank order like the
    data (src/gbt.jl:103).  Returns one ``FRange`` when every bank's axis
    continues the previous one (a full-band window of adjacent banks), else
    a float64 array of channel centres."""
    parts = []
    for h in list(np.asarray(headers, dtype=object).ravel()):
        c0, nc, cs = _chan_window(idxs, int(h["nchans"]))
        r = W.FRange(float(h["fch1"]) + float(h["foff"]) * c0, float(h["foff"]) * cs, nc)
        parts.append(W.fqav_range(r, fqavby) if fqavby > 1 else r)
    if not parts:
        return W.FRange(0.0, 1.0, 0)
    step = parts[0].step
    contiguous = all(p.step == step for p in parts)
    for a, b in zip(parts, parts[1:]):
        if not contiguous:
            break
        nxt = a.first + a.length * a.step
        contiguous = a.length > 0 and abs(b.first - nxt) <= 1e-9 * max(1.0, abs(nxt))
    if contiguous:
        return W.FRange(parts[0].first, step, sum(p.length for p in parts))
    return np.concatenate([p.values() for p in parts])


def _bank_geometry(f):
    """(kind, Julia shape, data offset) of a bank, from the per-file layout
    the read itself uses (cached per file version: one libhdf5 open per file,
    not one for the header and another for the data):
    "raw" = an uncompressed contiguous FBH5 ``data`` block or a 32-bit SIGPROC
    data block at that offset (read by preads); "h5" = another FBH5 layout;
    "other" = anything else, shape from the header
    (src/gbtworkerfunctions.jl:131-159); "array" = an in-memory array/tensor."""
    if not isinstance(f, (str, bytes)) and not hasattr(f, "__fspath__"):
        return "array", tuple(int(n) for n in f.shape), None
    from . import fbh5

    if readers.ishdf5(f):
        raw = fbh5.raw_layout(f)
        if raw is not None:
            return "raw", tuple(int(n) for n in raw[1]), int(raw[0])
        cd = fbh5.layout(f)["cdims"]
        if len(cd) == 3:
            return "h5", tuple(int(n) for n in cd[::-1]), None
    else:
        raw = readers.fil_raw_layout(f)
        if raw is not None:
            return "raw", tuple(int(n) for n in raw[1]), int(raw[0])
    h = readers.getheader(f)
    return "other", (int(h["nchans"]), int(h.get("nifs", 1)), int(h["nsamps"])), None


def _bank_shape(f):
    """(nchan, nif, ntime) of a bank (see _bank_geometry)."""
    return _bank_geometry(f)[1]


def _band_raw(ws, fs, geo, idxs, fqavby, op, tavby, band, root, force_copy, tm,
              peer_store=False):
    """Every bank a raw file of one geometry: each GPU reads its banks' windows
    as ONE stream of batches (bldp_file_runs_to_device: preads of every file
    into the pinned slot ring, H2D copies overlapping the reads) into one
    buffer, then the band is reduced straight into its vcat slots: one launch
    on the root (bldp_band_reduce_f32), or, with banks on several GPUs, one
    launch per GPU whose slots reach the root by a peer copy (or, peer_store,
    by the kernels' own stores over xGMI): bldp_band_reduce_multi_f32."""
    import time

    import torch

    from . import engine, filestream
    from .idxs import to_window

    jshape = geo[0][1]
    win = to_window(idxs, jshape) or [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
    runs0, dshape, rwin = filestream.plan_window(jshape, win, 0)
    groups = {}
    for b, w in enumerate(ws):
        groups.setdefault(int(w), []).append(b)
    views = [None] * len(fs)
    # the caller's current stream on every device: each reader thread queues
    # its copies' completion (and allocates its buffer) on it, so the reduce
    # queued below on the same stream is ordered after the copies even when
    # the caller runs under `with torch.cuda.stream(s)` (torch's current
    # stream is per thread: a reader thread's own would be the default one)
    cur = {d: torch.cuda.current_stream(d) for d in set(groups) | {root}}

    def read(item):
        dev, bl = item
        t = {}
        t0 = time.perf_counter()
        with torch.cuda.device(dev), torch.cuda.stream(cur[dev]):
            vs = filestream.files_to_device([fs[b] for b in bl], [geo[b][2] for b in bl], runs0,
                                            dshape, f"cuda:{dev}", timings=t)
        for b, v in zip(bl, vs):
            views[b] = v
        t["group_ms"] = (time.perf_counter() - t0) * 1e3
        return dev, t

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=len(groups)) as ex:  # one reader per GPU
        tread = dict(ex.map(read, groups.items()))
    tm["read"] = {str(d): t for d, t in tread.items()}
    tm["read_ms"] = (time.perf_counter() - t0) * 1e3
    t1 = time.perf_counter()
    if list(groups) == [root] and not force_copy:
        with torch.cuda.device(root):
            engine.band_reduce(views, fqavby, tavby, op, rwin, out=band)
        tm["reduce"] = "bldp_band_reduce_f32 (one launch)"
    else:
        engine.band_reduce_multi(views, fqavby, tavby, op, rwin, root=root, out=band,
                                 staged=force_copy, peer_store=peer_store and not force_copy)
        tm["reduce"] = "bldp_band_reduce_multi_f32" + (" (staged)" if force_copy else "")
    tm["reduce_queue_ms"] = (time.perf_counter() - t1) * 1e3


def _band_chunked(ws, fs, geo, idxs, fqavby, op, tavby, band, root, force_copy, tm,
                  peer_store=False):
    """Every bank a chunked FBH5 file (filter 32008 or no filter) of one
    geometry: each GPU reads and decodes its banks' chunks as ONE stream of
    batches (fbh5.band_window_chunked_dev: bldp_file_chunks_to_device) into
    one chunk grid per bank, then the band is reduced straight into its vcat
    slots, as _band_raw does for raw files (one launch on the root, or one
    launch per GPU and a peer copy of its slots).  False when the banks do not
    qualify (the caller reads bank by bank)."""
    import time

    import torch

    from . import engine, fbh5

    groups = {}
    for b, w in enumerate(ws):
        groups.setdefault(int(w), []).append(b)
    # the caller's current stream on every device (as in _band_raw)
    cur = {d: torch.cuda.current_stream(d) for d in set(groups) | {root}}
    views, rwins = [None] * len(fs), {}

    def read(item):
        dev, bl = item
        t = {}
        with torch.cuda.device(dev), torch.cuda.stream(cur[dev]):
            got = fbh5.band_window_chunked_dev([fs[b] for b in bl], idxs, f"cuda:{dev}",
                                               timings=t)
        if got is None:
            return dev, None
        for b, v in zip(bl, got[0]):
            views[b] = v
        rwins[dev] = got[1]
        return dev, t

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=len(groups)) as ex:  # one reader per GPU
        tread = dict(ex.map(read, groups.items()))
    if any(t is None for t in tread.values()) or \
            len({None if w is None else tuple(w) for w in rwins.values()}) != 1:
        return False
    rwin = next(iter(rwins.values()))
    tm["read"] = {str(d): t for d, t in tread.items()}
    tm["read_ms"] = (time.perf_counter() - t0) * 1e3
    t1 = time.perf_counter()
    if list(groups) == [root] and not force_copy:
        with torch.cuda.device(root):
            engine.band_reduce(views, fqavby, tavby, op, rwin, out=band)
        tm["reduce"] = "bldp_band_reduce_f32 (one launch)"
    else:
        engine.band_reduce_multi(views, fqavby, tavby, op, rwin, root=root, out=band,
                                 staged=force_copy, peer_store=peer_store and not force_copy)
        tm["reduce"] = "bldp_band_reduce_multi_f32" + (" (staged)" if force_copy else "")
    tm["reduce_queue_ms"] = (time.perf_counter() - t1) * 1e3
    return True


def _band_on_device(ws, fs, idxs, fqavby, op, tavby, nfpc, timings=None, staged=None,
                    peer_store=None):
    """One band stitched on the GPU (src/gbt.jl:103): every
    bank is read and reduced on its worker's GPU straight into its vcat slot
    of the band product on the first worker's GPU, the DC-spike patch runs on
    the stitched product in place (src/gbt.jl:101-102,111), and the band
    crosses PCIe once.  Banks that are all raw files of one geometry take
    _band_raw (one read stream per GPU, one reduce); others go bank by bank
    (a bank on another GPU is reduced there and its result copied into the
    slot).  None when the banks' products differ in shape or are not Float32:
    the caller then concatenates on the host.  ``timings``: a dict that
    receives the host timeline (ms)."""
    import os
    import time

    import torch

    from . import engine
    from .idxs import sanitizeidxs, to_window

    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    idxs = sanitizeidxs(idxs)
    geo = [_bank_geometry(f) for f in fs]
    shapes = [engine.out_shape(g[1], to_window(idxs, g[1]), fqavby, tavby) for g in geo]
    tm["geometry_ms"] = (time.perf_counter() - t0) * 1e3
    if len(set(shapes)) != 1 or 0 in shapes[0]:
        return None
    nco, ni, nto = shapes[0]
    nb, root = len(fs), int(ws[0])
    band = engine.fb_empty(nb * nco, ni, nto, device=f"cuda:{root}")
    # staged (or BLDP_BAND_FORCE_COPY=1 when not given) takes the other-GPU
    # branch (reduce, then copy into the slot) for every bank: how a one-GPU
    # box runs it.  An argument of this call: no process state is touched
    force_copy = (os.environ.get("BLDP_BAND_FORCE_COPY", "0") == "1" if staged is None
                  else bool(staged))
    # peer_store (or BLDP_BAND_PEER_STORE=1 when not given): a bank's GPU
    # other than the root stores its slot over xGMI from the reduce kernel
    # instead of reducing locally and copying (opt-in: that branch has not yet
    # run on a multi-GPU node)
    peer_store = (os.environ.get("BLDP_BAND_PEER_STORE", "0") == "1" if peer_store is None
                  else bool(peer_store))
    raw = (all(g[0] == "raw" for g in geo) and len({g[1] for g in geo}) == 1
           and os.environ.get("BLDP_NATIVE_READ", "1") != "0")
    # every bank a chunked FBH5 file of one geometry (the rawspec products:
    # filter 32008): the band's chunks read and decoded as one stream per GPU
    chunked = (not raw and all(g[0] == "h5" for g in geo) and len({g[1] for g in geo}) == 1
               and os.environ.get("BLDP_NATIVE_READ", "1") != "0")
    if chunked:
        chunked = _band_chunked(ws, fs, geo, idxs, fqavby, op, tavby, band, root, force_copy, tm,
                                peer_store)
    if raw:
        _band_raw(ws, fs, geo, idxs, fqavby, op, tavby, band, root, force_copy, tm, peer_store)
    elif not chunked:
        # every bank is read (compressed chunks decoded) on its own GPU and
        # reduced there straight into its vcat slot on the root: a kernel
        # store where the bank's GPU is the root (or, with peer_store, may
        # write the root's memory over xGMI: bldp_peer_access), else reduced
        # locally and copied into the slot by one stream-ordered
        # device-to-device copy.  No host wait per bank:
        # every reader queues on the caller's current stream of its device
        # (ordered with the root's despike and D2H below by the device
        # synchronize), and the band is complete when those streams drain.
        devs = sorted({int(w) for w in ws} | {root})
        cur = {d: torch.cuda.current_stream(d) for d in devs}
        direct = {d: (not force_copy)
                  and (d == root or (peer_store and engine.peer_access(d, root))) for d in devs}

        def bank(b):
            slot = band[b * nco:(b + 1) * nco]
            dev = int(ws[b])
            with torch.cuda.device(dev), torch.cuda.stream(cur[dev]):
                if direct[dev]:
                    return W.getdata_device(fs[b], idxs, fqavby, op, tavby, device=dev, out=slot)
                r = W.getdata_device(fs[b], idxs, fqavby, op, tavby, device=dev)
                if r is not None:  # (torch orders a cross-device copy on both devices' streams)
                    slot.copy_(r, non_blocking=True)
                return r

        t1 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=max(1, nb)) as ex:  # @spawnat per bank
            got = list(ex.map(bank, range(nb)))
        tm["banks_ms"] = (time.perf_counter() - t1) * 1e3
        if any(r is None for r in got):
            return None
    t2 = time.perf_counter()
    for d in sorted({int(w) for w in ws}):
        torch.cuda.synchronize(d)
    tm["sync_ms"] = (time.perf_counter() - t2) * 1e3
    with torch.cuda.device(root):
        t3 = time.perf_counter()
        if nfpc:
            engine.despike(band, nco // 64 if nfpc is True else int(nfpc))
        out = engine.fb_to_numpy(band, pinned=True)  # the one device -> host copy
        tm["despike_d2h_ms"] = (time.perf_counter() - t3) * 1e3
    tm["path"] = ("raw band" if raw else "chunked band" if chunked else "bank by bank") + \
        (" (staged)" if force_copy and not raw else "")
    tm["total_ms"] = (time.perf_counter() - t0) * 1e3
    return out


def _despike_host(d: np.ndarray, nfpc: int) -> np.ndarray:
    """d[spike:nfpc:end, :, :] .= d[spike-1:nfpc:end, :, :] with
    spike = nfpc÷2 + 1 (src/gbt.jl:101-102,111) on a host array of any element
    type, in place; the errors of bldp_despike_f32."""
    from . import _lib

    if nfpc < 2:
        raise _lib.BoundsError(_lib.BLDP_EBOUNDS, f"BoundsError: nfpc={nfpc} < 2")
    sp = nfpc // 2  # 0-based spike bin
    dst, src = d[sp::nfpc], d[sp - 1::nfpc]
    if dst.shape[0] != src.shape[0]:
        raise _lib.DimensionMismatch(_lib.BLDP_EDIM,
                                     f"DimensionMismatch: {dst.shape[0]} spike bins vs "
                                     f"{src.shape[0]} source bins (nchan={d.shape[0]}, nfpc={nfpc})")
    d[sp::nfpc] = src.copy()
    return d


def getband(workers, fnames, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1,
            despike_nfpc=None, freqs=False, stitch="device", staged=None, peer_store=None):
    """The stitched band product: reduce(vcat, getdata(...)) in the given
    bank order (src/gbt.jl:103).  ``workers``/``fnames`` are one band's banks
    (1-D), or a (nbank, nband) matrix like loadscan's ``ds``, whose columns are
    bands: then one stitched band per column is returned, as
    ``map(c -> reduce(vcat, c), eachcol(ds))`` (:103).  With ``despike_nfpc``
    the DC bin of every coarse channel is patched as in loadscan
    (src/gbt.jl:101-102,111); ``despike_nfpc=True`` takes loadscan's own
    ``nfpc = size(ds[1], 1) ÷ 64`` (64 coarse channels per bank, :101).
    ``freqs=True`` returns ``(band, bandaxis(...))`` (lists for a matrix).

    ``stitch="device"`` (default) stitches each band on the GPU
    (:func:`_band_on_device`); ``stitch="host"`` reduces every bank on its GPU,
    copies each bank's product to the host and concatenates there (also what
    bands of unequal bank products or non-Float32 data get).  ``staged=True``
    sends every bank of the device stitch through the staged branch (reduced
    on its own GPU, then copied into its slot) even where its GPU could write
    the root's memory directly: how a one-GPU box runs that branch (default:
    the environment's BLDP_BAND_FORCE_COPY, else off).  ``peer_store=True``
    lets a bank's GPU other than the root store its slot over xGMI straight
    from the reduce kernel (default: the environment's BLDP_BAND_PEER_STORE,
    else off: such banks are reduced on their GPU and copied into the slot)."""
    w = np.asarray(workers, dtype=object)
    f = np.asarray(fnames, dtype=object)
    if w.ndim not in (1, 2):
        raise AssertionError("getband takes one band (1-D) or a (nbank, nband) matrix")
    assert w.shape == f.shape, "workers and fnames must have the same size"
    if stitch not in ("device", "host"):
        raise ValueError("stitch must be 'device' or 'host'")
    wcol = [list(w)] if w.ndim == 1 else [list(w[:, j]) for j in range(w.shape[1])]
    fcol = [list(f)] if f.ndim == 1 else [list(f[:, j]) for j in range(f.shape[1])]
    op = W._opname(fqavfunc)
    bands = [None] * len(wcol)
    if stitch == "device" and op is not None:
        for j, (ws, fs) in enumerate(zip(wcol, fcol)):
            bands[j] = _band_on_device(ws, fs, idxs, fqavby, op, tavby, despike_nfpc,
                                       staged=staged, peer_store=peer_store)
    for j, (ws, fs) in enumerate(zip(wcol, fcol)):
        if bands[j] is not None:
            continue
        parts = list(getdata(ws, fs, idxs, fqavby, fqavfunc, tavby))
        nfpc = despike_nfpc
        if nfpc is True:
            nfpc = parts[0].shape[0] // 64  # size(ds[1], 1) ÷ 64
        band = np.asfortranarray(np.concatenate(parts, axis=0))
        if nfpc:
            if band.dtype == np.float32:
                from . import engine

                x = engine.fb_from_numpy(band, device=f"cuda:{int(ws[0])}")
                band = engine.fb_to_numpy(engine.despike(x, nfpc))
            else:  # other result types (integer sums, Float64) keep their type
                band = _despike_host(band, int(nfpc))
        bands[j] = band
    if freqs:
        axes = [bandaxis(getheaders(ws, fs), idxs, fqavby) for ws, fs in zip(wcol, fcol)]
        return (bands[0], axes[0]) if w.ndim == 1 else (bands, axes)
    return bands[0] if w.ndim == 1 else bands
