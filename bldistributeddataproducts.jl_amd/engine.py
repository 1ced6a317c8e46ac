"""Device-side operations on filterbank tensors, all through libbldp_hip.

Layout: a filterbank is a torch tensor whose LOGICAL shape is Julia's
``(nchan, nif, ntime)`` and whose memory is channel-fastest, i.e. strides
``(1, nchan, nchan*nif)`` — a ``permute(2, 1, 0)`` view of a contiguous
``[ntime][nif][nchan]`` buffer, the on-disk FBH5 order (SURVEY.md §8 notation).
Views with larger pitches (sub-windows of a bigger array) are accepted as-is;
anything else is rejected rather than silently copied.

torch supplies device memory and streams only; every byte of arithmetic runs
in the HIP kernels of libbldp_hip.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .idxs import window_shape

__all__ = [
    "fb_empty", "fb_from_numpy", "fb_to_numpy", "reduce", "band_reduce", "PreparedBandReduce",
    "band_reduce_multi",
    "stitch",
    "despike", "kurtosis", "band_kurtosis", "synth", "plan", "reduce_host", "kurtosis_host",
    "init", "finalize", "pinned",
]


def _torch():
    import torch

    return torch


def init(devices=None) -> None:
    """bldp_init: check the devices are gfx950, create their worker streams and
    a warm host-staging pipeline each, enable peer access between them.
    ``None`` = every visible device.  Optional (everything initialises lazily)."""
    L = _lib.lib()
    if devices is None:
        _lib.check(L.bldp_init(0, None), "bldp_init")
        return
    devs = [int(d) for d in devices]
    arr = (ctypes.c_int * len(devs))(*devs)
    _lib.check(L.bldp_init(len(devs), ctypes.cast(arr, ctypes.c_void_p)), "bldp_init")


def finalize() -> None:
    """bldp_finalize: drain the devices and free every library-owned resource."""
    _lib.check(_lib.lib().bldp_finalize(), "bldp_finalize")


class pinned:
    """Context manager page-locking a long-lived host numpy array for the
    host-array entry points (bldp_host_register / bldp_host_unregister)."""

    def __init__(self, a: np.ndarray):
        self.a = a

    def __enter__(self):
        if self.a.nbytes:
            _lib.check(_lib.lib().bldp_host_register(self.a.ctypes.data, self.a.nbytes),
                       "bldp_host_register")
        return self.a

    def __exit__(self, *exc):
        if self.a.nbytes:
            _lib.check(_lib.lib().bldp_host_unregister(self.a.ctypes.data), "bldp_host_unregister")
        return False


def fb_empty(nchan, nif, ntime, device=None, dtype=None):
    """Uninitialised Julia-order (nchan, nif, ntime) Float32 tensor on the GPU."""
    torch = _torch()
    dtype = dtype or torch.float32
    return torch.empty((int(ntime), int(nif), int(nchan)), dtype=dtype,
                       device=device or "cuda").permute(2, 1, 0)


def band_empty(nbank, nchan, nif, ntime, device=None, dtype=None):
    """A band's banks as Julia-order (nchan, nif, ntime) views of ONE device
    slab, bank b at element offset b*nchan*nif*ntime.  Streaming a band out of
    one slab measured 2.4% faster on MI355X than out of per-bank allocations
    (7.03 vs 6.86 TB/s on the 0000 band, bench.py --band-alloc)."""
    torch = _torch()
    dtype = dtype or torch.float32
    per = int(nchan) * int(nif) * int(ntime)
    slab = torch.empty(int(nbank) * per, dtype=dtype, device=device or "cuda")
    return [slab[b * per:(b + 1) * per].view(int(ntime), int(nif), int(nchan)).permute(2, 1, 0)
            for b in range(int(nbank))]


def fb_from_numpy(a: np.ndarray, device=None):
    """Host (nchan, nif, ntime) array -> device tensor with the same layout."""
    torch = _torch()
    a = np.asfortranarray(np.asarray(a, dtype=np.float32))
    if a.ndim != 3:
        raise ValueError("filterbank arrays are 3-D (nchan, nif, ntime)")
    t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 1, 0)))
    return t.to(device or "cuda").permute(2, 1, 0)


_d2h_streams: dict = {}


def device_to_host(c, stats=None) -> np.ndarray:
    """A contiguous device tensor into a new ordinary (pageable) numpy array
    of the same shape through the library's pinned slot ring
    (bldp_device_to_host: slot-sized DMAs overlapped with the slots' copy-out
    by the reader threads).  Ordered after the work queued on torch's current
    stream of the tensor's device.  No pinned memory is allocated or held: the
    result is the caller's ordinary memory (what torch's pinned caching
    allocator would have kept page-locked, rounded up to a power of two, for as
    long as the array lives and after)."""
    torch = _torch()
    if not c.is_contiguous():
        raise ValueError("device_to_host needs a contiguous tensor")
    h = np.empty(tuple(c.shape), dtype=np.dtype(str(c.dtype).replace("torch.", "")))
    if h.nbytes == 0:
        return h
    dev = c.device
    with torch.cuda.device(dev):
        cs = _d2h_streams.get(dev.index)
        if cs is None:
            cs = _d2h_streams[dev.index] = torch.cuda.Stream(dev, priority=-1)
        st = (ctypes.c_double * 4)()
        rc = _lib.lib().bldp_device_to_host(c.data_ptr(), h.ctypes.data, h.nbytes, cs.cuda_stream,
                                            _lib.stream_ptr(), st)
    _lib.check(rc, "bldp_device_to_host")
    if stats is not None:
        stats.update(first_dma_ms=st[0], total_ms=st[1], slots=int(st[2]), threads=int(st[3]))
    return h


def fb_to_numpy(t, pinned=False) -> np.ndarray:
    """Device tensor (Julia order) -> Fortran-ordered numpy array.  With
    ``pinned`` the copy goes through the library's pinned slot ring
    (device_to_host: DMA at PCIe speed instead of torch's staged copy into
    pageable memory, ~7 GB/s) into ordinary memory the array owns."""
    torch = _torch()
    c = t.permute(2, 1, 0).contiguous() if t.dim() == 3 else t.t().contiguous()
    if pinned and c.is_cuda:
        h = device_to_host(c)
    else:
        h = c.cpu().numpy()
    return np.asfortranarray(h.transpose(2, 1, 0) if t.dim() == 3 else h.T)


def peer_access(dev, peer) -> bool:
    """bldp_peer_access: may kernels on ``dev`` store straight into memory of
    ``peer`` (same device, or xGMI peer access, enabled here)?"""
    d = ctypes.c_int()
    _lib.check(_lib.lib().bldp_peer_access(int(dev), int(peer), ctypes.byref(d)), "bldp_peer_access")
    return bool(d.value)


def _abi_dims(t, allow_typed=False):
    """Map a channel-fastest tensor to (ptr, nchan, nif, ntime) of an array
    that contains it, so that its logical index (c, i, t) is element
    c + nchan*(i + nif*t) of the ABI array.

    Float32 only unless ``allow_typed``: every caller but the typed entry
    points (reduce / kurtosis, which branch to bldp_reduce_strided and
    bldp_kurtosis) hands the pointer to an ``_f32`` function."""
    code = _dtype_code(t.dtype)
    if code is None or (code != 0 and not allow_typed):
        raise TypeError(f"unsupported filterbank element type {t.dtype} (Float32 expected)")
    if not t.is_cuda:
        raise TypeError("device tensor expected (use getdata/reduce_host for host arrays)")
    if t.dim() != 3:
        raise ValueError("filterbank tensors are 3-D (nchan, nif, ntime)")
    n0, n1, n2 = t.shape
    s0, s1, s2 = t.stride()
    if n0 > 1 and s0 != 1:
        raise ValueError("channel axis must be the fastest (stride 1); use fb_empty layout")
    if n1 > 1 and n2 > 1:
        if s1 < n0 or s2 % s1 or s2 // s1 < n1:
            raise ValueError(f"unsupported strides {t.stride()} for shape {tuple(t.shape)}")
        nchan, nif = s1, s2 // s1
    elif n1 > 1:
        if s1 < n0:
            raise ValueError(f"unsupported strides {t.stride()}")
        nchan, nif = s1, n1
    else:
        nchan = s2 if (n2 > 1 and s2 >= n0) else n0
        if n2 > 1 and s2 < n0:
            raise ValueError(f"unsupported strides {t.stride()}")
        nif = 1
    return t.data_ptr(), int(nchan), int(nif), int(n2)


# bldp_dtype codes (include/bldp.h) by numpy element type
DTYPE_CODES = {np.dtype(np.float32): 0, np.dtype(np.float64): 1, np.dtype(np.uint8): 2,
               np.dtype(np.uint16): 3, np.dtype(np.uint32): 4, np.dtype(np.uint64): 5,
               np.dtype(np.int8): 6, np.dtype(np.int16): 7, np.dtype(np.int32): 8,
               np.dtype(np.int64): 9}
DTYPE_OF_CODE = {v: k for k, v in DTYPE_CODES.items()}


def _dtype_code(dt):
    """bldp_dtype of a numpy dtype or torch dtype (None if unsupported)."""
    if not isinstance(dt, np.dtype):
        try:
            dt = np.dtype(str(dt).replace("torch.", ""))
        except TypeError:
            return None
    return DTYPE_CODES.get(np.dtype(dt))


def out_dtype(dtype, op: str) -> np.dtype:
    """fqav's result element type for input `dtype` (Julia's; bldp_reduce_out_dtype):
    sum widens integers to (U)Int64, mean is Float64, max / min keep the type."""
    code = _dtype_code(dtype)
    if code is None:
        raise TypeError(f"unsupported element type {dtype}")
    rc = _lib.lib().bldp_reduce_out_dtype(code, _lib.OPS[op])
    _lib.check(min(rc, 0), "bldp_reduce_out_dtype")
    return DTYPE_OF_CODE[rc]


def _torch_dtype(dt: np.dtype):
    torch = _torch()
    return getattr(torch, np.dtype(dt).name)


def _check_bounds(win, shape):
    if win is None:
        return
    for ax in range(3):
        st, ct, sp = win[3 * ax: 3 * ax + 3]
        if ct > 0:
            last = st + (ct - 1) * sp
            if min(st, last) < 0 or max(st, last) >= shape[ax]:
                raise _lib.BoundsError(
                    _lib.BLDP_EBOUNDS,
                    f"BoundsError: window {st + 1}:{sp}:{last + 1} outside axis {ax + 1} of "
                    f"size {shape[ax]}")


def _full_win(win, shape):
    return list(win) if win is not None else [0, shape[0], 1, 0, shape[1], 1, 0, shape[2], 1]


def out_shape(shape, win, fqavby, tavby):
    nc, ni, nt = window_shape(win, shape)
    F, T = max(int(fqavby), 1), max(int(tavby), 1)
    if nc % F:
        raise _lib.DimensionMismatch(_lib.BLDP_EDIM,
                                     f"DimensionMismatch: fqavby={F} does not divide nchan={nc}")
    if nt % T:
        raise _lib.DimensionMismatch(_lib.BLDP_EDIM,
                                     f"DimensionMismatch: tavby={T} does not divide ntime={nt}")
    return nc // F, ni, nt // T


def reduce(x, fqavby=1, tavby=1, op="sum", win=None, out=None, stream=None):
    """fqav on the channel axis fused with time integration, on the GPU.

    x: device filterbank tensor; win: 9-int window (see idxs.to_window) or
    None; returns a Julia-order (nc/F, ni, nt/T) device tensor."""
    L = _lib.lib()
    shape = tuple(x.shape)
    _check_bounds(win, shape)
    nco, ni, nto = out_shape(shape, win, fqavby, tavby)
    torch = _torch()
    typed = x.dtype != torch.float32
    odt = _torch_dtype(out_dtype(x.dtype, op)) if typed else torch.float32
    if out is None:
        out = fb_empty(nco, ni, nto, device=x.device, dtype=odt)
    elif tuple(out.shape) != (nco, ni, nto) or out.dtype != odt:
        raise ValueError(f"out is {out.dtype} {tuple(out.shape)}, expected {odt} {(nco, ni, nto)}")
    optr, onc, oni, _ = _abi_dims(out, allow_typed=True) if out.numel() else (0, nco, ni, nto)
    ptr, nchan, nif, ntime = _abi_dims(x, allow_typed=True)
    keep, wp = _lib.win_arg(_full_win(win, shape))
    if typed:  # fqav's Julia result types for integer / Float64 data (bldp_reduce_strided)
        rc = L.bldp_reduce_strided(_dtype_code(x.dtype), ptr, nchan, nif, ntime, wp, int(fqavby),
                                   int(tavby), _lib.OPS[op], optr, onc, onc * oni,
                                   _lib.stream_ptr(stream))
        _lib.check(rc, "bldp_reduce_strided")
        return out
    rc = L.bldp_reduce_strided_f32(ptr, nchan, nif, ntime, wp, int(fqavby), int(tavby),
                                   _lib.OPS[op], optr, onc, onc * oni, _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_reduce_strided_f32")
    return out


class _Prepared:
    """A bldp_reduce_op_t handle: ``launch`` is one ctypes call that queues
    the kernel(s), ``launch_timed`` the same with two timing HipEvents,
    ``close`` releases it.  Keeps its tensors alive."""

    def _bind(self, L, h, keep):
        self._L, self._h, self._keep = L, h, keep
        self._fn, self._timed = L.bldp_reduce_launch, L.bldp_reduce_launch_timed

    def launch(self, stream=None) -> None:
        sp = stream if isinstance(stream, int) else _lib.stream_ptr(stream)
        rc = self._fn(self._h, sp)
        if rc:
            _lib.check(rc, "bldp_reduce_launch")

    def launch_timed(self, stream, ev_start, ev_stop) -> None:
        sp = stream if isinstance(stream, int) else _lib.stream_ptr(stream)
        rc = self._timed(self._h, sp, ev_start.ev, ev_stop.ev)
        if rc:
            _lib.check(rc, "bldp_reduce_launch_timed")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.bldp_reduce_release(self._h)
            self._h = None

    def __del__(self):
        self.close()


class PreparedReduce(_Prepared):
    """``reduce`` prepared once for fixed buffers, any element type
    (bldp_reduce_prepare): the per-file worker call of
    src/gbtworkerfunctions.jl:171-177 re-run on resident buffers costs one
    ctypes call and the kernel launch.  ``out`` as ``reduce`` makes it."""

    def __init__(self, x, fqavby=1, tavby=1, op="sum", win=None, out=None):
        torch = _torch()
        L = _lib.lib()
        shape = tuple(x.shape)
        _check_bounds(win, shape)
        nco, ni, nto = out_shape(shape, win, fqavby, tavby)
        odt = _torch_dtype(out_dtype(x.dtype, op)) if x.dtype != torch.float32 else torch.float32
        if out is None:
            out = fb_empty(nco, ni, nto, device=x.device, dtype=odt)
        elif tuple(out.shape) != (nco, ni, nto) or out.dtype != odt:
            raise ValueError(f"out is {out.dtype} {tuple(out.shape)}, expected {odt} "
                             f"{(nco, ni, nto)}")
        optr, onc, oni, _ = _abi_dims(out, allow_typed=True) if out.numel() else (0, nco, ni, nto)
        ptr, nchan, nif, ntime = _abi_dims(x, allow_typed=True)
        keep, wp = _lib.win_arg(_full_win(win, shape))
        h = ctypes.c_void_p()
        with torch.cuda.device(x.device):
            rc = L.bldp_reduce_prepare(_dtype_code(x.dtype), ptr, nchan, nif, ntime, wp,
                                       int(fqavby), int(tavby), _lib.OPS[op], optr, onc,
                                       onc * oni, ctypes.byref(h))
        _lib.check(rc, "bldp_reduce_prepare")
        self._bind(L, h, (x, keep))
        self.out = out


class PreparedKurtosis(_Prepared):
    """``kurtosis`` prepared once for fixed buffers, any element type
    (bldp_kurtosis_prepare): getkurtosis (src/gbtworkerfunctions.jl:197-202)
    re-run on a resident window for one ctypes call and the kernel launch."""

    def __init__(self, x, win=None, out=None):
        torch = _torch()
        L = _lib.lib()
        shape = tuple(x.shape)
        _check_bounds(win, shape)
        nc, ni, _ = window_shape(win, shape)
        if out is None:
            out = torch.empty((ni, nc), dtype=torch.float64, device=x.device).t()
        ptr, nchan, nif, ntime = _abi_dims(x, allow_typed=True)
        keep, wp = _lib.win_arg(_full_win(win, shape))
        h = ctypes.c_void_p()
        with torch.cuda.device(x.device):
            rc = L.bldp_kurtosis_prepare(_dtype_code(x.dtype), ptr, nchan, nif, ntime, wp,
                                         out.data_ptr() if out.numel() else None,
                                         ctypes.byref(h))
        _lib.check(rc, "bldp_kurtosis_prepare")
        self._bind(L, h, (x, keep))
        self.out = out


def plan(x, fqavby=1, tavby=1, op="sum", win=None) -> dict:
    """Launch plan the library picks for this call (path, lanes/group, ...)."""
    L = _lib.lib()
    shape = tuple(x.shape)
    _check_bounds(win, shape)
    ptr, nchan, nif, ntime = _abi_dims(x)
    info = (ctypes.c_int64 * 8)()
    keep, wp = _lib.win_arg(_full_win(win, shape))
    rc = L.bldp_reduce_plan_f32(ptr, nchan, nif, ntime, wp, int(fqavby), int(tavby),
                                _lib.OPS[op], None, info)
    _lib.check(rc, "bldp_reduce_plan_f32")
    keys = ["path", "lanes_per_group", "time_split_waves", "float4_per_lane", "time_chunks",
            "workgroups", "workspace_bytes", "vec_out"]
    d = dict(zip(keys, list(info)))
    d["path"] = _lib.PATHS[d["path"]]
    return d


def _band_args(banks, fqavby, tavby, win, out):
    """Checks of a one-GPU band reduce; (banks, geometry, out, ptr array, window keepalive)."""
    banks = list(banks)
    if not banks:
        raise ValueError("no banks")
    shape = tuple(banks[0].shape)
    geo = None
    for b in banks:
        if tuple(b.shape) != shape:
            raise ValueError("all banks of a band must have the same shape")
        g = _abi_dims(b)[1:]
        if geo is None:
            geo = g
        elif g != geo:
            raise ValueError("all banks of a band must have the same layout")
    _check_bounds(win, shape)
    nco, ni, nto = out_shape(shape, win, fqavby, tavby)
    nb = len(banks)
    if out is None:
        out = fb_empty(nb * nco, ni, nto, device=banks[0].device)
    if _dtype_code(out.dtype) != 0:
        raise TypeError(f"out must be Float32, not {out.dtype}")
    if tuple(out.shape) != (nb * nco, ni, nto) or (
            out.numel() and out.stride() != (1, nb * nco, nb * nco * ni) and ni * nto > 1):
        raise ValueError("out must be a dense Julia-order (nbank*nco, ni, nto) tensor")
    ptrs = (ctypes.c_void_p * nb)(*[b.data_ptr() for b in banks])
    keep, wp = _lib.win_arg(_full_win(win, shape))
    return banks, geo, out, ptrs, (keep, wp)


def band_reduce(banks, fqavby=1, tavby=1, op="sum", win=None, out=None, stream=None):
    """Reduce every bank of a band resident on ONE GPU and stitch them in bank
    order (reduce(vcat, ...), src/gbt.jl:103) in a single launch."""
    L = _lib.lib()
    banks, geo, out, ptrs, (keep, wp) = _band_args(banks, fqavby, tavby, win, out)
    nchan, nif, ntime = geo
    rc = L.bldp_band_reduce_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), nchan, nif, ntime,
                                wp, int(fqavby), int(tavby), _lib.OPS[op],
                                out.data_ptr() if out.numel() else None,
                                _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_band_reduce_f32")
    return out


class PreparedBandReduce:
    """band_reduce prepared once for fixed buffers (bldp_band_reduce_prepare_f32):
    checks, plan and kernel arguments are computed here, and ``launch`` only
    queues the kernel — one ctypes call, no Python-side work.  Results are
    those of ``band_reduce`` with the same arguments.  The banks and ``out``
    are kept alive by the object; ``close`` releases the handle."""

    def __init__(self, banks, fqavby=1, tavby=1, op="sum", win=None, out=None):
        L = _lib.lib()
        banks, geo, out, ptrs, (keep, wp) = _band_args(banks, fqavby, tavby, win, out)
        h = ctypes.c_void_p()
        with _torch().cuda.device(banks[0].device):
            rc = L.bldp_band_reduce_prepare_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p),
                                                *geo, wp, int(fqavby), int(tavby), _lib.OPS[op],
                                                out.data_ptr() if out.numel() else None,
                                                ctypes.byref(h))
        _lib.check(rc, "bldp_band_reduce_prepare_f32")
        self._L, self._h = L, h
        self._fn = L.bldp_reduce_launch
        self._timed = L.bldp_reduce_launch_timed
        self.banks, self.out = banks, out

    def launch(self, stream=None) -> None:
        """Queue the reduce on ``stream`` (a torch stream, a raw hipStream_t
        int, or None for torch's current stream)."""
        sp = stream if isinstance(stream, int) else _lib.stream_ptr(stream)
        rc = self._fn(self._h, sp)
        if rc:
            _lib.check(rc, "bldp_reduce_launch")

    def launch_timed(self, stream, ev_start, ev_stop) -> None:
        """``launch`` with the reduce's own dispatches carrying two timing
        ``_lib.HipEvent`` s (bldp_reduce_launch_timed): nothing is queued
        between this launch and the next."""
        sp = stream if isinstance(stream, int) else _lib.stream_ptr(stream)
        rc = self._timed(self._h, sp, ev_start.ev, ev_stop.ev)
        if rc:
            _lib.check(rc, "bldp_reduce_launch_timed")

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.bldp_reduce_release(self._h)
            self._h = None

    def __del__(self):
        self.close()


def band_reduce_multi(banks, fqavby=1, tavby=1, op="sum", win=None, root=0, out=None,
                      staged=False, peer_store=False):
    """One process, banks on several GPUs (bldp_band_reduce_multi_f32): each
    GPU reduces its banks (one launch per device for contiguous shards) into
    their vcat slots of the stitched product on `root` (into ``out`` when
    given: a dense Julia-order (nbank*nco, ni, nto) Float32 tensor there); a
    device other than the root reduces into staging and one peer copy moves
    its slots.  ``staged``: every bank takes the staged branch
    (BLDP_BAND_STAGED), the root's included; ``peer_store``: devices with peer
    access store their slots over xGMI from the kernels (BLDP_BAND_PEER_STORE,
    opt-in until a multi-GPU node has run it) -- per-call arguments, not
    process state."""
    torch = _torch()
    L = _lib.lib()
    banks = list(banks)
    shape = tuple(banks[0].shape)
    geo = _abi_dims(banks[0])[1:]
    for b in banks[1:]:
        if tuple(b.shape) != shape or _abi_dims(b)[1:] != geo:
            raise ValueError("all banks of a band must have the same shape and layout")
    _check_bounds(win, shape)
    nco, ni, nto = out_shape(shape, win, fqavby, tavby)
    if out is None:
        out = fb_empty(len(banks) * nco, ni, nto, device=torch.device("cuda", root))
    elif (_dtype_code(out.dtype) != 0 or tuple(out.shape) != (len(banks) * nco, ni, nto)
          or out.device != torch.device("cuda", root)
          or (out.numel() and ni * nto > 1 and out.stride() != (1, len(banks) * nco,
                                                                 len(banks) * nco * ni))):
        raise ValueError("out must be a dense Julia-order (nbank*nco, ni, nto) Float32 tensor "
                         "on the root device")
    devs = (ctypes.c_int * len(banks))(*[b.device.index for b in banks])
    ptrs = (ctypes.c_void_p * len(banks))(*[b.data_ptr() for b in banks])
    keep, wp = _lib.win_arg(_full_win(win, shape))
    for d in {b.device.index for b in banks}:
        torch.cuda.synchronize(d)  # inputs written on torch streams are complete
    rc = L.bldp_band_reduce_multi_f32(len(banks), ctypes.cast(devs, ctypes.c_void_p),
                                      ctypes.cast(ptrs, ctypes.c_void_p), *geo, wp,
                                      int(fqavby), int(tavby), _lib.OPS[op], int(root),
                                      out.data_ptr() if out.numel() else None,
                                      (_lib.BLDP_BAND_STAGED if staged else 0)
                                      | (_lib.BLDP_BAND_PEER_STORE if peer_store else 0))
    _lib.check(rc, "bldp_band_reduce_multi_f32")
    return out


def stitch(gathered, nbank, out=None, stream=None):
    """gathered: nbank dense (nc, ni, nt) blocks back to back (1-D or a
    [nbank, nt, ni, nc] contiguous tensor); returns vcat (nbank*nc, ni, nt)."""
    L = _lib.lib()
    g = gathered
    if g.dim() == 4:
        nb, nt, ni, nc = g.shape
    else:
        raise ValueError("gathered must be a contiguous [nbank, ntime, nif, nc] tensor")
    if nb != nbank or not g.is_contiguous():
        raise ValueError("gathered must be a contiguous [nbank, ntime, nif, nc] tensor")
    if out is None:
        out = fb_empty(nbank * nc, ni, nt, device=g.device)
    rc = L.bldp_stitch_f32(nbank, g.data_ptr(), nc, ni, nt, out.data_ptr(),
                           _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_stitch_f32")
    return out


def despike(x, nfpc, stream=None):
    """In place: every coarse channel's DC bin takes its left neighbour's
    value (src/gbt.jl:101-102,111).  Returns x."""
    L = _lib.lib()
    ptr, nchan, nif, ntime = _abi_dims(x)
    if nchan != x.shape[0] or (x.shape[1] > 1 and nif != x.shape[1]):
        raise ValueError("despike needs a dense Julia-order tensor")
    rc = L.bldp_despike_f32(ptr, x.shape[0], x.shape[1], x.shape[2], int(nfpc),
                            _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_despike_f32")
    return x


def kurtosis(x, win=None, stream=None):
    """Excess kurtosis over time per (channel, IF): (nc, ni) float64 tensor."""
    torch = _torch()
    L = _lib.lib()
    shape = tuple(x.shape)
    _check_bounds(win, shape)
    nc, ni, _ = window_shape(win, shape)
    out = torch.empty((ni, nc), dtype=torch.float64, device=x.device).t()
    ptr, nchan, nif, ntime = _abi_dims(x, allow_typed=True)
    keep, wp = _lib.win_arg(_full_win(win, shape))
    if x.dtype != torch.float32:  # StatsBase in Float64 for integer / Float64 rows
        rc = L.bldp_kurtosis(_dtype_code(x.dtype), ptr, nchan, nif, ntime, wp,
                             out.data_ptr() if out.numel() else None, _lib.stream_ptr(stream))
        _lib.check(rc, "bldp_kurtosis")
        return out
    rc = L.bldp_kurtosis_f32(ptr, nchan, nif, ntime, wp, out.data_ptr() if out.numel() else None,
                             None, _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_kurtosis_f32")
    return out


def kurtosis_plan(x, win=None) -> dict:
    """Kurtosis plan for this tensor and window: path ("regs", "mid", "leaf",
    "twopass"), K (level of the pairwise-sum blocks), leaf slots, workspace."""
    L = _lib.lib()
    shape = tuple(x.shape)
    _check_bounds(win, shape)
    ptr, nchan, nif, ntime = _abi_dims(x)
    info = (ctypes.c_int64 * 4)()
    keep, wp = _lib.win_arg(_full_win(win, shape))
    _lib.check(L.bldp_kurtosis_plan_f32(ptr, nchan, nif, ntime, wp, info), "bldp_kurtosis_plan_f32")
    return {"path": _lib.KURT_PATHS[info[0]], "K": info[1], "leaf_slots": info[2],
            "workspace_bytes": info[3]}


def band_kurtosis(banks, win=None, stream=None):
    """Kurtosis of every bank of a band on one GPU in one set of launches;
    returns a list of (nc, ni) float64 tensors (views of one buffer)."""
    torch = _torch()
    L = _lib.lib()
    banks = list(banks)
    if not banks:
        raise ValueError("no banks")
    shape = tuple(banks[0].shape)
    geo = _abi_dims(banks[0])[1:]
    for b in banks[1:]:
        if tuple(b.shape) != shape or _abi_dims(b)[1:] != geo:
            raise ValueError("all banks of a band must have the same shape and layout")
    _check_bounds(win, shape)
    nc, ni, _ = window_shape(win, shape)
    buf = torch.empty((len(banks), ni, nc), dtype=torch.float64, device=banks[0].device)
    ptrs = (ctypes.c_void_p * len(banks))(*[b.data_ptr() for b in banks])
    keep, wp = _lib.win_arg(_full_win(win, shape))
    rc = L.bldp_band_kurtosis_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), *geo, wp,
                                  buf.data_ptr() if buf.numel() else None,
                                  _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_band_kurtosis_f32")
    return [buf[k].t() for k in range(len(banks))]


def synth(nchan, nif, ntime, nfpc=1024, seed=0, kind=0, device=None, stream=None, out=None):
    """Synthetic BL-like filterbank generated on the GPU (bldp_synth_f32),
    into ``out`` (a dense Julia-order tensor, e.g. a band_empty view) if given."""
    L = _lib.lib()
    if out is None:
        out = fb_empty(nchan, nif, ntime, device=device)
    elif tuple(out.shape) != (nchan, nif, ntime) or (
            out.numel() and out.stride() != (1, nchan, nchan * nif)):
        raise ValueError("out must be a dense Julia-order (nchan, nif, ntime) tensor")
    rc = L.bldp_synth_f32(out.data_ptr() if out.numel() else None, nchan, nif, ntime, nfpc,
                          seed, kind, _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_synth_f32")
    return out


def reduce_host(a: np.ndarray, fqavby=1, tavby=1, op="sum", win=None, device=0) -> np.ndarray:
    """Host array in, host array out (bldp_reduce_host_f32): the window is
    streamed through the GPU and reduced there."""
    L = _lib.lib()
    a = np.asarray(a)
    if a.dtype != np.float32 or not a.flags.f_contiguous or a.ndim != 3:
        raise TypeError("host filterbank must be a Fortran-ordered float32 (nchan, nif, ntime)")
    shape = a.shape
    _check_bounds(win, shape)
    nco, ni, nto = out_shape(shape, win, fqavby, tavby)
    out = np.empty((nco, ni, nto), dtype=np.float32, order="F")
    keep, wp = _lib.win_arg(_full_win(win, shape))
    rc = L.bldp_reduce_host_f32(int(device), a.ctypes.data if a.size else None, shape[0],
                                shape[1], shape[2], wp, int(fqavby), int(tavby), _lib.OPS[op],
                                out.ctypes.data if out.size else None)
    _lib.check(rc, "bldp_reduce_host_f32")
    return out


def kurtosis_host(a: np.ndarray, win=None, device=0) -> np.ndarray:
    """Host array in, (nc, ni) float64 host array out (bldp_kurtosis_host_f32)."""
    L = _lib.lib()
    a = np.asarray(a)
    if a.dtype != np.float32 or not a.flags.f_contiguous or a.ndim != 3:
        raise TypeError("host filterbank must be a Fortran-ordered float32 (nchan, nif, ntime)")
    _check_bounds(win, a.shape)
    nc, ni, _ = window_shape(win, a.shape)
    out = np.empty((nc, ni), dtype=np.float64, order="F")
    keep, wp = _lib.win_arg(_full_win(win, a.shape))
    rc = L.bldp_kurtosis_host_f32(int(device), a.ctypes.data if a.size else None, a.shape[0],
                                  a.shape[1], a.shape[2], wp, out.ctypes.data if out.size else None)
    _lib.check(rc, "bldp_kurtosis_host_f32")
    return out


def reduce_host_typed(a: np.ndarray, fqavby=1, tavby=1, op="sum", win=None, device=0) -> np.ndarray:
    """Host array of any supported element type in, host array of fqav's
    Julia result type out (bldp_reduce_host): e.g. UInt8 SIGPROC data summed
    into UInt64, averaged into Float64, max / min kept as UInt8."""
    L = _lib.lib()
    a = np.asarray(a)
    code = _dtype_code(a.dtype)
    if code is None or a.ndim != 3:
        raise TypeError(f"unsupported host filterbank {a.dtype} {a.shape}")
    a = np.asfortranarray(a)
    shape = a.shape
    _check_bounds(win, shape)
    nco, ni, nto = out_shape(shape, win, fqavby, tavby)
    out = np.empty((nco, ni, nto), dtype=out_dtype(a.dtype, op), order="F")
    keep, wp = _lib.win_arg(_full_win(win, shape))
    rc = L.bldp_reduce_host(int(device), code, a.ctypes.data if a.size else None, shape[0],
                            shape[1], shape[2], wp, int(fqavby), int(tavby), _lib.OPS[op],
                            out.ctypes.data if out.size else None)
    _lib.check(rc, "bldp_reduce_host")
    return out


def kurtosis_host_typed(a: np.ndarray, win=None, device=0) -> np.ndarray:
    """Host array of any supported element type in, (nc, ni) float64 out
    (bldp_kurtosis_host; StatsBase's recipe in Float64 for non-Float32 rows,
    8- and 16-bit integer rows from exact integer power sums)."""
    L = _lib.lib()
    a = np.asarray(a)
    code = _dtype_code(a.dtype)
    if code is None or a.ndim != 3:
        raise TypeError(f"unsupported host filterbank {a.dtype} {a.shape}")
    a = np.asfortranarray(a)
    _check_bounds(win, a.shape)
    nc, ni, _ = window_shape(win, a.shape)
    out = np.empty((nc, ni), dtype=np.float64, order="F")
    keep, wp = _lib.win_arg(_full_win(win, a.shape))
    rc = L.bldp_kurtosis_host(int(device), code, a.ctypes.data if a.size else None, a.shape[0],
                              a.shape[1], a.shape[2], wp, out.ctypes.data if out.size else None)
    _lib.check(rc, "bldp_kurtosis_host")
    return out
