"""Mirror of ``GBT.WorkerFunctions`` (src/gbtworkerfunctions.jl) — the
worker-side read + reduce, with the reduction moved onto the MI355X.

Same names, argument meanings and error behaviour as the reference:

* ``fqav(A, n, f="sum")``  — :16-20 (array) and :27-33 (range);
* ``sanitizeidxs``          — :167-169 (re-exported from .idxs);
* ``getdata(fname, idxs, fqavby=1, fqavfunc="sum")`` — :191-195, plus the
  additive ``tavby`` time integration;
* ``getfbdata`` / ``getfbh5data`` — :171-177 / :179-189;
* ``getkurtosis``            — :197-202;
* ``getinventory`` / headers — :35-159 (host metadata, see .readers).

``fqavfunc`` is one of ``"sum" | "mean" | "max" | "min"`` (or the Python
builtins ``sum``/``max``/``min``, ``numpy.sum``/``mean``/``max``/``min``).
Any other callable is applied on the host exactly like the reference's
generic ``f(reshape(A, ...); dims=1)`` path (README.md:192-195) — that is the
reference behaviour for functions the GPU does not implement, not a fallback
of the GPU path.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _lib, engine, readers
from .idxs import COLON, JRange, sanitizeidxs, to_window  # noqa: F401  (re-exports)

__all__ = [
    "fqav", "FRange", "sanitizeidxs", "getdata", "getfbdata", "getfbh5data", "getkurtosis",
    "getinventory", "getfbheader", "getfbh5header", "getheader",
]


@dataclass(frozen=True)
class FRange:
    """Julia ``range(first; step, length)`` (a StepRangeLen) — the type
    ``fqav(r::AbstractRange, n)`` returns (src/gbtworkerfunctions.jl:32)."""

    first: float
    step: float
    length: int

    def __len__(self):
        return self.length

    @property
    def last(self) -> float:
        return self.first + (self.length - 1) * self.step

    def values(self) -> np.ndarray:
        return self.first + self.step * np.arange(self.length, dtype=np.float64)


def _opname(f) -> str | None:
    if isinstance(f, str):
        if f not in _lib.OPS:
            raise ValueError(f"fqavfunc {f!r} not one of {sorted(_lib.OPS)}")
        return f
    names = {sum: "sum", max: "max", min: "min", np.sum: "sum", np.mean: "mean",
             np.max: "max", np.min: "min", np.amax: "max", np.amin: "min"}
    return names.get(f)


def _is_tensor(x) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


def fqav_range(r, n: int):
    """fqav(r::AbstractRange, n) (src/gbtworkerfunctions.jl:27-33)."""
    if isinstance(r, JRange):
        first, step, length = float(r.first), float(r.step), len(r)
    elif isinstance(r, FRange):
        first, step, length = r.first, r.step, r.length
    else:
        raise TypeError("range expected")
    if n <= 1:  # :28
        return r
    import ctypes

    f, s, l = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    _lib.check(_lib.lib().bldp_fqav_range(first, step, length, int(n), ctypes.byref(f),
                                          ctypes.byref(s), ctypes.byref(l)), "bldp_fqav_range")
    return FRange(f.value, s.value, l.value)


def _host_generic(A: np.ndarray, n: int, f) -> np.ndarray:
    """Reference semantics for an arbitrary Julia-style f(X; dims=1): the
    result is whatever f returns, in f's own element type (fqav returns
    dropdims(f(reshape(A, ...); dims=1); dims=1), src/gbtworkerfunctions.jl:19:
    e.g. median or std of an integer array is Float64)."""
    if A.shape[0] % n:
        raise _lib.DimensionMismatch(_lib.BLDP_EDIM,
                                     f"DimensionMismatch: fqavby={n} does not divide {A.shape[0]}")
    R = np.asarray(A).reshape((n, A.shape[0] // n) + A.shape[1:], order="F")
    return np.asfortranarray(np.asarray(f(R, axis=0)))


def fqav(A, n: int, f="sum"):
    """Reduce every ``n`` elements of the first dimension of ``A`` with ``f``
    (src/gbtworkerfunctions.jl:16-20).  ``n <= 1`` returns ``A`` itself (:17).
    Device tensors stay on the device; host arrays go through the GPU and
    come back as host arrays."""
    if isinstance(A, (JRange, FRange)):
        return fqav_range(A, n)
    if n <= 1:
        return A
    op = _opname(f)
    if _is_tensor(A):
        if op is None:
            raise TypeError("only sum/mean/max/min run on device tensors")
        return engine.reduce(A, n, 1, op)
    A = np.asarray(A)
    if op is None:
        return _host_generic(A, n, f)
    a3 = A.reshape(A.shape + (1,) * (3 - A.ndim), order="F") if A.ndim < 3 else A
    if a3.ndim != 3:
        raise ValueError("fqav arrays are at most 3-D (nchan, nif, ntime)")
    out = _reduce_host(a3, n, 1, op, None, 0)
    return out.reshape((out.shape[0],) + A.shape[1:], order="F")


def _reduce_host(a, fqavby, tavby, op, win, device):
    """A host array through the GPU with fqav's Julia result type: Float32
    stays Float32; integer and Float64 arrays take the typed kernels (sum
    widened to (U)Int64, mean Float64, max / min the input type,
    src/gbtworkerfunctions.jl:19).  Nothing is converted on the way."""
    if a.dtype == np.float32:
        return engine.reduce_host(np.asfortranarray(a), fqavby, tavby, op, win, device=device)
    if engine._dtype_code(a.dtype) is None:
        raise TypeError(f"fqav: element type {a.dtype} is not supported (Float32, Float64, "
                        f"8- to 64-bit integers)")
    return engine.reduce_host_typed(a, fqavby, tavby, op, win, device=device)


def _reduce_array(x, idxs, fqavby, fqavfunc, tavby, device):
    idxs = sanitizeidxs(idxs)
    win = to_window(idxs, x.shape)
    op = _opname(fqavfunc)
    if op is None:
        if tavby > 1:
            raise TypeError("tavby needs fqavfunc in sum/mean/max/min")
        a = np.asarray(x)
        if win is not None:
            ax = [win[3 * k] + win[3 * k + 2] * np.arange(win[3 * k + 1]) for k in range(3)]
            a = a[np.ix_(*ax)]
        return fqav(a, fqavby, fqavfunc)
    if _is_tensor(x):
        return engine.reduce(x, fqavby, tavby, op, win)
    a = np.asarray(x)
    if a.dtype != np.float32 and fqavby <= 1 and tavby <= 1:
        # fqav(A, n <= 1) returns A (:17): the window itself, in its own type
        if engine._dtype_code(a.dtype) is None:
            raise TypeError(f"element type {a.dtype} is not supported")
        engine._check_bounds(win, a.shape)
        if win is None:
            return a
        ax = [win[3 * k] + win[3 * k + 2] * np.arange(win[3 * k + 1]) for k in range(3)]
        return np.asfortranarray(a[np.ix_(*ax)])
    return _reduce_host(a, fqavby, tavby, op, win, device)


def _raw_to_device(fname, raw, idxs, device):
    """The window of a raw (filter-free, contiguous float32) file on GPU
    ``device``: (Julia-order block tensor, window relative to it), or None for
    an empty window (the host path returns the empty result)."""
    from . import filestream

    base, jshape = raw
    win = to_window(idxs, jshape) or [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
    if win[1] * win[4] * win[7] == 0:
        filestream.plan_window(jshape, win)  # bounds check only
        return None
    x, _, rwin = filestream.window_to_device(fname, base, jshape, win, f"cuda:{int(device)}")
    return x, rwin


def _reduce_raw_file(fname, raw, idxs, fqavby, op, tavby, device):
    import torch

    got = _raw_to_device(fname, raw, idxs, device)
    if got is None:
        return None
    x, rwin = got
    with torch.cuda.device(x.device):
        return engine.fb_to_numpy(engine.reduce(x, fqavby, tavby, op, rwin))


def getfbdata(fbname, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1,
              device=0):
    """SIGPROC filterbank: mmap, window, reduce (src/gbtworkerfunctions.jl:171-177).
    32-bit data with a GPU reduction: only the window's rows / channel spans
    are read (parallel preads into pinned memory, streamed to the GPU)."""
    assert len(idxs) == 3, "idxs must have exactly three indices"  # :172
    idxs = sanitizeidxs(idxs)
    op = _opname(fqavfunc)
    if op is not None:
        raw = readers.fil_raw_layout(fbname)
        if raw is not None:
            r = _reduce_raw_file(fbname, raw, idxs, fqavby, op, tavby, device)
            if r is not None:
                return r
    _, data = readers.fil_mmap(fbname)
    try:
        return _reduce_array(data, idxs, fqavby, fqavfunc, tavby, device)
    finally:
        del data  # finalize(parent(dmmap)) (:175)


def getfbh5data(fbh5name, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1,
                device=0):
    """FBH5: read the window (whole dataset for (:,:,:)), then reduce
    (src/gbtworkerfunctions.jl:179-189)."""
    assert len(idxs) == 3, "idxs must have exactly three indices"  # :180
    idxs = sanitizeidxs(idxs)
    op = _opname(fqavfunc)
    from . import fbh5

    if op is not None and (fbh5.needs_bslz4(fbh5name) or fbh5.raw_chunked(fbh5name)):
        # compressed rawspec product: only the compressed chunks cross PCIe; they
        # are decoded, windowed and reduced on the GPU, the result comes back.
        # Unfiltered chunked data takes the same chunk reader without a decode.
        # (the decoded chunk grid plus the window inside it when the chunks
        # span the window's channels: no gather copy)
        x, rwin = fbh5._read_window_bslz4_dev(fbh5name, idxs, f"cuda:{device}",
                                              raw_chunks=not fbh5.needs_bslz4(fbh5name),
                                              dense=False)
        import torch

        with torch.cuda.device(x.device):
            return engine.fb_to_numpy(engine.reduce(x, fqavby, tavby, op, rwin))
    if op is not None:
        raw = fbh5.raw_layout(fbh5name)  # uncompressed contiguous: preads, no libhdf5 copy
        if raw is not None:
            r = _reduce_raw_file(fbh5name, raw, idxs, fqavby, op, tavby, device)
            if r is not None:
                return r
    data = readers.fbh5_read(fbh5name, idxs)
    return _reduce_array(data, (COLON, COLON, COLON), fqavby, fqavfunc, tavby, device)


def window_on_device(fname, idxs, device=0):
    """The Float32 window of a file (or host / device array) on GPU
    ``device`` as (tensor, window relative to it), reading it the way
    getfbh5data / getfbdata do (compressed chunks decoded on the GPU, raw
    data block preads, else libhdf5 / mmap then one H2D copy); None when the
    data are not Float32 (those keep their own types through the host-array
    path) or the window is empty."""
    import torch

    idxs = sanitizeidxs(idxs)
    dev = f"cuda:{int(device)}"
    if _is_tensor(fname):
        if fname.dtype != torch.float32:
            return None
        return fname, to_window(idxs, fname.shape)
    if isinstance(fname, (str, bytes)) or hasattr(fname, "__fspath__"):
        from . import fbh5

        h5 = readers.ishdf5(fname)
        if h5 and (fbh5.needs_bslz4(fname) or fbh5.raw_chunked(fname)):
            return fbh5._read_window_bslz4_dev(fname, idxs, dev,
                                               raw_chunks=not fbh5.needs_bslz4(fname), dense=False)
        raw = fbh5.raw_layout(fname) if h5 else readers.fil_raw_layout(fname)
        if raw is not None:
            return _raw_to_device(fname, raw, idxs, device)
        if h5:
            a, win = readers.fbh5_read(fname, idxs), None
        else:
            _, a = readers.fil_mmap(fname)
            win = to_window(idxs, a.shape)
    else:
        a = fname
        win = to_window(idxs, np.asarray(a).shape)
    a = np.asarray(a)
    if a.dtype != np.float32:
        return None
    if win is not None:
        a = np.asfortranarray(a[np.ix_(*[win[3 * k] + win[3 * k + 2] * np.arange(win[3 * k + 1])
                                         for k in range(3)])])
    if a.size == 0:
        return None
    return engine.fb_from_numpy(a, device=dev), None


def getdata_device(fname, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1,
                   device=0, out=None):
    """getdata with the result left on GPU ``device`` (a Julia-order Float32
    tensor), written into ``out`` when given — e.g. a bank's slot of a stitched
    band product (GBT.getband); None when the data are not Float32."""
    op = _opname(fqavfunc)
    if op is None:
        raise TypeError("the device path takes fqavfunc in sum/mean/max/min")
    got = window_on_device(fname, idxs, device)
    if got is None:
        return None
    x, rwin = got
    import torch

    with torch.cuda.device(x.device):
        return engine.reduce(x, fqavby, tavby, op, rwin, out=out)


def getdata(fname, idxs=(COLON, COLON, COLON), fqavby=1, fqavfunc="sum", tavby=1, device=0):
    """WorkerFunctions.getdata (src/gbtworkerfunctions.jl:191-195).

    ``fname`` may also be an in-memory filterbank: a Fortran-ordered
    (nchan, nif, ntime) float32 array (result on the host) or a Julia-order
    device tensor (result stays on the device)."""
    if not isinstance(fname, (str, bytes)) and not hasattr(fname, "__fspath__"):
        return _reduce_array(fname, idxs, fqavby, fqavfunc, tavby, device)
    idxs = sanitizeidxs(idxs)  # :192
    if readers.ishdf5(fname):  # :193
        return getfbh5data(fname, idxs, fqavby, fqavfunc, tavby, device)
    return getfbdata(fname, idxs, fqavby, fqavfunc, tavby, device)


def getkurtosis(fname, idxs=(COLON, COLON, COLON), device=0):
    """Excess kurtosis of every (channel, IF) row over time, Float64 (nc, ni)
    (src/gbtworkerfunctions.jl:197-202)."""
    idxs = sanitizeidxs(idxs)
    if _is_tensor(fname):
        return engine.kurtosis(fname, to_window(idxs, fname.shape))
    if isinstance(fname, (str, bytes)) or hasattr(fname, "__fspath__"):
        from . import fbh5

        h5 = readers.ishdf5(fname)
        if h5 and (fbh5.needs_bslz4(fname) or fbh5.raw_chunked(fname)):
            # compressed / chunked: the chunks go to the GPU, are decoded there
            # and the kurtosis runs on the window inside the chunk grid
            import torch

            x, rwin = fbh5._read_window_bslz4_dev(fname, idxs, f"cuda:{device}",
                                                  raw_chunks=not fbh5.needs_bslz4(fname),
                                                  dense=False)
            with torch.cuda.device(x.device):
                return engine.fb_to_numpy(engine.kurtosis(x, rwin))
        raw = fbh5.raw_layout(fname) if h5 else readers.fil_raw_layout(fname)
        got = _raw_to_device(fname, raw, idxs, device) if raw is not None else None
        if got is not None:  # window streamed to the GPU, kurtosis there
            import torch

            x, rwin = got
            with torch.cuda.device(x.device):
                return engine.fb_to_numpy(engine.kurtosis(x, rwin))
        if h5:
            a, idxs = readers.fbh5_read(fname, idxs), (COLON, COLON, COLON)
        else:
            _, a = readers.fil_mmap(fname)
    else:
        a = fname
    a = np.asarray(a)
    win = to_window(idxs, a.shape)
    if a.dtype != np.float32:  # StatsBase in Float64 for integer / Float64 rows (:200)
        if engine._dtype_code(a.dtype) is None:
            raise TypeError(f"getkurtosis: element type {a.dtype} is not supported")
        return engine.kurtosis_host_typed(a, win, device=device)
    return engine.kurtosis_host(np.asfortranarray(a), win, device=device)


getinventory = readers.getinventory
getfbheader = readers.getfbheader
getfbh5header = readers.getfbh5header
getheader = readers.getheader
