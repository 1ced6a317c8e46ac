"""TEST INFRASTRUCTURE ONLY — the parity oracle for libbldp_hip.

Two independent CPU restatements of the reference's worker-side reduction
(BLDistributedDataProducts.jl v0.3.2, src/gbtworkerfunctions.jl):

* ``C``: ctypes binding to ``oracle/liboracle.so`` (bldp_oracle.c), the
  authoritative checker and the ``cpu_baseline`` of bench.py;
* ``np_*``: a NumPy restatement written directly from the Julia source, used
  to cross-check the C restatement and to generate tests/golden fixtures.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg may
import this module.  The product path never does.

Parity status: pinned against the reference's own
known-answer tests only for ``fqav(::AbstractRange, n)`` (test/runtests.jl:5-6).
The array reductions are *parity unpinned* — Julia is absent here and the
reference ships no array fixtures — and are held instead to (a) agreement of
the two restatements, (b) integer-valued fixtures whose float32 sums are exact
in every summation order.

Array convention: Julia order.  A filterbank is a numpy array of logical shape
(nchan, nif, ntime), Fortran-contiguous (channel fastest), exactly the bytes
HDF5.jl / Blio hand to WorkerFunctions.getdata (README.md:165-168).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

OPS = {"sum": 0, "mean": 1, "max": 2, "min": 3}


class DimensionMismatch(ValueError):
    """Julia's DimensionMismatch (fqav reshape, src/gbtworkerfunctions.jl:18)."""


class BoundsErr(IndexError):
    """Julia's BoundsError (window outside the array)."""


# --------------------------------------------------------------------------
# C restatement (ctypes)
# --------------------------------------------------------------------------
_lib = None


def build() -> str:
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, I64, I = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        L.oracle_reduce.argtypes = [P, I64, I64, I64, P, I64, I64, I, P]
        L.oracle_reduce.restype = I
        L.oracle_kurtosis.argtypes = [P, I64, I64, I64, P, P]
        L.oracle_kurtosis.restype = I
        L.oracle_mean_f32.argtypes = [P, I64, I64, I64, P, P]
        L.oracle_mean_f32.restype = I
        L.oracle_stitch.argtypes = [I, P, I64, I64, I64, P]
        L.oracle_stitch.restype = I
        L.oracle_despike.argtypes = [P, I64, I64, I64, I64]
        L.oracle_despike.restype = I
        D = ctypes.c_double
        L.oracle_fqav_range.argtypes = [D, D, I64, I64, P, P, P]
        L.oracle_fqav_range.restype = None
        L.oracle_synth.argtypes = [P, I64, I64, I64, I64, ctypes.c_uint64, I]
        L.oracle_synth.restype = None
        L.oracle_reduce_banks_mt.argtypes = [I, P, I64, I64, I64, I64, I64, I, P]
        L.oracle_reduce_banks_mt.restype = I
        L.oracle_reduce_banks_pool.argtypes = [I, P, I64, I64, I64, I64, I64, I, P, I]
        L.oracle_reduce_banks_pool.restype = I
        _lib = L
    return _lib


def _fa(a: np.ndarray) -> np.ndarray:
    a = np.asarray(a, dtype=np.float32)
    if a.ndim != 3:
        raise ValueError("filterbank arrays are 3-D (nchan, nif, ntime)")
    return np.asfortranarray(a)


def _win(win):
    if win is None:
        return None, None
    w = (ctypes.c_int64 * 9)(*[int(x) for x in win])
    return w, ctypes.cast(w, ctypes.c_void_p)


def _check(rc: int, what: str):
    if rc == -2:
        raise DimensionMismatch(what)
    if rc == -6:
        raise BoundsErr(what)
    if rc != 0:
        raise ValueError(f"{what}: oracle error {rc}")


def window_shape(shape, win):
    if win is None:
        return tuple(shape)
    return (int(win[1]), int(win[4]), int(win[7]))


def reduce(a, fqavby=1, tavby=1, op="sum", win=None) -> np.ndarray:
    """C restatement of fqav on axis 1 fused with fqav on axis 3."""
    a = _fa(a)
    nc, ni, nt = window_shape(a.shape, win)
    F, T = max(int(fqavby), 1), max(int(tavby), 1)
    if nc % F or nt % T:
        raise DimensionMismatch(f"fqavby={F} / tavby={T} vs window {nc}x{nt}")
    out = np.empty((nc // F, ni, nt // T), dtype=np.float32, order="F")
    keep, wp = _win(win)
    rc = lib().oracle_reduce(a.ctypes.data, a.shape[0], a.shape[1], a.shape[2], wp, F, T,
                             OPS[op], out.ctypes.data)
    _check(rc, "oracle_reduce")
    return out


def kurtosis(a, win=None) -> np.ndarray:
    a = _fa(a)
    nc, ni, nt = window_shape(a.shape, win)
    out = np.empty((nc, ni), dtype=np.float64, order="F")
    keep, wp = _win(win)
    rc = lib().oracle_kurtosis(a.ctypes.data, a.shape[0], a.shape[1], a.shape[2], wp,
                               out.ctypes.data)
    _check(rc, "oracle_kurtosis")
    return out


def mean_f32(a, win=None) -> np.ndarray:
    """StatsBase's m of every (channel, IF) row: Julia's Float32 pairwise sum
    over time / length; (nc, ni) float32."""
    a = _fa(a)
    nc, ni, nt = window_shape(a.shape, win)
    out = np.empty((nc, ni), dtype=np.float32, order="F")
    keep, wp = _win(win)
    rc = lib().oracle_mean_f32(a.ctypes.data, a.shape[0], a.shape[1], a.shape[2], wp,
                               out.ctypes.data)
    _check(rc, "oracle_mean_f32")
    return out


def py_pairwise_sum(v) -> np.float32:
    """Base.mapreduce_impl(identity, +, v, 1, n) line by line (pure Python
    loops over np.float32 scalars; small n only): the third restatement of
    Julia's Float32 sum, written from base/reduce.jl's structure."""
    v = [np.float32(x) for x in v]

    def impl(ifirst, ilast, blksize=1024):
        if ifirst == ilast:
            return v[ifirst]
        if ifirst + blksize > ilast:
            a = v[ifirst] + v[ifirst + 1]
            for i in range(ifirst + 2, ilast + 1):
                a = np.float32(a + v[i])
            return np.float32(a)
        imid = ifirst + ((ilast - ifirst) >> 1)
        return np.float32(impl(ifirst, imid) + impl(imid + 1, ilast))

    return impl(0, len(v) - 1)


def stitch(banks) -> np.ndarray:
    banks = [_fa(b) for b in banks]
    nc, ni, nt = banks[0].shape
    ptrs = (ctypes.c_void_p * len(banks))(*[b.ctypes.data for b in banks])
    out = np.empty((nc * len(banks), ni, nt), dtype=np.float32, order="F")
    rc = lib().oracle_stitch(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), nc, ni, nt,
                             out.ctypes.data)
    _check(rc, "oracle_stitch")
    return out


def despike(d, nfpc) -> np.ndarray:
    d = _fa(d).copy(order="F")
    rc = lib().oracle_despike(d.ctypes.data, d.shape[0], d.shape[1], d.shape[2], int(nfpc))
    _check(rc, "oracle_despike")
    return d


def fqav_range(first, step, length, n):
    f, s, l = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    lib().oracle_fqav_range(float(first), float(step), int(length), int(n), ctypes.byref(f),
                            ctypes.byref(s), ctypes.byref(l))
    return f.value, s.value, l.value


def synth(nchan, nif, ntime, nfpc, seed, kind=0) -> np.ndarray:
    out = np.empty((nchan, nif, ntime), dtype=np.float32, order="F")
    lib().oracle_synth(out.ctypes.data, nchan, nif, ntime, nfpc, seed, kind)
    return out


def reduce_banks_mt(banks, fqavby, tavby, op="sum"):
    """CPU baseline: one thread per bank (one Distributed worker per bank)."""
    banks = [_fa(b) for b in banks]
    nchan, nif, ntime = banks[0].shape
    F, T = max(int(fqavby), 1), max(int(tavby), 1)
    outs = [np.empty((nchan // F, nif, ntime // T), np.float32, order="F") for _ in banks]
    ip = (ctypes.c_void_p * len(banks))(*[b.ctypes.data for b in banks])
    op_ = (ctypes.c_void_p * len(banks))(*[o.ctypes.data for o in outs])
    rc = lib().oracle_reduce_banks_mt(len(banks), ctypes.cast(ip, ctypes.c_void_p), nchan, nif,
                                      ntime, F, T, OPS[op], ctypes.cast(op_, ctypes.c_void_p))
    _check(rc, "oracle_reduce_banks_mt")
    return outs


def reduce_banks_pool(banks, fqavby, tavby, op="sum", nthreads=1):
    """CPU baseline on every core: the banks' output channels split into
    pieces over ``nthreads`` threads (same arithmetic as ``reduce``)."""
    banks = [_fa(b) for b in banks]
    nchan, nif, ntime = banks[0].shape
    F, T = max(int(fqavby), 1), max(int(tavby), 1)
    outs = [np.empty((nchan // F, nif, ntime // T), np.float32, order="F") for _ in banks]
    ip = (ctypes.c_void_p * len(banks))(*[b.ctypes.data for b in banks])
    op_ = (ctypes.c_void_p * len(banks))(*[o.ctypes.data for o in outs])
    rc = lib().oracle_reduce_banks_pool(len(banks), ctypes.cast(ip, ctypes.c_void_p), nchan, nif,
                                        ntime, F, T, OPS[op], ctypes.cast(op_, ctypes.c_void_p),
                                        int(nthreads))
    _check(rc, "oracle_reduce_banks_pool")
    return outs


# --------------------------------------------------------------------------
# NumPy restatement (independent of the C code)
# --------------------------------------------------------------------------
def np_window(a: np.ndarray, win) -> np.ndarray:
    """h5["data"][idxs...] with idxs given as 9 ints (0-based start, count, step)."""
    if win is None:
        return a
    ax = [win[3 * k] + win[3 * k + 2] * np.arange(win[3 * k + 1]) for k in range(3)]
    for k in range(3):
        if len(ax[k]) and (ax[k].min() < 0 or ax[k].max() >= a.shape[k]):
            raise BoundsErr(f"axis {k + 1}")
    return np.asfortranarray(a[np.ix_(*ax)])


def _fix_zero(m, R, axis, op):
    """numpy's max/min keep whichever signed zero came first; Julia orders
    -0.0 < +0.0.  Repair the all-zero-extremum groups."""
    zero = m == 0
    if not zero.any():
        return m
    if op == "max":
        pos = np.any((R == 0) & ~np.signbit(R), axis=axis)
        return np.where(zero, np.where(pos, np.float32(0.0), np.float32(-0.0)), m)
    neg = np.any((R == 0) & np.signbit(R), axis=axis)
    return np.where(zero, np.where(neg, np.float32(-0.0), np.float32(0.0)), m)


def np_fqav(a: np.ndarray, n: int, f: str = "sum") -> np.ndarray:
    """fqav(A, n; f) (src/gbtworkerfunctions.jl:16-20) on the first axis."""
    if n <= 1:  # :17 — returns A itself
        return a
    if a.shape[0] % n:  # :18 reshape -> DimensionMismatch
        raise DimensionMismatch(f"fqavby={n} does not divide {a.shape[0]}")
    R = a.reshape((n, a.shape[0] // n) + a.shape[1:], order="F")  # :18 (column-major)
    if f in ("sum", "mean"):  # :19 f(...; dims=1), Float64 accumulation here
        s = R.astype(np.float64).sum(axis=0)
        if f == "mean":
            s = s / n
        return np.asfortranarray((s + 0.0).astype(np.float32))
    m = R.max(axis=0) if f == "max" else R.min(axis=0)
    return np.asfortranarray(_fix_zero(m, R, 0, f))


def np_tavby(a: np.ndarray, n: int, f: str = "sum") -> np.ndarray:
    """Time integration: fqav applied to axis 3,
    permutedims(fqav(permutedims(A, (3,2,1)), n), (3,2,1))."""
    if n <= 1:
        return a
    return np.asfortranarray(np.transpose(np_fqav(np.transpose(a, (2, 1, 0)), n, f), (2, 1, 0)))


def np_reduce(a, fqavby=1, tavby=1, op="sum", win=None) -> np.ndarray:
    """Channel decimation then time integration, float64 throughout for
    sum/mean (the composition is computed in float64 before rounding)."""
    w = np_window(np.asarray(a, dtype=np.float32), win)
    if op in ("sum", "mean"):
        w64 = w.astype(np.float64)
        F, T = max(int(fqavby), 1), max(int(tavby), 1)
        if w64.shape[0] % F or w64.shape[2] % T:
            raise DimensionMismatch("factor does not divide window")
        R = w64.reshape((F, w64.shape[0] // F, w64.shape[1], T, w64.shape[2] // T), order="F")
        s = R.sum(axis=(0, 3))
        if op == "mean":
            s = s / (F * T)
        return np.asfortranarray((s + 0.0).astype(np.float32))
    return np_tavby(np_fqav(w, int(fqavby), op), int(tavby), op)


def np_pairwise_sum(rows: np.ndarray) -> np.ndarray:
    """Base.sum of each Float32 row (Base.mapreduce_impl, pairwise_blocksize
    1024): pieces of <= 1024 elements summed sequentially from their first
    element (np.add.accumulate is a sequential loop), halves split at
    ifirst + (ilast - ifirst) >> 1 and added back up the tree in Float32."""
    rows = np.asarray(rows, dtype=np.float32)

    def rec(lo, hi):  # inclusive, 0-based
        if hi - lo < 1024:
            return np.add.accumulate(rows[:, lo:hi + 1], axis=1, dtype=np.float32)[:, -1]
        mid = lo + ((hi - lo) >> 1)
        return (rec(lo, mid) + rec(mid + 1, hi)).astype(np.float32)

    if rows.shape[1] == 0:
        return np.full(rows.shape[0], np.nan, dtype=np.float32)
    return rec(0, rows.shape[1] - 1)


def np_kurtosis(a, win=None) -> np.ndarray:
    """getkurtosis (src/gbtworkerfunctions.jl:197-202), StatsBase recipe:
    m = mean(v) (Float32 pairwise sum / length), z and z2 in Float32,
    Float64 cm2 and cm4."""
    w = np_window(np.asarray(a, dtype=np.float32), win)
    nc, ni, nt = w.shape
    rows = w.reshape((nc * ni, nt), order="F")  # :199-200
    with np.errstate(invalid="ignore", over="ignore"):
        m = (np_pairwise_sum(rows) / np.float32(nt))[:, None]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        z = (rows - m).astype(np.float32)
        z2 = (z * z).astype(np.float32)
        cm2 = z2.astype(np.float64).sum(axis=1) / nt
        cm4 = (z2 * z2).astype(np.float64).sum(axis=1) / nt
        k = cm4 / (cm2 * cm2) - 3.0
    return np.asfortranarray(k.reshape((nc, ni), order="F"))  # :201


# --------------------------------------------------------------------------
# Element types other than Float32 (NumPy restatement; the C oracle covers the
# Float32 path).  Julia's result types (Base.add_sum widening, Statistics.mean,
# StatsBase.kurtosis in Float64) — see csrc/typed.hip.
# --------------------------------------------------------------------------
def jl_sum_type(dt) -> np.dtype:
    """Base.add_sum's result type: small unsigned -> UInt64, small signed ->
    Int64, everything else unchanged."""
    dt = np.dtype(dt)
    if dt.kind == "u":
        return np.dtype(np.uint64)
    if dt.kind == "i":
        return np.dtype(np.int64)
    return dt


def np_jl_sum_f64(x: np.ndarray, axis: int = 0) -> np.ndarray:
    """sum(x; dims=axis) of Float64 values as Julia's reducedim takes it:
    R = zero(Float64), then R + Base.mapreduce_impl over the axis (pairwise
    halves at ifirst + (ilast - ifirst) >> 1 down to pieces of <= 1024 summed in
    sequence from their first element; Base/reducedim.jl `_mapreducedim!`,
    Base/reduce.jl `mapreduce_impl`).  Axes of <= 16 take the other branch of
    `_mapreducedim!` (r = zero; r += A[i] in sequence), which gives the same
    value: 0.0 + a1 = a1 for every a1 but -0.0, and the final 0.0 + v below
    settles that case the same way."""
    x = np.moveaxis(np.asarray(x, dtype=np.float64), axis, -1)
    shape = x.shape[:-1]
    rows = x.reshape((-1, x.shape[-1]))
    s = np_pairwise_sum_f64(rows) if rows.shape[0] else np.zeros(0)
    return 0.0 + s.reshape(shape)


def np_reduce_typed(a, fqavby=1, tavby=1, op="sum", win=None) -> np.ndarray:
    """fqav (src/gbtworkerfunctions.jl:16-20) fused with the time integration
    for a non-Float32 array, with Julia's result element types: integer sums
    exact in (U)Int64 (wrapping); Float64 sums, and every mean, in the
    reference's order: each spectrum's F channels summed as Julia's
    sum(reshape(A, (F, :, ...)); dims=1) sums them (np_jl_sum_f64: pairwise
    above 1024), then the T spectral sums of a time block the same way (the
    time integration is fqav on axis 3); mean = that Float64
    sum of the values converted to Float64 (Statistics.mean's
    `_mean_promote`) / (F T); max / min in the input type."""
    w = np_window(np.asarray(a), win)
    F, T = max(int(fqavby), 1), max(int(tavby), 1)
    nc, ni, nt = w.shape
    if nc % F or nt % T:
        raise DimensionMismatch("factor does not divide window")
    # (F, co, ni, T, to): channel group on axis 0, time block on axis 3
    B = w.reshape((F, nc // F, ni, T, nt // T), order="F")
    if op in ("max", "min"):
        R = B.transpose(0, 3, 1, 2, 4).reshape((F * T, nc // F, ni, nt // T), order="F")
        if R.shape[0] == 0 or R.size == 0:
            return np.asfortranarray(np.empty(R.shape[1:], dtype=w.dtype))
        m = R.max(axis=0) if op == "max" else R.min(axis=0)
        if w.dtype.kind == "f":
            m = _fix_zero(m, R, 0, op)
        return np.asfortranarray(m.astype(w.dtype))
    st = jl_sum_type(w.dtype)
    if st.kind == "f" or op == "mean":
        with np.errstate(over="ignore", invalid="ignore"):
            spec = np_jl_sum_f64(B, axis=0)           # (co, ni, T, to)
            s = np_jl_sum_f64(spec, axis=2)           # (co, ni, to)
        if op == "mean":
            return np.asfortranarray(s / float(F * T))
        return np.asfortranarray(s)
    # exact, wrapping modulo 2^64 like Julia's (U)Int64
    R = B.reshape((F, nc // F, ni, T, nt // T), order="F").astype(st)
    s = R.sum(axis=(0, 3), dtype=st)
    return np.asfortranarray(s.astype(st))


def np_pairwise_sum_f64(rows: np.ndarray) -> np.ndarray:
    """Base.sum of each row converted to Float64 (mapreduce_impl, blocks of
    <= 1024 summed in sequence, halves at ifirst + (ilast - ifirst) >> 1)."""
    rows = np.asarray(rows, dtype=np.float64)

    def rec(lo, hi):
        if hi - lo < 1024:
            return np.add.accumulate(rows[:, lo:hi + 1], axis=1)[:, -1]
        mid = lo + ((hi - lo) >> 1)
        return rec(lo, mid) + rec(mid + 1, hi)

    if rows.shape[1] == 0:
        return np.zeros(rows.shape[0])
    return rec(0, rows.shape[1] - 1)


def np_kurtosis_typed(a, win=None) -> np.ndarray:
    """getkurtosis (src/gbtworkerfunctions.jl:197-202) of an integer or
    Float64 array: StatsBase.kurtosis(v) = kurtosis(v, mean(v)) entirely in
    Float64 — m = Base.sum (pairwise) / n, then z = v[i] - m, z2 = z*z,
    cm2 += z2, cm4 += z2*z2 in sequence, (cm4/n) / (cm2/n)^2 - 3."""
    w = np_window(np.asarray(a), win)
    nc, ni, nt = w.shape
    rows = w.reshape((nc * ni, nt), order="F").astype(np.float64)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore", under="ignore"):
        m = (np_pairwise_sum_f64(rows) / float(nt))[:, None]
        z = rows - m
        z2 = z * z
        if nt:
            cm2 = np.add.accumulate(z2, axis=1)[:, -1] / float(nt)
            cm4 = np.add.accumulate(z2 * z2, axis=1)[:, -1] / float(nt)
        else:
            cm2 = cm4 = np.full(nc * ni, np.nan)
        k = cm4 / (cm2 * cm2) - 3.0
    return np.asfortranarray(k.reshape((nc, ni), order="F"))


def np_stitch(banks) -> np.ndarray:
    """reduce(vcat, banks) (src/gbt.jl:103)."""
    return np.asfortranarray(np.concatenate([np.asarray(b) for b in banks], axis=0))


def np_despike(d, nfpc) -> np.ndarray:
    """d[spike:nfpc:end,:,:] .= d[spike-1:nfpc:end,:,:] (src/gbt.jl:101-102,111)."""
    d = np.array(d, dtype=np.float32, order="F", copy=True)
    spike = nfpc // 2 + 1
    if spike - 1 < 1:
        raise BoundsErr("spike-1 == 0")
    dst = np.arange(spike - 1, d.shape[0], nfpc)
    src = np.arange(spike - 2, d.shape[0], nfpc)
    if len(dst) != len(src):
        raise DimensionMismatch("spike/source lengths differ")
    d[dst] = d[src]
    return d


def np_fqav_range(first, step, length, n):
    """fqav(r::AbstractRange, n) (src/gbtworkerfunctions.jl:27-33)."""
    if n <= 1:
        return float(first), float(step), int(length)
    return first + (n - 1) * step / 2, float(n * step), length // n


def gamma_bandpass(nchan, nif, ntime, nfpc, seed):
    """NumPy synthetic BL-like power: gamma(2, 5e8) x per-coarse-channel
    scallop x DC spike at bin nfpc/2."""
    rng = np.random.default_rng(seed)
    g = rng.gamma(2.0, 5e8, size=(ntime, nif, nchan)).astype(np.float32)
    x = np.arange(nchan) % nfpc
    bp = (0.2 + 0.8 * np.sin(np.pi * (x + 0.5) / nfpc) ** 2).astype(np.float32)
    bp[x == nfpc // 2] *= 10.0
    return np.asfortranarray(np.transpose(g * bp, (2, 1, 0)))


# --------------------------------------------------------------------------
# HDF5 filter 32008 test encoder (bitshuffle + literal-only LZ4)
# --------------------------------------------------------------------------
def np_bitshuffle(a: np.ndarray) -> np.ndarray:
    """bitshuffle's bit transpose of one block (n % 8 == 0): bit plane
    r = (byte r//8, bit r%8) of every element, packed LSB-first."""
    b = np.frombuffer(np.ascontiguousarray(a).tobytes(), np.uint8).reshape(a.size, a.itemsize)
    bits = np.unpackbits(b, axis=1, bitorder="little")
    return np.packbits(bits.T, axis=1, bitorder="little").ravel()


def lz4_literals(data: bytes) -> bytes:
    """A valid LZ4 block holding `data` as one literal run (no matches)."""
    n = len(data)
    out = bytearray([min(n, 15) << 4])
    if n >= 15:
        r = n - 15
        while r >= 255:
            out.append(255)
            r -= 255
        out.append(r)
    return bytes(out) + data


def _lz4_len(out: bytearray, r: int) -> None:
    while r >= 255:
        out.append(255)
        r -= 255
    out.append(r)


def lz4_compress(src: bytes) -> bytes:
    """A greedy LZ4 block compressor (public LZ4 block format: token, literal
    length extension, literals, 16-bit little-endian offset, match length
    extension), for test data with real matches -- overlapping ones
    (offset < length) included.  Follows the format's end-of-block rules:
    the last 5 bytes are literals and no match starts within the last 12."""
    n = len(src)
    out = bytearray()
    table: dict = {}
    i = anchor = 0

    def emit(lit: bytes, off: int = 0, mlen: int = 0) -> None:
        ll = len(lit)
        ml = mlen - 4 if off else 0
        out.append((min(ll, 15) << 4) | (min(ml, 15) if off else 0))
        if ll >= 15:
            _lz4_len(out, ll - 15)
        out.extend(lit)
        if off:
            out.extend(off.to_bytes(2, "little"))
            if ml >= 15:
                _lz4_len(out, ml - 15)

    while i + 12 <= n:
        key = src[i:i + 4]
        cand = table.get(key)
        table[key] = i
        if cand is not None and i - cand <= 65535:
            m = 4
            while i + m < n - 5 and src[cand + m] == src[i + m]:
                m += 1
            emit(src[anchor:i], i - cand, m)
            i += m
            anchor = i
        else:
            i += 1
    emit(src[anchor:])
    return bytes(out)


def np_bslz4_encode(a: np.ndarray, block: int = 2048, lz4=None) -> bytes:
    """An HDF5-filter-32008 chunk (bitshuffle + LZ4) of `a`; LZ4 literal-only
    unless ``lz4`` (e.g. lz4_compress) is given."""
    import struct

    flat = np.ascontiguousarray(a, dtype=np.float32).ravel()
    n, es = flat.size, 4
    parts = [struct.pack(">QI", n * es, block * es)]
    nfull = n // block
    last = n % block
    last -= last % 8
    sizes = [block] * nfull + ([last] if last else [])
    pos = 0
    for sz in sizes:
        z = (lz4 or lz4_literals)(np_bitshuffle(flat[pos:pos + sz]).tobytes())
        parts.append(struct.pack(">I", len(z)) + z)
        pos += sz
    parts.append(flat[pos:].tobytes())
    return b"".join(parts)
