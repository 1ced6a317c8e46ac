"""GPU parity for element types other than Float32 (VERDICT r02 missing #2):
fqav and getkurtosis return the reference's result types — Base.add_sum
widening (UInt8/16/32 -> UInt64, Int8/16/32 -> Int64), Float64 means, max /
min in the input type, StatsBase.kurtosis in Float64
(src/gbtworkerfunctions.jl:16-20, 173-174, 188, 197-202) — and the values of
the NumPy restatement (oracle.np_reduce_typed / np_kurtosis_typed), through
the C ABI (bldp_reduce_strided, bldp_kurtosis, bldp_reduce_host,
bldp_kurtosis_host).

Tolerances: integer results are exact; Float64 sums follow the reference's
sequence (the F channels of a spectrum, spectrum after spectrum) and
kurtosis follows StatsBase's (Base.sum's pairwise mean, sequential moments),
so they are compared bit for bit as well (the oracle runs the same
sequence).  The reference itself may reassociate inside a 1024-element leaf
under @simd; that machine dependence is not something either restatement
pins."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import KURT_INT_FINISH, assert_kurtosis

pytestmark = pytest.mark.gpu

INT_TYPES = [np.uint8, np.uint16, np.uint32, np.uint64, np.int8, np.int16, np.int32, np.int64]
ALL_TYPES = INT_TYPES + [np.float64]


@pytest.fixture(scope="module")
def eng(pkg):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    pkg._lib.lib()
    return pkg.engine


def rand(dt, shape, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dt)
    if dt.kind == "f":
        return np.asfortranarray(rng.gamma(2.0, 3.0, shape).astype(dt))
    info = np.iinfo(dt)
    lo, hi = max(info.min, -(1 << 40)), min(info.max, 1 << 40)
    return np.asfortranarray(rng.integers(lo, hi, shape, endpoint=True).astype(dt))


def to_dev(eng, a):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 1, 0))).to("cuda")
    return t.permute(2, 1, 0)


def same(got, want):
    got, want = np.asarray(got), np.asarray(want)
    assert got.dtype == want.dtype, (got.dtype, want.dtype)
    assert got.shape == want.shape, (got.shape, want.shape)
    if got.dtype.kind == "f":
        return np.array_equal(got.view(np.uint64), want.view(np.uint64)) or \
            np.array_equal(got, want, equal_nan=True)
    return np.array_equal(got, want)


def kurt_same(got, want, dt, nt, msg=""):
    """Typed getkurtosis against the recipe: 8- and 16-bit rows take
    k_kurt_i8 / k_kurt_i16 (exact integer moments), within
    conftest.kurt_int_tol(nt) of it; every other type follows the recipe's
    sequence, bit for bit."""
    if np.dtype(dt).itemsize <= 2:
        assert np.asarray(got).dtype == np.asarray(want).dtype
        assert_kurtosis(got, want, "int", nt, msg)
    else:
        assert same(got, want), msg


def exact_kurtosis(a):
    """The exact excess kurtosis of every (channel, IF) row of an 8- or
    16-bit array, rounded once: power sums of d = x - centre (|d| <= 2^15),
    exact (d^2 = a 2^15 + b split so every Int64 sum stays below 2^63, the
    parts joined as Python integers), then X / Y^2 - 3 with Y = n S2 - S1^2,
    X = n^3 S4 - 4 n^2 S1 S3 + 6 n S1^2 S2 - 3 S1^4 (typed.hip k_kurt_i8 /
    k_kurt_i16; the kurtosis does not depend on the centre)."""
    from fractions import Fraction

    info = np.iinfo(a.dtype)
    d = a.astype(np.int64) - (info.min + info.max + 1) // 2
    n = a.shape[2]
    q = d * d
    hi, lo = q >> 15, q & 0x7FFF
    S1, S2 = d.sum(axis=2), q.sum(axis=2)
    S3h, S3l = (hi * d).sum(axis=2), (lo * d).sum(axis=2)
    S4a, S4b, S4c = (hi * hi).sum(axis=2), (2 * hi * lo).sum(axis=2), (lo * lo).sum(axis=2)
    out = np.empty(a.shape[:2])
    for idx in np.ndindex(*a.shape[:2]):
        s1, s2 = int(S1[idx]), int(S2[idx])
        s3 = (int(S3h[idx]) << 15) + int(S3l[idx])
        s4 = (int(S4a[idx]) << 30) + (int(S4b[idx]) << 15) + int(S4c[idx])
        y = n * s2 - s1 * s1
        x = n ** 3 * s4 - 4 * n * n * s1 * s3 + 6 * n * s1 * s1 * s2 - 3 * s1 ** 4
        out[idx] = np.nan if y == 0 else float(Fraction(x, y * y) - 3)
    return out


JULIA_OUT = {("sum", np.uint8): np.uint64, ("sum", np.uint16): np.uint64,
             ("sum", np.uint32): np.uint64, ("sum", np.uint64): np.uint64,
             ("sum", np.int8): np.int64, ("sum", np.int16): np.int64,
             ("sum", np.int32): np.int64, ("sum", np.int64): np.int64,
             ("sum", np.float64): np.float64}


@pytest.mark.parametrize("dt", ALL_TYPES, ids=lambda d: np.dtype(d).name)
def test_result_types_are_julias(pkg, eng, dt):
    for op in ("sum", "mean", "max", "min"):
        want = JULIA_OUT[("sum", dt)] if op == "sum" else np.float64 if op == "mean" else dt
        assert eng.out_dtype(np.dtype(dt), op) == np.dtype(want), (dt, op)
    assert eng.out_dtype(np.dtype(np.float32), "sum") == np.float32
    assert eng.out_dtype(np.dtype(np.float32), "mean") == np.float32


SHAPES = [(64, 1, 20, 4, 1), (96, 2, 12, 3, 4), (1000, 1, 7, 8, 1), (33, 3, 5, 1, 5),
          (4096, 1, 3, 64, 1)]


@pytest.mark.parametrize("dt", ALL_TYPES, ids=lambda d: np.dtype(d).name)
def test_reduce_typed_device_and_host(pkg, eng, orc, dt):
    for k, (nc, ni, nt, F, T) in enumerate(SHAPES):
        a = rand(dt, (nc, ni, nt), seed=k + 17 * np.dtype(dt).num)
        x = to_dev(eng, a)
        for op in ("sum", "mean", "max", "min"):
            want = orc.np_reduce_typed(a, F, T, op)
            got = eng.fb_to_numpy(eng.reduce(x, F, T, op))
            assert same(got, want), (dt, (nc, ni, nt, F, T), op)
            goth = eng.reduce_host_typed(a, F, T, op)
            assert same(goth, want), (dt, (nc, ni, nt, F, T), op, "host")
        # a strided window (reversed channels, every other spectrum)
        if nt >= 2 * T and nc >= 2 * F:
            w = [nc - 1, (nc // F) * F - F, -1, 0, ni, 1, 0, (nt // (2 * T)) * T, 2]
            for op in ("sum", "max"):
                want = orc.np_reduce_typed(a, F, T, op, w)
                assert same(eng.fb_to_numpy(eng.reduce(x, F, T, op, w)), want), (dt, op, w)
                assert same(eng.reduce_host_typed(a, F, T, op, w), want), (dt, op, w, "host")


@pytest.mark.parametrize("F,T", [(2048, 1), (4096, 2), (1500, 3), (8, 1100)])
def test_reduce_float64_wide_groups_pairwise(pkg, eng, orc, F, T):
    """Float64 sums (and integer means) of groups or time blocks longer than
    1024 take Base.mapreduce_impl's pairwise halves (src/gbtworkerfunctions.jl:19),
    bit for bit against the restatement pinned to Julia's loop
    (tests/test_oracle.py::test_typed_float64_sum_order_pinned)."""
    rng = np.random.default_rng(F + T)
    nc, nt = 3 * F, 2 * T
    b = np.asfortranarray(rng.standard_normal((nc, 1, nt)) * 1e8 + rng.standard_normal((nc, 1, nt)))
    x = to_dev(eng, b)
    for op in ("sum", "mean"):
        want = orc.np_reduce_typed(b, F, T, op)
        assert same(eng.fb_to_numpy(eng.reduce(x, F, T, op)), want), (F, T, op)
        assert same(eng.reduce_host_typed(b, F, T, op), want), (F, T, op, "host")
    big = np.asfortranarray(rng.integers(2**60, 2**62, (nc, 1, nt), dtype=np.int64))
    want = orc.np_reduce_typed(big, F, T, "mean")
    assert same(eng.fb_to_numpy(eng.reduce(to_dev(eng, big), F, T, "mean")), want), (F, T)
    # a strided window: every other channel, reversed time
    w = [0, F, 2, 0, 1, 1, nt - 1, T, -1]
    assert same(eng.fb_to_numpy(eng.reduce(x, F, T, "sum", w)),
                orc.np_reduce_typed(b, F, T, "sum", w)), (F, T, w)


def test_f32_entry_points_reject_other_types(pkg, eng):
    """Only reduce / kurtosis branch to the typed kernels; the Float32-only
    entry points refuse other element types instead of reading them as
    Float32."""
    import torch

    u = torch.zeros((256, 1, 8), dtype=torch.uint8, device="cuda")
    x = u.permute(2, 1, 0).contiguous().permute(2, 1, 0)
    for fn in (lambda: eng.band_reduce([x], 4, 1), lambda: eng.despike(x, 64),
               lambda: eng.band_kurtosis([x]), lambda: eng.plan(x, 4, 1),
               lambda: eng.kurtosis_plan(x)):
        with pytest.raises(TypeError):
            fn()
    f = eng.fb_empty(256, 1, 8)
    with pytest.raises(TypeError):
        eng.band_reduce([f], 4, 1, out=eng.fb_empty(64, 1, 8, dtype=torch.float64))


def test_reduce_typed_wraps_like_julia(pkg, eng, orc):
    """(U)Int64 sums wrap modulo 2^64, as Julia's do."""
    a = np.asfortranarray(np.full((8, 1, 2), np.iinfo(np.uint64).max, dtype=np.uint64))
    got = eng.reduce_host_typed(a, 4, 1, "sum")
    assert same(got, orc.np_reduce_typed(a, 4, 1, "sum"))
    assert got[0, 0, 0] == np.uint64(2**64 - 4)


@pytest.mark.parametrize("dt", ALL_TYPES, ids=lambda d: np.dtype(d).name)
def test_kurtosis_typed(pkg, eng, orc, dt):
    for k, (nc, ni, nt) in enumerate([(64, 1, 100), (37, 2, 1500), (5, 1, 5000), (3, 1, 1)]):
        a = rand(dt, (nc, ni, nt), seed=5 * k + np.dtype(dt).num)
        if np.dtype(dt).kind != "f":  # keep the Float64 mean's sums exact (< 2^53)
            a = np.asfortranarray((a.astype(np.int64) % 1000).astype(dt))
        want = orc.np_kurtosis_typed(a)
        got = eng.fb_to_numpy(eng.kurtosis(to_dev(eng, a)))
        kurt_same(got, want, dt, nt, (dt, (nc, ni, nt)))
        kurt_same(eng.kurtosis_host_typed(a), want, dt, nt, (dt, (nc, ni, nt), "host"))
    # windows: a spectrum range of every other channel; an empty time window -> NaN
    a = rand(dt, (40, 1, 300), seed=3)
    w = [1, 19, 2, 0, 1, 1, 10, 250, 1]
    kurt_same(eng.kurtosis_host_typed(a, w), orc.np_kurtosis_typed(a, w), dt, 250)
    e = eng.kurtosis_host_typed(a, [0, 40, 1, 0, 1, 1, 0, 0, 1])
    assert e.shape == (40, 1) and np.isnan(e).all()


@pytest.mark.parametrize("dt", [np.uint8, np.int8, np.uint16, np.int16],
                         ids=lambda d: np.dtype(d).name)
def test_kurtosis_typed_words(pkg, eng, orc, dt):
    """8- and 16-bit getkurtosis with a lane on each 32-bit word of 4 / 2
    channels (k_kurt_typed_w, the recipe's order; for 8-bit rows with plan
    option typed_kurt = 0): bit-identical to the one-lane-per-channel kernel
    (plan option typed_vec = 0) and to the oracle; the type's full range,
    spectrum counts around the 16-spectrum batches, two IFs, a channel window
    on a word boundary and one off it (the fallback).  By default these rows
    take k_kurt_i8 / k_kurt_i16, held to kurt_int_tol."""
    info = np.iinfo(dt)
    for k, (nc, ni, nt) in enumerate([(256, 2, 1000), (1024, 1, 77), (64, 1, 16), (128, 3, 15)]):
        rng = np.random.default_rng(k + np.dtype(dt).num)
        a = np.asfortranarray(rng.integers(info.min, info.max, (nc, ni, nt), endpoint=True)
                              .astype(dt))
        x = to_dev(eng, a)
        want = orc.np_kurtosis_typed(a)
        got = eng.fb_to_numpy(eng.kurtosis(x))
        kurt_same(got, want, dt, nt, (dt, (nc, ni, nt)))
        with pkg._lib.plan_option("typed_kurt", 0):
            rec = eng.fb_to_numpy(eng.kurtosis(x))
            assert same(rec, want), (dt, (nc, ni, nt))
            with pkg._lib.plan_option("typed_vec", 0):
                assert same(eng.fb_to_numpy(eng.kurtosis(x)), rec), (dt, (nc, ni, nt))
        for w in ([4, nc - 8, 1, 0, ni, 1, 3, nt - 3, 1], [1, nc - 4, 1, 0, ni, 1, 0, nt, 1]):
            kurt_same(eng.fb_to_numpy(eng.kurtosis(x, w)), orc.np_kurtosis_typed(a, w), dt,
                      w[7], (dt, (nc, ni, nt), w))


@pytest.mark.parametrize("dt", [np.uint8, np.int8, np.uint16, np.int16],
                         ids=lambda d: np.dtype(d).name)
def test_kurtosis_int_exact_moments(pkg, eng, orc, dt):
    """k_kurt_i8 / k_kurt_i16 (8- and 16-bit getkurtosis from exact integer
    power sums, time split over waves and, for long rows, over workgroups
    whose sums a second kernel adds): within conftest.KURT_INT_FINISH (relative on k + 3) of the exactly
    rounded kurtosis (Python integers), and within kurt_int_tol(nt) of the
    recipe (oracle); 4- and 8-byte words a lane (plan option typed_kurt 2 / 3)
    bit-identical.  The 0002 file geometry, one and several time chunks
    (the 0001 shape: few channels, long rows), the type's extremes (rows of
    only min / max: NaN as the recipe; two values), two IFs and a window."""
    info = np.iinfo(dt)
    rng = np.random.default_rng(99 + np.dtype(dt).num)
    for nc, ni, nt in ((65536, 1, 279), (512, 1, 200000), (256, 2, 4099), (8, 1, 17),
                       (64, 2, 1), (64, 1, 2), (16, 1, 4)):  # (1 spectrum: NaN, as the recipe)
        a = np.asfortranarray(rng.integers(info.min, info.max, (nc, ni, nt), endpoint=True)
                              .astype(dt))
        a[0, 0, :] = info.max  # constant rows: NaN
        a[1, 0, :] = info.min
        a[2, 0, :] = np.where(np.arange(nt) % 3 == 0, info.min, info.max)  # two values
        a[3, 0, :nt // 2] = info.min  # a long run then noise
        if nt == 1:
            assert np.isnan(orc.np_kurtosis_typed(a)).all()
        x = to_dev(eng, a)
        got = eng.fb_to_numpy(eng.kurtosis(x))
        for form in (2, 3):  # 4- and 8-byte words a lane: the same exact sums, the same bits
            with pkg._lib.plan_option("typed_kurt", form):
                assert same(eng.fb_to_numpy(eng.kurtosis(x)), got), (dt, nc, nt, form)
        csub = max(8, min(nc, 1024, 4_000_000 // (nt * ni)))  # (rows the exact check takes)
        sub = (slice(0, csub), slice(None))
        ex = exact_kurtosis(a[sub[0]])
        assert_kurtosis(got[sub], ex, "int", 1, (dt, nc, nt, "exact"))
        fin = np.isfinite(ex)
        err = np.abs(got[sub][fin] - ex[fin]) / np.abs(ex[fin] + 3)
        assert np.all(err <= KURT_INT_FINISH), (dt, nc, nt, float(err.max()) * 2 ** 53)
        if nc * ni * nt <= 5e6:
            assert_kurtosis(got, orc.np_kurtosis_typed(a), "int", nt, (dt, nc, nt))
    a = np.asfortranarray(rng.integers(info.min, info.max, (1000, 1, 300), endpoint=True)
                          .astype(dt))
    w = [8, 960, 1, 0, 1, 1, 5, 290, 1]  # word-aligned channel span, a time window
    got = eng.fb_to_numpy(eng.kurtosis(to_dev(eng, a), w))
    assert_kurtosis(got, orc.np_kurtosis_typed(a, w), "int", 290, (dt, "window"))
    with pkg._lib.plan_option("typed_kurt", 3):  # (8-byte aligned rows: 8-byte words)
        assert same(eng.fb_to_numpy(eng.kurtosis(to_dev(eng, a), w)), got), (dt, "window")


def test_worker_api_keeps_reference_types(pkg, eng, orc, tmp_path):
    """getdata / getkurtosis / fqav on 8- and 16-bit SIGPROC files and on a
    Float64 array: Julia's result types and values (no Float32 detour)."""
    W = pkg.WorkerFunctions
    rng = np.random.default_rng(8)
    for nbits, dt in ((8, np.uint8), (16, np.uint16)):
        a = np.asfortranarray(rng.integers(0, np.iinfo(dt).max, (256, 2, 50), endpoint=True)
                              .astype(dt))
        f = str(tmp_path / f"b{nbits}.fil")
        pkg.readers.write_fil(f, dict(fch1=8000.0, foff=-1.0, nchans=256, nifs=2, tsamp=1.0,
                                      nbits=nbits, telescope_id=6, machine_id=10, data_type=1,
                                      tstart=59000.0, source_name="X"), a)
        d = W.getdata(f)  # fqavby = 1: the data itself (fqav returns A, :17)
        assert d.dtype == dt and np.array_equal(d, a)
        for op in ("sum", "mean", "max", "min"):
            got = W.getdata(f, fqavby=16, fqavfunc=op)
            assert same(got, orc.np_reduce_typed(a, 16, 1, op)), (nbits, op)
        idxs = (pkg.JRange(1, 128), 2, pkg.JRange(5, 44))
        got = W.getdata(f, idxs, fqavby=8, tavby=4)
        w = [0, 128, 1, 1, 1, 1, 4, 40, 1]
        assert same(got, orc.np_reduce_typed(a, 8, 4, "sum", w))
        k = W.getkurtosis(f)
        kurt_same(k, orc.np_kurtosis_typed(a), dt, 50, nbits)
    b = np.asfortranarray(rng.standard_normal((512, 1, 30)))
    assert same(W.fqav(b, 8), orc.np_reduce_typed(b, 8, 1, "sum"))
    assert same(W.fqav(b, 8, "mean"), orc.np_reduce_typed(b, 8, 1, "mean"))
    assert W.fqav(b.astype(np.int16), 4).dtype == np.int64
    with pytest.raises(TypeError):
        W.fqav(b.astype(np.float16), 4)


@pytest.mark.parametrize("dt", ALL_TYPES, ids=lambda d: np.dtype(d).name)
def test_typed_vec_kernel_matches_oracle(pkg, eng, orc, dt):
    """The coalesced typed kernels (16-byte row loads, groups folded over
    lanes; blocks of <= 16 rows loaded in one batch: integer sums, max / min of every type, means of <= 32-bit
    integers) against the restatement, and bit-identical to the
    one-lane-per-group kernel (plan option typed_vec = 0): the SIGPROC 8-bit
    0002 geometry at fqavby 64, windows, several IFs, extremes of the type."""
    rng = np.random.default_rng(np.dtype(dt).num)
    sz = np.dtype(dt).itemsize
    shapes = [(65536, 1, 40, 64, 1), (4096, 2, 24, 16 // sz * 4, 3), (2048, 1, 17, 1024 // sz, 17),
              (768, 3, 10, 48, 2), (16384, 1, 9, 4096 // sz, 1),
              # short power-of-two blocks in one batch of <= 16 rows
              # (k_reduce_typed_vec16), a partial last batch of blocks
              (4096, 1, 68, 64, 4), (2048, 2, 40, 32, 8), (8192, 1, 48, 64, 16),
              (1024, 1, 300, 16, 1)]
    for nc, ni, nt, F, T in shapes:
        if nc % F:
            continue
        a = rand(dt, (nc, ni, nt), seed=nc + F)
        if np.dtype(dt).kind != "f":  # the type's extremes too
            info = np.iinfo(dt)
            a[0, 0, 0], a[1, 0, 0] = info.min, info.max
        else:
            a[0, 0, 0], a[3, 0, 0], a[5, 0, min(1, nt - 1)] = np.nan, -np.inf, -0.0
        x = to_dev(eng, a)
        for op in ("sum", "mean", "max", "min"):
            want = orc.np_reduce_typed(a, F, T, op)
            got = eng.fb_to_numpy(eng.reduce(x, F, T, op))
            assert same(got, want), (dt, (nc, ni, nt, F, T), op)
            with pkg._lib.plan_option("typed_vec", 0):
                assert same(eng.fb_to_numpy(eng.reduce(x, F, T, op)), got), (dt, op, "typed_vec 0")
        # a window: channels from group 2 on, spectra 2.. (a misaligned row start)
        w = [2 * F, nc - 2 * F, 1, 0, ni, 1, 1, (nt - 1) // T * T, 1]
        for op in ("sum", "max"):
            want = orc.np_reduce_typed(a, F, T, op, w)
            assert same(eng.fb_to_numpy(eng.reduce(x, F, T, op, w)), want), (dt, op, w)


@pytest.mark.parametrize("dt", ALL_TYPES + [np.float32], ids=lambda d: np.dtype(d).name)
def test_prepared_reduce_and_kurtosis(pkg, eng, dt):
    """bldp_reduce_prepare / bldp_kurtosis_prepare (ABI 5, any element type):
    each launch gives the unprepared call's result bit for bit, re-launches
    on new data in the same buffers see the new data, and the timed launch
    form records its events (the per-file call at one
    ctypes call and the kernel launch)."""
    import torch

    def same(got, want):  # (every element type here: bits, NaN = NaN)
        got, want = np.asarray(got), np.asarray(want)
        return got.dtype == want.dtype and got.shape == want.shape and \
            np.array_equal(got, want, equal_nan=got.dtype.kind == "f")

    for nc, ni, nt, F, T, win in ((4096, 1, 279, 64, 1, None), (1000, 2, 40, 8, 4, None),
                                  (512, 1, 70, 4, 7, [8, 480, 1, 0, 1, 1, 0, 70, 1]),
                                  (512, 1, 20000, 8, 16, None)):  # (long rows: time chunks)
        a = rand(dt, (nc, ni, nt), seed=nc + nt)
        x = to_dev(eng, a)
        for op in ("sum", "max"):
            pr = eng.PreparedReduce(x, F, T, op, win)
            pr.launch()
            assert same(eng.fb_to_numpy(pr.out), eng.fb_to_numpy(eng.reduce(x, F, T, op, win)))
            x.copy_(to_dev(eng, rand(dt, (nc, ni, nt), seed=nc + nt + 1)))
            e0, e1 = pkg._lib.HipEvent(timing=True), pkg._lib.HipEvent(timing=True)
            pr.launch_timed(None, e0, e1)
            torch.cuda.synchronize()
            assert e0.elapsed_time(e1) >= 0.0
            assert same(eng.fb_to_numpy(pr.out), eng.fb_to_numpy(eng.reduce(x, F, T, op, win)))
            pr.close()
        pk = eng.PreparedKurtosis(x, win)
        pk.launch()
        torch.cuda.synchronize()
        assert same(eng.fb_to_numpy(pk.out), eng.fb_to_numpy(eng.kurtosis(x, win)))
        pk.close()
    with pytest.raises(pkg.DimensionMismatch):
        eng.PreparedReduce(to_dev(eng, rand(dt, (100, 1, 8), seed=1)), 3, 1)
