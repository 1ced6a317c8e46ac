"""CPU: pin the oracle.  The reference's own KATs (test/runtests.jl:5-6), the
committed golden fixtures, and agreement of the C and NumPy restatements."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import KURT_LEAF_TOL, same_bits


def test_reference_range_kats(orc, golden):
    # GBT.fqav(1:4, 4) === 2.5:4.0:2.5 ; GBT.fqav(1:2:15, 4) === 4.0:8.0:12.0
    assert orc.fqav_range(1, 1, 4, 4) == (2.5, 4.0, 1)
    assert orc.fqav_range(1, 2, 8, 4) == (4.0, 8.0, 2)
    for k in golden.manifest["kat_range"]:
        assert list(orc.fqav_range(k["first"], k["step"], k["length"], k["n"])) == k["expect"]
        assert list(orc.np_fqav_range(k["first"], k["step"], k["length"], k["n"])) == k["expect"]


def test_range_passthrough_and_floor(orc):
    assert orc.fqav_range(10.0, 0.5, 7, 1) == (10.0, 0.5, 7)  # n <= 1 returns r (:28)
    assert orc.fqav_range(10.0, 0.5, 7, 0) == (10.0, 0.5, 7)
    f, s, n = orc.fqav_range(0.0, 1.0, 10, 4)  # length ÷ n floors (:31)
    assert (f, s, n) == (1.5, 4.0, 2)


@pytest.mark.parametrize("kind", ["reduce"])
def test_c_oracle_matches_golden(orc, golden, kind):
    for c in golden.cases(kind):
        a = golden.input(c["input"])
        got = orc.reduce(a, c["fqavby"], c["tavby"], c["op"], c["win"])
        want = golden.output(c)
        if c["exact"]:
            assert same_bits(got, want), c
        else:
            np.testing.assert_allclose(got, want, rtol=1e-6, err_msg=str(c))


def test_kurtosis_golden(orc, golden):
    for c in golden.cases("kurtosis"):
        got = orc.kurtosis(golden.input(c["input"]), c["win"])
        want = golden.output(c)
        assert np.array_equal(np.isnan(got), np.isnan(want))
        # the fixture comes from the NumPy restatement (pairwise Float32 mean,
        # Float64 sums in NumPy's order): same recipe, same m
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=0)
    full = golden.output(golden.cases("kurtosis")[0])
    assert np.isnan(full[5, 1])  # constant row -> NaN


def test_stitch_band_despike_golden(orc, golden):
    st = golden.cases("stitch")[0]
    banks = [golden.input(n) for n in st["input"]]
    assert same_bits(orc.stitch(banks), golden.output(st))
    bd = golden.cases("band")[0]
    got = orc.stitch([orc.reduce(b, bd["fqavby"], bd["tavby"], bd["op"]) for b in banks])
    assert same_bits(got, golden.output(bd))
    ds = golden.cases("despike")[0]
    a = golden.input(ds["input"])[:, :, : ds["ntime"]]
    assert same_bits(orc.despike(a, ds["nfpc"]), golden.output(ds))


@pytest.mark.parametrize("seed", range(6))
def test_c_and_numpy_restatements_agree(orc, seed):
    rng = np.random.default_rng(seed)
    nc = int(rng.choice([12, 48, 96, 256]))
    ni, nt = int(rng.integers(1, 4)), int(rng.integers(1, 40))
    a = np.asfortranarray(rng.gamma(2.0, 1e3, (nc, ni, nt)).astype(np.float32))
    Fs = [f for f in (1, 2, 3, 4, 6, 12) if nc % f == 0]
    Ts = [t for t in (1, 2, 3, 5) if nt % t == 0]
    for op in ("sum", "mean", "max", "min"):
        F, T = int(rng.choice(Fs)), int(rng.choice(Ts))
        c, n = orc.reduce(a, F, T, op), orc.np_reduce(a, F, T, op)
        if op in ("max", "min"):
            assert same_bits(c, n)
        else:
            np.testing.assert_allclose(c, n, rtol=1e-6)
    np.testing.assert_allclose(orc.kurtosis(a), orc.np_kurtosis(a), rtol=1e-12, atol=0)


@pytest.mark.parametrize("n", [1, 2, 3, 15, 16, 17, 1023, 1024, 1025, 2047, 2048, 2049, 3001,
                               4096, 4097, 70001])
def test_pairwise_mean_three_restatements(orc, n):
    """StatsBase's m = Float32 pairwise sum / n (Base.mapreduce_impl,
    blocksize 1024) from three independent restatements, bit for bit: the C
    oracle, the NumPy tree, and a literal pure-Python loop (small n)."""
    rng = np.random.default_rng(n)
    # integrated-power rows: mean/sigma from 30 to 30000, where the Float32
    # rounding of every partial sum matters
    R = np.repeat([30.0, 300.0, 3000.0, 30000.0], 4)[:, None]
    rows = (1e9 + 1e9 / R * rng.standard_normal((16, n))).astype(np.float32)
    a = np.asfortranarray(rows.reshape(16, 1, n))
    c = orc.mean_f32(a)[:, 0]
    npm = orc.np_pairwise_sum(rows) / np.float32(n)
    assert same_bits(c, npm.astype(np.float32))
    if n <= 5000:
        for r in range(16):
            assert same_bits(np.float32(orc.py_pairwise_sum(rows[r]) / np.float32(n)), c[r])
    # a Float64 sum rounded to Float32 is NOT this value for long rows: the
    # test data does exercise the Float32 rounding of the partial sums
    if n >= 1025:
        f64 = (rows.astype(np.float64).sum(axis=1) / n).astype(np.float32)
        assert not same_bits(f64, c)


def test_kurtosis_oracle_high_mean_rows(orc):
    """The regime of integrated BL power (mean/sigma = sqrt(N_avg) >> 1): the C
    oracle and the NumPy restatement agree, and a one-ulp change of m moves
    the excess kurtosis beyond the streamed path's worst-case bound (so the
    GPU tests resolve m on those rows)."""
    rng = np.random.default_rng(5)
    for nt in (16, 300, 1500, 5007):
        R = np.repeat([30.0, 300.0, 3000.0, 30000.0], 8)[:, None]
        rows = rng.gamma(R ** 2, 1e9 / R ** 2, (32, nt)).astype(np.float32)
        a = np.asfortranarray(rows.reshape(32, 1, nt))
        k = orc.kurtosis(a)[:, 0]
        np.testing.assert_allclose(k, orc.np_kurtosis(a)[:, 0], rtol=1e-12)
        m = orc.mean_f32(a)[:, 0]
        mp = np.nextafter(m, np.float32(np.inf))[:, None]
        z = (rows - mp).astype(np.float32)
        z2 = (z * z).astype(np.float32)
        k1 = (z2 * z2).astype(np.float64).sum(1) / nt / ((z2.astype(np.float64).sum(1) / nt) ** 2) - 3
        big = R[:, 0] >= 3000
        # the shift moves k by ~4 * skew * ulp(m) / sigma (sample skew varies)
        assert np.mean(np.abs(k1 - k)[big] > KURT_LEAF_TOL * np.abs(k[big] + 3)) >= 0.75


def test_errors(orc):
    a = np.zeros((12, 1, 6), np.float32, order="F")
    with pytest.raises(orc.DimensionMismatch):  # reshape in fqav (:18-19)
        orc.reduce(a, 5, 1)
    with pytest.raises(orc.DimensionMismatch):
        orc.reduce(a, 1, 4)
    with pytest.raises(orc.BoundsErr):
        orc.reduce(a, 1, 1, "sum", [10, 4, 1, 0, 1, 1, 0, 6, 1])
    with pytest.raises(orc.DimensionMismatch):  # spike/source lengths differ
        orc.despike(np.zeros((10, 1, 1), np.float32), 4)
    with pytest.raises(orc.BoundsErr):
        orc.despike(np.zeros((10, 1, 1), np.float32), 1)


def test_empty_and_passthrough(orc):
    a = np.zeros((8, 2, 0), np.float32, order="F")
    assert orc.reduce(a, 4, 1).shape == (2, 2, 0)
    b = np.arange(24, dtype=np.float32).reshape((4, 2, 3), order="F")
    assert same_bits(orc.reduce(b, 1, 1), b)  # n <= 1 returns the data unchanged
    assert same_bits(orc.reduce(b, 0, -3), b)


def test_julia_zero_and_nan_semantics(orc):
    a = np.array([-0.0, -0.0, -0.0, 0.0, 1.0, np.nan], np.float32).reshape((6, 1, 1), order="F")
    s = orc.reduce(a[:2], 2, 1, "sum")
    assert s[0, 0, 0] == 0 and not np.signbit(s[0, 0, 0])  # reducedim init +0.0
    pair = np.asfortranarray(a[2:4])  # (-0.0, +0.0): Julia orders -0.0 < +0.0
    assert not np.signbit(orc.reduce(pair, 2, 1, "max")[0, 0, 0])
    assert np.signbit(orc.reduce(pair, 2, 1, "min")[0, 0, 0])
    assert np.signbit(orc.reduce(np.asfortranarray(a[:2]), 2, 1, "max")[0, 0, 0])
    assert np.isnan(orc.reduce(a[4:6], 2, 1, "max")[0, 0, 0])
    assert np.isnan(orc.reduce(a[4:6], 2, 1, "min")[0, 0, 0])


def test_synth_generator_integer_kind(orc):
    a = orc.synth(64, 2, 5, 16, 3, kind=1)
    assert a.dtype == np.float32 and a.min() >= 0 and a.max() <= 255
    assert np.array_equal(a, np.round(a))
    b = orc.synth(64, 2, 5, 16, 3, kind=0)
    assert np.all(b > 0)


def test_baseline_threads_match_single(orc):
    rng = np.random.default_rng(3)
    banks = [np.asfortranarray(rng.integers(0, 256, (256, 1, 8)).astype(np.float32))
             for _ in range(4)]
    outs = orc.reduce_banks_mt(banks, 16, 4)
    for b, o in zip(banks, outs):
        assert same_bits(o, orc.reduce(b, 16, 4))
    for nth in (1, 3, 16):  # all-cores form: pieces of output channels over a pool
        for F, T, op in ((16, 4, "sum"), (1, 8, "mean"), (256, 1, "max")):
            outs = orc.reduce_banks_pool(banks, F, T, op, nth)
            for b, o in zip(banks, outs):
                assert same_bits(o, orc.reduce(b, F, T, op)), (nth, F, T, op)


# ---------------------------------------------------------------------------
# Non-Float32 element types (oracle.np_reduce_typed / np_kurtosis_typed),
# pinned against literal Python loops of the Julia source and against SciPy's
# independent kurtosis.
def py_kurtosis_statsbase(v):
    """StatsBase.kurtosis(v) for an integer / Float64 row, written as the
    package writes it: m = mean(v) (Base.sum pairwise / n), then one loop."""
    v = [float(x) for x in v]
    n = len(v)

    def impl(ifirst, ilast):  # Base.mapreduce_impl, pairwise_blocksize 1024
        if ifirst == ilast:
            return v[ifirst]
        if ifirst + 1024 > ilast:
            a = v[ifirst] + v[ifirst + 1]
            for i in range(ifirst + 2, ilast + 1):
                a = a + v[i]
            return a
        imid = ifirst + ((ilast - ifirst) >> 1)
        return impl(ifirst, imid) + impl(imid + 1, ilast)

    m = impl(0, n - 1) / n
    cm2 = cm4 = 0.0
    for x in v:
        z = x - m
        z2 = z * z
        cm2 += z2
        cm4 += z2 * z2
    cm4 /= n
    cm2 /= n
    return cm4 / (cm2 * cm2) - 3.0


@pytest.mark.parametrize("dt", [np.uint8, np.int16, np.float64])
def test_typed_kurtosis_oracle_pinned(orc, dt):
    import scipy.stats

    rng = np.random.default_rng(3)
    for nt in (2, 7, 1024, 1025, 2500):
        a = rng.gamma(2.0, 30.0, (3, 1, nt)).astype(dt)
        a = np.asfortranarray(a)
        got = orc.np_kurtosis_typed(a)
        for c in range(3):
            want = py_kurtosis_statsbase(a[c, 0, :])
            assert got[c, 0] == want, (dt, nt, c)  # same operations, same order
        np.testing.assert_allclose(got[:, 0], scipy.stats.kurtosis(a[:, 0, :].astype(np.float64),
                                                                   axis=1), rtol=1e-10)


def test_typed_reduce_oracle_pinned(orc):
    rng = np.random.default_rng(5)
    a = np.asfortranarray(rng.integers(0, 256, (12, 2, 6)).astype(np.uint8))
    F, T = 3, 2
    s = orc.np_reduce_typed(a, F, T, "sum")
    assert s.dtype == np.uint64 and s.shape == (4, 2, 3)
    for co in range(4):
        for i in range(2):
            for to in range(3):
                blk = [int(a[co * F + k, i, to * T + t]) for t in range(T) for k in range(F)]
                assert s[co, i, to] == sum(blk)
                assert orc.np_reduce_typed(a, F, T, "mean")[co, i, to] == \
                    (float(sum(blk[:F])) + float(sum(blk[F:]))) / (F * T)
                assert orc.np_reduce_typed(a, F, T, "max")[co, i, to] == max(blk)
    assert orc.np_reduce_typed(a, F, T, "max").dtype == np.uint8
    assert orc.np_reduce_typed(a.astype(np.int32), 3, 1, "sum").dtype == np.int64


def py_jl_sum(v):
    """sum(v) of Float64 values as Base's reducedim takes one slice: zero(T)
    plus mapreduce_impl (pairwise_blocksize 1024), written as Base writes it."""
    v = [float(x) for x in v]

    def impl(ifirst, ilast):
        if ifirst == ilast:
            return v[ifirst]
        if ilast - ifirst < 1024:
            a = v[ifirst] + v[ifirst + 1]
            for i in range(ifirst + 2, ilast + 1):
                a = a + v[i]
            return a
        imid = ifirst + ((ilast - ifirst) >> 1)
        return impl(ifirst, imid) + impl(imid + 1, ilast)

    return 0.0 + impl(0, len(v) - 1) if v else 0.0


@pytest.mark.parametrize("F,T", [(4, 2), (3, 1), (2048, 1), (4096, 2), (1500, 3), (5, 1100)])
def test_typed_float64_sum_order_pinned(orc, F, T):
    """Float64 fqav sums (and every typed mean) in Julia's order: each
    spectrum's F channels by mapreduce_impl (pairwise above 1024,
    src/gbtworkerfunctions.jl:19), then the T spectral sums of a time block the
    same way (time integration = fqav on axis 3).  Literal loops vs the
    vectorised restatement, bit for bit."""
    rng = np.random.default_rng(F * 7 + T)
    nco, nto = 2, 2
    b = np.asfortranarray(rng.standard_normal((nco * F, 1, nto * T)) * 1e8 +
                          rng.standard_normal((nco * F, 1, nto * T)))
    sb = orc.np_reduce_typed(b, F, T, "sum")
    mb = orc.np_reduce_typed(b, F, T, "mean")
    for co in range(nco):
        for to in range(nto):
            spec = [py_jl_sum(b[co * F:(co + 1) * F, 0, to * T + t]) for t in range(T)]
            want = py_jl_sum(spec)
            assert sb[co, 0, to] == want, (F, T, co, to)
            assert mb[co, 0, to] == want / (F * T)
    # integers: exact (U)Int64 sums; means in Float64 over the converted values
    # in the same order (sums beyond 2^53 round as Julia's do)
    big = np.asfortranarray(rng.integers(2**60, 2**62, (nco * F, 1, nto * T), dtype=np.int64))
    mi = orc.np_reduce_typed(big, F, T, "mean")
    for co in range(nco):
        for to in range(nto):
            spec = [py_jl_sum(big[co * F:(co + 1) * F, 0, to * T + t]) for t in range(T)]
            assert mi[co, 0, to] == py_jl_sum(spec) / (F * T)
