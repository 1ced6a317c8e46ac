"""GPU parity: every kernel of libbldp_hip against the CPU oracle and the
golden fixtures, through the C ABI.  Bit-exact for integer-valued data,
max/min, stitching, despiking and indexing; rtol 1e-5 for Float32 sums and
means of gamma-distributed data (the tolerance BASELINE.json names)."""
from __future__ import annotations

import numpy as np
import torch
import pytest

from conftest import assert_kurtosis, same_bits

pytestmark = pytest.mark.gpu

RTOL = 1e-5  # north_star: "within 1e-5 relative for Float32 sums"


def kurt_ok(eng, x, win, got, want, msg=""):
    """Kurtosis at the tolerance of the path the plan picked (conftest)."""
    shape = tuple(x.shape)
    nt = shape[2] if win is None else int(win[7])
    assert_kurtosis(got, want, eng.kurtosis_plan(x, win)["path"], nt, msg)


@pytest.fixture(scope="module")
def eng(pkg):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    pkg._lib.lib()  # loud failure if libbldp_hip.so is missing
    return pkg.engine


def dev(eng, a):
    return eng.fb_from_numpy(a, device="cuda:0")


def host(eng, t):
    return eng.fb_to_numpy(t)


def test_native_library_is_loaded(pkg, eng):
    import os

    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert "libbldp_hip.so" in maps


def test_golden_reduce(eng, golden):
    for c in golden.cases("reduce"):
        a = golden.input(c["input"])
        got = host(eng, eng.reduce(dev(eng, a), c["fqavby"], c["tavby"], c["op"], c["win"]))
        want = golden.output(c)
        if c["exact"]:
            assert same_bits(got, want), c
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL, err_msg=str(c))


def test_golden_band_stitch_despike_kurtosis(eng, golden):
    import torch

    st = golden.cases("stitch")[0]
    banks = [golden.input(n) for n in st["input"]]
    xs = [dev(eng, b) for b in banks]
    # bank-major gathered blocks -> vcat
    g = torch.stack([x.permute(2, 1, 0).contiguous() for x in xs])
    assert same_bits(host(eng, eng.stitch(g, len(xs))), golden.output(st))
    bd = golden.cases("band")[0]
    got = host(eng, eng.band_reduce(xs, bd["fqavby"], bd["tavby"], bd["op"]))
    assert same_bits(got, golden.output(bd))
    ds = golden.cases("despike")[0]
    a = golden.input(ds["input"])[:, :, : ds["ntime"]]
    x = dev(eng, np.asfortranarray(a))
    assert same_bits(host(eng, eng.despike(x, ds["nfpc"])), golden.output(ds))
    for c in golden.cases("kurtosis"):
        x = dev(eng, golden.input(c["input"]))
        kurt_ok(eng, x, c["win"], host(eng, eng.kurtosis(x, c["win"])), golden.output(c), c)


# (nchan, nif, ntime, F, T) covering the vector path at every lanes-per-group
# (F/4 = 1..64 and beyond), the narrow path (F = 1, 2), the scalar path (odd
# F), time splits across waves and across workgroups (long T).
SHAPES = [
    (4096, 1, 64, 4, 1), (4096, 1, 64, 8, 16), (4096, 2, 48, 16, 3), (4096, 1, 32, 32, 4),
    (4096, 1, 32, 64, 16), (8192, 1, 16, 128, 2), (8192, 1, 16, 256, 16),
    (16384, 1, 16, 1024, 16), (65536, 1, 4, 16384, 4), (6144, 1, 8, 12, 2),
    (6144, 1, 8, 384, 8), (4096, 1, 32, 1, 16), (4096, 3, 10, 2, 5), (4096, 1, 8, 1, 1),
    (96, 3, 10, 3, 5), (300, 2, 7, 5, 7), (512, 1, 8192, 8, 1024), (64, 1, 20000, 8, 20000),
    (512, 2, 4096, 1, 4096), (1020, 1, 2000, 6, 1000),
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_paths_integer_exact(eng, orc, shape):
    nc, ni, nt, F, T = shape
    rng = np.random.default_rng(abs(hash(shape)) % 2**32)
    a = np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
    exact = nc * nt * 255 < 2**24 or F * T * 255 < 2**24
    x = dev(eng, a)
    for op in ("sum", "max", "min", "mean"):
        got = host(eng, eng.reduce(x, F, T, op))
        want = orc.reduce(a, F, T, op)
        if op in ("max", "min") or (op == "sum" and exact):
            assert same_bits(got, want), (shape, op, eng.plan(x, F, T, op))
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL, err_msg=str((shape, op)))


# Interleaved vector path (F = 512..4096 with >= 4096 groups): a tail
# segment of fewer than 4 groups, several IFs and time blocks, every op.
IL_SHAPES = [(4098, 1, 16, 1024, 16), (8194, 2, 8, 512, 4), (4097, 1, 8, 2048, 8),
             (4099, 1, 4, 4096, 2),
             # short time blocks, one per workgroup: T = 1 is the reference's
             # fqav, no integration
             (4098, 1, 16, 1024, 1), (4097, 2, 20, 512, 1), (4096, 1, 5, 2048, 1),
             (4099, 1, 36, 1024, 4),
             # tiles >= 8 rows deep, grid x a multiple of 8: the per-XCD segment
             # order (RedArgs::il_xcd)
             (4096, 1, 32, 1024, 16), (4096, 2, 16, 512, 8), (2048, 1, 16, 2048, 8)]


@pytest.mark.parametrize("shape", IL_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_interleaved_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=nco + F, kind=1)  # integers 0..255
    a = host(eng, x)
    for op in ("sum", "max", "min", "mean"):
        assert eng.plan(x, F, T, op)["path"] == "interleaved"
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (shape, op)  # F*T*255 < 2^24
    # band launch: 3 banks written into their stitched slots
    banks = [x] + [eng.synth(nco * F, ni, nt, 1024, seed=b, kind=1) for b in (1, 2)]
    got = host(eng, eng.band_reduce(banks, F, T))
    assert same_bits(got, orc.stitch([orc.reduce(host(eng, b), F, T) for b in banks]))


# Row kernel (F = 4..256, powers of two, one float4 column per lane): a
# partial last 1024-channel segment, several IFs / time blocks / banks.
ROW_SHAPES = [(1025, 1, 8, 4, 8), (600, 2, 12, 8, 4), (300, 1, 16, 16, 8), (150, 3, 6, 32, 2),
              (65, 1, 24, 64, 8), (16384 + 3, 1, 32, 64, 16), (33, 2, 4, 128, 4), (17, 1, 8, 256, 8)]


@pytest.mark.parametrize("shape", ROW_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_row_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=nco + F, kind=1)  # integers 0..255
    a = host(eng, x)
    for op in ("sum", "max", "min", "mean"):
        assert eng.plan(x, F, T, op)["path"] == "row", (shape, eng.plan(x, F, T, op))
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (shape, op)  # F*T*255 < 2^24
    banks = [x] + [eng.synth(nco * F, ni, nt, 1024, seed=b, kind=1) for b in (1, 2)]
    got = host(eng, eng.band_reduce(banks, F, T))
    assert same_bits(got, orc.stitch([orc.reduce(host(eng, b), F, T) for b in banks]))


@pytest.mark.parametrize("F,T", [(64, 16), (16, 8), (256, 16)])
def test_reduce_row_xcd_order_integer_exact(eng, orc, F, T):
    """Rows 4 MiB apart and tiles >= 8 rows deep: the row kernels take the
    per-XCD segment order (RedArgs::il_xcd); a permutation of the tiles, so
    bit-exact against the oracle like the default order."""
    nc, nt = 1 << 20, 2 * T
    x = eng.synth(nc, 1, nt, 1024, seed=F + T, kind=1)  # integers 0..255
    a = host(eng, x)
    assert eng.plan(x, F, T, "sum")["path"] == "row"
    for op in ("sum", "max"):
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (F, T, op)


@pytest.mark.parametrize("T", [1, 2, 4])
def test_reduce_narrowt_xcd_order_integer_exact(eng, orc, T):
    """F = 2 with short time blocks on a >= 1 GiB launch: k_reduce_narrowt in
    the per-XCD segment order (RedArgs::il_xcd); bit-exact against the
    oracle."""
    nc, nt = 1 << 20, 256
    x = eng.synth(nc, 1, nt, 1024, seed=T, kind=1)  # integers 0..255, 1 GiB
    assert eng.plan(x, 2, T, "sum")["path"] == "narrow"
    got = host(eng, eng.reduce(x, 2, T, "sum"))
    assert same_bits(got, orc.reduce(host(eng, x), 2, T, "sum")), T


@pytest.mark.parametrize("F,T", [(64, 1), (16, 2)])
def test_reduce_rowt_xcd_order_integer_exact(eng, orc, F, T):
    """A short-time-block launch of >= 1 GiB: k_reduce_rowt in the per-XCD
    segment order (RedArgs::il_xcd); bit-exact against the oracle."""
    nc, nt = 1 << 20, 256
    x = eng.synth(nc, 1, nt, 1024, seed=F + T, kind=1)  # integers 0..255, 1 GiB
    assert eng.plan(x, F, T, "sum")["path"] == "row"
    got = host(eng, eng.reduce(x, F, T, "sum"))
    assert same_bits(got, orc.reduce(host(eng, x), F, T, "sum")), (F, T)


# Short time blocks (T in {1, 2, 4}; T = 1 is the reference's fqav with no
# time integration): k_reduce_rowt takes 16 / T time blocks per workgroup,
# the last group partial, and windows of <= 128 float4 columns (the 512-channel
# 0001 product) share a workgroup between 2 or 4 time groups; bit-exact, and
# the same bits k_reduce_row gives.
# Launches of fewer than 64 workgroups per CU with 16 rows per lane take 8 rows
# per lane (TPB = 8 / T); the last two shapes are large enough for 16.
ROWT_SHAPES = [(1025, 2, 37, 16, 1), (64, 1, 279, 64, 1), (33, 3, 10, 4, 2), (257, 1, 28, 256, 4),
               (300, 2, 1, 8, 1), (64, 1, 200, 8, 1), (64, 2, 150, 8, 2), (20, 1, 70, 8, 1),
               (4096, 2, 2051, 16, 1), (128, 1, 8200, 256, 4),
               # tavby = 3 and 8 (BLDP_T38): 5 / 2 blocks per workgroup (2 / 1 when small)
               (1025, 2, 36, 16, 3), (64, 1, 279, 64, 3), (257, 1, 48, 256, 8), (33, 3, 30, 4, 3),
               (20, 1, 69, 8, 3), (64, 2, 152, 8, 8), (300, 1, 96, 32, 3), (4096, 2, 2052, 16, 3)]


@pytest.mark.parametrize("shape", ROWT_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_short_time_blocks_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=7 * nco + F, kind=1)
    a = host(eng, x)
    nto = nt // T
    tpb = 16 // T if nto > 1 else 1
    cols = nco * F // 4  # float4 columns; <= 128 of them: 2 or 4 time groups per workgroup
    tsub = 1 if tpb == 1 else 4 if cols <= 64 else 2 if cols <= 128 else 1
    blocks_c = -(-cols // 256)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    small = blocks_c * ni * -(-(-(-nto // tpb)) // tsub) < 64 * ncu
    if tpb > 1 and (small or (cols <= 128 and (T == 1 or F >= 64))):
        # small launch (4 rows per lane at T <= 2) or narrow window: 8 rows
        tpb = 4 // T if small and T <= 2 else 8 // T
        if tpb == 1:  # (tavby = 8: one block per workgroup, k_reduce_row's grid)
            tsub = 1
    for op in ("sum", "max", "min", "mean"):
        plan = eng.plan(x, F, T, op)
        assert plan["path"] == "row", (shape, plan)
        assert plan["workgroups"] == blocks_c * ni * -(-(-(-nto // tpb)) // tsub), (shape, plan)
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (shape, op)
    if a.nbytes > 1 << 28:
        assert tpb == 16 // T, (shape, tpb)
        return  # (the large shapes: the 16-row kernel; windows and bands run above)
    # a time window starting inside the data, and a band of three banks
    if nt > T:
        w = [0, nco * F, 1, 0, ni, 1, 1, (nt - 1) // T * T, 1]
        got = host(eng, eng.reduce(x, F, T, "sum", w))
        assert same_bits(got, orc.reduce(a, F, T, "sum", w)), (shape, "window")
    banks = [x] + [eng.synth(nco * F, ni, nt, 1024, seed=b, kind=1) for b in (1, 2)]
    got = host(eng, eng.band_reduce(banks, F, T))
    assert same_bits(got, orc.stitch([orc.reduce(host(eng, b), F, T) for b in banks]))


# Small groups that are not a power of two (F = 3, 5, 6, 7, 12) with short time
# blocks: k_reduce_lanet, one lane per group and NRW / T time blocks per
# workgroup (the last time group partial); the 0002-band windows of 65535 and
# 65532 channels among them; bit-exact on integer data, windows and bands.
LANET_SHAPES = [(1000, 1, 37, 3, 1), (21845, 1, 18, 3, 1), (300, 2, 20, 5, 2), (257, 1, 33, 6, 1),
                (100, 3, 12, 7, 4), (513, 1, 19, 12, 1), (5461, 1, 9, 12, 1), (200, 1, 8, 12, 2),
                (70, 2, 24, 3, 4), (90, 1, 18, 6, 2), (600, 2, 16, 12, 4), (300, 1, 12, 5, 4),
                # segments shifted onto 64-byte product lines: nco % 256 > 240 takes one
                # more column block; odd nco moves every row's (and bank's) alignment
                (241, 2, 17, 3, 1), (497, 1, 10, 7, 2), (767, 3, 9, 5, 1), (16, 1, 5, 12, 1),
                # tavby = 3 and 8 (BLDP_T38): 2 / 1 blocks of 6 / 8 rows per lane
                (1000, 1, 36, 3, 3), (300, 2, 24, 5, 8), (513, 1, 18, 12, 3), (90, 1, 33, 7, 3),
                (600, 2, 16, 12, 8), (170, 1, 39, 6, 3)]


def lanet_rows(F):
    return 8


@pytest.mark.parametrize("shape", LANET_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_small_odd_groups_short_time_blocks_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=11 * nco + F + nt, kind=1)
    a = host(eng, x)
    nto, tpb = nt // T, lanet_rows(F) // T
    for op in ("sum", "max", "min", "mean"):
        plan = eng.plan(x, F, T, op)
        assert plan["path"] == "lane", (shape, plan)
        # (nco + 15): each row's segments start on a 64-byte line of the product;
        # windows of nco + 15 <= 128 / 64 pack 2 / 4 time groups per workgroup
        tsub = 4 if nco + 15 <= 64 else 2 if nco + 15 <= 128 else 1
        if F == 12:  # k_reduce_col3: 64 groups x 16 / T time blocks per workgroup
            assert plan["workgroups"] == -(-nco // 64) * ni * -(-nto // max(1, 4 // T)), \
                (shape, plan)
        else:
            assert plan["workgroups"] == \
                -(-(nco + 15) // 256) * ni * -(-(-(-nto // tpb)) // tsub), (shape, plan)
        got = host(eng, eng.reduce(x, F, T, op))
        want = orc.reduce(a, F, T, op)
        if op == "mean" and (F * T) & (F * T - 1):
            np.testing.assert_allclose(got, want, rtol=RTOL)  # s / (F T) in Float32 vs Float64
        else:
            assert same_bits(got, want), (shape, op)
    # a window one group and one spectrum in, and a band of three banks
    if nco > 1 and nt > T:
        w = [F, (nco - 1) * F, 1, 0, ni, 1, 1, (nt - 1) // T * T, 1]
        got = host(eng, eng.reduce(x, F, T, "sum", w))
        assert same_bits(got, orc.reduce(a, F, T, "sum", w)), (shape, "window")
    banks = [x] + [eng.synth(nco * F, ni, nt, 1024, seed=b, kind=1) for b in (1, 2)]
    got = host(eng, eng.band_reduce(banks, F, T))
    assert same_bits(got, orc.stitch([orc.reduce(host(eng, b), F, T) for b in banks]))


def test_reduce_small_odd_groups_gamma_rtol(eng, orc):
    """Float data through k_reduce_lanet at the 1e-5 tolerance."""
    for F, T in ((3, 1), (12, 1), (5, 2), (7, 4)):
        nc = 4096 // F * F
        a = orc.gamma_bandpass(nc, 1, 40, 1024, 31 * F + T)
        x = dev(eng, a)
        assert eng.plan(x, F, T)["path"] == "lane"
        for op in ("sum", "mean"):
            np.testing.assert_allclose(host(eng, eng.reduce(x, F, T, op)), orc.reduce(a, F, T, op),
                                       rtol=RTOL, err_msg=str((F, T, op)))
        for op in ("max", "min"):
            assert same_bits(host(eng, eng.reduce(x, F, T, op)), orc.reduce(a, F, T, op))


# Large groups (F = 512..4096) with short time blocks on windows with few
# groups per row or more (IF, time block) pairs than the interleaved kernel's
# grid holds (fqavby = 512 on the 512-channel 0001 product: one output per
# spectrum): k_reduce_wavet, one wave per group and 4 x 16 / (T K4) time
# blocks; bit-exact, and the same bits k_reduce_vec gives.
WAVET_SHAPES = [(1, 1, 300, 512, 1), (2, 2, 40, 1024, 2), (3, 1, 64, 4096, 4), (1, 1, 66000, 512, 1),
                (2, 1, 37, 2048, 1),
                # tavby = 3 (BLDP_T38)
                (1, 1, 300, 512, 3), (2, 2, 42, 4096, 3), (3, 1, 63, 1024, 3)]


@pytest.mark.parametrize("shape", WAVET_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_large_groups_short_time_blocks_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=3 * nco + F + nt, kind=1)
    a = host(eng, x)
    nto, k4 = nt // T, F // 256
    tb = max(1, 16 // (T * k4))  # time blocks per batch
    rw = tb * (1 if tb >= 2 else 4)  # per wave: one batch, or 4 of one block
    for op in ("sum", "max", "min", "mean"):
        plan = eng.plan(x, F, T, op)
        assert plan["path"] == "vector", (shape, plan)
        assert plan["workgroups"] == nco * ni * -(-nto // (4 * rw)), (shape, plan)
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (shape, op)
    if nt > T:
        w = [0, nco * F, 1, 0, ni, 1, 1, (nt - 1) // T * T, 1]
        got = host(eng, eng.reduce(x, F, T, "sum", w))
        assert same_bits(got, orc.reduce(a, F, T, "sum", w)), (shape, "window")


# The narrow path (fqavby = 1, 2) with short time blocks: k_reduce_narrowt,
# 16 / T time blocks per workgroup (2 or 4 time groups per workgroup on
# windows of <= 128 float4 columns); bit-exact, the same bits as k_reduce_narrow.
NARROWT_SHAPES = [(512, 1, 300, 2, 1), (128, 2, 50, 2, 2), (2048, 1, 32, 1, 4), (256, 3, 20, 1, 2),
                  (6000, 1, 17, 2, 1), (4096, 1, 37, 1, 1), (100, 2, 9, 1, 1),  # (F = T = 1: the copy)
                  (512, 1, 300, 2, 3), (100, 2, 30, 2, 3), (2048, 3, 33, 2, 3)]  # tavby = 3


@pytest.mark.parametrize("shape", NARROWT_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_narrow_short_time_blocks_integer_exact(eng, orc, shape):
    nco, ni, nt, F, T = shape
    x = eng.synth(nco * F, ni, nt, 1024, seed=5 * nco + F + nt, kind=1)
    a = host(eng, x)
    nto, cols = nt // T, nco * F // 4
    tsub = 4 if cols <= 64 else 2 if cols <= 128 else 1
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    tpb = 16 // T  # 8 / 4 rows per lane on small launches and, at T = 1, narrow windows
    if -(-cols // 256) * ni * -(-(-(-nto // tpb)) // tsub) < 64 * ncu or (cols <= 128 and T == 1):
        tpb = 4 // T if T <= 2 else 8 // T
    for op in ("sum", "max", "min", "mean"):
        plan = eng.plan(x, F, T, op)
        assert plan["path"] == "narrow", (shape, plan)
        assert plan["workgroups"] == -(-cols // 256) * ni * -(-(-(-nto // tpb)) // tsub), \
            (shape, plan)
        got = host(eng, eng.reduce(x, F, T, op))
        assert same_bits(got, orc.reduce(a, F, T, op)), (shape, op)
    w = [0, nco * F, 1, 0, ni, 1, 1, (nt - 1) // T * T, 1]
    got = host(eng, eng.reduce(x, F, T, "sum", w))
    assert same_bits(got, orc.reduce(a, F, T, "sum", w)), (shape, "window")


# Time integration (fqavby = 1, the narrow kernel): partial last segments,
# several IFs / time blocks / banks, every op, a time-offset window.
TIME_SHAPES = [(4100, 1, 32, 16), (4096, 3, 40, 5), (1 << 20, 2, 48, 16), (1 << 23, 1, 16, 16),
               (8 * 1024 + 4, 1, 64, 64)]


@pytest.mark.parametrize("shape", TIME_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_reduce_time_integer_exact(eng, orc, shape):
    nc, ni, nt, T = shape
    x = eng.synth(nc, ni, nt, 1024, seed=nc + T, kind=1)  # integers 0..255
    a = host(eng, x)
    for op in ("sum", "max", "min", "mean"):
        got = host(eng, eng.reduce(x, 1, T, op))
        want = orc.reduce(a, 1, T, op)
        if op == "mean" and T & (T - 1):
            np.testing.assert_allclose(got, want, rtol=RTOL)
        else:
            assert same_bits(got, want), (shape, op)
    # band: 3 banks written into their stitched slots, a window from spectrum 4
    w = [0, nc, 1, 0, ni, 1, 3, (nt - 3) // T * T, 1]
    banks = [x] + [eng.synth(nc, ni, nt, 1024, seed=b, kind=1) for b in (1, 2)]
    got = host(eng, eng.band_reduce(banks, 1, T, "sum", w))
    assert same_bits(got, orc.stitch([orc.reduce(host(eng, b), 1, T, "sum", w) for b in banks]))


def test_plan_covers_all_paths(eng):
    import torch

    x = eng.fb_empty(4096, 1, 64)
    assert eng.plan(x, 64, 16)["path"] == "vector"
    assert eng.plan(x, 1, 16)["path"] == "narrow"
    assert eng.plan(x, 2, 16)["path"] == "narrow"
    assert eng.plan(eng.fb_empty(4095, 1, 4), 3, 1)["path"] == "lane"
    assert eng.plan(eng.fb_empty(4095, 1, 4), 4095, 1)["path"] == "scalar"
    y = eng.fb_empty(512, 1, 8192)
    assert eng.plan(y, 8, 8192)["time_chunks"] > 1
    assert eng.plan(y, 8, 1024)["time_split_waves"] in (2, 4)
    del torch


@pytest.mark.parametrize("F,T", [(64, 16), (1024, 16), (8, 64), (1, 8), (4, 1)])
def test_reduce_gamma_rtol(eng, orc, F, T):
    a = orc.gamma_bandpass(16384, 1, 128, 1024, F * 100 + T)
    x = dev(eng, a)
    for op in ("sum", "mean", "max", "min"):
        got = host(eng, eng.reduce(x, F, T, op))
        want = orc.reduce(a, F, T, op)
        if op in ("max", "min"):
            assert same_bits(got, want)
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL)


WINDOWS = [
    [32, 512, 1, 1, 1, 1, 4, 32, 1],        # (33:544, 2, 5:36): unaligned start? 32 -> aligned
    [33, 512, 1, 0, 2, 1, 0, 48, 1],        # misaligned start -> dword-aligned vector loads / tile
    [1020, 96, -3, 0, 2, 1, 44, 12, -3],    # reversed strided channels and times
    [5, 120, 8, 0, 2, 1, 0, 48, 1],         # strided channels
    [0, 1024, 1, 1, 1, 1, 0, 24, 2],        # every other spectrum
    [0, 1024, 1, 0, 2, 1, 7, 1, 1],         # an Integer time index (i:i)
]


@pytest.mark.parametrize("win", WINDOWS, ids=range(len(WINDOWS)))
def test_windows(eng, orc, win):
    rng = np.random.default_rng(5)
    a = np.asfortranarray(rng.integers(0, 256, (1024, 2, 48)).astype(np.float32))
    x = dev(eng, a)
    for F, T in [(1, 1), (4, 4), (8, 2), (3, 6), (16, 1)]:
        if win[1] % F or win[7] % T:
            continue
        for op in ("sum", "max"):
            got = host(eng, eng.reduce(x, F, T, op, win))
            assert same_bits(got, orc.reduce(a, F, T, op, win)), (win, F, T, op)


# Tile path (misaligned starts, odd F, channel steps 2..8, groups up to one
# tile row, several IFs, long T split across workgroups):
# (nchan, nif, ntime, window, F, T).  Integer data keeps every sum exact.
TILE_CASES = [
    (4096, 1, 32, [1, 4032, 1, 0, 1, 1, 0, 32, 1], 64, 16),
    (4096, 2, 16, [3, 4092, 1, 0, 2, 1, 0, 16, 1], 3, 4),
    (4096, 1, 16, [0, 4095, 1, 0, 1, 1, 0, 16, 1], 5, 1),
    (8192, 1, 8, [2, 8184, 1, 0, 1, 1, 0, 8, 1], 1, 8),
    (8192, 1, 8, [2, 8186, 1, 0, 1, 1, 0, 8, 1], 2, 2),
    (8192, 1, 4, [1, 8186, 1, 0, 1, 1, 0, 4, 1], 4093, 1),
    (8192, 1, 4, [5, 8000, 1, 0, 1, 1, 0, 4, 1], 1000, 2),
    (8192, 1, 8, [0, 4096, 2, 0, 1, 1, 0, 8, 1], 16, 4),
    (8192, 1, 8, [7, 2720, 3, 0, 1, 1, 0, 8, 1], 17, 8),
    (8192, 1, 8, [3, 1020, 8, 0, 1, 1, 0, 8, 1], 12, 8),
    (1028, 1, 5000, [1, 1024, 1, 0, 1, 1, 0, 5000, 1], 4, 5000),
    (4096, 3, 16, [1, 1020, 1, 1, 2, 1, 0, 16, 1], 20, 4),
    (65540, 1, 24, [1, 65536, 1, 0, 1, 1, 4, 16, 1], 1024, 16),
]


def misaligned_paths(win, F, T=16):
    """Paths a window that starts off a 16-byte boundary takes (16-byte row
    pitches; BLDP_UNALIGNED_VEC=2): unit-step windows with F = 1 or F % 4 == 0,
    F <= 256 read their own float4 columns with dword-aligned 16-byte loads on
    the vector / narrow paths;
    F = 1 windows whose channel count is not a multiple of 4 take the
    realigning narrow kernel; the rest the tile path."""
    if win[2] != 1:
        return {"tile"}
    if F == 1:
        return {"narrow"} if win[1] % 4 == 0 else {"narrow_mis"}
    if F in (3, 5, 6, 7, 12) and T in (1, 2, 3, 4, 8):
        return {"lane"}  # k_reduce_lanet: short time blocks of small odd groups
    if F == 3:
        return {"lane"}  # one dwordx3 per lane (BLDP_LANE3)
    if F % 4 == 0 and F <= 256:
        return {"vector", "row"}
    return {"tile"}


@pytest.mark.parametrize("case", TILE_CASES, ids=range(len(TILE_CASES)))
def test_tile_path(eng, orc, case):
    nc, ni, nt, win, F, T = case
    rng = np.random.default_rng(nc + F)
    a = np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
    x = dev(eng, a)
    assert eng.plan(x, F, T, "sum", win)["path"] in misaligned_paths(win, F, T)
    for op in ("sum", "max", "min", "mean"):
        got = host(eng, eng.reduce(x, F, T, op, win))
        want = orc.reduce(a, F, T, op, win)
        if op == "mean":
            np.testing.assert_allclose(got, want, rtol=RTOL)
        else:
            assert same_bits(got, want), (case, op)


def test_tile_path_special_values(eng, orc):
    a = np.zeros((68, 1, 4), np.float32, order="F")
    a[1:5, 0, 0] = -0.0
    a[5:9, 0, 1] = [-0.0, 0.0, -0.0, -0.0]
    a[9:13, 0, 2] = [1.0, np.nan, 2.0, 3.0]
    a[13:17, 0, 3] = [np.inf, 1.0, -np.inf, 0.0]
    a[17:21, 0, 0] = [np.inf, 1.0, 5.0, 0.0]
    x = dev(eng, a)
    for F, T in [(4, 1), (2, 2), (1, 4), (3, 4), (20, 1)]:
        win = [1, 60, 1, 0, 1, 1, 0, 4, 1]
        assert eng.plan(x, F, T, "max", win)["path"] in misaligned_paths(win, F, T)
        for op in ("sum", "max", "min"):
            got = host(eng, eng.reduce(x, F, T, op, win))
            want = orc.reduce(a, F, T, op, win)
            if op == "sum":
                assert np.array_equal(np.isnan(got), np.isnan(want))
                fin = np.isfinite(want)
                assert np.array_equal(got[fin], want[fin])
            else:
                assert same_bits(got, want), (F, T, op)

def test_subview_tensor(eng, orc):
    rng = np.random.default_rng(9)
    a = np.asfortranarray(rng.integers(0, 256, (2048, 2, 40)).astype(np.float32))
    x = dev(eng, a)[256:1280, 1:2, 8:40]  # a view with the parent's pitches
    got = host(eng, eng.reduce(x, 64, 8))
    want = orc.reduce(a, 64, 8, "sum", [256, 1024, 1, 1, 1, 1, 8, 32, 1])
    assert same_bits(got, want)


def test_strided_output_writes_stitched_slot(eng, orc):
    import torch

    rng = np.random.default_rng(4)
    a = np.asfortranarray(rng.integers(0, 256, (1024, 1, 16)).astype(np.float32))
    out = eng.fb_empty(4 * 64, 1, 4)
    out.fill_(-1.0)
    eng.reduce(dev(eng, a), 16, 4, "sum", out=out[128:192])
    o = host(eng, out)
    assert same_bits(o[128:192], orc.reduce(a, 16, 4))
    assert np.all(o[:128] == -1) and np.all(o[192:] == -1)
    del torch


def test_band_reduce_8_banks(eng, orc):
    banks = [orc.gamma_bandpass(65536, 1, 64, 1024, 100 + b) for b in range(8)]
    xs = [dev(eng, b) for b in banks]
    got = host(eng, eng.band_reduce(xs, 64, 16))
    want = orc.stitch([orc.reduce(b, 64, 16) for b in banks])
    np.testing.assert_allclose(got, want, rtol=RTOL)
    got = host(eng, eng.band_reduce(xs, 1024, 64, "max"))
    assert same_bits(got, orc.stitch([orc.reduce(b, 1024, 64, "max") for b in banks]))


def test_special_values(eng, orc):
    a = np.zeros((64, 1, 4), np.float32, order="F")
    a[0:4, 0, 0] = -0.0
    a[4:8, 0, 0] = [-0.0, 0.0, -0.0, -0.0]
    a[8:12, 0, 0] = [1.0, np.nan, 2.0, 3.0]
    a[12:16, 0, 0] = [np.inf, 1.0, -np.inf, 0.0]
    a[16:20, 0, 0] = [np.inf, 1.0, 5.0, 0.0]
    a[20:24, 0, 0] = [3e38, 3e38, 0, 0]  # overflow to inf in f32
    x = dev(eng, a)
    for F, T in [(4, 1), (4, 2), (1, 4), (16, 4)]:
        for op in ("sum", "max", "min"):
            got = host(eng, eng.reduce(x, F, T, op))
            want = orc.reduce(a, F, T, op)
            if op == "sum":
                assert np.array_equal(np.isnan(got), np.isnan(want))
                fin = np.isfinite(want)
                assert np.array_equal(got[~fin & ~np.isnan(want)], want[~fin & ~np.isnan(want)])
            else:
                assert same_bits(got, want), (F, T, op)


def test_errors_and_empty(eng, pkg):
    x = eng.fb_empty(96, 1, 10)
    with pytest.raises(pkg.DimensionMismatch):
        eng.reduce(x, 7, 1)
    with pytest.raises(pkg.DimensionMismatch):
        eng.reduce(x, 1, 3)
    with pytest.raises(pkg.BoundsError):
        eng.reduce(x, 1, 1, "sum", [90, 10, 1, 0, 1, 1, 0, 10, 1])
    e = eng.reduce(eng.fb_empty(96, 1, 0), 4, 1)
    assert tuple(e.shape) == (24, 1, 0)
    e = eng.reduce(x, 4, 1, "sum", [0, 0, 1, 0, 1, 1, 0, 10, 1])
    assert tuple(e.shape) == (0, 1, 10)


def test_host_pipeline(eng, orc):
    rng = np.random.default_rng(12)
    a = np.asfortranarray(rng.integers(0, 256, (4096, 2, 300)).astype(np.float32))
    for win, F, T in [(None, 64, 10), ([128, 2048, 1, 1, 1, 1, 20, 200, 1], 16, 8),
                      ([4000, 500, -2, 0, 2, 1, 299, 100, -3], 4, 5)]:
        got = eng.reduce_host(a, F, T, "sum", win)
        assert same_bits(got, orc.reduce(a, F, T, "sum", win)), win


def test_kurtosis_long_and_strided(eng, orc):
    rng = np.random.default_rng(1)
    a = np.asfortranarray((rng.standard_normal((512, 1, 20000)) ** 2).astype(np.float32) * 1e9)
    x = dev(eng, a)
    kurt_ok(eng, x, None, host(eng, eng.kurtosis(x)), orc.kurtosis(a))
    b = np.asfortranarray((rng.standard_normal((257, 3, 300)) ** 2).astype(np.float32))
    w = [3, 200, 1, 1, 2, 1, 10, 250, 1]
    y = dev(eng, b)
    kurt_ok(eng, y, w, host(eng, eng.kurtosis(y, w)), orc.kurtosis(b, w))


def test_synth_integer_kind_matches_oracle(eng, orc):
    t = eng.synth(1000, 2, 7, 64, seed=5, kind=1)
    assert same_bits(host(eng, t), orc.synth(1000, 2, 7, 64, 5, kind=1))
    g = host(eng, eng.synth(1024, 1, 8, 64, seed=5, kind=0))
    np.testing.assert_allclose(g, orc.synth(1024, 1, 8, 64, 5, kind=0), rtol=1e-5)


def test_full_size_bank_properties(eng):
    """cfg3 geometry (2^26 ch x 16 spectra, F=1024, T=16) at full size:
    size-independent properties instead of the oracle (which would take
    minutes): integer data makes every sum exact, so the total of the
    outputs equals the total of the input, and max/min of the outputs
    equal the global max/min; one channel group is recomputed on the host."""
    import torch

    x = eng.synth(1 << 26, 1, 16, 1 << 20, seed=3, kind=1)
    s = eng.reduce(x, 1024, 16, "sum")
    assert tuple(s.shape) == (65536, 1, 1)
    assert s.double().sum().item() == x.double().sum().item()
    assert eng.reduce(x, 1024, 16, "max").max().item() == x.max().item()
    assert eng.reduce(x, 1024, 16, "min").min().item() == x.min().item()
    k = 12345
    blk = x[k * 1024:(k + 1) * 1024].double().sum().item()
    assert s[k, 0, 0].item() == blk
    # time integration alone: sum over time of each channel
    t = eng.reduce(x, 1, 16, "sum")
    assert torch.equal(t[:, 0, 0].double(), x[:, 0, :].double().sum(dim=1))


def test_full_size_cfg3_band_slab(eng):
    """The north-star band at full size (8 x 2^26 ch x 16 spectra = 32 GiB in
    one slab, F=1024, T=16, one launch): on integer data every bank's
    stitched slot sums to that bank's total, and spot groups of every bank
    match a host recomputation (exact)."""
    import torch

    n = 1 << 26
    banks = eng.band_empty(8, n, 1, 16)
    for b, v in enumerate(banks):
        eng.synth(n, 1, 16, 1 << 20, seed=30 + b, kind=1, out=v)
    out = eng.band_reduce(banks, 1024, 16, "sum")
    assert tuple(out.shape) == (8 * 65536, 1, 1)
    assert eng.plan(banks[0], 1024, 16)["path"] == "interleaved"
    for b, v in enumerate(banks):
        slot = out[b * 65536:(b + 1) * 65536, 0, 0].double()
        assert slot.sum().item() == v.double().sum().item(), b
        for k in (0, 777 * (b + 1), 65535):
            assert slot[k].item() == v[k * 1024:(k + 1) * 1024].double().sum().item(), (b, k)
    mx = eng.band_reduce(banks, 1024, 16, "max")
    assert torch.equal(mx[3 * 65536:4 * 65536, 0, 0],
                       banks[3][:, 0, :].reshape(65536, 1024, 16).amax(dim=(1, 2)))
    del banks, out, mx
    torch.cuda.empty_cache()


def test_band_kurtosis(eng, orc):
    rng = np.random.default_rng(21)
    banks = [np.asfortranarray((rng.standard_normal((1024, 2, 300)) ** 2).astype(np.float32))
             for _ in range(5)]
    xs = [dev(eng, b) for b in banks]
    w = [4, 1000, 1, 0, 2, 1, 10, 280, 1]
    ks = eng.band_kurtosis(xs, w)
    assert len(ks) == 5
    for b, x, k in zip(banks, xs, ks):
        kurt_ok(eng, x, w, host(eng, k), orc.kurtosis(b, w))
    long = [np.asfortranarray((rng.standard_normal((64, 1, 30000)) ** 2).astype(np.float32))
            for _ in range(3)]
    xs = [dev(eng, b) for b in long]
    ks = eng.band_kurtosis(xs)  # many leaves, tree merge
    for b, x, k in zip(long, xs, ks):
        kurt_ok(eng, x, None, host(eng, k), orc.kurtosis(b))


def test_full_size_cfg4_and_cfg2_banks(eng, orc):
    """cfg4 (0001: 512 ch x 880000 spectra, window 1:879616, F=8, T=1024) at
    full size on integer data: exact totals and a spot group; cfg2 (8 banks of
    0002) against the oracle directly."""
    x = eng.synth(512, 1, 880000, 8, seed=4, kind=1)
    w = [0, 512, 1, 0, 1, 1, 0, 879616, 1]
    s = eng.reduce(x, 8, 1024, "sum", w)
    assert tuple(s.shape) == (64, 1, 859)
    assert s.double().sum().item() == x[:, :, :879616].double().sum().item()
    blk = x[8 * 5:8 * 6, 0, 1024 * 700:1024 * 701].double().sum().item()
    assert s[5, 0, 700].item() == blk
    assert eng.reduce(x, 8, 1024, "max", w).max().item() == x[:, :, :879616].max().item()
    banks = [orc.gamma_bandpass(65536, 1, 279, 1024, 200 + b) for b in range(8)]
    got = host(eng, eng.band_reduce([dev(eng, b) for b in banks], 64, 16, "sum",
                                    [0, 65536, 1, 0, 1, 1, 0, 272, 1]))
    want = orc.stitch([orc.reduce(b, 64, 16, "sum", [0, 65536, 1, 0, 1, 1, 0, 272, 1])
                       for b in banks])
    np.testing.assert_allclose(got, want, rtol=RTOL)


@pytest.mark.parametrize("nt", [1, 2, 7, 12, 16, 17, 32, 33])
@pytest.mark.parametrize("nc,ni", [(4096, 2), (4100, 1)])
def test_kurtosis_short_windows(eng, orc, nt, nc, ni):
    """nt <= 32 runs the register-resident single-read kernel (exact-count
    code at 16 and 32; whole waves store through LDS, a partial wave per
    lane), bit-exact; 33 the register tile."""
    rng = np.random.default_rng(nt + nc)
    a = np.asfortranarray((rng.standard_normal((nc, ni, nt)) ** 2).astype(np.float32) * 1e6)
    x = dev(eng, a)
    want = orc.kurtosis(a)
    kurt_ok(eng, x, None, host(eng, eng.kurtosis(x)), want)
    r = a[::-1].copy(order="F")
    ks = eng.band_kurtosis([x, dev(eng, r)])
    kurt_ok(eng, x, None, host(eng, ks[0]), want)
    kurt_ok(eng, x, None, host(eng, ks[1]), orc.kurtosis(r))


@pytest.mark.parametrize("nt", [33, 100, 128, 129, 272, 384, 385, 512, 513])
def test_kurtosis_mid_windows(eng, orc, nt):
    """33..512 spectra: k_kurt_mid keeps a 64-channel tile in registers (one
    read); a partial last tile; a window with channel/time offsets; 513 goes
    to the chunk-merge kernels."""
    rng = np.random.default_rng(1000 + nt)
    a = np.asfortranarray((rng.standard_normal((1100, 2, nt + 3)) ** 2).astype(np.float32)
                          * 1e6)
    a[5, 1, :] = 7.0  # a constant row -> NaN, as StatsBase
    b = a[:, :, :nt].copy(order="F")
    x = dev(eng, b)
    kurt_ok(eng, x, None, host(eng, eng.kurtosis(x)), orc.kurtosis(b))
    w = [8, 1088, 1, 0, 2, 1, 3, nt, 1]  # idxs = (9:1096, :, 4:nt+3)
    y = dev(eng, a)
    kurt_ok(eng, y, w, host(eng, eng.kurtosis(y, w)), orc.kurtosis(a, w))


def test_band_reduce_multi_device_api(eng, orc, pkg):
    """The single-process multi-GPU entry point; on a one-GPU box every bank
    sits on device 0 (the peer path runs on the driver's 8-GPU node)."""
    import torch

    banks = [orc.gamma_bandpass(8192, 2, 48, 1024, 300 + b) for b in range(8)]
    xs = [dev(eng, b) for b in banks]
    w = [0, 8192, 1, 0, 2, 1, 0, 48, 1]
    got = host(eng, eng.band_reduce_multi(xs, 64, 16, "sum", w))
    want = orc.stitch([orc.reduce(b, 64, 16, "sum", w) for b in banks])
    np.testing.assert_allclose(got, want, rtol=RTOL)
    assert same_bits(got, host(eng, eng.band_reduce(xs, 64, 16, "sum", w)))
    L = pkg._lib.lib()
    import ctypes

    devs = (ctypes.c_int * 2)(0, torch.cuda.device_count())  # no such device
    ptrs = (ctypes.c_void_p * 2)(xs[0].data_ptr(), xs[1].data_ptr())
    rc = L.bldp_band_reduce_multi_f32(2, devs, ptrs, 8192, 2, 48, None, 64, 16, 0, 0, None, 0)
    assert rc == pkg._lib.BLDP_EINVAL
    devs = (ctypes.c_int * 2)(0, 0)
    rc = L.bldp_band_reduce_multi_f32(2, devs, ptrs, 8192, 2, 48, None, 64, 16, 0, 0, None, 6)
    assert rc == pkg._lib.BLDP_EINVAL  # unknown flag bits
    d = ctypes.c_int(-1)
    assert L.bldp_peer_access(0, 0, ctypes.byref(d)) == 0 and d.value == 1
    assert L.bldp_peer_access(0, torch.cuda.device_count(), ctypes.byref(d)) == \
        pkg._lib.BLDP_EINVAL
    assert eng.peer_access(0, 0)


def test_band_reduce_multi_staged_branch(eng, orc):
    """BLDP_BAND_STAGED (staged=True) sends every bank of
    bldp_band_reduce_multi_f32 through the staged branch a bank off the root
    takes without peer access (local reduce into a staging buffer, then one
    strided hipMemcpy2DAsync into the bank's slot of the root's product):
    bit-exact against the single-launch band reduce, for a one-row and a
    many-row product."""
    rng = np.random.default_rng(88)
    for shape, F, T, w in (((8192, 2, 48), 64, 16, [0, 8192, 1, 0, 2, 1, 0, 48, 1]),
                           ((4096, 1, 64), 1024, 64, None),
                           ((1000, 3, 20), 8, 5, [4, 992, 1, 0, 3, 1, 0, 20, 1])):
        banks = [np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32))
                 for _ in range(5)]
        xs = [dev(eng, b) for b in banks]
        got = host(eng, eng.band_reduce_multi(xs, F, T, "sum", w, staged=True))
        assert same_bits(got, host(eng, eng.band_reduce(xs, F, T, "sum", w))), shape
        assert same_bits(got, orc.stitch([orc.reduce(b, F, T, "sum", w) for b in banks]))


def _random_case(rng):
    """A random window / factors / op over a small random array, biased so
    that every plan (row, vector, narrow, tile, scalar, time chunks) shows up
    (the interleaved kernel needs >= 4096 large groups: IL_SHAPES)."""
    nchan = int(rng.choice([rng.integers(1, 300), rng.integers(300, 5000), 4096, 8192, 16384]))
    nif = int(rng.integers(1, 4))
    ntime = int(rng.choice([rng.integers(1, 70), rng.integers(70, 400)]))
    cs = int(rng.choice([1, 1, 1, 1, 1, 2, 3, -1, -2, 5, 9]))
    c0 = int(rng.integers(0, nchan))
    if rng.random() < 0.5:
        c0 -= c0 % 4  # 16-byte aligned start
    if rng.random() < 0.25:
        c0 = 0
    cmax = (nchan - 1 - c0) // cs + 1 if cs > 0 else c0 // (-cs) + 1
    F = int(rng.choice([1, 2, 3, 4, 8, 16, 64, 256, 5, 12, 32]))
    if cmax // F == 0:
        F = 1
    g = cmax // F
    ngroups = int(rng.integers(1, g + 1)) if rng.random() < 0.95 else 0
    if ngroups and rng.random() < 0.5:
        ngroups = g  # the widest window this start allows
    nc = ngroups * F
    i0 = int(rng.integers(0, nif))
    ni = int(rng.integers(1, nif - i0 + 1))
    T = int(rng.choice([1, 2, 3, 4, 8, 16, 7, 32, 128]))
    t0 = int(rng.integers(0, ntime)) if rng.random() < 0.7 else 0
    if (ntime - t0) // T == 0:
        T = 1
    m = (ntime - t0) // T
    nto = int(rng.integers(1, m + 1)) if rng.random() < 0.95 else 0
    win = [c0, nc, cs, i0, ni, 1, t0, nto * T, 1]
    op = str(rng.choice(["sum", "max", "min", "mean"]))
    return (nchan, nif, ntime), win, F, T, op


@pytest.mark.parametrize("seed", range(8))
def test_reduce_random_windows_against_oracle(eng, orc, seed):
    """300 random (shape, window, fqavby, tavby, op) cases per seed on
    integer data: bit-exact against the oracle whenever the Float32 group
    sums are exact (< 2^24), rtol 1e-5 otherwise; every plan the planner can
    pick is reached."""
    rng = np.random.default_rng(1234 + seed)
    seen = set()
    for _ in range(40):
        shape, win, F, T, op = _random_case(rng)
        a = np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32))
        x = dev(eng, a)
        got = host(eng, eng.reduce(x, F, T, op, win))
        want = orc.reduce(a, F, T, op, win)
        assert got.shape == want.shape, (shape, win, F, T, op)
        if win[1] * win[4] * win[7]:
            seen.add(eng.plan(x, F, T, op, win)["path"])
        if op in ("max", "min") or (op == "sum" and F * T * 255 < 2 ** 24):
            assert same_bits(got, want), (shape, win, F, T, op)
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL, err_msg=str((shape, win, F, T, op)))
    assert seen  # the plan set is reported for coverage inspection


@pytest.mark.parametrize("seed", range(4))
def test_kurtosis_random_windows_against_oracle(eng, orc, seed):
    """Random windows for getkurtosis: register (<= 32 spectra), tile (<= 512)
    and two-pass kernels, aligned and unaligned channel windows."""
    rng = np.random.default_rng(777 + seed)
    for _ in range(12):
        shape, win, _, _, _ = _random_case(rng)
        nt = int(rng.choice([rng.integers(1, 40), rng.integers(40, 600), rng.integers(600, 1500)]))
        shape = (shape[0], shape[1], nt)
        win[6] = int(rng.integers(0, nt))
        win[7] = int(rng.integers(0, nt - win[6] + 1))
        a = np.asfortranarray((rng.standard_normal(shape) ** 2).astype(np.float32) * 100)
        x = dev(eng, a)
        kurt_ok(eng, x, win, host(eng, eng.kurtosis(x, win)), orc.kurtosis(a, win), (shape, win))


@pytest.mark.parametrize("seed", range(3))
def test_host_and_band_random_windows(eng, orc, seed):
    """Random windows through the host-array drop-in (bldp_reduce_host_f32,
    staged through pinned pipelines) and through band launches of 1-5 banks
    (stitched output slots)."""
    rng = np.random.default_rng(4242 + seed)
    for _ in range(12):
        shape, win, F, T, op = _random_case(rng)
        a = np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32))
        exact = op in ("max", "min") or (op == "sum" and F * T * 255 < 2 ** 24)
        got = eng.reduce_host(a, F, T, op, win)
        want = orc.reduce(a, F, T, op, win)
        if exact:
            assert same_bits(got, want), (shape, win, F, T, op)
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL)
        nb = int(rng.integers(1, 6))
        banks = [a] + [np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32))
                       for _ in range(nb - 1)]
        got = host(eng, eng.band_reduce([dev(eng, b) for b in banks], F, T, op, win))
        want = orc.stitch([orc.reduce(b, F, T, op, win) for b in banks])
        if exact:
            assert same_bits(got, want), (nb, shape, win, F, T, op)
        else:
            np.testing.assert_allclose(got, want, rtol=RTOL)


def _random_axis(rng, lo, n):
    """(start, count, step) inside [lo, lo + n): steps of either sign."""
    step = int(rng.choice([1, 1, 1, 2, 3, -1, -2]))
    a, b = sorted(int(v) for v in rng.integers(lo, lo + n, 2))
    if step < 0:
        a, b = b, a
    count = (b - a) // step + 1
    return a, int(rng.integers(0, count + 1)) if rng.random() < 0.1 else count, step


@pytest.mark.parametrize("seed", range(3))
def test_unchunk_random_boxes(eng, pkg, seed):
    """bldp_unchunk_f32 directly: a random chunk box (chunk dims, grid, box
    origin) packed chunk by chunk in grid order, and random windows of either
    step sign inside it; bit-exact against numpy indexing of the unpacked box
    (the decoded-FBH5 gather, src/gbtworkerfunctions.jl:185)."""
    import ctypes

    import torch

    rng = np.random.default_rng(99 + seed)
    L = pkg._lib.lib()
    for _ in range(25):
        ct, ci, cc = int(rng.integers(1, 6)), int(rng.integers(1, 3)), int(rng.integers(1, 70))
        gt, gi, gc = int(rng.integers(1, 5)), int(rng.integers(1, 3)), int(rng.integers(1, 5))
        bt0, bi0, bc0 = (ct * int(rng.integers(0, 4)), ci * int(rng.integers(0, 2)),
                         cc * int(rng.integers(0, 4)))
        box = rng.integers(0, 1 << 20, (gt * ct, gi * ci, gc * cc)).astype(np.float32)
        packed = np.concatenate([
            box[a * ct:(a + 1) * ct, b * ci:(b + 1) * ci, c * cc:(c + 1) * cc].ravel()
            for a in range(gt) for b in range(gi) for c in range(gc)])
        (t0, nt, ts), (i0, ni, is_), (c0, nc, cs) = (
            _random_axis(rng, bt0, gt * ct), _random_axis(rng, bi0, gi * ci),
            _random_axis(rng, bc0, gc * cc))
        win = [c0, nc, cs, i0, ni, is_, t0, nt, ts]
        sel = lambda s, n, st, lo: s - lo + st * np.arange(n)  # noqa: E731
        want = box[np.ix_(sel(t0, nt, ts, bt0), sel(i0, ni, is_, bi0), sel(c0, nc, cs, bc0))]
        pk = torch.from_numpy(packed).to("cuda:0")
        out = eng.fb_empty(nc, ni, nt, device="cuda:0")
        i3 = lambda *v: (ctypes.c_int64 * 3)(*v)  # noqa: E731
        rc = L.bldp_unchunk_f32(pk.data_ptr(), i3(ct, ci, cc), i3(bt0, bi0, bc0), i3(gt, gi, gc),
                                (ctypes.c_int64 * 9)(*win), out.data_ptr() if out.numel() else None,
                                pkg._lib.stream_ptr())
        assert rc == 0, pkg._lib.last_error()
        got = host(eng, out)
        assert got.shape == (nc, ni, nt)
        assert same_bits(got, np.asfortranarray(want.transpose(2, 1, 0))), (
            (ct, ci, cc), (gt, gi, gc), (bt0, bi0, bc0), win)


@pytest.mark.parametrize("seed", range(2))
def test_stitch_despike_random(eng, orc, seed):
    """Random bank counts and block shapes through bldp_stitch_f32 (vcat of
    bank-major gathered blocks, src/gbt.jl:103) and random nfpc through
    bldp_despike_f32 (src/gbt.jl:101-102,111): bit-exact copies."""
    import torch

    rng = np.random.default_rng(31 + seed)
    for _ in range(20):
        nb = int(rng.integers(1, 9))
        nc, ni, nt = int(rng.integers(1, 3000)), int(rng.integers(1, 4)), int(rng.integers(1, 9))
        blocks = [rng.standard_normal((nc, ni, nt)).astype(np.float32, order="F")
                  for _ in range(nb)]
        g = torch.from_numpy(np.stack([b.transpose(2, 1, 0) for b in blocks])).to("cuda:0")
        got = host(eng, eng.stitch(g.contiguous(), nb))
        assert same_bits(got, orc.stitch(blocks)), (nb, nc, ni, nt)
        nfpc = int(rng.integers(2, 65))
        whole = nfpc * int(rng.integers(1, 40))
        d = np.asfortranarray(rng.standard_normal((whole, ni, nt)).astype(np.float32))
        got = host(eng, eng.despike(dev(eng, d), nfpc))
        assert same_bits(got, orc.despike(d, nfpc)), (whole, ni, nt, nfpc)


@pytest.mark.parametrize("nt", [513, 1024, 1025, 5007])
def test_kurtosis_long_windows_leaf_merge(eng, orc, nt):
    """> 512 spectra: k_kurt_leaf streams each leaf of Julia's pairwise sum
    once and the tree kernels merge them.  Covers ragged leaves, a constant
    row (NaN, as StatsBase), an RFI-like outlier in the first spectrum of a
    row (the leaf's shift point; StatsBase's Float32 z^4 overflows to Inf
    there, which the merge reproduces from the row's extremes), a row whose
    mean dwarfs its spread, a window with channel/time offsets and a band
    launch."""
    rng = np.random.default_rng(7000 + nt)
    a = np.asfortranarray((rng.standard_normal((1100, 2, nt + 5)) ** 2).astype(np.float32)
                          * 1e6)
    a[5, 1, :] = 7.0
    a[9, 0, 0] = 3e12
    a[11, 1, :] += np.float32(3e9)  # mean / sigma ~ 2000
    x = a[:, :, :nt].copy(order="F")
    xd = dev(eng, x)
    want = orc.kurtosis(x)
    kurt_ok(eng, xd, None, host(eng, eng.kurtosis(xd)), want)
    w = [8, 1088, 1, 0, 2, 1, 5, nt, 1]  # idxs = (9:1096, :, 6:nt+5)
    y = dev(eng, a)
    kurt_ok(eng, y, w, host(eng, eng.kurtosis(y, w)), orc.kurtosis(a, w))
    r = x[::-1].copy(order="F")
    ks = eng.band_kurtosis([xd, dev(eng, r)])
    kurt_ok(eng, xd, None, host(eng, ks[0]), want)
    kurt_ok(eng, xd, None, host(eng, ks[1]), orc.kurtosis(r))


@pytest.mark.parametrize("c0", [1, 2, 3, 5])
@pytest.mark.parametrize("F", [1])
def test_narrow_misaligned_windows(eng, orc, c0, F):
    """Windows starting off a 16-byte boundary with F = 1 (time integration
    of a zoom window, e.g. idxs = (2:n, :, :)): the narrow kernel on the
    window's own (dword-aligned) float4 columns when the channel count is a
    multiple of 4, else the realigning narrow kernel (aligned float4 columns
    summed over T, realigned by lane shuffle).  Integer data, bit-exact for
    every op, two IFs, a ragged last tile, stitched band slots, and a long
    time block split into chunks."""
    rng = np.random.default_rng(10 * c0 + F)
    a = np.asfortranarray(rng.integers(0, 256, (4100, 2, 48)).astype(np.float32))
    nc = (4100 - c0) - (4100 - c0) % 2
    x = dev(eng, a)
    for T, tw in ((8, 48), (48, 48), (3, 12)):
        w = [c0, nc, 1, 0, 2, 1, 0, tw, 1]
        assert eng.plan(x, F, T, "sum", w)["path"] in misaligned_paths(w, F)
        for op in ("sum", "mean", "max", "min"):
            got = host(eng, eng.reduce(x, F, T, op, w))
            want = orc.reduce(a, F, T, op, w)
            if op == "mean":
                np.testing.assert_allclose(got, want, rtol=RTOL)
            else:
                assert same_bits(got, want), (T, op)
    banks = [a] + [np.asfortranarray(rng.integers(0, 256, a.shape).astype(np.float32))
                   for _ in range(2)]
    w = [c0, nc, 1, 1, 1, 1, 4, 40, 1]
    got = host(eng, eng.band_reduce([dev(eng, b) for b in banks], F, 8, "sum", w))
    assert same_bits(got, orc.stitch([orc.reduce(b, F, 8, "sum", w) for b in banks]))
    # few tiles, long time block: partials over time chunks + the finalize
    b = np.asfortranarray(rng.integers(0, 256, (72, 1, 20000)).astype(np.float32))
    y = dev(eng, b)
    for ncw, path in ((64, "narrow"), (62, "narrow_mis")):
        w = [c0, ncw, 1, 0, 1, 1, 0, 20000, 1]
        p = eng.plan(y, F, 20000, "sum", w)
        assert p["path"] == path and p["time_chunks"] > 1
        assert same_bits(host(eng, eng.reduce(y, F, 20000, "sum", w)),
                         orc.reduce(b, F, 20000, "sum", w))


# Unaligned vector paths (BLDP_UNALIGNED_VEC=2): windows that start off a
# 16-byte boundary, and arrays whose channel pitch is not a multiple of 4
# floats (odd nchan), read their own float4 columns with dword-aligned 16-byte
# loads.  (nchan, nif, ntime, window, F, T, expected paths)
UNALIGNED_CASES = [
    (4100, 2, 48, [1, 4096, 1, 0, 2, 1, 0, 48, 1], 64, 16, {"row", "vector"}),
    (4100, 1, 48, [3, 4096, 1, 0, 1, 1, 0, 48, 1], 4, 48, {"row", "vector"}),
    (4100, 2, 32, [2, 4080, 1, 1, 1, 1, 0, 32, 1], 20, 8, {"vector"}),
    (4100, 1, 64, [1, 4096, 1, 0, 1, 1, 0, 64, 1], 256, 2, {"row"}),
    (4100, 1, 16, [1, 4096, 1, 0, 1, 1, 0, 16, 1], 1, 16, {"narrow"}),
    (516, 1, 20000, [3, 512, 1, 0, 1, 1, 0, 19456, 1], 8, 1024, {"vector"}),  # cfg4-like
    (4097, 3, 40, [0, 4096, 1, 0, 3, 1, 0, 40, 1], 1024, 8, {"interleaved"}),  # odd pitch
    (4097, 2, 40, [1, 4096, 1, 0, 2, 1, 0, 40, 1], 64, 8, {"row"}),            # odd pitch
    (4097, 2, 40, [1, 4092, 1, 0, 2, 1, 0, 40, 1], 2, 8, {"narrow"}),         # odd pitch
    (4097, 1, 24, [1, 4095, 1, 0, 1, 1, 0, 24, 1], 3, 8, {"lane"}),           # odd pitch, odd F
    (4097, 2, 24, [2, 4090, 1, 0, 2, 1, 0, 24, 1], 5, 4, {"lane"}),
    (4100, 1, 40, [3, 4092, 1, 0, 1, 1, 0, 40, 1], 6, 8, {"lane"}),           # (lanet at tavby 8)
    (4100, 1, 40, [0, 4095, 1, 0, 1, 1, 0, 40, 1], 7, 20, {"tile"}),
    (4097, 1, 40, [3, 4092, 1, 0, 1, 1, 0, 40, 1], 6, 8, {"lane"}),           # odd pitch
    (4097, 1, 40, [0, 4095, 1, 0, 1, 1, 0, 40, 1], 7, 20, {"lane"}),          # odd pitch
    (4097, 1, 40, [1, 4094, 1, 0, 1, 1, 0, 40, 1], 2, 8, {"lane"}),           # odd pitch
    (71, 1, 30000, [1, 63, 1, 0, 1, 1, 0, 30000, 1], 3, 30000, {"lane"}),  # time chunks
    (4095, 1, 8, [0, 4095, 1, 0, 1, 1, 0, 8, 1], 5, 8, {"lane"}),             # ends at the array end
    (4096, 2, 8, [4, 4089, 1, 0, 2, 1, 0, 8, 1], 3, 8, {"lane"}),
    (4097, 1, 24, [1, 4095, 1, 0, 1, 1, 0, 24, 1], 4095, 8, {"scalar"}),      # odd pitch, wide F
]


@pytest.mark.parametrize("case", UNALIGNED_CASES, ids=range(len(UNALIGNED_CASES)))
def test_unaligned_vector_paths(eng, orc, case):
    """Integer data: bit-exact for sum/max/min against the oracle, mean at
    RTOL; the path is the one the plan rule names; a 3-bank stitched band."""
    nc, ni, nt, win, F, T, paths = case
    rng = np.random.default_rng(nc * 7 + F)
    a = np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
    x = dev(eng, a)
    assert eng.plan(x, F, T, "sum", win)["path"] in paths, case
    for op in ("sum", "max", "min", "mean"):
        got = host(eng, eng.reduce(x, F, T, op, win))
        want = orc.reduce(a, F, T, op, win)
        if op == "mean":
            np.testing.assert_allclose(got, want, rtol=RTOL)
        else:
            assert same_bits(got, want), (case, op)
    banks = [a] + [np.asfortranarray(rng.integers(0, 256, a.shape).astype(np.float32))
                   for _ in range(2)]
    got = host(eng, eng.band_reduce([dev(eng, b) for b in banks], F, T, "sum", win))
    assert same_bits(got, orc.stitch([orc.reduce(b, F, T, "sum", win) for b in banks]))


def test_unaligned_vector_special_values(eng, orc):
    """NaN / Inf / -0.0 through the unaligned row and narrow paths (Julia's
    max/min semantics, bit-exact)."""
    a = np.zeros((68, 1, 4), np.float32, order="F")
    a[1:5, 0, 0] = -0.0
    a[5:9, 0, 1] = [-0.0, 0.0, -0.0, -0.0]
    a[9:13, 0, 2] = [1.0, np.nan, 2.0, 3.0]
    a[13:17, 0, 3] = [np.inf, 1.0, -np.inf, 0.0]
    a[17:21, 0, 0] = [np.inf, 1.0, 5.0, 0.0]
    x = dev(eng, a)
    win = [1, 64, 1, 0, 1, 1, 0, 4, 1]
    for F, T in [(4, 1), (8, 2), (1, 4), (16, 4)]:
        assert eng.plan(x, F, T, "max", win)["path"] in ("row", "vector", "narrow")
        for op in ("sum", "max", "min"):
            got = host(eng, eng.reduce(x, F, T, op, win))
            want = orc.reduce(a, F, T, op, win)
            if op == "sum":
                assert np.array_equal(np.isnan(got), np.isnan(want))
                fin = np.isfinite(want)
                assert np.array_equal(got[fin], want[fin])
            else:
                assert same_bits(got, want), (F, T, op)


# Time blocks that are not a multiple of a kernel's row batch (tavby = 3, 8, 9,
# 15, 17, 24): the rows after the last full batch are loaded together and then
# chained in row order (BLDP_TAIL_BATCH); row, narrow, misaligned narrow and
# vector plans, bit-exact on integer data, with a partial window.
TAIL_CASES = [(64, None, ("row", "vector")), (2, None, ("narrow",)), (1, None, ("narrow",)),
              (8, None, ("vector", "row")), (1, [1, 4094, 1, 0, 1, 1, 0, None, 1], ("narrow_mis",)),
              (12, None, ("vector", "lane")), (24, None, ("vector",)), (48, None, ("vector",)),
              (96, None, ("vector",)), (768, None, ("vector", "interleaved"))]


@pytest.mark.parametrize("T", [3, 8, 9, 15, 17, 24])
@pytest.mark.parametrize("case", TAIL_CASES, ids=lambda c: f"F{c[0]}-{c[2][0]}")
def test_reduce_block_tails_integer_exact(eng, orc, case, T):
    F, w, path = case
    nt = 3 * T + 5  # three blocks and a few spectra over
    x = eng.synth(4096, 1, nt, 1024, seed=97 * F + T, kind=1)
    a = host(eng, x)
    win = list(w) if w is not None else [0, 4096 // F * F, 1, 0, 1, 1, 0, None, 1]
    win[7] = nt // T * T
    for op in ("sum", "max", "min"):
        plan = eng.plan(x, F, T, op, win)
        assert plan["path"] in path, (F, T, plan)
        got = host(eng, eng.reduce(x, F, T, op, win))
        assert same_bits(got, orc.reduce(a, F, T, op, win)), (F, T, op, path)


# Groups wider than 4096 channels (fqavby = 16384, 65536: K4 > 16 float4 per
# lane per row) with few outputs split their rows over waves and time chunks by
# the work in a row (BLDP_WIDE_SPLIT); max / min bit-exact, sums within 1e-5.
@pytest.mark.parametrize("F", [16384, 65536])
@pytest.mark.parametrize("T", [3, 8, 9, 31])
def test_reduce_wide_groups_time_split(eng, orc, F, T):
    nt = 279 // T * T
    x = eng.synth(65536, 1, 279, 1024, seed=F + T, kind=1)
    a = host(eng, x)
    w = [0, 65536, 1, 0, 1, 1, 0, nt, 1]
    plan = eng.plan(x, F, T, "sum", w)
    assert plan["path"] == "vector", plan
    for op in ("max", "min"):
        got = host(eng, eng.reduce(x, F, T, op, w))
        assert same_bits(got, orc.reduce(a, F, T, op, w)), (F, T, op, plan)
    # (sums of F x T bytes pass 2^24: Float32 rounds them, so the 1e-5 bound)
    got = host(eng, eng.reduce(x, F, T, "sum", w))
    np.testing.assert_allclose(got, orc.reduce(a, F, T, "sum", w), rtol=RTOL)
    g = orc.gamma_bandpass(65536, 1, nt, 1024, 3 * T)
    got = host(eng, eng.reduce(dev(eng, g), F, T, "mean"))
    np.testing.assert_allclose(got, orc.reduce(g, F, T, "mean"), rtol=RTOL)


@pytest.mark.parametrize("nc", [512, 1024])
def test_wavet_bank_pack_stitched(pkg, eng, orc, nc):
    """k_reduce_wavet with one wave per (bank, group) of a <= 16-group
    stitched row (plan option wave_bpack: the 0001 band at fqavby = 512)
    against the per-wave form and the oracle: 2, 3, 8 (and 16 at one group a
    bank) banks, T = 1, 2, 3, 4, partial last workgroups, every op."""
    rng = np.random.default_rng(nc)
    for nb in ((2, 3, 8, 16) if nc == 512 else (2, 3, 8)):
        for T, nt, ni in ((1, 1001, 1), (2, 402, 1), (3, 303, 1), (4, 100, 1), (1, 64, 3)):
            data = [np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
                    for _ in range(nb)]
            xs = [dev(eng, a) for a in data]
            assert eng.plan(xs[0], 512, T, "sum")["path"] == "vector"
            for op in ("sum", "mean", "max", "min"):
                got = host(eng, eng.band_reduce(xs, 512, T, op))
                with pkg._lib.plan_option("wave_bpack", 0):
                    ref = host(eng, eng.band_reduce(xs, 512, T, op))
                assert same_bits(got, ref), (nc, nb, T, op)
                want = orc.stitch([orc.reduce(a, 512, T, op) for a in data])
                assert same_bits(got, want), (nc, nb, T, op)


@pytest.mark.parametrize("T", [1, 2, 3, 4, 8])
def test_col3_fqavby12_short_blocks(pkg, eng, orc, T):
    """k_reduce_col3 (fqavby = 12 with short time blocks: float4 columns,
    three lanes a group, 64 groups of the stitched row per workgroup) against
    the oracle: integer data bit for bit (and equal to k_reduce_lanet, plan
    option col3 = 0), Float32 data within RTOL; 1, 2, 3 and 8 banks, the 0001
    row width and a wide row, a misaligned channel window, two IFs, partial
    last time groups."""
    rng = np.random.default_rng(T)
    for nc, ni, nt, nbs in ((512, 1, 16 * T * 7 + T, (1, 2, 3, 8)), (8192, 2, 24 * T, (1, 3))):
        for nb in nbs:
            ints = [np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
                    for _ in range(nb)]
            xs = [dev(eng, a) for a in ints]
            for win in (None, [1, nc // 12 * 12 - 12, 1, 0, ni, 1, 0, nt, 1]):
                w = win or [0, nc // 12 * 12, 1, 0, ni, 1, 0, nt, 1]
                for op in ("sum", "mean", "max", "min"):
                    got = host(eng, eng.band_reduce(xs, 12, T, op, w))
                    want = orc.stitch([orc.reduce(a, 12, T, op, w) for a in ints])
                    assert same_bits(got, want), (nc, nb, T, op, w)
                    with pkg._lib.plan_option("col3", 0):
                        ref = host(eng, eng.band_reduce(xs, 12, T, op, w))
                    assert same_bits(got, ref), (nc, nb, T, op, w)
            gam = [orc.gamma_bandpass(nc, ni, nt, 64, 31 * T + k) for k in range(nb)]
            xs = [dev(eng, a) for a in gam]
            w = [0, nc // 12 * 12, 1, 0, ni, 1, 0, nt, 1]
            got = host(eng, eng.band_reduce(xs, 12, T, "sum", w))
            want = orc.stitch([orc.reduce(a, 12, T, "sum", w) for a in gam])
            np.testing.assert_allclose(got, want, rtol=RTOL)


@pytest.mark.parametrize("F", [3, 5, 6, 7])
def test_lanes_along_stitched_rows(pkg, eng, orc, F):
    """k_reduce_lanes (plan option lane_bpack: k_reduce_lanet's lanes along
    the stitched product row of a band of narrow banks, the 0001 band at
    fqavby = 3) against k_reduce_lanet and the oracle: 2, 3 and 8 banks,
    T = 1, 2, 3, 4, 8, partial last time groups, a channel window, every op."""
    rng = np.random.default_rng(F + 7)
    nc = 512 // F * F
    for nb in (2, 3, 8):
        for T, nt, ni in ((1, 1001, 1), (2, 300, 1), (3, 297, 1), (4, 100, 1), (8, 200, 1),
                          (1, 120, 2)):
            data = [np.asfortranarray(rng.integers(0, 256, (512, ni, nt)).astype(np.float32))
                    for _ in range(nb)]
            xs = [dev(eng, a) for a in data]
            for win in ([0, nc, 1, 0, ni, 1, 0, nt, 1], [F, nc - F, 1, 0, ni, 1, 0, nt, 1]):
                for op in ("sum", "mean", "max", "min"):
                    got = host(eng, eng.band_reduce(xs, F, T, op, win))
                    with pkg._lib.plan_option("lane_bpack", 0):
                        ref = host(eng, eng.band_reduce(xs, F, T, op, win))
                    assert same_bits(got, ref), (F, nb, T, op, win)
                    want = orc.stitch([orc.reduce(a, F, T, op, win) for a in data])
                    assert same_bits(got, want), (F, nb, T, op, win)


@pytest.mark.parametrize("F", [64, 128, 16])
def test_rowt_bank_pack_stitched(pkg, eng, orc, F):
    """k_reduce_rowt with its lane sets over consecutive banks (plan option
    row_bpack: a stitched band of narrow banks, the 0001 band at fqavby = 64,
    so each product row gets whole segments of two banks) against the time-
    group form and the oracle: 2, 3 (odd: no packing), 4 and 8 banks, T = 1,
    2, 4, partial last time groups, every op; F = 16 (128-byte segments) is
    never packed."""
    rng = np.random.default_rng(F + 1)
    for nb in (2, 3, 4, 8):
        for T, nt, ni in ((1, 4001, 1), (2, 1000, 1), (4, 968, 1), (1, 300, 2)):
            data = [np.asfortranarray(rng.integers(0, 256, (512, ni, nt)).astype(np.float32))
                    for _ in range(nb)]
            xs = [dev(eng, a) for a in data]
            for op in ("sum", "mean", "max", "min"):
                got = host(eng, eng.band_reduce(xs, F, T, op))
                with pkg._lib.plan_option("row_bpack", 0):
                    ref = host(eng, eng.band_reduce(xs, F, T, op))
                assert same_bits(got, ref), (F, nb, T, op)
                want = orc.stitch([orc.reduce(a, F, T, op) for a in data])
                assert same_bits(got, want), (F, nb, T, op)



@pytest.mark.parametrize("F", [4, 16, 64, 256])
def test_row_split_forms_bit_identical(pkg, eng, orc, F):
    """k_reduce_row and its row-split forms (k_reduce_rows, a time block's
    16-row batches over 2 / 4 slices of a workgroup: the single-file launch
    of the per-file getdata shape) give the same bits, for every op; integer
    data matches the oracle exactly, gamma data within RTOL; partial last
    column blocks, several banks, an IF axis and a stitched band."""
    rng = np.random.default_rng(F)
    # (shapes with >= 16 waves' worth of row tiles: fewer take the vector
    # path's time split over waves instead of the row kernel)
    for nc, ni, nt, T, nb in ((65536, 1, 272, 16, 1), (65536 + 4 * F, 8, 64, 32, 1),
                              (65536, 1, 272, 16, 3)):
        ints = [np.asfortranarray(rng.integers(0, 256, (nc, ni, nt)).astype(np.float32))
                for _ in range(nb)]
        gam = [orc.gamma_bandpass(nc, ni, nt, 64, 100 * F + k) for k in range(nb)]
        for data, exact in ((ints, True), (gam, False)):
            xs = [dev(eng, a) for a in data]
            for op in ("sum", "mean", "max", "min"):
                outs = {}
                for S in (1, 2, 4):
                    with pkg._lib.plan_option("row_split", S):
                        pl = eng.plan(xs[0], F, T, op)
                        assert pl["path"] == "row" and pl["time_split_waves"] == S, pl
                        outs[S] = host(eng, eng.band_reduce(xs, F, T, op))
                assert same_bits(outs[2], outs[1]) and same_bits(outs[4], outs[1]), (nc, F, T, op)
                want = orc.stitch([orc.reduce(a, F, T, op) for a in data])
                if exact or op in ("max", "min"):
                    assert same_bits(outs[1], want), (nc, F, T, op)
                else:
                    np.testing.assert_allclose(outs[1], want, rtol=RTOL)
    # the planner's own choice on one 0002 file at fqavby = 64, tavby = 16
    x = dev(eng, np.zeros((65536, 1, 16), np.float32))
    assert eng.plan(x, 64, 16)["time_split_waves"] in (2, 4)


def test_rowt_small_launch_tavby8_long_narrow_window(eng, orc):
    """A small launch at tavby = 8 on a narrow window (256 channels) with more
    than 65535 time blocks: the 8-rows-per-lane downgrade would be
    k_reduce_row, whose grid y (IF x time block) cannot hold them, so the
    plan keeps k_reduce_rowt; the result matches the oracle."""
    rng = np.random.default_rng(8)
    nto = 70000
    a = np.asfortranarray(rng.integers(0, 256, (256, 1, 8 * nto)).astype(np.float32))
    x = dev(eng, a)
    for F in (4, 64):
        got = host(eng, eng.reduce(x, F, 8))
        assert same_bits(got, orc.reduce(a, F, 8)), F
    # and where the grid does hold them, T = 8 on a small launch is k_reduce_row
    b = np.asfortranarray(rng.integers(0, 256, (65536, 1, 272)).astype(np.float32))
    y = dev(eng, b)
    assert eng.plan(y, 64, 8)["path"] == "row"
    assert same_bits(host(eng, eng.reduce(y, 64, 8)), orc.reduce(b, 64, 8))


# Every runtime plan option (bldp_plan_option) at every value: each form of a
# plan the planner can take must give the oracle's results (integer data:
# exact in any summation order), so a plan choice is a pure speed choice.
PLAN_OPTION_VALUES = {
    "row_split": (1, 2, 4), "ts_fill": (0, 1), "narrow_mis": (0, 1),
    "t38": (0, 1), "wide_split": (0, 1), "narrow_tpb": (0, 1, 2), "lane": (0, 1),
    "lane3": (0, 1), "lanet": (0, 1), "lanet_pack": (0, 1), "vec_il": (0, 1), "vec_row": (0, 1),
    "row_tpb": (0, 1), "rowt_pack": (0, 1), "rowt_small": (0, 64, 100000), "wavet": (0, 1),
    "unaligned_vec": (0, 1, 2), "row_bpack": (0, 1), "lane_bpack": (0, 1),
    "wave_bpack": (0, 1), "col3": (0, 1), "rowt_narrow8": (0, 1),
    "st_plain": (0, 1, 2),
}
# (nchan, nif, ntime, window, F, T): shapes where the options above change the plan
PLAN_OPTION_SHAPES = [
    (65536, 1, 64, None, 64, 16), (65536, 1, 64, None, 64, 1), (65536, 1, 48, None, 64, 3),
    (65536, 1, 64, None, 64, 8), (512, 1, 4096, None, 8, 1), (512, 1, 4096, None, 64, 4),
    (512, 1, 2048, None, 8, 512), (512, 1, 4096, None, 512, 1), (65536, 1, 16, None, 1024, 16),
    (65536, 1, 16, None, 1024, 1), (65535, 1, 24, None, 3, 1), (65532, 1, 24, None, 12, 2),
    (4096, 2, 40, [1, 4092, 1, 0, 2, 1, 0, 40, 1], 1, 4),
    (4096, 2, 40, [2, 4092, 1, 0, 2, 1, 0, 40, 1], 2, 5),
    (4096, 1, 40, [3, 4032, 1, 0, 1, 1, 0, 40, 1], 64, 8), (4095, 1, 40, None, 3, 10),
    (4095, 1, 40, None, 5, 1), (65536, 1, 24, None, 65536, 8), (4096, 1, 64, None, 2, 1),
    (4096, 1, 64, None, 1, 1), (4096, 1, 63, None, 2, 3), (131072, 1, 8, None, 4, 8),
    # 0001-like narrow rows on the lane path (k_reduce_lanet)
    (512, 1, 4096, [0, 510, 1, 0, 1, 1, 0, 4096, 1], 3, 1),
    (512, 1, 4000, [0, 504, 1, 0, 1, 1, 0, 4000, 1], 12, 1),
    (512, 2, 100, [0, 510, 1, 0, 2, 1, 0, 100, 1], 3, 2),
    (512, 1, 1000, [1, 507, 1, 0, 1, 1, 0, 1000, 1], 3, 4),
    (512, 1, 300, [0, 510, 1, 0, 1, 1, 0, 300, 1], 6, 1),
    (512, 1, 300, [0, 504, 1, 0, 1, 1, 0, 300, 1], 7, 1),
    # narrow rows at fqavby 64 / 128 (row_bpack on the two-bank stitch)
    (512, 1, 4001, None, 64, 1), (512, 1, 1000, None, 128, 2),
    # interleaved groups with two IFs, a window, an odd group count (the last
    # segment half full) and time blocks shorter than the rows in flight
    (8192, 2, 40, [256, 7680, 1, 0, 2, 1, 0, 40, 1], 512, 5),
]


@pytest.mark.parametrize("name", sorted(PLAN_OPTION_VALUES))
def test_plan_options_every_form(pkg, eng, orc, name):
    rng = np.random.default_rng(len(name))
    cases = []
    for nc, ni, nt, win, F, T in PLAN_OPTION_SHAPES:
        top = min(255, (2 ** 24 - 1) // (F * T))  # every Float32 group sum exact (< 2^24)
        a = np.asfortranarray(rng.integers(0, top + 1, (nc, ni, nt)).astype(np.float32))
        cases.append((a, dev(eng, a), win, F, T))
    paths = set()
    for val in PLAN_OPTION_VALUES[name]:
        with pkg._lib.plan_option(name, val):
            for a, x, win, F, T in cases:
                for op in ("sum", "max"):
                    paths.add(eng.plan(x, F, T, op, win)["path"])
                    got = host(eng, eng.reduce(x, F, T, op, win))
                    assert same_bits(got, orc.reduce(a, F, T, op, win)), \
                        (name, val, a.shape, win, F, T, op)
                # two banks stitched
                got = host(eng, eng.band_reduce([x, x], F, T, "sum", win))
                want = orc.reduce(a, F, T, "sum", win)
                assert same_bits(got, orc.stitch([want, want])), (name, val, a.shape, F, T)
    assert paths


KURT_OPTION_VALUES = {"kurt_exact": (0, 1), "kurt_mid_cpl": (1, 2), "kurt_mid_small": (0, 1),
                      "kurt_leaf_narrow": (0, 4), "kurt_leaf_tile": (0, 1),
                      "unaligned_vec": (0, 2)}


@pytest.mark.parametrize("name", sorted(KURT_OPTION_VALUES))
def test_kurtosis_plan_options_every_form(pkg, eng, orc, name):
    """The kurtosis plan options at every value against the oracle, each at
    the tolerance of the path the plan took."""
    rng = np.random.default_rng(7 + len(name))
    shapes = [(4096, 1, 16, None), (4096, 1, 32, None), (8192, 1, 48, None), (8192, 1, 279, None),
              (512, 1, 3000, None), (512, 2, 1500, None), (4096, 1, 40, [1, 4092, 1, 0, 1, 1, 0, 40, 1])]
    for nc, ni, nt, win in shapes:
        a = np.asfortranarray(rng.gamma(20.0, 1e6, (nc, ni, nt)).astype(np.float32))
        x = dev(eng, a)
        want = orc.kurtosis(a, win)
        for val in KURT_OPTION_VALUES[name]:
            with pkg._lib.plan_option(name, val):
                kurt_ok(eng, x, win, host(eng, eng.kurtosis(x, win)), want, (name, val, nc, nt))
