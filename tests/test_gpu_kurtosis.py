"""GPU parity of getkurtosis (src/gbtworkerfunctions.jl:197-202) against the
oracle, in the regime the product is used in: integrated BL power, whose
mean/sigma = sqrt(N_avg) runs from tens to tens of thousands.  There a
one-ulp change of StatsBase's Float32 mean m moves the excess kurtosis by
~4 * skew * ulp(m) / sigma, so every path must reproduce Julia's pairwise
Float32 sum exactly (tests/test_oracle.py pins the oracle's).

Tolerances (tests/conftest.py assert_kurtosis), by the path that ran:
  regs     (<= 32 spectra)      bit-exact
  mid      (33..512, or <= 32 without float4 columns)  6 nt 2^-53 relative
                                 on k + 3 (Float64 order)
  leaf     (> 512, float4 columns)  13 * 2^-24 * 1.05 relative on k + 3
                                 (Float32 rounding of z^2, z^4 in the recipe)
  twopass  (> 512 without float4 columns)  6 nt 2^-53 relative on k + 3
"float4 columns": unit channel step and a channel count that is a multiple of
4; the start and the pitches need only dword alignment (gfx950 16-byte loads).
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import assert_kurtosis

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(pkg):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    pkg._lib.lib()
    return pkg.engine


def dev(eng, a):
    return eng.fb_from_numpy(a, device="cuda:0")


def host(eng, t):
    return eng.fb_to_numpy(t)


def power_rows(rng, nc, ni, nt, nfpc=64):
    """Integrated-power filterbank: channel c has mean/sigma R[c % 5] of
    {1.4, 30, 300, 3000, 30000} (gamma with shape R^2, i.e. N_avg = R^2
    spectra of chi^2(2) power), times a per-coarse-channel scallop."""
    R = np.array([np.sqrt(2.0), 30.0, 300.0, 3000.0, 30000.0])[np.arange(nc) % 5]
    x = np.arange(nc) % nfpc
    bp = 0.2 + 0.8 * np.sin(np.pi * (x + 0.5) / nfpc) ** 2
    g = rng.gamma((R ** 2)[None, None, :], (1e9 / R ** 2 * bp)[None, None, :], (nt, ni, nc))
    return np.asfortranarray(g.astype(np.float32).transpose(2, 1, 0))


def unaligned(nt):
    """The path of a window whose channels cannot be read as float4 (count
    not a multiple of 4, or a channel step)."""
    return "mid" if nt <= 512 else "twopass"


def check(eng, orc, a, win=None, expect=None, msg=""):
    x = dev(eng, a)
    plan = eng.kurtosis_plan(x, win)
    if expect:
        assert plan["path"] == expect, (plan, msg)
    got = host(eng, eng.kurtosis(x, win))
    want = orc.kurtosis(a, win)
    nt = orc.window_shape(a.shape, win)[2]
    assert_kurtosis(got, want, plan["path"], nt, (msg, win))
    return plan


PATH_NT = [(7, "regs"), (16, "regs"), (32, "regs"), (33, "mid"), (48, "mid"), (64, "mid"),
           (65, "mid"), (100, "mid"), (272, "mid"),
           (385, "mid"), (512, "mid"), (513, "leaf"), (1024, "leaf"), (1025, "leaf"),
           (2048, "leaf"), (2049, "leaf"), (5007, "leaf"), (20000, "leaf")]


@pytest.mark.parametrize("nt,path", PATH_NT, ids=[f"{n}-{p}" for n, p in PATH_NT])
def test_kurtosis_integrated_power_rows(eng, orc, nt, path):
    """Every path on integrated-power rows (mean/sigma up to 3e4), aligned and
    unaligned (two-pass) windows, a band launch."""
    rng = np.random.default_rng(nt)
    nc = 1000 if nt <= 512 else 260
    a = power_rows(rng, nc, 2, nt)
    check(eng, orc, a, None, path, "aligned")
    # unaligned channel start -> lane-per-channel tile or two passes (same m)
    w = [1, nc - 3, 1, 0, 2, 1, 0, nt, 1]
    check(eng, orc, a, w, unaligned(nt), "unaligned")
    # time window starting inside the data (aligned channels, shifted leaves)
    if nt > 8:
        w = [4, nc - 4, 1, 1, 1, 1, 3, nt - 5, 1]
        check(eng, orc, a, w, None, "time window")
    b = power_rows(rng, nc, 2, nt)
    ks = eng.band_kurtosis([dev(eng, a), dev(eng, b)])
    pth = eng.kurtosis_plan(dev(eng, a))["path"]
    for arr, k in zip((a, b), ks):
        assert_kurtosis(host(eng, k), orc.kurtosis(arr), pth, nt, "band")


@pytest.mark.parametrize("nt", [513, 1000, 1024, 1025, 3000, 8192])
def test_kurtosis_short_windows_of_narrow_products(eng, orc, nt):
    """Short windows of a narrow product (the 0001 shape: 512 channels, a
    band of 3 banks): few leaves and few channels, so every leaf is read
    whole into registers (k_kurt_tile: the recipe itself for nt <= 1024, leaf
    partials and the tree above that).  Also a window whose channel count is
    not a multiple of a workgroup's channels and that starts off a float4."""
    rng = np.random.default_rng(7000 + nt)
    arrs = [power_rows(rng, 512, 1, nt + 3) for _ in range(3)]
    for w in ([0, 512, 1, 0, 1, 1, 0, nt, 1], [4, 500, 1, 0, 1, 1, 3, nt, 1]):
        assert eng.kurtosis_plan(dev(eng, arrs[0]), w)["path"] == "leaf"
        ks = eng.band_kurtosis([dev(eng, a) for a in arrs], w)
        for a, k in zip(arrs, ks):
            assert_kurtosis(host(eng, k), orc.kurtosis(a, w), "leaf", nt, w)


@pytest.mark.parametrize("nt,nc", [(140000, 64), (600000, 16), (2200001, 8)])
def test_kurtosis_tree_passes(eng, orc, nt, nc):
    """Long windows whose pairwise tree has K > 6 levels above the blocks, so
    the merge runs 1 or 2 tree passes before the per-output wave (nt =
    140000: K = 7; 600000: K = 9, the cfg4 depth; 2200001: K = 11), aligned
    and unaligned."""
    rng = np.random.default_rng(nt)
    a = power_rows(rng, nc, 1, nt)
    p = check(eng, orc, a, None, "leaf", "aligned")
    assert p["K"] > 6
    check(eng, orc, a, [1, nc - 2, 1, 0, 1, 1, 0, nt, 1], "twopass", "unaligned")


def test_kurtosis_cfg4_band_spot_rows(eng, orc):
    """cfg4 at full size (8 banks x 512 ch x 880000 spectra, window 1:879616,
    one band launch): spot rows of two banks against the oracle, one bank
    shifted to integrated-power levels (mean/sigma ~ 140)."""
    import torch

    n = 880000
    banks = eng.band_empty(8, 512, 1, n)
    for b, v in enumerate(banks):
        eng.synth(512, 1, n, 8, seed=400 + b, kind=0, out=v)
    banks[3].add_(1e11)
    w = [0, 512, 1, 0, 1, 1, 0, 879616, 1]
    assert eng.kurtosis_plan(banks[0], w)["path"] == "leaf"
    ks = eng.band_kurtosis(banks, w)
    for b in (0, 3):
        a = np.asfortranarray(banks[b][:64].cpu().numpy())
        sub = [0, 64, 1, 0, 1, 1, 0, 879616, 1]
        assert_kurtosis(host(eng, ks[b])[:64], orc.kurtosis(a, sub), "leaf", 879616, b)
        a = np.asfortranarray(banks[b][448:].cpu().numpy())
        assert_kurtosis(host(eng, ks[b])[448:], orc.kurtosis(a, sub), "leaf", 879616, b)
    del banks, ks
    torch.cuda.empty_cache()


@pytest.mark.parametrize("nt", [1, 2, 16, 300, 1500, 5000])
def test_kurtosis_special_rows(eng, orc, nt):
    """Rows the recipe turns into NaN or Inf, on every path: a constant row
    (0/0), an outlier whose Float32 z^4 (or z^2) overflows, a NaN, an Inf,
    values so small that every Float32 z^2 underflows, a row of one repeated
    value plus a few ulps (m decides everything there)."""
    rng = np.random.default_rng(50 + nt)
    a = power_rows(rng, 64, 1, nt)
    a[1, 0, :] = 7.0
    a[2, 0, 0] = 3e12                       # z^4 overflows
    a[3, 0, nt // 2] = 2e19                 # z^2 overflows
    a[4, 0, nt - 1] = np.nan
    a[5, 0, 0] = np.inf
    a[6, 0, :] = (rng.random(nt) * 1e-30).astype(np.float32)  # z^2 underflows
    ulp = np.spacing(np.float32(1e9))
    a[7, 0, :] = np.float32(1e9) + ulp * rng.integers(-3, 4, nt).astype(np.float32)
    a[8, 0, :] = -a[0, 0, :]
    check(eng, orc, a, None, None, "aligned")
    check(eng, orc, a, [1, 62, 1, 0, 1, 1, 0, nt, 1], unaligned(nt), "unaligned")


@pytest.mark.parametrize("nt,path", [(16, "regs"), (32, "regs"), (100, "mid"), (384, "mid"),
                                     (600, "leaf"), (5007, "leaf")])
def test_kurtosis_unaligned_float4_windows(eng, orc, nt, path):
    """Windows starting off a 16-byte boundary whose channel count is a
    multiple of 4, and arrays with an odd channel pitch: the register and
    streamed-leaf paths on dword-aligned 16-byte loads (bit-exact on regs),
    k_kurt_mid2 on dword-aligned 8-byte loads (100 and 384 spectra: 13 and 48
    per wave)."""
    rng = np.random.default_rng(1000 + nt)
    a = power_rows(rng, 260, 2, nt)
    check(eng, orc, a, [1, 256, 1, 0, 2, 1, 0, nt, 1], path, "c0=1")
    check(eng, orc, a, [3, 252, 1, 1, 1, 1, 0, nt, 1], path, "c0=3, second IF")
    b = power_rows(rng, 257, 2, nt)  # channel pitch 257 floats
    check(eng, orc, b, [1, 256, 1, 0, 2, 1, 0, nt, 1], path, "odd pitch")
    check(eng, orc, b, [0, 256, 1, 1, 1, 1, 0, nt, 1], path, "odd pitch, c0=0")
    ks = eng.band_kurtosis([dev(eng, b), dev(eng, b)], [2, 252, 1, 0, 2, 1, 0, nt, 1])
    want = orc.kurtosis(b, [2, 252, 1, 0, 2, 1, 0, nt, 1])
    for k in ks:
        assert_kurtosis(host(eng, k), want, path, nt, "band")


def test_kurtosis_empty_and_degenerate_windows(eng, orc):
    a = power_rows(np.random.default_rng(3), 64, 2, 40)
    x = dev(eng, a)
    assert tuple(eng.kurtosis(x, [0, 0, 1, 0, 2, 1, 0, 40, 1]).shape) == (0, 2)
    k = host(eng, eng.kurtosis(x, [0, 64, 1, 0, 2, 1, 5, 0, 1]))  # no spectra: NaN
    assert k.shape == (64, 2) and np.isnan(k).all()
    assert np.isnan(orc.kurtosis(a, [0, 64, 1, 0, 2, 1, 5, 0, 1])).all()
    check(eng, orc, a, [63, 64, -1, 1, 2, -1, 39, 40, -1], "mid", "reversed")
    check(eng, orc, a, [0, 32, 2, 0, 2, 1, 0, 20, 2], "mid", "strided")
    b = power_rows(np.random.default_rng(4), 64, 2, 1500)
    check(eng, orc, b, [63, 64, -1, 1, 2, -1, 1499, 1500, -1], "twopass", "reversed long")


def test_kurtosis_caller_workspace(eng, orc, pkg):
    """bldp_kurtosis_f32 with a caller-owned workspace of
    bldp_kurtosis_workspace_size bytes (enough for the aligned and the
    unaligned plan of the window)."""
    import torch

    L = pkg._lib.lib()
    rng = np.random.default_rng(9)
    a = power_rows(rng, 256, 1, 3000)
    for win in (None, [1, 254, 1, 0, 1, 1, 7, 2990, 1]):
        keep, wp = pkg._lib.win_arg(win if win is not None else [0, 256, 1, 0, 1, 1, 0, 3000, 1])
        sz = L.bldp_kurtosis_workspace_size(256, 1, 3000, wp)
        ws = torch.full((sz + 8,), 255, dtype=torch.uint8, device="cuda:0")
        x = dev(eng, a)
        nc = 256 if win is None else 254
        out = torch.empty((nc,), dtype=torch.float64, device="cuda:0")
        rc = L.bldp_kurtosis_f32(x.data_ptr(), 256, 1, 3000, wp, out.data_ptr(), ws.data_ptr(),
                                 pkg._lib.stream_ptr())
        assert rc == 0, pkg._lib.last_error()
        path = eng.kurtosis_plan(x, win)["path"]
        want = orc.kurtosis(a, win)[:, 0]
        assert_kurtosis(out.cpu().numpy(), want, path, 3000 if win is None else 2990)


def test_kurtosis_host_drop_in_long_window(eng, orc):
    """bldp_kurtosis_host_f32 (the Julia drop-in on a host array) stages the
    window and runs the same kernels."""
    rng = np.random.default_rng(77)
    a = power_rows(rng, 512, 1, 4000)
    got = eng.kurtosis_host(a)
    assert_kurtosis(got, orc.kurtosis(a), "leaf", 4000)
    w = [2, 500, 1, 0, 1, 1, 10, 3000, 1]
    got = eng.kurtosis_host(a, w)  # (leaf or two-pass, by the staged buffer's alignment)
    assert_kurtosis(got, orc.kurtosis(a, w), "leaf", 3000)


def test_kurtosis_and_chunked_reduce_from_threads_share_scratch(eng, orc):
    """Host threads sharing torch's current stream (the GBT fan-out runs one
    thread per (worker, file)) and the library scratch of that stream:
    long-window kurtosis (leaf partials + tree) and time-chunked reductions
    (partials + finalize) from 8 threads at once, every result against the
    oracle.  The scratch lease serialises the calls' launches on the stream."""
    from concurrent.futures import ThreadPoolExecutor

    import torch

    rng = np.random.default_rng(123)
    arrs = [power_rows(rng, 256, 1, int(n)) for n in (1500, 2600, 5007, 7000)] * 2
    ints = [np.asfortranarray(rng.integers(0, 256, (64, 1, 20000)).astype(np.float32))
            for _ in range(4)]
    xs = [dev(eng, a) for a in arrs]
    ys = [dev(eng, a) for a in ints]
    assert eng.plan(ys[0], 8, 20000)["time_chunks"] > 1  # scratch partials

    def kjob(x):
        return host(eng, eng.kurtosis(x))

    def rjob(y):
        return host(eng, eng.reduce(y, 8, 20000))

    for _ in range(3):
        with ThreadPoolExecutor(8) as ex:
            ks = list(ex.map(kjob, xs))
            rs = list(ex.map(rjob, ys * 2))
        torch.cuda.synchronize()
        for a, k in zip(arrs, ks):
            assert_kurtosis(k, orc.kurtosis(a), "leaf", a.shape[2])
        for a, r in zip(ints * 2, rs):
            assert np.array_equal(r, orc.reduce(a, 8, 20000))
