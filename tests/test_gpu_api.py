"""GPU, end to end through the reference-shaped API: files on disk (FBH5 and
SIGPROC) -> WorkerFunctions.getdata / GBT.getdata / getband / getkurtosis,
and the N-rank band exchange with the real kernels (gloo transport, two ranks
sharing cuda:0)."""
from __future__ import annotations

import os

import numpy as np
import pytest

from conftest import assert_kurtosis, same_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def files(pkg, orc, tmp_path_factory):
    d = tmp_path_factory.mktemp("banks")
    rng = np.random.default_rng(2026)
    banks, names = [], []
    for b in range(8):
        a = np.asfortranarray(rng.integers(0, 256, (4096, 1, 40)).astype(np.float32))
        banks.append(a)
        hdr = dict(fch1=8400.0 - b * 187.5, foff=-187.5 / 4096, nchans=4096, nifs=1,
                   tsamp=1.07, source_name="HIP1234")
        if b % 2 == 0:
            p = d / f"BLP0{b}" / f"blc0{b}_guppi_59000_12345_HIP1234_0011.rawspec.0002.h5"
            p.parent.mkdir()
            pkg.fbh5.write(p, dict(hdr, nfpc=64), a, chunks=(8, 1, 1024))
        else:
            p = d / f"BLP0{b}" / f"blc0{b}_guppi_59000_12345_HIP1234_0011.rawspec.0002.fil"
            p.parent.mkdir()
            pkg.readers.write_fil(p, dict(hdr, telescope_id=6, machine_id=10, data_type=1,
                                          tstart=59000.5, nbits=32), a)
        names.append(str(p))
    return banks, names


def test_worker_getdata_files(pkg, orc, files):
    banks, names = files
    J, C = pkg.JRange, pkg.COLON
    for a, f in zip(banks, names):
        got = pkg.WorkerFunctions.getdata(f, (C, C, J(1, 32)), fqavby=64, tavby=8)
        assert same_bits(got, orc.reduce(a, 64, 8, "sum", [0, 4096, 1, 0, 1, 1, 0, 32, 1]))
        got = pkg.WorkerFunctions.getdata(f, (J(1025, 2048), 1, C), fqavby=16, fqavfunc="max")
        assert same_bits(got, orc.reduce(a, 16, 1, "max", [1024, 1024, 1, 0, 1, 1, 0, 40, 1]))
    with pytest.raises(pkg.DimensionMismatch):
        pkg.WorkerFunctions.getdata(names[0], fqavby=3)


def test_gbt_getdata_getband_kurtosis(pkg, orc, files):
    banks, names = files
    J, C = pkg.JRange, pkg.COLON
    workers = [0] * len(names)  # every "worker" is this box's GPU 0
    res = pkg.GBT.getdata(workers, names, (C, C, J(1, 40)), fqavby=64, tavby=10)
    assert res.shape == (8,)
    for a, r in zip(banks, res):
        assert same_bits(r, orc.reduce(a, 64, 10))
    band = pkg.GBT.getband(workers, names, (C, C, C), fqavby=64, tavby=10)
    assert same_bits(band, orc.stitch([orc.reduce(a, 64, 10) for a in banks]))
    full = pkg.GBT.getband(workers, names, (C, C, J(1, 3)), despike_nfpc=64)
    want = orc.despike(orc.stitch([np.asfortranarray(a[:, :, :3]) for a in banks]), 64)
    assert same_bits(full, want)
    band2, ax = pkg.GBT.getband(workers, names, (C, C, J(1, 3)), freqs=True, despike_nfpc=True)
    assert same_bits(band2, want)  # loadscan's nfpc = 4096 ÷ 64 = 64 (src/gbt.jl:100)
    foff = -187.5 / 4096
    assert isinstance(ax, pkg.worker.FRange) and len(ax) == band2.shape[0] == 8 * 4096
    assert ax.first == 8400.0 and ax.step == foff
    _, ax = pkg.GBT.getband(workers, names, (C, C, J(1, 3)), fqavby=64, freqs=True)
    np.testing.assert_allclose(ax.values(), 8400.0 + 63 * foff / 2 + 64 * foff * np.arange(512),
                               rtol=0, atol=1e-9)
    with pytest.raises(pkg.BoundsError):  # nfpc = 64 ÷ 64 = 1: d[0:1:end] in the reference
        pkg.GBT.getband(workers, names, (C, C, J(1, 3)), fqavby=64, despike_nfpc=True)
    ks = pkg.GBT.getkurtosis(workers[:2], names[:2], (J(1, 512), C, C))
    for a, k in zip(banks[:2], ks):
        # (the loosest path bound: the staged buffer's alignment picks the path)
        assert_kurtosis(k, orc.kurtosis(a, [0, 512, 1, 0, 1, 1, 0, 40, 1]), "leaf", 40)
    hdrs = pkg.GBT.getheaders(workers[:2], names[:2])
    assert hdrs[0]["nfpc"] == 64 and hdrs[1]["nfpc"] == 64  # FBH5 attr / round(187.5/64/abs(foff))
    # a (nbank, nband) matrix like loadscan's ds: one stitched band per column,
    # map(c -> reduce(vcat, c), eachcol(ds)) (src/gbt.jl:103)
    wm = np.array(workers, dtype=object).reshape(4, 2)
    fm = np.array(names, dtype=object).reshape(4, 2)
    bands = pkg.GBT.getband(wm, fm, (C, C, C), fqavby=64, tavby=10)
    assert len(bands) == 2
    for j in range(2):
        col = [banks[2 * r + j] for r in range(4)]  # fm[:, j]
        assert same_bits(bands[j], orc.stitch([orc.reduce(a, 64, 10) for a in col]))
    bands, axes = pkg.GBT.getband(wm, fm, (C, C, J(1, 3)), freqs=True)
    assert len(axes) == 2 and len(axes[1]) == bands[1].shape[0] == 4 * 4096
    with pytest.raises(AssertionError):
        pkg.GBT.getband(np.zeros((2, 2, 2), object), np.zeros((2, 2, 2), object))


@pytest.mark.parametrize("force_copy", ["0", "1"])
def test_getband_device_stitch_matches_host_concat(pkg, orc, files, monkeypatch, force_copy):
    """GBT.getband's device stitch (every bank reduced into its vcat slot on
    the GPU, despike in place, one copy to the host) is bit-exact against the
    host concatenation of per-bank results, with and without despike; with
    BLDP_BAND_FORCE_COPY=1 every bank takes the other-GPU branch (reduced on
    its own device, then copied into the slot)."""
    monkeypatch.setenv("BLDP_BAND_FORCE_COPY", force_copy)
    banks, names = files
    J, C = pkg.JRange, pkg.COLON
    workers = [0] * len(names)
    for idxs, F, T, op, nfpc in (((C, C, C), 64, 10, "sum", None),
                                 ((C, C, J(1, 32)), 1, 8, "mean", None),
                                 ((C, C, J(1, 3)), 1, 1, "sum", 64),
                                 ((J(1, 2048), C, J(2, 40)), 2, 1, "max", True)):
        dev = pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                              despike_nfpc=nfpc)
        host = pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                               despike_nfpc=nfpc, stitch="host")
        assert same_bits(dev, host), (idxs, F, T, op, nfpc)
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), banks[0].shape)
        want = orc.stitch([orc.reduce(a, F, T, op, win) for a in banks])
        if nfpc:
            want = orc.despike(want, want.shape[0] // 8 // 64 if nfpc is True else nfpc)
        assert same_bits(dev, want), (idxs, F, T, op, nfpc)
    # banks whose products differ in shape: the host concatenation takes over
    short = [names[0], names[1]]
    assert pkg.GBT._band_on_device([0, 0], [banks[0], banks[1][:2048]], (C, C, C), 1, "sum", 1,
                                   None) is None
    got = pkg.GBT.getband([0, 0], short, (C, C, C), fqavby=4)
    assert same_bits(got, orc.stitch([orc.reduce(a, 4, 1) for a in banks[:2]]))


@pytest.mark.parametrize("force_copy", ["0", "1"])
def test_getband_raw_band_one_stream(pkg, orc, tmp_path, monkeypatch, force_copy):
    """Banks that are all raw files of one geometry (uncompressed contiguous
    FBH5 and 32-bit SIGPROC, data at different file offsets) take the band
    read: one stream of preads / H2D batches for every bank
    (bldp_file_runs_to_device) and one reduce into the vcat slots
    (bldp_band_reduce_f32; with BLDP_BAND_FORCE_COPY=1 the multi-GPU form,
    bldp_band_reduce_multi_f32, on its staged branch).  Bit-exact against the
    host concatenation and the oracle, with and without despike, whole rows
    and channel sub-spans (zoom windows read span by span)."""
    monkeypatch.setenv("BLDP_BAND_FORCE_COPY", force_copy)
    rng = np.random.default_rng(77)
    J, C = pkg.JRange, pkg.COLON
    nc = 1 << 18
    banks, names = [], []
    for b in range(6):
        a = np.asfortranarray(rng.integers(0, 256, (nc, 1, 24)).astype(np.float32))
        hdr = dict(fch1=8400.0 - b * 187.5, foff=-187.5 / nc, nchans=nc, nifs=1, tsamp=1.07)
        if b % 2 == 0:
            p = tmp_path / f"raw{b}.h5"
            pkg.fbh5.write(p, dict(hdr, nfpc=1024), a)
        else:
            p = tmp_path / f"raw{b}.fil"
            pkg.readers.write_fil(p, dict(hdr, telescope_id=6, machine_id=10, data_type=1,
                                          tstart=59000.5, nbits=32, source_name="X"), a)
        banks.append(a)
        names.append(str(p))
    workers = [0] * len(names)
    for idxs, F, T, op, nfpc in (((C, C, C), 64, 8, "sum", None),
                                 ((C, C, J(3, 18)), 16, 4, "max", 1024),
                                 ((J(4097, 4096 + 65536), C, J(1, 24)), 1024, 24, "mean", None),
                                 ((C, C, J(1, 2)), 1, 1, "sum", True)):
        tm = {}
        dev = pkg.GBT._band_on_device(workers, names, idxs, F, op, T, nfpc, timings=tm)
        assert tm["path"] == "raw band", tm
        host = pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                               despike_nfpc=nfpc, stitch="host")
        assert same_bits(dev, host), (idxs, F, T, op, nfpc)
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), banks[0].shape)
        want = orc.stitch([orc.reduce(a, F, T, op, win) for a in banks])
        if nfpc:
            want = orc.despike(want, want.shape[0] // len(banks) // 64 if nfpc is True else nfpc)
        assert same_bits(dev, want), (idxs, F, T, op, nfpc)
        assert same_bits(pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                                         despike_nfpc=nfpc), want)


@pytest.mark.parametrize("staged", [False, True])
@pytest.mark.parametrize("branch", ["chunked band", "bank by bank"])
def test_getband_compressed_banks_device_stitch(pkg, orc, tmp_path, monkeypatch, staged, branch):
    """A band of compressed (HDF5 filter 32008) banks.  "chunked band": every
    bank's chunks read and decoded as one stream of batches per GPU
    (bldp_file_chunks_to_device) into one chunk grid per bank, then one band
    reduce into the vcat slots (staged: bldp_band_reduce_multi_f32's staged
    branch).  "bank by bank" (the fallback for banks that do not share a
    layout): each bank's chunks are decoded on its GPU and the reduce there
    writes the root's vcat slot directly (bldp_peer_access; one GPU: the same
    device), or, staged, reduces locally and one stream-ordered device copy
    fills the slot; no host wait per bank.  Bit-exact against the host
    concatenation and the oracle, with and without despike (src/gbt.jl:75-78,
    101-103; src/gbtworkerfunctions.jl:181-187)."""
    if branch == "bank by bank":
        monkeypatch.setattr(pkg.GBT, "_band_chunked", lambda *a, **k: False)
    rng = np.random.default_rng(4242)
    J, C = pkg.JRange, pkg.COLON
    banks, names = [], []
    for b in range(8):
        a = np.asfortranarray(rng.integers(0, 200, (4096, 1, 48)).astype(np.float32))
        f = str(tmp_path / f"z{b}.rawspec.0002.h5")
        pkg.fbh5.write_bslz4(f, dict(foff=-187.5 / 4096, fch1=8400.0 - 187.5 * b, nfpc=64), a,
                             (16, 1, 4096),
                             lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
        banks.append(a)
        names.append(f)
    workers = [0] * len(names)
    for idxs, F, T, op, nfpc in (((C, C, C), 64, 16, "sum", None),
                                 ((C, C, J(1, 32)), 1, 8, "mean", 64),
                                 ((J(1, 2048), C, J(2, 47)), 4, 1, "max", True)):
        tm = {}
        dev = pkg.GBT._band_on_device(workers, names, idxs, F, op, T, nfpc, timings=tm,
                                      staged=staged)
        assert tm["path"] == branch + (" (staged)" if staged else ""), tm
        host = pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                               despike_nfpc=nfpc, stitch="host")
        assert same_bits(dev, host), (idxs, F, T, op, nfpc)
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), banks[0].shape)
        want = orc.stitch([orc.reduce(a, F, T, op, win) for a in banks])
        if nfpc:
            want = orc.despike(want, want.shape[0] // 8 // 64 if nfpc is True else nfpc)
        assert same_bits(dev, want), (idxs, F, T, op, nfpc)
        assert same_bits(pkg.GBT.getband(workers, names, idxs, fqavby=F, tavby=T, fqavfunc=op,
                                         despike_nfpc=nfpc, staged=staged), want)


def test_getband_chunked_band_mixed_filters_and_fallback(pkg, orc, tmp_path):
    """The chunked-band read takes compressed and unfiltered chunked banks of
    one geometry together (unfiltered chunks copied raw, a chunk never written
    read as 0), with the window inside one chunk column (the chunk grid is the
    window's array) or across several (each bank's window gathered from its
    grid, bldp_unchunk_f32), and hands banks of different chunk layouts back
    to the bank-by-bank branch; all bit-exact against the oracle."""
    rng = np.random.default_rng(515)
    J, C = pkg.JRange, pkg.COLON
    enc = lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress)  # noqa: E731
    for chunk, want_path in (((8, 1, 2048), "chunked band"), ((8, 1, 512), "chunked band"),
                             (None, "bank by bank")):
        banks, names = [], []
        for b in range(4):
            a = np.asfortranarray(rng.integers(0, 200, (2048, 1, 40)).astype(np.float32))
            ck = chunk or ((8, 1, 2048) if b < 2 else (8, 1, 1024))  # None: two layouts
            f = str(tmp_path / f"m{b}_{chunk[2] if chunk else 0}.h5")
            if b % 2:
                pkg.fbh5.write(f, dict(foff=-1.0, nfpc=64), a, chunks=ck)
            else:
                pkg.fbh5.write_bslz4(f, dict(foff=-1.0, nfpc=64), a, ck, enc)
            banks.append(a)
            names.append(f)
        for idxs, F, T, op in (((C, C, C), 64, 8, "sum"), ((J(129, 2048), C, J(3, 34)), 8, 4, "max")):
            tm = {}
            got = pkg.GBT._band_on_device([0] * 4, names, idxs, F, op, T, None, timings=tm)
            assert tm["path"] == want_path, (chunk, tm)
            win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), banks[0].shape)
            want = orc.stitch([orc.reduce(a, F, T, op, win) for a in banks])
            assert same_bits(got, want), (chunk, idxs, F, T, op)
    # a compressed band with a chunk never written (fill value 0)
    a = np.asfortranarray(rng.integers(0, 200, (2048, 1, 32)).astype(np.float32))
    c = np.ascontiguousarray(a.transpose(2, 1, 0))
    items, want_a = [], a.copy(order="F")
    for k in range(4):
        if k == 2:
            items.append(None)
            want_a[:, :, 8 * k:8 * k + 8] = 0.0
        else:
            items.append(enc(np.ascontiguousarray(c[8 * k:8 * k + 8])))
    names = []
    for b in range(3):
        f = str(tmp_path / f"hole{b}.h5")
        pkg.fbh5.write_bslz4_chunks(f, dict(foff=-1.0, nfpc=64), (2048, 1, 32), (8, 1, 2048), items)
        names.append(f)
    tm = {}
    got = pkg.GBT._band_on_device([0] * 3, names, (C, C, C), 16, "sum", 4, None, timings=tm)
    assert tm["path"] == "chunked band", tm
    assert same_bits(got, orc.stitch([orc.reduce(want_a, 16, 4)] * 3))


@pytest.mark.parametrize("kind", ["raw", "compressed"])
def test_getband_under_a_caller_stream(pkg, orc, tmp_path, kind):
    """getband called inside `with torch.cuda.stream(s)`: the
    reader threads queue their copies' completion on the caller's stream, so
    the reduce the caller's thread queues on s reads landed bank data.  The
    caller's stream is kept busy first, so a reduce not ordered after the
    copies would read the buffer before they land."""
    import torch

    rng = np.random.default_rng(31)
    C = pkg.COLON
    nc = 1 << 18 if kind == "raw" else 4096
    banks, names = [], []
    for b in range(4):
        a = np.asfortranarray(rng.integers(0, 256, (nc, 1, 16)).astype(np.float32))
        f = str(tmp_path / f"s{b}.h5")
        if kind == "raw":
            pkg.fbh5.write(f, dict(foff=-1.0, nfpc=1024), a)
        else:
            pkg.fbh5.write_bslz4(f, dict(foff=-1.0, nfpc=64), a, (16, 1, 4096),
                                 lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
        banks.append(a)
        names.append(f)
    want = orc.stitch([orc.reduce(a, 64, 8) for a in banks])
    s = torch.cuda.Stream()
    junk = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
    for _ in range(3):
        with torch.cuda.stream(s):
            for _ in range(20):  # ~0.1 s of queued work ahead of the band on s
                junk.mul_(1.0)
            tm = {}
            got = pkg.GBT._band_on_device([0] * 4, names, (C, C, C), 64, "sum", 8, None,
                                          timings=tm)
        assert tm["path"] == ("raw band" if kind == "raw" else "chunked band"), tm
        assert same_bits(got, want)
    torch.cuda.synchronize()


def test_getband_staged_leaves_other_threads_plans_alone(pkg, orc, tmp_path):
    """The staged/direct choice of the band reduce is an argument of the call
    (BLDP_BAND_STAGED), not process state: while one
    thread runs getband(staged=True) over raw banks, another thread's
    plan-sensitive reduces keep their plans and their bits."""
    import threading

    import torch

    eng = pkg.engine
    rng = np.random.default_rng(9)
    C = pkg.COLON
    names, banks = [], []
    for b in range(4):
        a = np.asfortranarray(rng.integers(0, 256, (1 << 16, 1, 16)).astype(np.float32))
        f = str(tmp_path / f"t{b}.h5")
        pkg.fbh5.write(f, dict(foff=-1.0, nfpc=1024), a)
        names.append(f)
        banks.append(a)
    want_band = orc.stitch([orc.reduce(a, 64, 16) for a in banks])
    shapes = [((65536, 1, 279), 64, 16, [0, 65536, 1, 0, 1, 1, 0, 272, 1]),
              ((4096, 1, 64), 1024, 64, None), ((512, 1, 4096), 8, 1, None)]
    xs = []
    for shape, F, T, w in shapes:
        a = np.asfortranarray(rng.integers(0, 256, shape).astype(np.float32))
        x = eng.fb_from_numpy(a)
        xs.append((a, x, F, T, w, eng.plan(x, F, T, "sum", w), orc.reduce(a, F, T, "sum", w)))
    stop, errs = threading.Event(), []

    def bander():
        try:
            while not stop.is_set():
                got = pkg.GBT.getband([0] * 4, names, (C, C, C), fqavby=64, tavby=16, staged=True)
                assert same_bits(got, want_band)
        except Exception as e:  # noqa: BLE001 (reported below)
            errs.append(e)

    th = threading.Thread(target=bander)
    th.start()
    try:
        for _ in range(30):
            for a, x, F, T, w, plan0, want in xs:
                assert eng.plan(x, F, T, "sum", w) == plan0
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    got = eng.fb_to_numpy(eng.reduce(x, F, T, "sum", w))
                assert same_bits(got, want)
    finally:
        stop.set()
        th.join()
    assert not errs, errs


def test_device_to_host_through_the_slot_ring(pkg):
    """bldp_device_to_host (fb_to_numpy(pinned=True), getband's one D2H): the
    band lands in ordinary numpy memory through the library's pinned slots,
    bit-exact, for sizes below one slot, a ragged multiple, and more than the
    whole ring (slot reuse); ordered after the producer's stream; nothing
    pinned is handed out."""
    import ctypes

    import torch

    eng = pkg.engine
    for n in (1, 1000, (32 << 20) // 4 + 3, (300 << 20) // 4 + 5):
        x = torch.arange(n, dtype=torch.int32, device="cuda")
        st = {}
        h = eng.device_to_host(x, stats=st)
        assert h.dtype == np.int32 and h.shape == (n,)
        assert np.array_equal(h, np.arange(n, dtype=np.int32)), n
        assert st["slots"] >= 1 and st["threads"] >= 1
        assert h.base is None or not isinstance(h.base, torch.Tensor)
    # ordered after the work queued on the caller's (producer's) stream
    s = torch.cuda.Stream()
    y = torch.zeros(1 << 26, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for _ in range(10):
            y.add_(1.0)
        h = eng.device_to_host(y)
    assert (h == 10.0).all()
    # the Julia-order product copy getband makes
    z = eng.fb_empty(4096, 2, 7)
    z.copy_(torch.arange(4096 * 2 * 7, dtype=torch.float32, device="cuda").view(7, 2, 4096)
            .permute(2, 1, 0))
    got = eng.fb_to_numpy(z, pinned=True)
    assert got.flags.f_contiguous and same_bits(got, eng.fb_to_numpy(z))
    L = pkg._lib.lib()
    assert L.bldp_device_to_host(None, None, 0, None, None, None) == 0
    assert L.bldp_device_to_host(None, None, 16, None, None, None) == pkg._lib.BLDP_EINVAL
    assert L.bldp_device_to_host(ctypes.c_void_p(16), None, -1, None, None, None) == \
        pkg._lib.BLDP_EINVAL


def test_gbt_getkurtosis_fanout_long_windows(pkg, orc, tmp_path):
    """GBT.getkurtosis over 6 files on one device with > 512 spectra: one
    thread per (worker, file) on the same stream and scratch (the leaf
    partials and tree levels), each result against the oracle."""
    rng = np.random.default_rng(61)
    arrs, names = [], []
    for b in range(6):
        a = np.asfortranarray((rng.gamma(400.0, 1e6, (256, 1, 1500 + 300 * b))).astype(np.float32))
        p = tmp_path / f"k{b}.h5"
        pkg.fbh5.write(p, dict(fch1=1000.0, foff=-0.1, nchans=256, nifs=1, tsamp=1.0, nfpc=64), a)
        arrs.append(a)
        names.append(str(p))
    for _ in range(2):
        ks = pkg.GBT.getkurtosis([0] * 6, names)
        for a, k in zip(arrs, ks):
            assert_kurtosis(k, orc.kurtosis(a), "leaf", a.shape[2])


def _rank(rank, world, port, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__ as entry

    pkg, orc = entry.load_package(), entry.load_oracle()
    eng = pkg.engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    banks = [orc.gamma_bandpass(8192, 1, 64, 1024, 50 + b) for b in range(8)]
    mine = [eng.fb_from_numpy(banks[b], "cuda:0") for b in pkg.band.banks_for_rank(8, rank, world)]

    def reduce_fn(bs, F, T, op, win):  # real kernel; gloo moves host tensors
        return eng.band_reduce(bs, F, T, op, win).cpu()

    def stitch_fn(g, n):  # real stitch kernel on the gathered blocks
        return eng.stitch(g.cuda(), n).cpu()

    res = pkg.band.band_reduce_dist(mine, 64, 16, "sum", None, reduce_fn=reduce_fn,
                                    stitch_fn=stitch_fn)
    if rank == 0:
        want = orc.stitch([orc.reduce(b, 64, 16) for b in banks])
        got = res.permute(2, 1, 0).contiguous().numpy().transpose(2, 1, 0)
        q.put(bool(np.allclose(got, want, rtol=1e-5)) and got.shape == want.shape)
    else:
        q.put(res is None)
    dist.destroy_process_group()
    del rng, torch


def test_band_dist_two_ranks_real_kernels():
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=300)
    assert all(p.exitcode == 0 for p in ps)
    assert all(q.get(timeout=5) for _ in ps)


def _nccl_pipeline_rank(port, q, kind="torch"):
    """One rank of an RCCL (torch "nccl") process group driving BandPipeline
    (torch.distributed.gather) or NativeBandPipeline (bldp_band_gather_f32 on
    its own stream) with the gather on: what every rank of bench.py N>1 runs."""
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__ as entry

    pkg, orc = entry.load_package(), entry.load_oracle()
    eng = pkg.engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    ok = []
    for ni, F, T, nt in ((1, 1024, 16, 16), (2, 64, 4, 32)):  # single-row and stitched
        banks = [orc.gamma_bandpass(8192, ni, nt, 1024, 70 + b) for b in range(4)]
        dbanks = [eng.fb_from_numpy(b, "cuda:0") for b in banks]
        want = orc.stitch([orc.reduce(b, F, T) for b in banks])
        if kind == "native":
            pipe = pkg.band.NativeBandPipeline(4 * 8192 // F, ni, nt // T, device="cuda:0")
        else:
            pipe = pkg.band.BandPipeline(4 * 8192 // F, ni, nt // T, device="cuda:0",
                                         gather_single=True)
        for _ in range(3):  # slots reused: the gather of step k overlaps step k+1
            slot = pipe.begin()
            eng.band_reduce(dbanks, F, T, "sum", None, out=pipe.local(slot))
            res = pipe.exchange(slot)
            pipe.wait(slot)
            torch.cuda.synchronize()
            got = eng.fb_to_numpy(res)
            ok.append(got.shape == want.shape and bool(np.allclose(got, want, rtol=1e-5)))
        pipe.drain()
        if kind == "native":
            pipe.close()
    t = torch.tensor([1.0, 2.0], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
    ok.append(t.tolist() == [1.0, 2.0])
    dist.barrier()
    dist.destroy_process_group()
    q.put(ok)


@pytest.mark.parametrize("kind", ["torch", "native"])
def test_band_pipeline_over_rccl_one_rank(kind):
    """The N>1 exchange of bench.py (async RCCL gather to the root, then the
    stitch kernel; torch.distributed.gather or the C ABI's ncclGather on the
    pipeline's own stream) on a one-rank group, the most of it one GPU can run
    (RCCL refuses two ranks on one device)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_pipeline_rank,
                    args=(29900 + os.getpid() % 90 + (kind == "native"), q, kind))
    p.start()
    p.join(timeout=240)
    assert p.exitcode == 0
    ok = q.get(timeout=5)
    assert ok and all(ok), ok


def test_bench_pipeline_flag():
    """bench.py --pipeline: the N>1 step (reduce + RCCL gather + stitch) timed
    on a one-rank group."""
    import json
    import subprocess
    import sys

    from conftest import REPO

    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3",
                        "--warmup", "1", "--config", "cfg2", "--pipeline", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    c = d["config"]
    assert d["n_gpus"] == 1 and d["value"] > 0 and "RCCL (nccl backend) gather" in c["parallelism"]
    assert c["dist_backend"] == "nccl" and c["world_size"] == 1 and c["device_count"] >= 1
    assert c["exchange"] == "native" and "bldp_band_gather_f32" in c["parallelism"]


def _bslz4_fixtures():
    import json

    from conftest import GOLDEN

    z = np.load(os.path.join(GOLDEN, "bslz4_v1.npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, "bslz4_manifest.json")) as f:
        return z, json.load(f)["cases"]


def test_bslz4_gpu_decoder_matches_bitshuffle_library(pkg):
    z, cases = _bslz4_fixtures()
    chunks = [z["chunk_" + c["name"]].tobytes() for c in cases]
    out = pkg.fbh5.bslz4_decode_dev(chunks, device="cuda:0").cpu().numpy()
    pos = 0
    for c in cases:
        raw = z["raw_" + c["name"]].ravel()
        assert np.array_equal(out[pos:pos + raw.size].view(np.uint32), raw.view(np.uint32)), \
            c["name"]
        pos += raw.size
    assert pos == out.size


def test_bslz4_gpu_rejects_chunks_larger_than_their_slot(pkg):
    """A chunk whose header claims more (or fewer) bytes than its output slot
    is refused on the host before any launch (BLDP_EINVAL): nothing is written
    into the neighbouring slots."""
    import struct

    import torch

    z, _ = _bslz4_fixtures()
    good = z["chunk_int_runs_b512"].tobytes()
    raw = z["raw_int_runs_b512"].ravel()
    nb = raw.nbytes
    L, lib = pkg._lib.lib(), pkg._lib
    for claim in (2 * nb, nb - 32):
        evil = struct.pack(">Q", claim) + good[8:]  # same blocks, forged byte count
        blobs = [good, evil, good]
        comp = np.frombuffer(b"".join(blobs), np.uint8)
        coff = np.array([0, len(good), len(good) + len(evil)], np.uint64)
        clen = np.array([len(b) for b in blobs], np.uint64)
        ooff = np.array([0, nb, 2 * nb], np.uint64)
        olen = np.full(3, nb, np.uint64)
        out = torch.full((3 * nb // 4,), -1, dtype=torch.int32, device="cuda:0")
        cdev = torch.from_numpy(comp.copy()).cuda()
        rc = L.bldp_bslz4_decode_dev(3, comp.ctypes.data, cdev.data_ptr(), coff.ctypes.data,
                                     clen.ctypes.data, 4, out.data_ptr(), ooff.ctypes.data,
                                     olen.ctypes.data, lib.stream_ptr())
        assert rc == lib.BLDP_EINVAL and "slot" in lib.last_error()
        torch.cuda.synchronize()
        assert (out == -1).all()  # refused before the launch: no slot touched
    with pytest.raises(ValueError):  # the Python wrapper checks the slots too
        pkg.fbh5.bslz4_decode_dev([good, good], device="cuda:0",
                                  out=torch.empty(nb // 4, dtype=torch.float32, device="cuda:0"),
                                  out_offsets=[0, nb // 2])


def test_bslz4_gpu_rejects_corrupt_blocks(pkg):
    import struct

    bad = struct.pack(">QI", 2048 * 4, 2048 * 4) + struct.pack(">I", 3) + b"\0\0\0"
    with pytest.raises(pkg.BLDPError):  # passes the host plan, fails in the kernel
        pkg.fbh5.bslz4_decode_dev([bad], device="cuda:0")
    z, _ = _bslz4_fixtures()
    good = z["chunk_int_runs_b512"].tobytes()
    out = pkg.fbh5.bslz4_decode_dev([good], device="cuda:0")  # the device still works
    assert np.array_equal(out.cpu().numpy(), z["raw_int_runs_b512"].ravel())
    # asynchronous form: a good and a corrupt call share one error word, which
    # bldp_bslz4_error reports after the fact
    import torch

    L, lib = pkg._lib.lib(), pkg._lib
    err = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    res = torch.empty(max(z["raw_int_runs_b512"].nbytes, 2048 * 4), dtype=torch.uint8,
                      device="cuda:0")
    for blob in (good, bad):
        h = np.frombuffer(blob, np.uint8)
        dv = torch.from_numpy(h.copy()).cuda()
        o = np.zeros(1, np.uint64)
        n = np.array([len(blob)], np.uint64)
        olen = np.array([pkg.fbh5.bslz4_info(blob)[0]], np.uint64)
        assert L.bldp_bslz4_decode_dev_async(1, h.ctypes.data, dv.data_ptr(), o.ctypes.data,
                                             n.ctypes.data, 4, res.data_ptr(), o.ctypes.data,
                                             olen.ctypes.data, err.data_ptr(),
                                             lib.stream_ptr()) == 0
        if blob is good:
            assert L.bldp_bslz4_error(err.data_ptr(), lib.stream_ptr()) == 0
    assert L.bldp_bslz4_error(err.data_ptr(), lib.stream_ptr()) == lib.BLDP_EINVAL
    assert "corrupt" in lib.last_error() or "overruns" in lib.last_error()


@pytest.mark.parametrize("parsed_index,native", [(True, True), (True, False), (False, True)])
def test_fbh5_bslz4_on_gpu_end_to_end(pkg, orc, tmp_path, monkeypatch, parsed_index, native):
    """Compressed FBH5 through the GPU decoder; chunks read by parallel preads
    at the parsed chunk index (the library's reader threads,
    bldp_chunks_to_device, or with BLDP_NATIVE_READ=0 the Python reader), and
    (parsed_index=False) one H5Dread_chunk at a time, as for files outside the
    parser's scope."""
    monkeypatch.setenv("BLDP_NATIVE_READ", "1" if native else "0")
    J, C = pkg.JRange, pkg.COLON
    d = np.asfortranarray(np.random.default_rng(8).integers(0, 256, (4096, 2, 40))
                          .astype(np.float32))
    p = tmp_path / "blc00_guppi_59000_12345_HIP1234_0011.rawspec.0002.h5"
    pkg.fbh5.write_bslz4(p, dict(foff=-0.002861, nfpc=1024), d, (16, 1, 1024),
                         lambda blk: orc.np_bslz4_encode(blk, 2048))
    if not parsed_index:
        monkeypatch.setattr(pkg.h5chunks, "chunk_table", lambda *a, **k: None)
    tm = {}
    x = pkg.fbh5._read_window_bslz4_dev(p, (C, C, C), "cuda:0", timings=tm)
    assert tm["parsed_chunk_index"] is parsed_index
    assert same_bits(pkg.engine.fb_to_numpy(x), d)
    x = pkg.fbh5.read_window_bslz4(p, (J(1025, 3072), C, J(5, 36)), device="cuda:0")
    assert same_bits(pkg.engine.fb_to_numpy(x), np.asfortranarray(d[1024:3072, :, 4:36]))
    got = pkg.WorkerFunctions.getdata(str(p), (C, C, J(1, 32)), fqavby=64, tavby=8)
    assert same_bits(got, orc.reduce(d, 64, 8, "sum", [0, 4096, 1, 0, 2, 1, 0, 32, 1]))
    got = pkg.GBT.getdata([0], [str(p)], (J(4096, -1, 1), 1, C), fqavby=16, fqavfunc="max")
    assert same_bits(got[0], orc.reduce(d, 16, 1, "max", [4095, 4096, -1, 0, 1, 1, 0, 40, 1]))


# --- library runtime: bldp_init / bldp_finalize, staging pool, pinning ------

def test_init_finalize_and_lazy_reinit(pkg, orc):
    eng = pkg.engine
    eng.init()
    eng.init([0])  # idempotent
    with pytest.raises(pkg._lib.ArgumentError):
        eng.init([99])
    rng = np.random.default_rng(31)
    a = np.asfortranarray(rng.integers(0, 256, (1024, 1, 64)).astype(np.float32))
    assert same_bits(eng.reduce_host(a, 16, 4), orc.reduce(a, 16, 4))
    eng.finalize()
    eng.finalize()  # nothing left to free
    assert same_bits(eng.reduce_host(a, 16, 4), orc.reduce(a, 16, 4))  # lazily re-created
    assert same_bits(eng.reduce_host(a, 8, 2, "max"), orc.reduce(a, 8, 2, "max"))


def test_concurrent_host_callers_share_one_gpu(pkg, orc):
    # GBT.getdata fans one call per (worker, file) out concurrently
    # (src/gbt.jl:75-77); several workers may map to one GPU.
    from concurrent.futures import ThreadPoolExecutor

    eng = pkg.engine
    rng = np.random.default_rng(32)
    arrs = [np.asfortranarray(rng.integers(0, 256, (4096, 1, 96 + 16 * k)).astype(np.float32))
            for k in range(8)]
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda a: eng.reduce_host(a, 64, 16), arrs * 3))
    for g, a in zip(got, arrs * 3):
        assert same_bits(g, orc.reduce(a, 64, 16))
    with ThreadPoolExecutor(8) as ex:
        kur = list(ex.map(eng.kurtosis_host, arrs))
    for k, a in zip(kur, arrs):
        assert_kurtosis(k, orc.kurtosis(a), "leaf", a.shape[2])


def test_host_paths_do_not_leak_device_memory(pkg, orc):
    import torch

    eng = pkg.engine
    rng = np.random.default_rng(33)
    # long time block with few outputs -> chunked plan with library scratch;
    # values 0..31 keep every 8 x 60000 group sum below 2^24 (exact in Float32)
    a = np.asfortranarray(rng.integers(0, 32, (64, 1, 60000)).astype(np.float32))
    want = orc.reduce(a, 8, 60000)
    for _ in range(2):
        eng.reduce_host(a, 8, 60000)
        eng.kurtosis_host(a)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(20):
        got = eng.reduce_host(a, 8, 60000)
        eng.kurtosis_host(a)
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert same_bits(got, want)
    assert free0 - free1 < (16 << 20), (free0, free1)


def test_pinned_host_buffer(pkg, orc):
    eng = pkg.engine
    rng = np.random.default_rng(34)
    a = np.asfortranarray(rng.integers(0, 256, (8192, 1, 64)).astype(np.float32))
    with eng.pinned(a):
        got = eng.reduce_host(a, 64, 16)
    assert same_bits(got, orc.reduce(a, 64, 16))
    with pytest.raises(pkg._lib.ArgumentError):
        pkg._lib.check(pkg._lib.lib().bldp_host_register(None, 0))


@pytest.mark.parametrize("native", [True, False])
def test_raw_files_stream_to_gpu(pkg, orc, tmp_path, monkeypatch, native):
    """Uncompressed contiguous FBH5 and 32-bit SIGPROC files: getdata and
    getkurtosis read only the window (parallel preads into pinned slots,
    several batches: the library's reader threads, bldp_runs_to_device, or the
    Python reader with BLDP_NATIVE_READ=0) and reduce on the GPU; exact on
    integer data."""
    monkeypatch.setenv("BLDP_NATIVE_READ", "1" if native else "0")
    fs = pkg.filestream
    monkeypatch.setattr(fs, "BATCH_BYTES", 1 << 20)
    monkeypatch.setattr(fs, "PIECE_BYTES", 192 << 10)
    monkeypatch.setattr(fs, "SUBSPAN_MIN_BYTES", 4096)
    rng = np.random.default_rng(91)
    a = np.asfortranarray(rng.integers(0, 256, (4096, 2, 300)).astype(np.float32))
    h5, fil = str(tmp_path / "r.h5"), str(tmp_path / "r.fil")
    pkg.fbh5.write(h5, dict(foff=-187.5 / 4096, nfpc=64), a)
    pkg.readers.write_fil(fil, dict(fch1=8000.0, foff=-187.5 / 4096, nchans=4096, nifs=2,
                                    tsamp=1.0, nbits=32, telescope_id=6, machine_id=10,
                                    data_type=1, tstart=59000.0, source_name="X"), a)
    J, C = pkg.JRange, pkg.COLON
    W = pkg.WorkerFunctions
    cases = [((C, C, C), 64, 4, "sum"), ((C, 2, J(1, 288)), 16, 8, "max"),
             ((J(1025, 2048), C, J(300, -3, 1)), 8, 4, "sum"),   # channel span per row
             ((J(4096, -1, 1), C, J(11, 7, 300)), 4, 1, "min")]
    for f in (h5, fil):
        for idxs, F, T, op in cases:
            win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), a.shape)
            got = W.getdata(f, idxs, fqavby=F, fqavfunc=op, tavby=T)
            assert same_bits(got, orc.reduce(a, F, T, op, win)), (f, idxs)
        kw = [1024, 1024, 1, 0, 2, 1, 0, 300, 1]
        got = W.getkurtosis(f, (J(1025, 2048), C, C))
        assert_kurtosis(got, orc.kurtosis(a, kw), "leaf", 300)
    tm = {}
    runs, dshape, rwin = fs.plan_window(a.shape, [0, 4096, 1, 0, 2, 1, 0, 300, 1],
                                        pkg.fbh5.raw_layout(h5)[0])
    buf = fs.read_runs_to_device(h5, runs, "cuda:0", timings=tm)
    assert tm["batches"] > 4 and buf.numel() == a.nbytes
    assert same_bits(pkg.engine.fb_to_numpy(buf.view(torch_f32()).view(300, 2, 4096)
                                            .permute(2, 1, 0)), a)


@pytest.mark.parametrize("ramp", ["1", "0"])
def test_raw_reader_ramped_batches(pkg, orc, tmp_path, monkeypatch, ramp):
    """bldp_runs_to_device / bldp_file_runs_to_device cut blocks of more than
    4 slots into batches of slot/4, slot/2, slots..., slot/2, slot/4
    (BLDP_RUNS_RAMP=0: slot-sized).  With 4 MiB slots: one 20 MB raw file
    (whole, and a channel span per row: many runs crossing batch boundaries)
    and a band of three raw files through the band read, bit-exact."""
    monkeypatch.setenv("BLDP_RUNS_RAMP", ramp)
    monkeypatch.setenv("BLDP_NATIVE_READ", "1")
    monkeypatch.setattr(pkg.filestream, "NATIVE_BATCH_BYTES", 4 << 20)
    rng = np.random.default_rng(13)
    J, C = pkg.JRange, pkg.COLON
    banks, names = [], []
    for b in range(3):
        a = np.asfortranarray(rng.integers(0, 256, (4096, 2, 600)).astype(np.float32))
        p = str(tmp_path / f"r{b}.h5")
        pkg.fbh5.write(p, dict(foff=-187.5 / 4096, nfpc=64), a)
        banks.append(a)
        names.append(p)
    W = pkg.WorkerFunctions
    for idxs, F, T in (((C, C, C), 1, 1), ((J(1025, 2048), C, J(3, 598)), 4, 2)):
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), banks[0].shape)
        got = W.getdata(names[0], idxs, fqavby=F, tavby=T)
        assert same_bits(got, orc.reduce(banks[0], F, T, "sum", win)), idxs
    tm = {}
    got = pkg.GBT._band_on_device([0] * 3, names, (C, C, C), 64, "sum", 8, None, timings=tm)
    assert tm["path"] == "raw band", tm
    assert same_bits(got, orc.stitch([orc.reduce(a, 64, 8) for a in banks]))


def test_truncated_file_raises_read_error(pkg, tmp_path, monkeypatch):
    """A read past the end of a file (truncated after its layout was taken, or
    a stale index) is an I/O error (BLDP_EIO -> ReadError, an OSError), not an
    argument error."""
    monkeypatch.setenv("BLDP_NATIVE_READ", "1")
    a = np.asfortranarray(np.ones((4096, 1, 64), np.float32))
    fil = str(tmp_path / "t.fil")
    pkg.readers.write_fil(fil, dict(fch1=8000.0, foff=-1.0, nchans=4096, nifs=1, tsamp=1.0,
                                    nbits=32, telescope_id=6, machine_id=10, data_type=1,
                                    tstart=59000.0, source_name="X"), a)
    raw = pkg.readers.fil_raw_layout(fil)
    assert raw is not None
    os.truncate(fil, os.path.getsize(fil) - 4096 * 4 * 10)  # the last 10 spectra gone
    C = pkg.COLON
    with pytest.raises(pkg.ReadError) as e:
        pkg.worker._reduce_raw_file(fil, raw, (C, C, C), 64, "sum", 1, 0)
    assert isinstance(e.value, OSError) and e.value.code == pkg._lib.BLDP_EIO
    assert "truncated" in str(e.value)


def torch_f32():
    import torch

    return torch.float32


def test_c_abi_demo_binary():
    """examples/c_abi_demo.c: the ABI driven from plain C (host arrays,
    windows, int codes, bldp_last_error), as a Julia ccall drives it."""
    import subprocess

    from conftest import REPO

    exe = os.path.join(REPO, "build", "c_abi_demo")
    assert os.path.exists(exe), "run __graft_entry__.build() first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_native_band_gather_world1(pkg, orc):
    """The C-ABI band exchange (bldp_comm_* + bldp_band_gather_f32, RCCL
    ncclGather) on a one-rank communicator: the gathered band equals the
    rank's slice, single-row and multi-row (stitch) outputs."""
    import torch

    eng = pkg.engine
    nb = pkg.band.NativeBand(0, 1, 0, pkg.band.NativeBand.new_id())
    try:
        for ni, F, T in ((1, 1024, 32), (2, 1024, 32), (2, 64, 8)):
            banks = [eng.synth(4096, ni, 32, 64, seed=b, kind=1) for b in range(3)]
            local = eng.band_reduce(banks, F, T)
            got = nb.gather(local)
            torch.cuda.synchronize()
            assert same_bits(eng.fb_to_numpy(got), eng.fb_to_numpy(local))
    finally:
        nb.close()


@pytest.mark.parametrize("F,T,nbank", [(64, 16, 1), (64, 16, 3), (256, 16, 2), (4, 1, 2),
                                        (1024, 16, 1), (8, 2048, 1)])
def test_prepared_reduce_and_timed_launch(pkg, orc, F, T, nbank):
    """bldp_band_reduce_prepare_f32 + bldp_reduce_launch / _launch_timed give
    band_reduce's bits on every path (row split, rowt, interleaved, chunked +
    finalize: the timed form's events span both dispatches), launched again
    on the same buffers; the dispatch-carried events time the launch."""
    import torch

    eng, HipEvent = pkg.engine, pkg._lib.HipEvent
    nt = 64 if T < 2048 else 4096
    banks = [eng.synth(16384, 1, nt + 3, 1024, seed=7 * b + F, kind=1) for b in range(nbank)]
    win = [0, 16384, 1, 0, 1, 1, 0, nt, 1]
    want = eng.fb_to_numpy(eng.band_reduce(banks, F, T, "sum", win))
    prep = eng.PreparedBandReduce(banks, F, T, "sum", win)
    try:
        sp = int(torch.cuda.current_stream().cuda_stream)
        e0, e1 = HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False)
        for k in range(3):
            prep.out.fill_(float("nan"))
            if k == 1:
                prep.launch(sp)
            else:
                prep.launch_timed(sp, e0, e1)
            torch.cuda.synchronize()
            assert same_bits(eng.fb_to_numpy(prep.out), want), k
        assert 0 < e0.elapsed_time(e1) < 1000
        b0 = orc.reduce(eng.fb_to_numpy(banks[0]), F, T, "sum", win)
        assert same_bits(want[:16384 // F], b0)
    finally:
        prep.close()
    L = pkg._lib.lib()
    assert L.bldp_reduce_launch_timed(None, None, None, None) == pkg._lib.BLDP_EINVAL


def test_bench_json_contract():
    """bench.py prints one JSON line with the keys the driver reads (a short
    cfg1 run; the default cfg3 run is the round-end bench)."""
    import json
    import subprocess
    import sys

    from conftest import REPO

    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "3",
                        "--warmup", "1", "--config", "cfg1", "--cpu-seconds", "0.5"],
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and 0 < rf["frac"] < 1 and rf["peak"] == 8000.0
    # the per-launch kernel time (its own pass) and the timed span per launch, which
    # is at most the step; the clock-settle launches ran before the warmup
    assert rf["kernel_ms"] > 0 and rf["span_ms_per_launch"] > 0
    assert rf["span_ms_per_launch"] <= d["ms_per_step"] * 1.05
    assert d["settle_launches"] > 0
    # the box's pure-read rate for the launch's bytes, and the reduce beside it
    pr = rf["box_read_probe"]
    assert pr["bytes"] == rf["bytes_per_launch"] // 16 * 16 and 0 < pr["GBps"] < 20000.0
    assert rf["frac_of_box_read"] == pytest.approx(rf["achieved"] / pr["GBps"], rel=1e-3)
    # cfg1 (71 MB a launch) runs cold by default: the launches rotate over
    # >= 1 GiB of copies, the probe too, and the warm figure is beside it
    assert rf["cache"].startswith("cold") and pr["copies"] >= 15
    assert rf["warm"]["kernel_ms"] > 0 and rf["warm"]["frac"] > 0
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert "workload" in d["config"]


def test_unfiltered_chunked_fbh5_on_gpu(pkg, orc, tmp_path):
    """Chunked FBH5 without a filter (edge chunks padded by HDF5): the chunk
    reader moves the stored chunks to the GPU, which gathers the window and
    reduces it (no decode)."""
    J, C = pkg.JRange, pkg.COLON
    a = np.asfortranarray(np.random.default_rng(12).integers(0, 256, (1000, 3, 50))
                          .astype(np.float32))
    p = str(tmp_path / "chunked.h5")
    pkg.fbh5.write(p, dict(foff=-1.0, nfpc=100), a, chunks=(7, 1, 100))
    assert pkg.fbh5.raw_chunked(p) and not pkg.fbh5.needs_bslz4(p)
    for idxs, F, T, op in [((C, C, C), 10, 5, "sum"), ((J(101, 900), 2, J(3, 50)), 8, 4, "max"),
                           ((J(1000, -1, 1), C, J(50, -7, 1)), 4, 1, "min")]:
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), a.shape)
        got = pkg.WorkerFunctions.getdata(p, idxs, fqavby=F, fqavfunc=op, tavby=T)
        assert same_bits(got, orc.reduce(a, F, T, op, win)), idxs


@pytest.mark.parametrize("ci", [1, 2])
def test_chunks_spanning_the_channels_reduce_in_place(pkg, orc, tmp_path, ci):
    """Chunks that span the whole channel axis (gi = gc = 1, the rawspec
    layout): getdata reduces the window straight out of the decoded chunk grid
    (no gather), for windows with channel / IF / time steps, reversed axes,
    integer indices and partial first and last chunks; compressed and
    unfiltered files, every op, against the oracle (integer data: exact)."""
    J, C = pkg.JRange, pkg.COLON
    rng = np.random.default_rng(40 + ci)
    nc, ni, nt = 1500, 2, 61
    a = np.asfortranarray(rng.integers(0, 128, (nc, ni, nt)).astype(np.float32))
    comp, plain = str(tmp_path / "c.h5"), str(tmp_path / "p.h5")
    chunk = (8, ci, nc)
    pkg.fbh5.write_bslz4(comp, dict(foff=-1.0), a, chunk,
                         lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
    pkg.fbh5.write(plain, dict(foff=-1.0), a, chunks=chunk)
    cases = [((C, C, C), 4, 1, "sum"), ((J(3, 1498), C, J(5, 60)), 8, 4, "max"),
             ((J(1, 2, 1500), 2, J(2, 3, 59)), 5, 2, "min"),
             ((J(1500, -1, 1), J(2, -1, 1), J(61, -2, 1)), 3, 31, "sum"),
             ((J(11, 3, 1490), C, 17), 1, 1, "sum")]
    for idxs, F, T, op in cases:
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), a.shape) or \
            [0, nc, 1, 0, ni, 1, 0, nt, 1]
        want = orc.reduce(a, F, T, op, win)
        for f in (comp, plain):
            x, rwin = pkg.fbh5._read_window_bslz4_dev(f, pkg.sanitizeidxs(idxs), "cuda:0",
                                                      raw_chunks=f == plain, dense=False)
            # the chunk box is one chunk wide in IF unless the window takes
            # both IFs from one-IF chunks
            assert (rwin is not None) == (ci == 2 or win[4] == 1), (idxs, ci)
            got = pkg.WorkerFunctions.getdata(f, idxs, fqavby=F, fqavfunc=op, tavby=T)
            assert same_bits(got, want), (f, idxs, F, T, op)


def test_getkurtosis_compressed_and_chunked_files(pkg, orc, tmp_path):
    """getkurtosis on a bitshuffle/LZ4 FBH5 and an unfiltered chunked one: the
    chunks are decoded on the GPU and the kurtosis runs on the window inside
    the chunk grid (chunks spanning the channels) or on the gathered window
    (narrower chunks); long and short windows against the oracle."""
    from conftest import assert_kurtosis

    J, C = pkg.JRange, pkg.COLON
    rng = np.random.default_rng(77)
    nc, ni, nt = 512, 1, 1500
    a = np.asfortranarray(rng.gamma(4.0, 1e9, (nc, ni, nt)).astype(np.float32))
    W, eng = pkg.WorkerFunctions, pkg.engine
    for chunk in ((16, 1, nc), (16, 1, 96)):
        comp, plain = str(tmp_path / f"c{chunk[2]}.h5"), str(tmp_path / f"p{chunk[2]}.h5")
        pkg.fbh5.write_bslz4(comp, dict(foff=-1.0), a, chunk,
                             lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
        pkg.fbh5.write(plain, dict(foff=-1.0), a, chunks=chunk)
        for idxs in ((C, C, C), (J(5, 508), C, J(7, 1406)), (J(2, 2, 511), C, J(1, 300))):
            win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), a.shape) or \
                [0, nc, 1, 0, ni, 1, 0, nt, 1]
            want = orc.kurtosis(a, win)
            for f in (comp, plain):
                got = W.getkurtosis(f, idxs)
                x, rwin = pkg.fbh5._read_window_bslz4_dev(f, pkg.sanitizeidxs(idxs), "cuda:0",
                                                          raw_chunks=f == plain, dense=False)
                path = eng.kurtosis_plan(x, rwin)["path"]
                assert_kurtosis(got, want, path, win[7], (f, idxs))


@pytest.mark.parametrize("native", [True, False])
def test_compressed_file_missing_and_unfiltered_chunks(pkg, orc, tmp_path, monkeypatch, native):
    """HDF5 chunk states the readers must honour: a chunk never written reads
    as the fill value 0, a chunk stored with filter mask bit 0 set holds raw
    elements (the filter was skipped for it), the rest are bitshuffle/LZ4.
    getdata and getkurtosis through the native and the Python readers against
    the oracle on the array those states describe (integer data: exact)."""
    from conftest import assert_kurtosis

    monkeypatch.setenv("BLDP_NATIVE_READ", "1" if native else "0")
    J, C = pkg.JRange, pkg.COLON
    rng = np.random.default_rng(5150)
    nc, ni, nt = 512, 2, 70
    a = np.asfortranarray(rng.integers(0, 200, (nc, ni, nt)).astype(np.float32))
    chunk = (8, 1, 512)  # C order (t, i, c): 9 x 2 chunks, the last time block partial
    c = np.ascontiguousarray(a.transpose(2, 1, 0))  # [t][i][c]
    items, want = [], a.copy(order="F")
    for k, t0 in enumerate(range(0, nt, 8)):
        for i0 in range(ni):
            blk = np.zeros(chunk, np.float32)
            part = c[t0:t0 + 8, i0:i0 + 1, :]
            blk[:part.shape[0]] = part
            if (k, i0) in ((2, 0), (6, 1)):
                items.append(None)  # never written
                want[:, i0, t0:t0 + 8] = 0.0
            elif (k, i0) in ((4, 1), (8, 0)):
                items.append((1, blk.tobytes()))  # stored raw, filter skipped
            else:
                items.append(orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
    p = str(tmp_path / "holes.h5")
    pkg.fbh5.write_bslz4_chunks(p, dict(foff=-1.0), (nc, ni, nt), chunk, items)
    for idxs, F, T, op in [((C, C, C), 4, 5, "sum"), ((J(3, 510), 2, J(9, 64)), 4, 8, "max"),
                           ((C, 1, J(70, -1, 1)), 8, 1, "min")]:
        win = pkg.idxs.to_window(pkg.sanitizeidxs(idxs), a.shape) or \
            [0, nc, 1, 0, ni, 1, 0, nt, 1]
        got = pkg.WorkerFunctions.getdata(p, idxs, fqavby=F, fqavfunc=op, tavby=T)
        assert same_bits(got, orc.reduce(want, F, T, op, win)), idxs
    k = pkg.WorkerFunctions.getkurtosis(p, (C, C, C))
    assert_kurtosis(k, orc.kurtosis(want), "mid", nt)


def test_gbt_fanout_over_compressed_and_raw_files(pkg, orc, tmp_path):
    """GBT.getdata fans one call per (worker, file) out on threads
    (src/gbt.jl:75-77): compressed, unfiltered-chunked and contiguous files
    read at once on one device share the native reader (one read call at a
    time per device) and the decode scratch; every result against the oracle."""
    J, C = pkg.JRange, pkg.COLON
    rng = np.random.default_rng(808)
    names, arrs = [], []
    for k in range(6):
        a = np.asfortranarray(rng.integers(0, 128, (1024, 1, 96 + 8 * k)).astype(np.float32))
        f = str(tmp_path / f"f{k}.h5")
        if k % 3 == 0:
            pkg.fbh5.write_bslz4(f, dict(foff=-1.0), a, (16, 1, 1024),
                                 lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
        elif k % 3 == 1:
            pkg.fbh5.write(f, dict(foff=-1.0), a, chunks=(16, 1, 256))
        else:
            pkg.fbh5.write(f, dict(foff=-1.0), a)
        names.append(f)
        arrs.append(a)
    for _ in range(3):
        got = pkg.GBT.getdata([0] * 6, names, (J(1, 1024), C, J(1, 96)), fqavby=16, tavby=8)
        for g, a in zip(got, arrs):
            assert same_bits(g, orc.reduce(a, 16, 8, "sum", [0, 1024, 1, 0, 1, 1, 0, 96, 1]))


def test_bslz4_gpu_decoder_random_lz4(pkg, orc):
    """The GPU decoder on the same kind of random chunks (real LZ4 matches,
    all block sizes, raw tails), 40 chunks in one call."""
    from test_host import _random_bslz4_cases

    cases = _random_bslz4_cases(orc, 100, 40)
    out = pkg.fbh5.bslz4_decode_dev([c for _, c in cases], device="cuda:0").cpu().numpy()
    pos = 0
    for a, c in cases:
        got = out[pos:pos + a.size]
        assert np.array_equal(got.view(np.uint32), a.view(np.uint32)), (a.size, len(c))
        pos += a.size
    assert pos == out.size


@pytest.mark.parametrize("seed", range(2))
def test_compressed_and_raw_files_random_windows(pkg, orc, tmp_path, seed):
    """Random chunk geometries and windows: a bitshuffle/LZ4 FBH5 (real LZ4
    matches), an unfiltered chunked FBH5 and a contiguous one, each through
    WorkerFunctions.getdata on the GPU, against the oracle (exact on integer
    data)."""
    rng = np.random.default_rng(31 + seed)
    nc, ni, nt = int(rng.integers(200, 3000)), int(rng.integers(1, 3)), int(rng.integers(20, 90))
    a = np.asfortranarray(rng.integers(0, 64, (nc, ni, nt)).astype(np.float32))
    chunk = (int(rng.integers(1, 17)), 1, int(rng.integers(64, 1500)))
    comp, plain, cont = (str(tmp_path / f"{k}.h5") for k in ("c", "p", "u"))
    pkg.fbh5.write_bslz4(comp, dict(foff=-1.0), a, chunk,
                         lambda blk: orc.np_bslz4_encode(blk, 512, lz4=orc.lz4_compress))
    pkg.fbh5.write(plain, dict(foff=-1.0), a, chunks=chunk)
    pkg.fbh5.write(cont, dict(foff=-1.0), a)
    J, C = pkg.JRange, pkg.COLON
    for _ in range(6):
        F = int(rng.choice([1, 2, 4, 5, 8]))
        T = int(rng.choice([1, 2, 3, 4]))
        c0 = int(rng.integers(1, nc // 2))
        ncw = (int(rng.integers(F, nc - c0 + 1)) // F) * F
        t0 = int(rng.integers(1, nt // 2))
        ntw = (int(rng.integers(T, nt - t0 + 1)) // T) * T
        idxs = (J(c0, c0 + ncw - 1), C, J(t0, t0 + ntw - 1))
        op = str(rng.choice(["sum", "max", "min"]))
        win = [c0 - 1, ncw, 1, 0, ni, 1, t0 - 1, ntw, 1]
        want = orc.reduce(a, F, T, op, win)
        for f in (comp, plain, cont):
            got = pkg.WorkerFunctions.getdata(f, idxs, fqavby=F, fqavfunc=op, tavby=T)
            assert same_bits(got, want), (f, idxs, F, T, op, chunk)


def test_chunk_reader_stages_through_the_slot_ring(pkg, tmp_path):
    """The native chunk reader stages compressed reads through the device's
    pinned slot ring (bldp_chunks_to_device with host_pinned NULL), the ring
    bldp_runs_to_device uses, so no pinned buffer the size of the window is
    allocated.  Cases, each bit-exact against the data written:
    - a 260 MB window of mixed chunks (bitshuffle/LZ4, stored unfiltered with
      per-chunk values, never written): more batches than the ring has
      slots, so slots are reused;
    - unfiltered chunks of 40 MiB, larger than a 32 MiB slot: the ring grows;
    - raw-file reads in between, which take the ring back to 8 x 32 MiB."""
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "bslz4_v1.npz"))
    comp, dec = z["chunk_gamma_chunk_b2048"].tobytes(), z["raw_gamma_chunk_b2048"]
    C = pkg.COLON
    ct, cc = 16, 4096
    gt, gc = 80, 16
    want = np.empty((gt * ct, 1, gc * cc), np.float32)  # C order (time, IF, chan)
    chunks = []
    for t in range(gt):
        for c in range(gc):
            k = t * gc + c
            blk = want[t * ct:(t + 1) * ct, :, c * cc:(c + 1) * cc]
            if k % 7 == 3:  # stored without the filter: values unique to the chunk
                v = (np.arange(ct * cc, dtype=np.float32).reshape(ct, 1, cc) + 65536.0 * k)
                blk[...] = v
                chunks.append((1, v.tobytes()))
            elif k % 11 == 5:  # never written: the fill value
                blk[...] = 0.0
                chunks.append(None)
            else:
                blk[...] = dec
                chunks.append(comp)
    big = str(tmp_path / "mixed.h5")
    pkg.fbh5.write_bslz4_chunks(big, dict(foff=-1.0), (gc * cc, 1, gt * ct), (ct, 1, cc), chunks)
    wide = np.asfortranarray(
        np.arange(2 * 160 * 65536, dtype=np.float32).reshape(65536, 1, 320, order="F"))
    wide_f = str(tmp_path / "wide.h5")
    pkg.fbh5.write_bslz4_chunks(
        wide_f, dict(foff=-1.0), (65536, 1, 320), (160, 1, 65536),
        [(1, np.ascontiguousarray(wide[:, :, 160 * i:160 * (i + 1)].transpose(2, 1, 0)).tobytes())
         for i in range(2)])
    raw = np.asfortranarray(np.random.default_rng(3).integers(0, 256, (8192, 1, 64))
                            .astype(np.float32))
    raw_f = str(tmp_path / "raw.h5")
    pkg.fbh5.write(raw_f, dict(foff=-1.0), raw)
    want_j = np.asfortranarray(want.transpose(2, 1, 0))
    for f, w in ((big, want_j), (raw_f, raw), (wide_f, wide), (raw_f, raw), (big, want_j),
                 (wide_f, wide)):
        got = pkg.WorkerFunctions.getdata(f, (C, C, C))
        assert same_bits(got, w), f
    J = pkg.JRange
    got = pkg.WorkerFunctions.getdata(big, (J(4000, 40000), C, J(17, 1000)), fqavby=1)
    assert same_bits(got, want_j[3999:40000, :, 16:1000])


def test_cfg5_share_full_size_host_path(pkg, orc):
    """One GPU's share of cfg5 (bank b of 4 bands x {0000, 0001, 0002}) at the
    full per-array sizes (4 GiB, 1.8 GB, 73 MB) through bldp_reduce_host_f32
    from pinned host memory, as bench.py --mode host streams it (SURVEY §8d
    D2(5), the GBT.getdata fan-out src/gbt.jl:69-79): the 0002 arrays
    (gamma power) against the oracle; the 0000/0001 arrays as integer data,
    bit-exact against the device-resident reduce and checked by exact
    totals and spot groups."""
    import torch

    eng = pkg.engine
    prods = [  # name, nchan, ntime, window, F, T, nfpc, product
        ("0000", 1 << 26, 16, 16, 1024, 16, 1 << 20, 0),
        ("0001", 512, 880000, 879616, 8, 1024, 8, 1),
        ("0002", 65536, 279, 272, 64, 16, 1024, 2)]
    bank = 3
    for name, nchan, ntime, tw, F, T, nfpc, pr in prods:
        h = torch.empty((ntime, 1, nchan), dtype=torch.float32, pin_memory=True)
        win = None if tw == ntime else [0, nchan, 1, 0, 1, 1, 0, tw, 1]
        for band in range(4):
            seed = 1000 * band + 10 * bank + pr
            t = eng.synth(nchan, 1, ntime, nfpc, seed=seed, kind=0 if name == "0002" else 1)
            h.copy_(t.permute(2, 1, 0))
            a = h.numpy().transpose(2, 1, 0)  # Julia order, Fortran-contiguous, pinned
            got = eng.reduce_host(a, F, T, "sum", win)
            assert got.shape == (nchan // F, 1, tw // T)
            if name == "0002":
                np.testing.assert_allclose(got, orc.reduce(a, F, T, "sum", win), rtol=1e-5)
                continue
            ref = eng.fb_to_numpy(eng.reduce(t, F, T, "sum", win))
            assert same_bits(got, ref), (name, band)
            assert got.astype(np.float64).sum() == t[:, :, :tw].double().sum().item()
            for g in (0, (nchan // F) // 2 + band, nchan // F - 1):
                blk = a[g * F:(g + 1) * F, 0, :T].astype(np.float64).sum()
                assert got[g, 0, 0] == blk, (name, band, g)
            del t
        del h
        torch.cuda.empty_cache()


def test_read_probe(pkg):
    """tools/hbm_probe (build/libbldp_probe.so, a measurement tool outside the
    product library): the pure-read reference bench.py reports (timed by
    dispatch-carried events), its grid forms, and its argument checks."""
    import sys

    import torch

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "tools"))
    import hbm_probe

    r = hbm_probe.read_probe(64 << 20, launches=5, pkg=pkg)
    # (a 64 MiB buffer read over and over partly stays in the 256 MB
    # Infinity Cache: 8.7 TB/s measured, above the HBM peak)
    assert r["bytes"] == 64 << 20 and r["form"] in hbm_probe.PROBE_FORMS and 500 < r["GBps"] < 20000
    L = hbm_probe.lib()
    buf = torch.zeros(1 << 20, dtype=torch.float32, device="cuda")
    for g in (0, 1, 2, 4):  # ragged tail (a partial chunk) in every form
        for m in range(8):
            assert L.bldp_probe_read(buf.data_ptr(), (4 << 20) - 48, m << 8 | g, None, None,
                                     None) == 0
    assert L.bldp_probe_read(None, 0, 0, None, None, None) == 0
    assert L.bldp_probe_read(buf.data_ptr() + 4, 1024, 0, None, None, None) != 0
    assert L.bldp_probe_read(buf.data_ptr(), -16, 0, None, None, None) != 0
    assert L.bldp_probe_read(buf.data_ptr(), 1024, -1, None, None, None) != 0
    assert L.bldp_probe_read(buf.data_ptr(), 1024, 2048, None, None, None) != 0
    torch.cuda.synchronize()
