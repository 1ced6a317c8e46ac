"""CPU: host-side logic — Julia index handling (sanitizeidxs, ranges), the
SIGPROC reader, the inventory walk, the GBT fan-out shape, and the sharded
band exchange (world_size 2, gloo)."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest


def test_sanitizeidxs_and_window(pkg):
    J, C = pkg.JRange, pkg.COLON
    # Integers become i:i so results stay 3-D (src/gbtworkerfunctions.jl:167-169)
    assert pkg.sanitizeidxs((C, 2, J(5, 10))) == (C, J(2, 2), J(5, 10))
    to_window = pkg.idxs.to_window
    assert to_window((C, C, C), (10, 2, 7)) is None
    assert to_window((J(3, 8), 1, C), (10, 2, 7)) == [2, 6, 1, 0, 1, 1, 0, 7, 1]
    assert to_window((J(9, -2, 1), C, J(1, 3, 7)), (10, 2, 7)) == [8, 5, -2, 0, 2, 1, 0, 3, 3]
    assert len(J(1, 2, 15)) == 8 and len(J(5, 4)) == 0 and list(J(1, 3, 7)) == [1, 4, 7]
    with pytest.raises(AssertionError):
        to_window((C, C), (1, 1, 1))  # @assert length(idxs) == 3
    with pytest.raises(TypeError):
        to_window((range(3), C, C), (10, 1, 1))


def test_fqav_range_mirror(pkg):
    # GBT.fqav(1:4, 4) === 2.5:4.0:2.5 ; GBT.fqav(1:2:15, 4) === 4.0:8.0:12.0
    r = pkg.GBT.fqav(pkg.JRange(1, 4), 4)
    assert (r.first, r.step, len(r), r.last) == (2.5, 4.0, 1, 2.5)
    r = pkg.GBT.fqav(pkg.JRange(1, 2, 15), 4)
    assert (r.first, r.step, len(r), r.last) == (4.0, 8.0, 2, 12.0)
    rr = pkg.JRange(1, 9)
    assert pkg.fqav(rr, 1) is rr


def test_bandaxis(pkg):
    J, C = pkg.JRange, pkg.COLON
    foff = -187.5 / 1024
    hdrs = [dict(fch1=8400.0 - b * 187.5, foff=foff, nchans=1024) for b in range(8)]
    ax = pkg.GBT.bandaxis(hdrs, (C, C, C), 16)  # adjacent banks: one range
    assert isinstance(ax, pkg.worker.FRange) and len(ax) == 512
    np.testing.assert_allclose(ax.values(), 8400.0 + 15 * foff / 2 + 16 * foff * np.arange(512),
                               rtol=0, atol=1e-9)
    assert pkg.GBT.bandaxis(hdrs, (C, C, C), 1).step == foff
    # a channel window per bank: the pieces no longer continue each other
    ax = pkg.GBT.bandaxis(hdrs[:2], (J(3, 2, 9), 1, C), 2)
    want = [8400.0 + foff * (2 + 1), 8400.0 + foff * (6 + 1)]  # fqav(3:2:9 -> 2 centres)
    want += [w - 187.5 for w in want]
    np.testing.assert_allclose(ax, want, rtol=0, atol=1e-9)
    with pytest.raises(IndexError):
        pkg.GBT.bandaxis(hdrs, (J(1, 2000), C, C))
    with pytest.raises(AssertionError):
        pkg.GBT.bandaxis(hdrs, (C, C))
    assert len(pkg.GBT.bandaxis([], (C, C, C))) == 0


def test_fqav_passthrough_and_generic_host(pkg):
    a = np.arange(24, dtype=np.float32).reshape((4, 2, 3), order="F")
    assert pkg.fqav(a, 1) is a  # n <= 1 returns A itself (:17)
    med = pkg.fqav(a, 2, np.median)  # any f(X; dims) runs as the reference does
    np.testing.assert_array_equal(med, np.median(a.reshape((2, 2, 2, 3), order="F"), axis=0))
    with pytest.raises(pkg.DimensionMismatch):
        pkg.fqav(a, 3, np.median)


def test_fqav_generic_keeps_f_result_type(pkg):
    """fqav returns f(reshape(A, ...); dims=1) as f makes it
    (src/gbtworkerfunctions.jl:19): median / std of an Int16 array are Float64
    (Julia's Statistics), not truncated back to Int16."""
    a = np.asfortranarray(np.array([1, 2, 4, 7, -3, 8, 10, 11], dtype=np.int16).reshape((8, 1, 1)))
    med = pkg.fqav(a, 2, np.median)
    assert med.dtype == np.float64
    np.testing.assert_array_equal(med[:, 0, 0], [1.5, 5.5, 2.5, 10.5])
    sd = pkg.fqav(a, 4, np.std)
    assert sd.dtype == np.float64 and sd.shape == (2, 1, 1)
    assert pkg.fqav(a.astype(np.float32), 2, np.median).dtype == np.float32


def test_sigproc_roundtrip_and_header(pkg, tmp_path):
    rd = pkg.readers
    data = np.asfortranarray(np.random.default_rng(0).random((64, 2, 5)).astype(np.float32))
    hdr = dict(telescope_id=6, machine_id=10, data_type=1, source_name="VOYAGER1",
               tstart=59000.5, tsamp=18.253611, fch1=8438.96484375, foff=-2.7939677238464355e-06,
               nchans=64, nifs=2, nbits=32)
    f = tmp_path / "guppi_59000_00001_VOYAGER1_0001.rawspec.0000.fil"
    rd.write_fil(f, hdr, data)
    assert not rd.ishdf5(f)
    h, mm = rd.fil_mmap(f)
    assert h["nsamps"] == 5 and mm.shape == (64, 2, 5)
    np.testing.assert_array_equal(np.asarray(mm), data)
    gh = rd.getfbheader(f)
    assert gh["nfpc"] == 1048576  # round(Int32, 187.5/64/abs(foff)) (:134)
    assert "header_size" not in gh and "sample_size" not in gh


def test_ishdf5_signature(pkg, tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\0" * 100)
    assert pkg.readers.ishdf5(p)
    q = tmp_path / "y.h5"
    q.write_bytes(b"\0" * 512 + b"\x89HDF\r\n\x1a\n" + b"\0" * 100)
    assert pkg.readers.ishdf5(q)


def test_inventory_walk(pkg, tmp_path):
    root = tmp_path / "datax"
    good = root / "AGBT22B_999_01" / "GUPPI" / "BLP42"
    good.mkdir(parents=True)
    (good / "blc42_guppi_59000_12345_HIP1234_0011.rawspec.0002.h5").write_bytes(b"")
    (good / "blc42_guppi_59000_12345_HIP1234_0011.rawspec.0000.h5").write_bytes(b"")
    (good / "junk.0002.h5").write_bytes(b"")  # does not match the guppi regex -> warn
    (root / "AGBT22B_999_01" / "GUPPI" / "XYZ").mkdir()  # player regex filters it out
    (root / "notasession").mkdir()
    warns = []
    inv = pkg.readers.getinventory(root=str(root), worker=3, warn=warns.append)
    assert len(inv) == 1 and len(warns) == 1
    e = inv[0]
    assert (e["imjd"], e["smjd"], e["session"], e["scan"], e["src_name"], e["band"], e["bank"],
            e["worker"]) == (59000, 12345, "AGBT22B_999_01", "0011", "HIP1234", 4, 2, 3)
    assert e["host"] == socket.gethostname() and e["file"].endswith("0002.h5")
    assert tuple(e) == pkg.readers.INVENTORY_FIELDS
    assert pkg.readers.getinventory(root=str(tmp_path / "missing")) == []
    invs = pkg.GBT.getinventories([1, 2], root=str(root))
    assert [len(i) for i in invs] == [1, 1] and invs[1][0]["worker"] == 2


def test_datahosts(pkg):
    h = pkg.GBT.datahosts()
    assert len(h) == 64 and h[0] == "blc00" and h[-1] == "blc77"
    assert pkg.GBT.datahosts("x")[9] == "xblc11"


def test_getdata_size_assert(pkg):
    with pytest.raises(AssertionError):
        pkg.GBT.getdata([0, 1], ["a"])


def test_banks_for_rank(pkg):
    b = pkg.band.banks_for_rank
    assert [list(b(8, r, 4)) for r in range(4)] == [[0, 1], [2, 3], [4, 5], [6, 7]]
    assert list(b(8, 0, 1)) == list(range(8))
    with pytest.raises(ValueError):
        b(8, 0, 3)


def _band_worker(rank, world, port, F, T, ni, nt, q):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__ as entry

    pkg, orc = entry.load_package(), entry.load_oracle()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(42)
    banks = [np.asfortranarray(rng.integers(0, 256, (256, ni, nt)).astype(np.float32))
             for _ in range(8)]
    mine = [banks[b] for b in pkg.band.banks_for_rank(8, rank, world)]

    def to_t(a):  # Julia-order CPU tensor with channel-fastest strides
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 1, 0))).permute(2, 1, 0)

    def reduce_fn(bs, F_, T_, op, win):  # CPU stand-in for engine.band_reduce
        return to_t(orc.stitch([orc.reduce(b, F_, T_, op, win) for b in bs]))

    def stitch_fn(g, n):  # CPU stand-in for engine.stitch: [n, nto, ni, nc] -> vcat
        parts = [np.asfortranarray(g[k].numpy().transpose(2, 1, 0)) for k in range(n)]
        return to_t(orc.stitch(parts))

    res = pkg.band.band_reduce_dist(mine, F, T, "sum", None, reduce_fn=reduce_fn,
                                    stitch_fn=stitch_fn)
    want = orc.stitch([orc.reduce(b, F, T) for b in banks])

    def check(r):
        got = r.permute(2, 1, 0).contiguous().numpy().transpose(2, 1, 0)
        return bool(np.array_equal(got, want)) and got.shape == want.shape

    ok = check(res) if rank == 0 else res is None
    # the pipelined exchange bench.py times: 3 steps over 2 slots, each slot
    # filled with this rank's slice before its gather
    loc = reduce_fn(mine, F, T, "sum", None)
    pipe = pkg.band.BandPipeline(*loc.shape, device="cpu", stitch_fn=stitch_fn)
    for _ in range(3):
        s = pipe.begin()
        pipe.local(s).copy_(loc)
        r = pipe.exchange(s)
        ok = ok and (check(r) if rank == 0 else r is None)
    pipe.drain()
    q.put(ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("F,T,ni,nt,world", [(16, 4, 2, 8, 2), (256, 8, 1, 8, 2),
                                             (16, 4, 2, 8, 4), (256, 8, 1, 8, 8)])
def test_band_exchange_gloo(F, T, ni, nt, world):
    """The N-rank band exchange (as bench.py runs it at N = 2, 4, 8) on CPU."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + F + 3 * world
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, F, T, ni, nt, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    results = [q.get(timeout=5) for _ in procs]
    assert all(p.exitcode == 0 for p in procs)
    assert all(results)


def test_fbh5_read_and_header(pkg, tmp_path):
    fb, J, C = pkg.fbh5, pkg.JRange, pkg.COLON
    d = np.asfortranarray(np.random.default_rng(1).random((64, 2, 10)).astype(np.float32))
    p = tmp_path / "blc42_guppi_59000_12345_HIP1234_0011.rawspec.0002.h5"
    fb.write(p, dict(fch1=8400.0, foff=-2.861022949e-3, nchans=64, nifs=2, tsamp=1.07,
                     source_name="HIP1234", nfpc=1024), d, chunks=(4, 1, 16))
    assert pkg.readers.ishdf5(p)
    assert np.array_equal(fb.read_window(p, (C, C, C)), d)  # h5["data"][] (:183)
    w = fb.read_window(p, (J(60, -3, 5), 2, J(2, 2, 9)))  # hyperslab (:185)
    assert np.array_equal(w, d[59:3:-3][:, 1:2, 1:9:2]) and w.shape == (19, 1, 4)
    with pytest.raises(pkg.BoundsError):
        fb.read_window(p, (J(1, 65), C, C))
    h = pkg.readers.getheader(p)
    assert list(h) == sorted(h)  # sorted by key (:153)
    assert "DIMENSION_LABELS" not in h  # dropped (:145)
    assert h["nsamps"] == 10 and h["data_size"] == 64 * 2 * 10 * 4 and h["nfpc"] == 1024
    q = tmp_path / "nonfpc.h5"
    fb.write(q, dict(foff=-2.7939677238464355e-06), d, deflate=4)
    assert fb.header(q)["nfpc"] == 1048576
    with pytest.raises(NameError):  # the reference's :147-150 bug, on request
        fb.header(q, reference_bug=True)
    assert np.array_equal(fb.read_window(q, (C, C, C)), d)


def _bslz4_fixtures():
    import json

    from conftest import GOLDEN

    z = np.load(os.path.join(GOLDEN, "bslz4_v1.npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, "bslz4_manifest.json")) as f:
        m = json.load(f)
    return z, m["cases"]


def test_bslz4_host_decoder_matches_bitshuffle_library(pkg):
    """Chunks produced by the bitshuffle + LZ4 C libraries (imagecodecs,
    oracle/gen_bslz4_fixtures.py) decode bit-exactly."""
    z, cases = _bslz4_fixtures()
    assert len(cases) >= 14
    for c in cases:
        raw = z["raw_" + c["name"]].ravel()
        got = pkg.fbh5.bslz4_decode_host(z["chunk_" + c["name"]].tobytes())
        assert np.array_equal(got.view(np.uint32), raw.view(np.uint32)), c["name"]


def test_bslz4_encoder_roundtrip_and_corruption(pkg, orc):
    import struct

    a = (np.random.default_rng(3).random(2048 * 2 + 77) * 100).astype(np.float32)
    for block in (2048, 128):
        enc = orc.np_bslz4_encode(a, block)
        assert pkg.fbh5.bslz4_info(enc) == (a.nbytes, block * 4)
        assert np.array_equal(pkg.fbh5.bslz4_decode_host(enc), a)
    bad = struct.pack(">QI", 2048 * 4, 2048 * 4) + struct.pack(">I", 3) + b"\0\0\0"
    with pytest.raises(pkg.BLDPError):  # a match with offset 0
        pkg.fbh5.bslz4_decode_host(bad)
    with pytest.raises(pkg.BLDPError):  # truncated chunk
        pkg.fbh5.bslz4_decode_host(orc.np_bslz4_encode(a)[:-9])
    with pytest.raises(pkg.BLDPError):  # block size field overruns the chunk
        b = bytearray(orc.np_bslz4_encode(a))
        b[12:16] = struct.pack(">I", 1 << 30)
        pkg.fbh5.bslz4_decode_host(bytes(b))


def test_fbh5_bslz4_window_host_decode(pkg, orc, tmp_path):
    """A bitshuffle/LZ4 FBH5 file without the HDF5 plugin: chunks are read raw
    (H5Dread_chunk) and decoded by libbldp_hip, windows match the data."""
    J, C = pkg.JRange, pkg.COLON
    d = np.asfortranarray(np.random.default_rng(8).random((1000, 2, 20)).astype(np.float32))
    p = tmp_path / "bslz4.h5"
    pkg.fbh5.write_bslz4(p, dict(foff=-0.002861, nfpc=1024), d, (8, 1, 256),
                         lambda blk: orc.np_bslz4_encode(blk, 512))
    assert pkg.fbh5.needs_bslz4(p)
    lay = pkg.fbh5.layout(p)
    assert lay["chunk"] == (8, 1, 256) and lay["filters"][0]["id"] == 32008
    assert np.array_equal(pkg.fbh5.read_window(p, (C, C, C)), d)
    w = pkg.fbh5.read_window(p, (J(990, -7, 3), 2, J(3, 2, 19)))
    assert np.array_equal(w, d[989:1:-7][:, 1:2, 2:19:2])
    # real LZ4 streams (with matches) from the bitshuffle library as chunks
    z, _ = _bslz4_fixtures()
    chunks = [z["chunk_gamma_chunk_b2048"].tobytes(), z["chunk_gamma_chunk_b512"].tobytes()]
    raw = z["raw_gamma_chunk_b2048"]  # (16, 1, 4096) C order [t][i][c]
    full = np.concatenate([raw, raw], axis=0).transpose(2, 1, 0)  # Julia (4096, 1, 32)
    q = tmp_path / "lib.h5"
    it = iter(chunks)
    pkg.fbh5.write_bslz4(q, dict(foff=-0.002861), full, (16, 1, 4096), lambda blk: next(it))
    assert np.array_equal(pkg.fbh5.read_window(q, (C, C, C)), np.asfortranarray(full))


def test_fbh5_read_chunks_into_one_buffer(pkg, orc, tmp_path):
    """The pinned-buffer read path (chunks read by libhdf5 straight into one
    caller buffer) returns the same bytes as per-chunk reads."""
    J, C = pkg.JRange, pkg.COLON
    d = np.asfortranarray(np.random.default_rng(4).random((600, 1, 24)).astype(np.float32))
    p = tmp_path / "c.h5"
    pkg.fbh5.write_bslz4(p, {}, d, (8, 1, 256), lambda blk: orc.np_bslz4_encode(blk, 256))
    bufs = []

    def alloc(n):
        b = np.zeros(n + 16, np.uint8)
        bufs.append(b)
        return b.ctypes.data, b

    per = pkg.fbh5.read_chunks(p, (J(100, 590), C, J(3, 20)))
    one = pkg.fbh5.read_chunks(p, (J(100, 590), C, J(3, 20)), alloc)
    assert per[:5] == one[:5] and one[4] == (3, 1, 3)
    chunks, keep = one[5]
    assert len(chunks) == len(per[5]) == 9
    for (m1, b), (m2, off, nb) in zip(per[5], chunks):
        assert m1 == m2 and keep[off:off + nb].tobytes() == b


RAW_WINDOWS = [
    None,
    [0, 1000, 1, 0, 3, 1, 5, 20, 1],
    [999, 500, -2, 2, 3, -1, 36, 12, -3],
    [10, 1, 1, 1, 1, 1, 0, 37, 1],
    [100, 300, 1, 0, 3, 1, 3, 10, 3],
    [400, 100, 1, 1, 2, 1, 0, 37, 1],
]


@pytest.mark.parametrize("subspan", [False, True])
def test_raw_file_window_plans(pkg, orc, tmp_path, monkeypatch, subspan):
    """filestream.plan_window: the byte runs of a window of an uncompressed
    contiguous FBH5 dataset / a 32-bit SIGPROC data block, read back on the
    host, hold exactly the window once the relative window is applied (both
    the whole-row and the channel-span-per-row plans)."""
    fs = pkg.filestream
    if subspan:
        monkeypatch.setattr(fs, "SUBSPAN_MIN_BYTES", 1)
    rng = np.random.default_rng(77)
    a = np.asfortranarray(rng.integers(0, 256, (1000, 3, 37)).astype(np.float32))
    h5, fil = str(tmp_path / "u.h5"), str(tmp_path / "u.fil")
    pkg.fbh5.write(h5, dict(foff=-1.0, nfpc=64), a)
    pkg.readers.write_fil(fil, dict(fch1=8000.0, foff=-1.0, nchans=1000, nifs=3, tsamp=1.0,
                                    nbits=32, telescope_id=6, machine_id=10, data_type=1,
                                    tstart=59000.0, source_name="X"), a)
    for f, raw in ((h5, pkg.fbh5.raw_layout(h5)), (fil, pkg.readers.fil_raw_layout(fil))):
        assert raw is not None and tuple(raw[1]) == a.shape
        for win in RAW_WINDOWS:
            w = win or [0, 1000, 1, 0, 3, 1, 0, 37, 1]
            runs, dshape, rwin = fs.plan_window(raw[1], w, raw[0])
            blk = fs.read_runs_host(f, runs).view(np.float32)
            blk = blk.reshape(dshape[::-1]).transpose(2, 1, 0)
            assert np.array_equal(orc.np_window(blk, rwin), orc.np_window(a, w)), (f, win)
            if subspan and (w[1] - 1) * abs(w[2]) + 1 < 500:
                assert dshape[0] < 1000  # channel span only
    with pytest.raises(pkg.BoundsError):
        fs.plan_window(a.shape, [0, 1001, 1, 0, 3, 1, 0, 37, 1])
    # not raw: chunked FBH5, 8-bit SIGPROC
    pkg.fbh5.write(h5, dict(foff=-1.0), a, chunks=(8, 1, 100))
    assert pkg.fbh5.raw_layout(h5) is None
    pkg.readers.write_fil(fil, dict(fch1=8000.0, foff=-1.0, nchans=1000, nifs=3, tsamp=1.0,
                                    nbits=8, telescope_id=6, machine_id=10, data_type=1,
                                    tstart=59000.0, source_name="X"), a.astype(np.uint8))
    assert pkg.readers.fil_raw_layout(fil) is None


def test_h5_chunk_index_parser(pkg, tmp_path):
    """h5chunks.chunk_table reads the chunk B-tree of ``data`` from the file;
    every entry must equal libhdf5's H5Dget_chunk_info_by_coord, and files
    outside its scope (contiguous layout) give None."""
    import ctypes

    from conftest import GOLDEN

    h5chunks = pkg.h5chunks
    fb = pkg.fbh5
    z = np.load(os.path.join(GOLDEN, "bslz4_v1.npz"), allow_pickle=False)
    chunk = z["chunk_gamma_chunk_b2048"].tobytes()
    c = str(tmp_path / "c.h5")
    fb.write_bslz4_chunks(c, dict(foff=-1.0, nfpc=64), (4096, 1, 16 * 300), (16, 1, 4096),
                          (chunk for _ in range(300)))
    a = np.asfortranarray(np.random.default_rng(1).random((1000, 3, 50), dtype=np.float32))
    dfl, cont = str(tmp_path / "d.h5"), str(tmp_path / "u.h5")
    fb.write(dfl, dict(foff=-1.0), a, chunks=(7, 1, 100), deflate=1)
    fb.write(cont, dict(foff=-1.0), a)
    H = fb.h5().L
    for f, nchunks in ((c, 300), (dfl, 8 * 3 * 10), (cont, None)):
        fid = H.H5Fopen(f.encode(), 0, 0)
        d = H.H5Dopen2(fid, b"data", 0)
        try:
            tab = h5chunks.chunk_table(f, H, d)
            if nchunks is None:
                assert tab is None
                continue
            assert len(tab["index"]) == nchunks
            for k, ent in tab["index"].items():
                off = (ctypes.c_uint64 * 3)(*k)
                m, ad, sz = ctypes.c_uint(), ctypes.c_uint64(), ctypes.c_uint64()
                assert H.H5Dget_chunk_info_by_coord(d, off, ctypes.byref(m), ctypes.byref(ad),
                                                    ctypes.byref(sz)) >= 0
                assert (ad.value, sz.value, m.value) == ent
        finally:
            H.H5Dclose(d)
            H.H5Fclose(fid)


def test_raw_file_window_plans_random(pkg, orc, tmp_path, monkeypatch):
    """filestream.plan_window on random windows (steps of either sign on every
    axis, both read plans) against numpy indexing of the same file."""
    fs = pkg.filestream
    rng = np.random.default_rng(5)
    a = np.asfortranarray(rng.integers(0, 256, (300, 3, 41)).astype(np.float32))
    f = str(tmp_path / "r.fil")
    pkg.readers.write_fil(f, dict(fch1=8000.0, foff=-1.0, nchans=300, nifs=3, tsamp=1.0,
                                  nbits=32, telescope_id=6, machine_id=10, data_type=1,
                                  tstart=59000.0, source_name="X"), a)
    base, jshape = pkg.readers.fil_raw_layout(f)
    for sub in (False, True):
        monkeypatch.setattr(fs, "SUBSPAN_MIN_BYTES", 1 if sub else 1 << 30)
        for _ in range(200):
            w = []
            for n in jshape:
                st = int(rng.integers(0, n))
                sp = int(rng.choice([1, 1, 2, 3, -1, -2]))
                cmax = (n - 1 - st) // sp + 1 if sp > 0 else st // (-sp) + 1
                w += [st, int(rng.integers(0, cmax + 1)), sp]
            runs, dshape, rwin = fs.plan_window(jshape, w, base)
            if not len(runs):
                assert w[1] * w[4] * w[7] == 0
                continue
            blk = fs.read_runs_host(f, runs).view(np.float32)
            blk = blk.reshape(dshape[::-1]).transpose(2, 1, 0)
            assert np.array_equal(orc.np_window(blk, rwin), orc.np_window(a, w)), w


def _random_bslz4_cases(orc, seed, count):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        n = int(rng.integers(1, 20000))
        kind = k % 5
        if kind == 0:
            a = np.zeros(n, np.float32)
        elif kind == 1:
            a = rng.integers(0, 4, n).astype(np.float32)
        elif kind == 2:
            a = rng.random(n).astype(np.float32)
        elif kind == 3:
            a = np.tile(rng.random(int(rng.integers(1, 40))).astype(np.float32), n)[:n]
        else:  # gamma power with a bandpass, like a filterbank
            a = (rng.gamma(2.0, 5e8, n) * (0.2 + 0.8 * np.cos(np.arange(n) / 200.0) ** 2)
                 ).astype(np.float32)
        block = int(rng.choice([8, 64, 256, 1024, 2048, 4096]))
        out.append((a, orc.np_bslz4_encode(a, block, lz4=orc.lz4_compress)))
    return out


def test_bslz4_host_decoder_random_lz4(pkg, orc):
    """The host bitshuffle/LZ4 decoder on random chunks whose LZ4 blocks carry
    real matches (overlapping ones included; oracle.lz4_compress), block sizes
    8..4096 elements, element counts with a raw tail."""
    for a, c in _random_bslz4_cases(orc, 99, 40):
        d = pkg.fbh5.bslz4_decode_host(c)
        assert np.array_equal(d.view(np.uint32), a.view(np.uint32)), (a.size, len(c))


def test_compressed_read_planning(pkg):
    """The vectorised planning of the compressed-FBH5 device read: batches
    are contiguous chunk ranges covering every chunk (a small first batch),
    and the pread tasks cover every stored chunk byte exactly once, each at
    the file offset of its chunk (adjacent chunks merged into one read)."""
    fb = pkg.fbh5
    rng = np.random.default_rng(5)
    for _ in range(20):
        n = int(rng.integers(1, 60))
        sizes = rng.integers(0, 50, n).astype(np.int64)
        sizes[rng.random(n) < 0.2] = 0
        b = fb._batches_of(sizes, 30, 120)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(x[1] == y[0] and x[0] < x[1] for x, y in zip(b, b[1:]))
        offsets = np.zeros(n, np.int64)
        offsets[1:] = np.cumsum(sizes[:-1])
        faddr = np.cumsum(sizes + rng.integers(0, 2, n) * 7) + 1000  # some gaps
        seen = np.zeros(int(sizes.sum()), np.int64)
        for k0, k1 in b:
            for task in fb._read_tasks(faddr, sizes, offsets, k0, k1, piece=16):
                for fo, do, m in task:
                    assert 0 < m <= 16
                    for q in range(m):
                        k = int(np.searchsorted(offsets, do + q, side="right")) - 1
                        while sizes[k] == 0:
                            k -= 1
                        assert fo + q == faddr[k] + (do + q - offsets[k])
                        seen[do + q] += 1
        assert np.all(seen == 1)


def test_file_metadata_cache_follows_rewrites(pkg, tmp_path):
    """layout/raw_layout/chunk_index are memoised per file version: a file
    rewritten in place (new size / inode / change time) is parsed again."""
    import time

    fb = pkg.fbh5
    p = tmp_path / "m.h5"
    a = np.zeros((64, 1, 8), np.float32, order="F")
    fb.write(p, dict(foff=-1.0, nfpc=8), a, chunks=(4, 1, 64))
    assert fb.layout(p)["cdims"] == (8, 1, 64)
    assert fb.layout(p) is fb.layout(p)  # cached
    time.sleep(0.01)
    fb.write(p, dict(foff=-1.0, nfpc=8), np.zeros((128, 1, 4), np.float32, order="F"))
    assert fb.layout(p)["cdims"] == (4, 1, 128)
    assert fb.raw_layout(p) is not None


def test_bench_spawns_its_ranks_without_a_launcher():
    """`python bench.py --gpus N` with no torch.distributed.run: bench.py starts
    the N rank processes itself (before touching torch or HIP), they meet over
    127.0.0.1, and rank 0 alone prints the JSON line (the launch and exchange
    path, no GPU work: --mode rendezvous)."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--mode", "rendezvous"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["world_size"] == 2
    assert d["config"]["gathered_ranks"] == [0, 1] and d["value"] == 2.0


def test_bench_spawned_ranks_fail_fast():
    """One self-spawned rank dies before the rendezvous: bench.py stops the
    others (blocked in init_process_group, whose own timeout is 30 min) and
    returns that rank's status within seconds (spawn_ranks polls its ranks)."""
    import subprocess
    import sys
    import time

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for bad in ("1", "0"):
        env["BENCH_RENDEZVOUS_FAIL_RANK"] = bad
        t0 = time.time()
        r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                            "--dist-backend", "gloo", "--mode", "rendezvous"],
                           capture_output=True, text=True, timeout=120, env=env)
        el = time.time() - t0
        assert r.returncode == 3, (bad, r.returncode, r.stderr[-2000:])
        assert el < 60, el
        assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_spawned_ranks_deadline():
    """A self-spawned rank that hangs (here: before the rendezvous, where its
    peer blocks in init_process_group; on a GPU node, in an RCCL collective)
    never exits, so no exit status reports it: spawn_ranks stops every rank
    at --rank-deadline and bench.py returns 124."""
    import subprocess
    import sys
    import time

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BENCH_RENDEZVOUS_HANG_RANK"] = "1"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--mode", "rendezvous", "--rank-deadline", "20"],
                       capture_output=True, text=True, timeout=120, env=env)
    el = time.time() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert 20 <= el < 60, el
    assert "deadline" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_despike_host_keeps_the_result_type(pkg):
    """getband's host despike for non-Float32 bands (integer sums, Float64):
    d[spike:nfpc:end, :, :] .= d[spike-1:nfpc:end, :, :] with spike = nfpc÷2+1
    (src/gbt.jl:101-102,111) in the band's own element type (the
    Float32 device despike cast a UInt64 / Float64 band to Float32)."""
    nfpc = 8
    d = np.asfortranarray((np.arange(32 * 2 * 3, dtype=np.uint64) * (2 ** 40 + 3)).reshape(
        (32, 2, 3), order="F"))
    want = d.copy(order="F")
    for c in range(nfpc // 2, 32, nfpc):  # 0-based spike bin nfpc/2 takes its left neighbour
        want[c] = want[c - 1]
    got = pkg.GBT._despike_host(d.copy(order="F"), nfpc)
    assert got.dtype == np.uint64 and np.array_equal(got, want)
    f = np.asfortranarray(np.random.default_rng(1).standard_normal((16, 1, 2)))
    g = pkg.GBT._despike_host(f.copy(order="F"), 4)
    assert g.dtype == np.float64 and np.array_equal(g[2::4], f[1::4])
    with pytest.raises(pkg.BoundsError):
        pkg.GBT._despike_host(f.copy(order="F"), 1)
    with pytest.raises(pkg.DimensionMismatch):  # 3 spike bins vs 4 source bins
        pkg.GBT._despike_host(np.zeros((14, 1, 1)), 4)
