"""CPU: the C-ABI library loads, exports every symbol include/bldp.h declares,
and its host-only entry points (shape, plan, range, argument checks) behave
like the reference without a GPU."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO


def declared_symbols():
    src = open(os.path.join(REPO, "include", "bldp.h")).read()
    return sorted(set(re.findall(r"BLDP_API\s+\w+\s+(bldp_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def L(pkg):
    return pkg._lib.lib()


def test_header_and_binding_agree(pkg):
    decl = declared_symbols()
    assert len(decl) >= 15
    assert sorted(pkg._lib.SIGNATURES) == decl


def test_library_exports_every_declared_symbol(pkg, L):
    out = subprocess.run(["nm", "-D", "--defined-only", pkg._lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (bldp_\w+)", out))
    missing = set(declared_symbols()) - exported
    assert not missing, missing
    for s in declared_symbols():
        assert getattr(L, s) is not None
    assert L.bldp_abi_version() == pkg._lib.ABI_VERSION == 5


def test_library_is_gfx950_code(pkg):
    blob = open(pkg._lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_error_path(pkg, L):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    n = ctypes.c_int(-1)
    rc = L.bldp_device_count(ctypes.byref(n))
    assert rc == pkg._lib.BLDP_EHIP
    assert "device" in pkg._lib.last_error().lower()


def test_reduce_shape_and_errors(pkg, L):
    sh = (ctypes.c_int64 * 3)()
    assert L.bldp_reduce_shape(65536, 1, 279, None, 64, 1, sh) == 0
    assert list(sh) == [1024, 1, 279]
    keep, wp = pkg._lib.win_arg([0, 65536, 1, 0, 1, 1, 0, 272, 1])  # idxs=(:, :, 1:272)
    assert L.bldp_reduce_shape(65536, 1, 279, wp, 64, 16, sh) == 0
    assert list(sh) == [1024, 1, 17]
    assert L.bldp_reduce_shape(65536, 1, 279, None, 64, 16, sh) == pkg._lib.BLDP_EDIM
    assert "tavby=16" in pkg._lib.last_error()
    assert L.bldp_reduce_shape(100, 1, 10, None, 3, 1, sh) == pkg._lib.BLDP_EDIM
    assert "DimensionMismatch" in pkg._lib.last_error()
    keep, wp = pkg._lib.win_arg([90, 20, 1, 0, 1, 1, 0, 10, 1])
    assert L.bldp_reduce_shape(100, 1, 10, wp, 1, 1, sh) == pkg._lib.BLDP_EBOUNDS
    keep, wp = pkg._lib.win_arg([0, 10, 0, 0, 1, 1, 0, 10, 1])
    assert L.bldp_reduce_shape(100, 1, 10, wp, 1, 1, sh) == pkg._lib.BLDP_EINVAL
    # n <= 1 disables an axis (fqav returns A, src/gbtworkerfunctions.jl:17)
    assert L.bldp_reduce_shape(7, 3, 5, None, 0, -2, sh) == 0 and list(sh) == [7, 3, 5]


def test_fqav_range_kats_through_abi(L):
    f, s, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
    assert L.bldp_fqav_range(1.0, 1.0, 4, 4, ctypes.byref(f), ctypes.byref(s), ctypes.byref(n)) == 0
    assert (f.value, s.value, n.value) == (2.5, 4.0, 1)  # test/runtests.jl:5
    assert L.bldp_fqav_range(1.0, 2.0, 8, 4, ctypes.byref(f), ctypes.byref(s), ctypes.byref(n)) == 0
    assert (f.value, s.value, n.value) == (4.0, 8.0, 2)  # test/runtests.jl:6


def plan(pkg, L, ptr, nchan, nif, ntime, F, T, win=None):
    info = (ctypes.c_int64 * 8)()
    keep, wp = pkg._lib.win_arg(win)
    rc = L.bldp_reduce_plan_f32(ptr, nchan, nif, ntime, wp, F, T, 0, None, info)
    assert rc == 0, pkg._lib.last_error()
    return list(info)


def test_launch_plans_host_only(pkg, L):
    A = 1 << 20  # any 16-byte aligned address
    # cfg3 bank: interleaved vector path, 2 groups of 1024 channels per
    # workgroup (each 4 float4 per row per lane-column)
    p = plan(pkg, L, A, 1 << 26, 1, 16, 1024, 16)
    assert p[0] == 4 and p[1] == 64 and p[3] == 4 and p[4] == 1
    assert p[5] == 65536 // 2
    # F = 512 / 2048 / 4096 interleave too; F = 8192 and split time blocks do not
    assert plan(pkg, L, A, 1 << 26, 1, 16, 512, 16)[0] == 4
    assert plan(pkg, L, A, 1 << 26, 1, 16, 2048, 16)[0] == 4
    assert plan(pkg, L, A, 1 << 26, 1, 16, 4096, 16)[0] == 4
    assert plan(pkg, L, A, 1 << 26, 1, 16, 8192, 16)[0] == 0
    assert plan(pkg, L, A, 4096, 1, 4096, 1024, 4096)[0] == 0
    # cfg1: F=64 -> 16 lanes per group, one float4 each: the row kernel; one
    # file is a small launch (< 64 tiles per CU), so each 16-row block is
    # split over 4 workgroup slices (k_reduce_rows: 256 channels per
    # workgroup), 2 at F = 256; a 0000 bank is not split; forced forms
    w272 = [0, 65536, 1, 0, 1, 1, 0, 272, 1]
    p = plan(pkg, L, A, 65536, 1, 279, 64, 16, w272)
    assert p[0] == 5 and p[1] == 16 and p[2] == 4 and p[3] == 1 and p[5] == 256 * 17
    p = plan(pkg, L, A, 65536, 1, 279, 256, 16, w272)
    assert p[0] == 5 and p[2] == 2 and p[5] == 128 * 17
    p = plan(pkg, L, A, 1 << 26, 1, 16, 64, 16)
    assert p[0] == 5 and p[2] == 1 and p[5] == 65536
    for S, wg in ((1, 64 * 17), (2, 128 * 17), (4, 256 * 17)):
        with pkg._lib.plan_option("row_split", S):
            p = plan(pkg, L, A, 65536, 1, 279, 64, 16, w272)
            assert p[0] == 5 and p[2] == S and p[5] == wg, (S, p)
    # tavby = 9 (no whole 16-row batch): k_reduce_row, whatever the option says
    with pkg._lib.plan_option("row_split", 4):
        p = plan(pkg, L, A, 65536, 1, 279, 64, 9, [0, 65536, 1, 0, 1, 1, 0, 270, 1])
        assert p[0] == 5 and p[2] == 1
    with pytest.raises(pkg._lib.ArgumentError):
        pkg._lib.check(L.bldp_plan_option(b"no_such_option", 1, None))
    # a small launch at tavby = 8: one 8-row block per workgroup (k_reduce_row)
    # where its grid holds the time blocks, else k_reduce_rowt
    assert plan(pkg, L, A, 65536, 1, 279, 64, 8, w272)[5] == 64 * 34
    p = plan(pkg, L, A, 256, 1, 8 * 70000, 4, 8)
    assert p[0] == 5 and p[5] == -(-70000 // 2 // 4)
    # too few tiles for one wave per tile: waves split time, generic kernel
    assert plan(pkg, L, A, 4096, 1, 64, 64, 16)[0] == 0
    # cfg4: narrow channel, long time -> time split waves and/or chunks
    p = plan(pkg, L, A, 512, 1, 879616, 8, 1024)
    assert p[0] == 0 and p[1] == 2 and (p[2] > 1 or p[4] > 1)
    # F=1 time-only: narrow path; F = 2, 3, 5, 6, 7 with an odd pitch (the tile
    # path needs 16-byte pitches): one lane per output; odd pitch with a wide
    # F: scalar
    assert plan(pkg, L, A, 4096, 1, 16, 1, 16)[0] == 1
    assert plan(pkg, L, A, 4095, 1, 16, 3, 1)[0] == 7
    assert plan(pkg, L, A + 2, 4095, 1, 16, 3, 1)[0] == 2
    assert plan(pkg, L, A, 4095, 1, 16, 4095, 1)[0] == 2
    # a dword-aligned pointer or window start off a 16-byte boundary: dword-aligned
    # 16-byte loads on the row / narrow / interleaved kernels (BLDP_UNALIGNED_VEC);
    # a pointer that is not even dword-aligned: scalar
    assert plan(pkg, L, A + 4, 4096, 1, 16, 64, 1)[0] == 5
    assert plan(pkg, L, A + 2, 4096, 1, 16, 64, 1)[0] == 2
    assert plan(pkg, L, A, 4096, 1, 16, 64, 16, [1, 4032, 1, 0, 1, 1, 0, 16, 1])[0] in (0, 5)
    assert plan(pkg, L, A, 4096, 1, 16, 1, 1, [1, 4092, 1, 0, 1, 1, 0, 16, 1])[0] == 1
    assert plan(pkg, L, A, 4097, 1, 8, 1024, 8, [0, 4096, 1, 0, 1, 1, 0, 8, 1])[0] == 4
    # F = 3, 5, 6, 7, 12 with short time blocks (T = 1, 2, 3, 4, 8): one lane per
    # group, several time blocks per workgroup (k_reduce_lanet); with long time
    # blocks and 16-byte pitches the tile path keeps them, except F = 3 (one
    # dwordx3 per lane: the lane kernel everywhere)
    assert plan(pkg, L, A, 4096, 1, 16, 3, 1, [0, 4095, 1, 0, 1, 1, 0, 16, 1])[0] == 7
    assert plan(pkg, L, A, 4096, 1, 16, 12, 1, [0, 4092, 1, 0, 1, 1, 0, 16, 1])[0] == 7
    assert plan(pkg, L, A, 4096, 1, 16, 3, 16, [0, 4095, 1, 0, 1, 1, 0, 16, 1])[0] == 7
    assert plan(pkg, L, A, 4096, 1, 16, 5, 16, [0, 4095, 1, 0, 1, 1, 0, 16, 1])[0] == 3
    # tile path: odd F > 7, misaligned channel start with F >= 512, short channel step
    assert plan(pkg, L, A, 4096, 1, 16, 9, 1, [0, 4095, 1, 0, 1, 1, 0, 16, 1])[0] == 3
    assert plan(pkg, L, A, 4096, 1, 16, 1024, 16, [1, 3072, 1, 0, 1, 1, 0, 16, 1])[0] == 3
    # misaligned start, F = 1, a channel count that is not a multiple of 4:
    # the realigning narrow kernel
    assert plan(pkg, L, A, 4096, 1, 16, 1, 1, [1, 4094, 1, 0, 1, 1, 0, 16, 1])[0] == 6
    assert plan(pkg, L, A, 4096, 1, 16, 2, 4, [3, 4092, 1, 0, 1, 1, 0, 16, 1])[0] == 3  # F=2: tile
    assert plan(pkg, L, A, 4096, 1, 16, 1, 1, [0, 2048, 2, 0, 1, 1, 0, 16, 1])[0] == 3
    assert plan(pkg, L, A, 4096, 1, 16, 16, 1, [0, 2048, 2, 0, 1, 1, 0, 16, 1])[0] == 3
    # ... but not a reversed step, a step > 8, or a group wider than a tile row
    assert plan(pkg, L, A, 4096, 1, 16, 16, 1, [4095, 2048, -2, 0, 1, 1, 0, 16, 1])[0] == 2
    assert plan(pkg, L, A, 4096, 1, 16, 16, 1, [0, 256, 16, 0, 1, 1, 0, 16, 1])[0] == 2
    assert plan(pkg, L, A, 8192, 1, 4, 4094, 1, [1, 8188, 1, 0, 1, 1, 0, 4, 1])[0] == 2
    assert plan(pkg, L, A, 8192, 1, 4, 4093, 1, [1, 8186, 1, 0, 1, 1, 0, 4, 1])[0] == 3
    # one long time block with few outputs -> chunked across workgroups
    p = plan(pkg, L, A, 64, 1, 100000, 8, 100000)
    assert p[4] > 1 and p[6] > 0


def test_null_pointer_rejected(pkg, L):
    assert L.bldp_reduce_f32(None, 64, 1, 4, None, 4, 1, 0, None, None) == pkg._lib.BLDP_EINVAL
    assert L.bldp_reduce_f32(None, 64, 1, 4, None, 4, 1, 9, None, None) == pkg._lib.BLDP_EINVAL
    assert "op" in pkg._lib.last_error()


def test_empty_calls_are_noops(pkg, L):
    assert L.bldp_reduce_f32(None, 64, 1, 0, None, 4, 1, 0, None, None) == 0
    assert L.bldp_despike_f32(None, 0, 1, 1, 16, None) == 0
    sz = L.bldp_kurtosis_workspace_size(512, 1, 880000, None)
    assert sz > 512 * 8


def test_despike_and_stitch_argument_checks(pkg, L):
    assert L.bldp_despike_f32(None, 10, 1, 1, 4, None) == pkg._lib.BLDP_EDIM
    assert L.bldp_despike_f32(None, 10, 1, 1, 1, None) == pkg._lib.BLDP_EBOUNDS
    assert L.bldp_stitch_f32(0, None, 4, 1, 1, None, None) == pkg._lib.BLDP_EINVAL
    buf = np.zeros(16, np.float32)
    assert L.bldp_stitch_f32(2, buf.ctypes.data, 4, 2, 1, buf.ctypes.data, None) == \
        pkg._lib.BLDP_EINVAL


def test_native_comm_host_checks(pkg, L):
    """bldp_comm_*: an RCCL unique id is made on the host; the argument
    checks answer without a GPU (the cross-GPU band stitch
    through the C ABI)."""
    import ctypes

    nid = pkg.band.NativeBand.new_id()
    assert len(nid) == pkg._lib.BLDP_COMM_ID_BYTES and any(nid)
    assert L.bldp_comm_id(None) == pkg._lib.BLDP_EINVAL
    assert L.bldp_band_gather_f32(None, 0, None, 4, None, None) == pkg._lib.BLDP_EINVAL
    assert "communicator" in pkg._lib.last_error()
    assert L.bldp_comm_destroy(None) == pkg._lib.BLDP_OK
    h = ctypes.c_void_p()
    assert L.bldp_comm_init(0, 2, 2, None, ctypes.byref(h)) == pkg._lib.BLDP_EINVAL


def test_empty_windows_plan_without_fault(pkg, L):
    """Regression (found by the random-window test): an empty window with a
    long time block used to divide by zero while planning the time split
    (SIGFPE in the host process).  Planning, reducing and kurtosis of empty
    windows are no-ops."""
    A = 1 << 20
    for win, F, T in (([155, 115, 1, 1, 1, 1, 25, 0, 1], 5, 128),
                      ([0, 0, 1, 0, 1, 1, 0, 64, 1], 8, 64),
                      ([0, 64, 1, 0, 0, 1, 0, 256, 1], 8, 256)):
        info = (ctypes.c_int64 * 8)()
        keep, wp = pkg._lib.win_arg(win)
        assert L.bldp_reduce_plan_f32(A, 271, 2, 300, wp, F, T, 0, None, info) == 0
        assert L.bldp_reduce_f32(A, 271, 2, 300, wp, F, T, 0, None, None) == 0
        assert L.bldp_kurtosis_workspace_size(271, 2, 300, wp) >= 0


def test_unchunk_argument_checks(pkg, L):
    """bldp_unchunk_f32 (the device gather from decoded FBH5 chunks) checks
    the window against the chunk box on the host, before any launch: no
    window element may fall outside the decoded bytes, and counts/steps that
    would overflow the last-index product are refused too."""
    i3 = lambda *v: (ctypes.c_int64 * 3)(*v)  # noqa: E731
    chunk, box0, grid = i3(4, 1, 64), i3(8, 0, 128), i3(2, 1, 3)  # t 8..15, c 128..319

    def call(win, packed=None, out=None):
        return L.bldp_unchunk_f32(packed, chunk, box0, grid, (ctypes.c_int64 * 9)(*win), out,
                                  None)

    ok = [128, 192, 1, 0, 1, 1, 8, 8, 1]
    assert call(ok) == pkg._lib.BLDP_EINVAL  # in bounds: only the null buffers remain
    assert "null" in pkg._lib.last_error()
    for bad in ([127, 4, 1, 0, 1, 1, 8, 2, 1],       # channel before the box
                [300, 21, 1, 0, 1, 1, 8, 2, 1],      # channel past the box
                [319, 193, -1, 0, 1, 1, 8, 1, 1],    # reversed, one past the start
                [128, 2, 1, 0, 1, 1, 15, 2, 1],      # time past the box
                [128, 2, 1, 0, 2, 1, 8, 1, 1],       # IF past the box
                [128, 1 << 62, 4, 0, 1, 1, 8, 1, 1],  # count x step would overflow
                [128, 2, 1 << 62, 0, 1, 1, 8, 1, 1],
                [128, 2, -(1 << 62), 0, 1, 1, 8, 1, 1]):
        assert call(bad) == pkg._lib.BLDP_EBOUNDS, bad
    assert call([128, 0, 1, 0, 1, 1, 8, 2, 1]) == 0  # empty window: no-op, no pointers
    assert call([128, 2, 1, 0, 1, 1, 8, 2, -1]) == pkg._lib.BLDP_EBOUNDS  # t 8, 7
    assert L.bldp_unchunk_f32(None, i3(0, 1, 64), box0, grid, (ctypes.c_int64 * 9)(*ok), None,
                              None) == pkg._lib.BLDP_EINVAL
    assert L.bldp_unchunk_f32(None, None, box0, grid, None, None, None) == pkg._lib.BLDP_EINVAL


def test_kurtosis_empty_windows_long_time_plan_without_fault(pkg, L):
    """Regression for the kurtosis planner's sibling of the SIGFPE above (an
    empty channel or IF window with more than 512 spectra divided by zero
    while sizing the merge): workspace size, plan and the calls themselves are
    host-side no-ops for empty windows, whatever the time span."""
    A = 1 << 20
    ptrs = (ctypes.c_void_p * 2)(A, A)
    for win in ([5, 0, 1, 0, 2, 1, 0, 5000, 1],      # no channels, 5000 spectra
                [0, 64, 1, 1, 0, 1, 0, 880000, 1],    # no IFs
                [0, 0, 1, 0, 0, 1, 10, 600, 1]):
        keep, wp = pkg._lib.win_arg(win)
        assert L.bldp_kurtosis_workspace_size(271, 2, 880000, wp) == 0
        info = (ctypes.c_int64 * 4)()
        assert L.bldp_kurtosis_plan_f32(A, 271, 2, 880000, wp, info) == 0
        assert L.bldp_kurtosis_f32(A, 271, 2, 880000, wp, None, None, None) == 0
        assert L.bldp_band_kurtosis_f32(2, ptrs, 271, 2, 880000, wp, None, None) == 0


def _pw_leaves(n):
    """Leaves of Base.mapreduce_impl's recursion over [0, n) (0-based, inclusive)."""
    out = []

    def rec(lo, hi):
        if hi - lo < 1024:
            out.append((lo, hi - lo + 1))
        else:
            mid = lo + ((hi - lo) >> 1)
            rec(lo, mid)
            rec(mid + 1, hi)

    rec(0, n - 1)
    return out


@pytest.mark.parametrize("n", [1, 33, 512, 513, 1024, 1025, 2048, 2049, 4095, 4096, 4097,
                               70001, 131073, 879616, 880000, 2200001])
def test_kurtosis_plan_pairwise_blocks(pkg, L, n):
    """bldp_kurtosis_plan_f32 reports the level K of the pairwise-sum blocks
    and 2^(K+1) leaf slots; slot s = 2j + h of block j (kurtosis.hip pw_leaf,
    restated here) reproduces exactly the leaves of Julia's recursion, in
    order, so the kernels' Float32 leaf sums and the perfect tree above them
    are Base.sum's."""
    A = 1 << 20
    info = (ctypes.c_int64 * 4)()
    assert L.bldp_kurtosis_plan_f32(A, 64, 1, n, None, info) == 0
    path, K, nslot, ws = list(info)
    assert path == (0 if n <= 32 else 1 if n <= 512 else 2)
    assert nslot == 2 << K

    def node(L_, j):
        lo, ln = 0, n
        for l_ in range(L_ - 1, -1, -1):
            left = (ln + 1) >> 1
            if (j >> l_) & 1:
                lo, ln = lo + left, ln - left
            else:
                ln = left
        return lo, ln

    leaves = []
    for s in range(nslot):
        lo, ln = node(K, s >> 1)
        if ln > 1024:
            left = (ln + 1) >> 1
            lo, ln = (lo + left, ln - left) if s & 1 else (lo, left)
        elif s & 1:
            ln = 0
        if ln:
            leaves.append((lo, ln))
    assert leaves == _pw_leaves(n)
    # the tree above level K is perfect: every node there is split (> 1024)
    for lev in range(K):
        assert all(node(lev, j)[1] > 1024 for j in range(1 << lev))
    if path == 2:
        assert ws >= 64 * nslot * (4 * 8 + 3 * 4)
    # a dword-aligned (not 16-byte aligned) pointer keeps the float4 plan
    # (gfx950 16-byte loads at dword alignment); a channel count that is not a
    # multiple of 4 takes the register tile up to 512 spectra (any alignment),
    # else two passes
    assert L.bldp_kurtosis_plan_f32(A + 4, 64, 1, n, None, info) == 0
    assert info[0] == path and info[1] == K
    w = (ctypes.c_int64 * 9)(1, 62, 1, 0, 1, 1, 0, n, 1)
    assert L.bldp_kurtosis_plan_f32(A, 64, 1, n, w, info) == 0
    assert info[0] == (1 if n <= 512 else 3) and info[1] == K


def test_bslz4_slot_size_checked_before_launch(pkg, L):
    """the device decode takes each chunk's output slot size and
    refuses a chunk whose header claims another size on the host, before any
    launch (so this runs without a GPU: the device pointers are never used)."""
    import struct

    body = struct.pack(">I", 3) + b"\0\0\0"
    for claim, slot in ((2 * 8192, 8192), (8192 - 32, 8192)):
        chunk = struct.pack(">QI", claim, 8192) + body
        h = np.frombuffer(chunk, np.uint8)
        off = np.zeros(1, np.uint64)
        n = np.array([len(chunk)], np.uint64)
        olen = np.array([slot], np.uint64)
        fake = 1 << 20  # never dereferenced: the check precedes every HIP call
        rc = L.bldp_bslz4_decode_dev(1, h.ctypes.data, fake, off.ctypes.data, n.ctypes.data, 4,
                                     fake, off.ctypes.data, olen.ctypes.data, None)
        assert rc == pkg._lib.BLDP_EINVAL and "slot" in pkg._lib.last_error()
        rc = L.bldp_bslz4_decode_dev_async(1, h.ctypes.data, fake, off.ctypes.data,
                                           n.ctypes.data, 4, fake, off.ctypes.data,
                                           olen.ctypes.data, fake, None)
        assert rc == pkg._lib.BLDP_EINVAL
    assert L.bldp_bslz4_decode_dev(1, h.ctypes.data, fake, off.ctypes.data, n.ctypes.data, 4,
                                   fake, off.ctypes.data, None, None) == pkg._lib.BLDP_EINVAL


def test_chunks_to_device_validates_before_any_read(pkg, L):
    """bldp_chunks_to_device (the native chunk reader) checks its tables on the
    host before it reads or touches a device: batches that do not end at the
    last chunk, negative sizes, an unfiltered chunk of the wrong size,
    compressed chunks without an output."""
    fake = 1 << 20  # never dereferenced: every check precedes the reads
    fa = np.array([0, 100], np.int64)
    sz = np.array([100, 100], np.int64)
    of = np.array([0, 100], np.int64)
    mk = np.zeros(2, np.uint32)

    def call(fa=fa, sz=sz, of=of, mk=mk, bend=(2,), out=fake, ocb=400, stage=200, obytes=800):
        be = np.array(bend, np.int64)
        return L.bldp_chunks_to_device(-1, len(sz), fa.ctypes.data, sz.ctypes.data,
                                       of.ctypes.data, mk.ctypes.data, len(be), be.ctypes.data,
                                       fake, fake, stage, out, ocb, obytes, fake, None, None, None)

    assert call(bend=(1,)) == pkg._lib.BLDP_EINVAL and "end at chunk" in pkg._lib.last_error()
    assert call(bend=(2, 1)) == pkg._lib.BLDP_EINVAL
    assert call(sz=np.array([100, -1], np.int64)) == pkg._lib.BLDP_EINVAL
    assert call(mk=np.ones(2, np.uint32)) == pkg._lib.BLDP_EINVAL  # raw chunk of 100 B, slot 400
    assert call(out=None) == pkg._lib.BLDP_EINVAL and "output" in pkg._lib.last_error()
    assert call(stage=199) == pkg._lib.BLDP_EINVAL and "staging" in pkg._lib.last_error()
    assert call(obytes=799) == pkg._lib.BLDP_EINVAL and "exceed" in pkg._lib.last_error()
    assert L.bldp_chunks_to_device(-1, 0, None, None, None, None, 0, None, None, None, 0, None, 0,
                                   0, None, None, None, None) == 0  # nothing to do
    # host_pinned NULL (the library's slot ring): the same checks, before any
    # ring is allocated or a device is touched
    be = np.array([1], np.int64)
    assert L.bldp_chunks_to_device(-1, len(sz), fa.ctypes.data, sz.ctypes.data, of.ctypes.data,
                                   mk.ctypes.data, 1, be.ctypes.data, None, fake, 200, fake, 400,
                                   800, fake, None, None, None) == pkg._lib.BLDP_EINVAL
    assert "end at chunk" in pkg._lib.last_error()
    assert L.bldp_chunks_to_device(-1, len(sz), fa.ctypes.data, sz.ctypes.data, of.ctypes.data,
                                   mk.ctypes.data, 1, be.ctypes.data, None, None, 200, fake, 400,
                                   800, fake, None, None, None) == pkg._lib.BLDP_EINVAL


def test_runs_to_device_validates_before_any_read(pkg, L):
    """bldp_runs_to_device rejects bad tables and slot geometry on the host."""
    fake = 1 << 20
    fo = np.array([0, 10], np.int64)
    ln = np.array([10, -1], np.int64)
    assert L.bldp_runs_to_device(-1, 2, fo.ctypes.data, ln.ctypes.data, fake, 20, 64 << 20, 4,
                                 None, None, None) == pkg._lib.BLDP_EINVAL
    ln = np.array([10, 10], np.int64)
    assert L.bldp_runs_to_device(-1, 2, fo.ctypes.data, ln.ctypes.data, fake, 20, 1024, 4,
                                 None, None, None) == pkg._lib.BLDP_EINVAL  # slots < 1 MiB
    assert L.bldp_runs_to_device(-1, 2, fo.ctypes.data, ln.ctypes.data, fake, 20, 64 << 20, 1,
                                 None, None, None) == pkg._lib.BLDP_EINVAL  # one slot
    assert L.bldp_runs_to_device(-1, 2, fo.ctypes.data, ln.ctypes.data, fake, 19, 64 << 20, 4,
                                 None, None, None) == pkg._lib.BLDP_EINVAL  # 20 bytes into 19
    assert L.bldp_runs_to_device(-1, 0, None, None, None, 0, 64 << 20, 4, None, None, None) == 0


# ---- the Julia binding's ccalls against the header --------------------------
# Julia is absent here and on the GPU box, so julia/BLDPHip.jl cannot run; its
# ABI contract can still be checked: every ccall names a declared entry point
# with the same return type and the same argument types, position by position.
_C_TO_JL = {"int": "Cint", "int64_t": "Int64", "size_t": "Csize_t", "uint64_t": "UInt64",
            "uint32_t": "UInt32", "uint8_t": "UInt8", "char": "UInt8", "float": "Float32",
            "double": "Float64", "void": "Cvoid", "bldp_reduce_op_t": "Ptr{Cvoid}",
            "unsigned": "Cuint"}


def _c_param_to_jl(p):
    p = p.replace("const", " ").strip()
    arrays = p.count("[")
    p = re.sub(r"\[[^\]]*\]", "", p)
    stars = p.count("*")
    words = p.replace("*", " ").split()
    base = words[0] if words else ""
    t = _C_TO_JL[base]
    for _ in range(stars + arrays):
        t = "Ptr{%s}" % t
    return t


def _header_signatures():
    src = open(os.path.join(REPO, "include", "bldp.h")).read()
    sigs = {}
    for ret, name, params in re.findall(r"BLDP_API\s+(\w+)\s+(bldp_\w+)\s*\(([^)]*)\)\s*;", src):
        params = " ".join(params.split())
        args = [] if params in ("", "void") else [_c_param_to_jl(x) for x in params.split(",")]
        sigs[name] = (_C_TO_JL[ret], args)
    return sigs


def _split_top(s):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _julia_ccalls():
    src = open(os.path.join(REPO, "bldistributeddataproducts.jl_amd", "julia", "BLDPHip.jl")).read()
    calls = re.findall(r"ccall\(\(:(bldp_\w+),\s*libbldp\),\s*(\w+),\s*\(([^()]*)\)", src, re.S)
    return [(n, r, _split_top(" ".join(a.split()))) for n, r, a in calls]


def test_julia_binding_ccalls_match_the_header():
    sigs = _header_signatures()
    calls = _julia_ccalls()
    assert len(calls) >= 12
    for name, ret, args in calls:
        assert name in sigs, name
        want_ret, want_args = sigs[name]
        assert ret == want_ret, (name, ret, want_ret)
        # Julia passes a C array parameter as Ptr{T} and const pointers alike
        assert args == want_args, (name, args, want_args)
    # the binding covers the Julia worker's whole drop-in surface
    named = {n for n, _, _ in calls}
    for n in ("bldp_reduce_host_f32", "bldp_kurtosis_host_f32", "bldp_reduce_shape",
              "bldp_last_error", "bldp_band_gather_f32", "bldp_comm_init"):
        assert n in named, n


def test_julia_binding_abi_version_is_the_headers():
    """BLDPHip.__init__ refuses a library whose bldp_abi_version differs from
    the ABI_VERSION it was written against: that constant must be the
    header's BLDP_ABI_VERSION (the ccall signatures above are checked against
    the same header), or every Julia worker fails at load."""
    hdr = open(os.path.join(REPO, "include", "bldp.h")).read()
    jl = open(os.path.join(REPO, "bldistributeddataproducts.jl_amd", "julia", "BLDPHip.jl")).read()
    want = int(re.search(r"#define BLDP_ABI_VERSION (\d+)", hdr).group(1))
    got = int(re.search(r"^const ABI_VERSION = (\d+)$", jl, re.M).group(1))
    assert got == want, (got, want)


def test_typed_entry_points_host_checks(pkg, L):
    """Julia's fqav result element types (bldp_reduce_out_dtype, host only) and
    the typed entry points' argument checks (nothing is launched)."""
    D = {"f32": 0, "f64": 1, "u8": 2, "u16": 3, "u32": 4, "u64": 5, "i8": 6, "i16": 7, "i32": 8,
         "i64": 9}
    for t in ("u8", "u16", "u32", "u64"):
        assert L.bldp_reduce_out_dtype(D[t], 0) == D["u64"]
    for t in ("i8", "i16", "i32", "i64"):
        assert L.bldp_reduce_out_dtype(D[t], 0) == D["i64"]
    for t in D:
        assert L.bldp_reduce_out_dtype(D[t], 1) == (D["f32"] if t == "f32" else D["f64"])
        assert L.bldp_reduce_out_dtype(D[t], 2) == D[t] == L.bldp_reduce_out_dtype(D[t], 3)
    assert L.bldp_reduce_out_dtype(D["f64"], 0) == D["f64"]
    assert L.bldp_reduce_out_dtype(42, 0) == pkg._lib.BLDP_EINVAL
    assert L.bldp_reduce_out_dtype(D["u8"], 9) == pkg._lib.BLDP_EINVAL
    assert L.bldp_reduce_strided(42, None, 64, 1, 4, None, 4, 1, 0, None, 16, 16, None) == \
        pkg._lib.BLDP_EINVAL
    assert L.bldp_reduce_strided(D["u8"], None, 64, 1, 4, None, 3, 1, 0, None, 16, 16, None) == \
        pkg._lib.BLDP_EDIM
    assert L.bldp_reduce_strided(D["u8"], None, 64, 1, 4, None, 4, 1, 0, None, 16, 16, None) == \
        pkg._lib.BLDP_EINVAL  # null pointers
    assert L.bldp_kurtosis(42, None, 64, 1, 4, None, None, None) == pkg._lib.BLDP_EINVAL
    w = (ctypes.c_int64 * 9)(0, 65, 1, 0, 1, 1, 0, 4, 1)
    assert L.bldp_kurtosis(D["u16"], None, 64, 1, 4, w, None, None) == pkg._lib.BLDP_EBOUNDS
    assert pkg.engine.out_dtype(np.dtype(np.uint8), "sum") == np.uint64
    assert pkg.engine.out_dtype(np.dtype(np.int16), "mean") == np.float64


def test_plan_options_documented_and_accepted(pkg, L):
    """Every plan option named in include/bldp.h is accepted by
    bldp_plan_option, reads back what was set, and resets with -1; the
    planner's defaults come back after the reset."""
    src = open(os.path.join(REPO, "include", "bldp.h")).read()
    block = src[src.index("Process-wide plan options"):src.index("BLDP_API int bldp_plan_option")]
    names = re.findall(r'"([a-z0-9_]+)"', block)
    assert len(names) >= 20, names
    A = 1 << 20
    base = plan(pkg, L, A, 65536, 1, 279, 64, 16, [0, 65536, 1, 0, 1, 1, 0, 272, 1])
    for n in names:
        v = 1
        prev = ctypes.c_int64(99)
        assert L.bldp_plan_option(n.encode(), v, ctypes.byref(prev)) == 0, n
        assert prev.value == -1, (n, prev.value)
        assert L.bldp_plan_option(n.encode(), -1, ctypes.byref(prev)) == 0, n
        assert prev.value == v, (n, prev.value)
    assert plan(pkg, L, A, 65536, 1, 279, 64, 16, [0, 65536, 1, 0, 1, 1, 0, 272, 1]) == base
    # an option changes the plan it names, and the reset restores it
    with pkg._lib.plan_option("vec_row", 0):
        assert plan(pkg, L, A, 65536, 1, 279, 64, 16, [0, 65536, 1, 0, 1, 1, 0, 272, 1])[0] == 0
    assert plan(pkg, L, A, 65536, 1, 279, 64, 16, [0, 65536, 1, 0, 1, 1, 0, 272, 1]) == base


def test_plan_option_domains_checked(pkg, L):
    """bldp_plan_option rejects values outside an option's domain (ADVICE r04:
    huge values multiplied by the CU count, out-of-domain forms silently
    coerced) with BLDP_EINVAL and leaves the option unchanged; the removed
    options (force_staged, il_persist, max_wg_per_cu: ABI 4) are unknown."""
    cases = {"row_split": ((1, 2, 4), (0, 3, 5, 8)), "st_plain": ((0, 1, 2), (3, 100)),
             "unaligned_vec": ((0, 2), (3,)),
             "lane": ((0, 1), (2,)), "wavet": ((0, 1), (2,)), "narrow_mis": ((0, 1), (2,)),
             "kurt_leaf_tile": ((0, 1), (2,)),
             "kurt_mid_cpl": ((1, 2), (0, 3)), "vec_il": ((0, 1), (2, 1 << 40)),
             "rowt_small": ((0, 64, 100000), (1 << 21, 1 << 62)),
             "typed_kurt": ((0, 1, 2, 3), (4,))}
    for n, (good, bad) in cases.items():
        for v in good:
            assert L.bldp_plan_option(n.encode(), v, None) == 0, (n, v)
        for v in bad:
            prev = ctypes.c_int64(99)
            assert L.bldp_plan_option(n.encode(), v, ctypes.byref(prev)) == pkg._lib.BLDP_EINVAL, \
                (n, v)
            assert prev.value == 99  # not written on error
            assert n in pkg._lib.last_error()
        assert L.bldp_plan_option(n.encode(), -1, None) == 0
        assert L.bldp_plan_option(n.encode(), -7, None) == 0  # any negative: the default
    for n in ("force_staged", "il_persist", "max_wg_per_cu", "typed_rows", "typed_pipe"):
        assert L.bldp_plan_option(n.encode(), 1, None) == pkg._lib.BLDP_EINVAL, n
