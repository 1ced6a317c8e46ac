"""FBH5 (filterbank-in-HDF5) window reads and headers through libhdf5 (ctypes).

This takes the role HDF5.jl plays in the reference:

* ``h5open(f) do h5; h5["data"][idxs...]; end`` (src/gbtworkerfunctions.jl:181-187);
* ``attributes(h5["data"])`` (:141-155).

FBH5 stores ``data`` in C order as ``[nsamps][nifs][nchans]``. HDF5.jl
reverses the dimensions, so Julia sees ``(nchans, nifs, nsamps)``, and this
module returns the same thing: a Fortran-ordered float32 array of shape
``(nc, ni, nt)``.

* A Julia window becomes one HDF5 hyperslab (start, stride, count on the
  reversed axes). Negative-step ranges are read forward and flipped.
* The element type is converted to native float32 by libhdf5.

Compressed rawspec products need the bitshuffle filter (HDF5 filter 32008,
H5Zbitshuffle in the reference, Project.toml:10). They read only if that
filter plugin is registered with libhdf5 (``HDF5_PLUGIN_PATH``); otherwise
libhdf5 reports the missing filter and we raise. Uncompressed and
deflate-compressed files always read.

The library is located via ``$BLDP_LIBHDF5`` first, then a short list of
common paths (this image ships libhdf5 1.10 in /opt/conda/lib).
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

from ._lib import BLDPError, BoundsError
from .idxs import to_window

hid_t = ctypes.c_int64
herr_t = ctypes.c_int
hsize_t = ctypes.c_uint64

_CANDIDATES = ["/opt/conda/lib/libhdf5.so", "libhdf5.so", "libhdf5_serial.so",
               "/usr/lib/x86_64-linux-gnu/hdf5/serial/libhdf5.so"]

H5F_ACC_RDONLY, H5F_ACC_TRUNC, H5P_DEFAULT, H5S_ALL, H5S_SELECT_SET = 0, 2, 0, 0, 0
H5T_INTEGER, H5T_FLOAT, H5T_STRING = 0, 1, 3
H5S_SCALAR = 0

_h5 = None


class _H5:
    def __init__(self, path):
        L = ctypes.CDLL(path)
        sig = {
            "H5open": ([], herr_t), "H5Fopen": ([ctypes.c_char_p, ctypes.c_uint, hid_t], hid_t),
            "H5Fcreate": ([ctypes.c_char_p, ctypes.c_uint, hid_t, hid_t], hid_t),
            "H5Fclose": ([hid_t], herr_t), "H5Dopen2": ([hid_t, ctypes.c_char_p, hid_t], hid_t),
            "H5Dclose": ([hid_t], herr_t), "H5Dget_space": ([hid_t], hid_t),
            "H5Dget_type": ([hid_t], hid_t),
            "H5Dread": ([hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p], herr_t),
            "H5Dwrite": ([hid_t, hid_t, hid_t, hid_t, hid_t, ctypes.c_void_p], herr_t),
            "H5Dcreate2": ([hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t, hid_t], hid_t),
            "H5Sclose": ([hid_t], herr_t),
            "H5Sget_simple_extent_ndims": ([hid_t], ctypes.c_int),
            "H5Sget_simple_extent_dims": ([hid_t, ctypes.c_void_p, ctypes.c_void_p],
                                          ctypes.c_int),
            "H5Sget_simple_extent_npoints": ([hid_t], ctypes.c_int64),
            "H5Screate_simple": ([ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p], hid_t),
            "H5Screate": ([ctypes.c_int], hid_t),
            "H5Sselect_hyperslab": ([hid_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p], herr_t),
            "H5Tclose": ([hid_t], herr_t), "H5Tget_class": ([hid_t], ctypes.c_int),
            "H5Tget_size": ([hid_t], ctypes.c_size_t), "H5Tcopy": ([hid_t], hid_t),
            "H5Tset_size": ([hid_t, ctypes.c_size_t], herr_t),
            "H5Tis_variable_str": ([hid_t], ctypes.c_int),
            "H5Tget_sign": ([hid_t], ctypes.c_int),
            "H5Aget_num_attrs": ([hid_t], ctypes.c_int),
            "H5Aopen_by_idx": ([hid_t, ctypes.c_char_p, ctypes.c_int, ctypes.c_int, hsize_t,
                                hid_t, hid_t], hid_t),
            "H5Aget_name": ([hid_t, ctypes.c_size_t, ctypes.c_char_p], ctypes.c_ssize_t),
            "H5Aget_type": ([hid_t], hid_t), "H5Aget_space": ([hid_t], hid_t),
            "H5Aread": ([hid_t, hid_t, ctypes.c_void_p], herr_t),
            "H5Awrite": ([hid_t, hid_t, ctypes.c_void_p], herr_t),
            "H5Acreate2": ([hid_t, ctypes.c_char_p, hid_t, hid_t, hid_t, hid_t], hid_t),
            "H5Aclose": ([hid_t], herr_t),
            "H5Pcreate": ([hid_t], hid_t), "H5Pclose": ([hid_t], herr_t),
            "H5Pset_chunk": ([hid_t, ctypes.c_int, ctypes.c_void_p], herr_t),
            "H5Pset_deflate": ([hid_t, ctypes.c_uint], herr_t),
            "H5Dvlen_reclaim": ([hid_t, hid_t, hid_t, ctypes.c_void_p], herr_t),
            "H5Eset_auto2": ([hid_t, ctypes.c_void_p, ctypes.c_void_p], herr_t),
            "H5Dget_create_plist": ([hid_t], hid_t),
            "H5Pget_layout": ([hid_t], ctypes.c_int),
            "H5Pget_chunk": ([hid_t, ctypes.c_int, ctypes.c_void_p], ctypes.c_int),
            "H5Pget_nfilters": ([hid_t], ctypes.c_int),
            "H5Pget_filter2": ([hid_t, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_size_t, ctypes.c_char_p,
                                ctypes.c_void_p], ctypes.c_int),
            "H5Pset_filter": ([hid_t, ctypes.c_int, ctypes.c_uint, ctypes.c_size_t,
                               ctypes.c_void_p], herr_t),
            "H5Zfilter_avail": ([ctypes.c_int], ctypes.c_int),
            "H5Dget_chunk_storage_size": ([hid_t, ctypes.c_void_p, ctypes.c_void_p], herr_t),
            "H5Dget_offset": ([hid_t], ctypes.c_uint64),
            "H5Oget_info2": ([hid_t, ctypes.c_void_p, ctypes.c_uint], herr_t),
            "H5Dget_chunk_info_by_coord": ([hid_t, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p], herr_t),
            "H5Tget_order": ([hid_t], ctypes.c_int),
            "H5Dread_chunk": ([hid_t, hid_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p],
                              herr_t),
            "H5Dwrite_chunk": ([hid_t, hid_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                ctypes.c_void_p], herr_t),
        }
        for name, (a, r) in sig.items():
            f = getattr(L, name)
            f.argtypes, f.restype = a, r
        if L.H5open() < 0:
            raise BLDPError(-1, f"H5open failed ({path})")
        L.H5Eset_auto2(0, None, None)  # errors come back as return codes, not stderr
        g = lambda n: hid_t.in_dll(L, n).value  # noqa: E731
        self.NATIVE_FLOAT, self.NATIVE_DOUBLE = g("H5T_NATIVE_FLOAT_g"), g("H5T_NATIVE_DOUBLE_g")
        self.NATIVE_LLONG, self.NATIVE_ULLONG = g("H5T_NATIVE_LLONG_g"), g("H5T_NATIVE_ULLONG_g")
        self.NATIVE_INT = g("H5T_NATIVE_INT_g")
        self.C_S1 = g("H5T_C_S1_g")
        self.DATASET_CREATE = g("H5P_CLS_DATASET_CREATE_ID_g")
        self.L, self.path = L, path


def h5():
    global _h5
    if _h5 is None:
        paths = [os.environ.get("BLDP_LIBHDF5")] + _CANDIDATES
        errs = []
        for p in paths:
            if not p:
                continue
            try:
                _h5 = _H5(p)
                break
            except OSError as e:
                errs.append(f"{p}: {e}")
        if _h5 is None:
            raise BLDPError(-1, "libhdf5 not found (set BLDP_LIBHDF5): " + "; ".join(errs))
    return _h5


def _ok(v, what):
    if v < 0:
        raise BLDPError(-1, f"libhdf5: {what} failed")
    return v


def _hs(vals):
    return (hsize_t * len(vals))(*[int(v) for v in vals])


def _dims(space) -> tuple:
    H = h5().L
    nd = H.H5Sget_simple_extent_ndims(space)
    d = (hsize_t * max(nd, 1))()
    H.H5Sget_simple_extent_dims(space, d, None)
    return tuple(int(d[k]) for k in range(nd))


def read_window(fname, idxs) -> np.ndarray:
    """h5["data"][idxs...] as a Fortran-ordered float32 (nc, ni, nt) array
    (src/gbtworkerfunctions.jl:181-187; whole dataset for (:,:,:)).
    Bitshuffle/LZ4 chunks that libhdf5 cannot decode (no filter plugin) are
    read raw and decoded by libbldp_hip (host C++ decoder)."""
    if needs_bslz4(fname):
        return read_window_bslz4(fname, idxs, device=None)
    H5 = h5()
    H = H5.L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            fs = _ok(H.H5Dget_space(d), "get_space")
            try:
                cdims = _dims(fs)
                if len(cdims) != 3:
                    raise BLDPError(-1, f"{fname}: data is {len(cdims)}-D, expected 3")
                jshape = cdims[::-1]  # (nchans, nifs, nsamps)
                win = to_window(idxs, jshape)
                if win is None:
                    win = [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
                start, step, count, flip = [], [], [], []
                for ax in range(3):
                    st, ct, sp = win[3 * ax: 3 * ax + 3]
                    if ct > 0:
                        last = st + (ct - 1) * sp
                        if min(st, last) < 0 or max(st, last) >= jshape[ax]:
                            raise BoundsError(-6, f"BoundsError: axis {ax + 1} window "
                                                  f"{st + 1}:{sp}:{last + 1} of {jshape[ax]}")
                        if sp < 0:
                            st, sp = last, -sp
                    start.append(st)
                    step.append(sp)
                    count.append(ct)
                    flip.append(win[3 * ax + 2] < 0)
                nc, ni, nt = count
                buf = np.empty((nt, ni, nc), dtype=np.float32)
                if buf.size:
                    _ok(H.H5Sselect_hyperslab(fs, H5S_SELECT_SET, _hs(start[::-1]),
                                              _hs(step[::-1]), _hs(count[::-1]), None),
                        "select_hyperslab")
                    ms = _ok(H.H5Screate_simple(3, _hs([nt, ni, nc]), None), "memspace")
                    try:
                        _ok(H.H5Dread(d, H5.NATIVE_FLOAT, ms, fs, H5P_DEFAULT,
                                      buf.ctypes.data),
                            f"read {fname} (compressed with an unregistered filter?)")
                    finally:
                        H.H5Sclose(ms)
                out = buf.transpose(2, 1, 0)  # Julia order, Fortran-contiguous view
                for ax in range(3):
                    if flip[ax]:
                        out = np.flip(out, axis=ax)
                return np.asfortranarray(out)
            finally:
                H.H5Sclose(fs)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)


def _read_attr(H5, a):
    H = H5.L
    t = H.H5Aget_type(a)
    sp = H.H5Aget_space(a)
    try:
        n = H.H5Sget_simple_extent_npoints(sp)
        scalar = H.H5Sget_simple_extent_ndims(sp) == 0
        cls = H.H5Tget_class(t)
        if cls == H5T_STRING:
            if H.H5Tis_variable_str(t) > 0:
                ptrs = (ctypes.c_char_p * n)()
                _ok(H.H5Aread(a, t, ptrs), "read vlen string attr")
                vals = [p.decode() if p else "" for p in ptrs]
                H.H5Dvlen_reclaim(t, sp, H5P_DEFAULT, ptrs)
            else:
                size = H.H5Tget_size(t)
                raw = ctypes.create_string_buffer(size * n)
                _ok(H.H5Aread(a, t, raw), "read string attr")
                vals = [raw.raw[k * size:(k + 1) * size].split(b"\0", 1)[0].decode()
                        for k in range(n)]
        elif cls == H5T_INTEGER:
            signed = H.H5Tget_sign(t) != 0
            arr = np.empty(n, np.int64 if signed else np.uint64)
            _ok(H.H5Aread(a, H5.NATIVE_LLONG if signed else H5.NATIVE_ULLONG,
                          arr.ctypes.data), "read int attr")
            vals = [int(v) for v in arr]
        elif cls == H5T_FLOAT:
            arr = np.empty(n, np.float64)
            _ok(H.H5Aread(a, H5.NATIVE_DOUBLE, arr.ctypes.data), "read float attr")
            vals = [float(v) for v in arr]
        else:
            return None
        return vals[0] if scalar else vals
    finally:
        H.H5Sclose(sp)
        H.H5Tclose(t)


def header(fname, reference_bug: bool = False) -> dict:
    """getfbh5header (src/gbtworkerfunctions.jl:141-155): the attributes of
    ``data`` except DIMENSION_LABELS, plus nfpc when absent, data_size and
    nsamps, sorted by key.

    The reference computes the missing nfpc from an undefined ``fbh`` and
    pushes a bare value instead of a pair (:147-150), so such files throw
    there.  ``reference_bug=True`` reproduces that failure; the default
    computes ``nfpc = round(Int32, 187.5/64/abs(foff))`` as getfbheader does
    (:134)."""
    H5 = h5()
    H = H5.L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            attrs = {}
            for k in range(H.H5Aget_num_attrs(d)):
                a = _ok(H.H5Aopen_by_idx(d, b".", 0, 0, k, H5P_DEFAULT, H5P_DEFAULT), "attr")
                try:
                    nm = ctypes.create_string_buffer(256)
                    H.H5Aget_name(a, 256, nm)
                    name = nm.value.decode()
                    if name != "DIMENSION_LABELS":  # :145
                        attrs[name] = _read_attr(H5, a)
                finally:
                    H.H5Aclose(a)
            t = H.H5Dget_type(d)
            elsize = H.H5Tget_size(t)
            H.H5Tclose(t)
            fs = H.H5Dget_space(d)
            cdims = _dims(fs)
            H.H5Sclose(fs)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)
    if "nfpc" not in attrs:  # :147-150
        if reference_bug:
            raise NameError("UndefVarError: fbh not defined (src/gbtworkerfunctions.jl:149)")
        attrs["nfpc"] = int(np.int32(round(187.5 / 64 / abs(attrs["foff"]))))
    attrs["data_size"] = int(elsize * int(np.prod(cdims)))  # :151
    attrs["nsamps"] = int(cdims[0])  # :152 size(data, ndims(data)) -> first C dim
    return dict(sorted(attrs.items()))  # :153


def write(fname, attrs: dict, data: np.ndarray, chunks=None, deflate: int = 0) -> None:
    """Write an FBH5-layout file (dataset ``data`` = C-order [t][i][c] float32
    plus scalar attributes and DIMENSION_LABELS) — used to make test inputs."""
    H5 = h5()
    H = H5.L
    a = np.asfortranarray(np.asarray(data, dtype=np.float32))
    cdims = a.shape[::-1]
    f = _ok(H.H5Fcreate(os.fsencode(fname), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), "create")
    try:
        sp = _ok(H.H5Screate_simple(3, _hs(cdims), None), "space")
        dcpl = _ok(H.H5Pcreate(H5.DATASET_CREATE), "dcpl")
        if chunks or deflate:
            _ok(H.H5Pset_chunk(dcpl, 3, _hs(chunks or cdims)), "set_chunk")
        if deflate:
            _ok(H.H5Pset_deflate(dcpl, deflate), "set_deflate")
        d = _ok(H.H5Dcreate2(f, b"data", H5.NATIVE_FLOAT, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT),
                "create dataset")
        H.H5Pclose(dcpl)
        H.H5Sclose(sp)
        try:
            c = np.ascontiguousarray(a.transpose(2, 1, 0))
            _ok(H.H5Dwrite(d, H5.NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, c.ctypes.data),
                "write")
            items = dict(attrs)
            items.setdefault("DIMENSION_LABELS", ["time", "feed_id", "frequency"])
            for k, v in items.items():
                _write_attr(H5, d, k, v)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)


def _write_attr(H5, obj, name, v):
    H = H5.L
    if isinstance(v, (list, tuple)) and v and isinstance(v[0], str):
        size = max(len(s) for s in v) + 1
        t = H.H5Tcopy(H5.C_S1)
        H.H5Tset_size(t, size)
        sp = H.H5Screate_simple(1, _hs([len(v)]), None)
        buf = ctypes.create_string_buffer(b"".join(s.encode().ljust(size, b"\0") for s in v))
        mt, close_t = t, True
    elif isinstance(v, str):
        t = H.H5Tcopy(H5.C_S1)
        H.H5Tset_size(t, len(v) + 1)
        sp = H.H5Screate(H5S_SCALAR)
        buf = ctypes.create_string_buffer(v.encode())
        mt, close_t = t, True
    elif isinstance(v, (bool, int, np.integer)):
        sp = H.H5Screate(H5S_SCALAR)
        buf = ctypes.c_int32(int(v)) if name == "nfpc" else ctypes.c_int64(int(v))
        mt = H5.NATIVE_INT if name == "nfpc" else H5.NATIVE_LLONG
        t, close_t = mt, False
    else:
        sp = H.H5Screate(H5S_SCALAR)
        buf = ctypes.c_double(float(v))
        t = mt = H5.NATIVE_DOUBLE
        close_t = False
    a = _ok(H.H5Acreate2(obj, name.encode(), t, sp, H5P_DEFAULT, H5P_DEFAULT), f"attr {name}")
    try:
        _ok(H.H5Awrite(a, mt, ctypes.byref(buf) if not isinstance(buf, ctypes.Array) else buf),
            f"write attr {name}")
    finally:
        H.H5Aclose(a)
        H.H5Sclose(sp)
        if close_t:
            H.H5Tclose(t)


# --------------------------------------------------------------------------
# HDF5 filter 32008 (bitshuffle + LZ4) chunk decoding through libbldp_hip
# --------------------------------------------------------------------------
BSHUF_FILTER_ID = 32008


def bslz4_info(chunk: bytes) -> tuple[int, int]:
    """(uncompressed bytes, block bytes) of a bitshuffle-LZ4 chunk."""
    from . import _lib

    nb, bb = ctypes.c_uint64(), ctypes.c_uint32()
    buf = np.frombuffer(chunk, np.uint8)
    _lib.check(_lib.lib().bldp_bslz4_info(buf.ctypes.data, buf.size, ctypes.byref(nb),
                                          ctypes.byref(bb)), "bldp_bslz4_info")
    return nb.value, bb.value


def bslz4_decode_host(chunk: bytes, dtype=np.float32) -> np.ndarray:
    """Decode one chunk on the host (C++ in libbldp_hip)."""
    from . import _lib

    nb, _ = bslz4_info(chunk)
    es = np.dtype(dtype).itemsize
    out = np.empty(nb // es, dtype=dtype)
    buf = np.frombuffer(chunk, np.uint8)
    _lib.check(_lib.lib().bldp_bslz4_decode_host(buf.ctypes.data, buf.size, es,
                                                 out.ctypes.data if out.size else None, nb),
               "bldp_bslz4_decode_host")
    return out


def bslz4_decode_dev(chunks, dtype=np.float32, device=None, stream=None, out=None,
                     out_offsets=None):
    """Decode a list of chunks on the GPU in one launch: only the compressed
    bytes cross PCIe.  Without ``out`` the chunks land back to back in a new
    1-D device tensor; with ``out``/``out_offsets`` (bytes) they land there."""
    import torch

    from . import _lib

    es = np.dtype(dtype).itemsize
    sizes = [bslz4_info(c)[0] for c in chunks]
    comp = np.frombuffer(b"".join(bytes(c) for c in chunks), np.uint8)
    coff = np.cumsum([0] + [len(c) for c in chunks[:-1]]).astype(np.uint64)
    clen = np.array([len(c) for c in chunks], np.uint64)
    if out is None:
        dev = torch.device(device or "cuda")
        tdt = {4: torch.float32, 8: torch.float64, 2: torch.int16, 1: torch.uint8}[es]
        out = torch.empty(sum(sizes) // es, dtype=tdt, device=dev)
        ooff = np.cumsum([0] + sizes[:-1]).astype(np.uint64)
    else:
        dev = out.device
        ooff = np.asarray(out_offsets, np.uint64)
        cap = out.numel() * out.element_size()
        if len(ooff) != len(chunks) or any(int(o) + s > cap for o, s in zip(ooff, sizes)):
            raise ValueError("decoded chunks do not fit the output tensor")
    olen = np.array(sizes, np.uint64)  # each chunk's slot: the size its header states
    cdev = torch.from_numpy(comp.copy()).to(dev) if comp.size else None
    rc = _lib.lib().bldp_bslz4_decode_dev(
        len(chunks), comp.ctypes.data, cdev.data_ptr() if cdev is not None else None,
        coff.ctypes.data, clen.ctypes.data, es, out.data_ptr(), ooff.ctypes.data,
        olen.ctypes.data, _lib.stream_ptr(stream))
    _lib.check(rc, "bldp_bslz4_decode_dev")
    return out


# --------------------------------------------------------------------------
# Chunked datasets with filter 32008: direct chunk reads + our decoder
# --------------------------------------------------------------------------
H5D_CHUNKED = 2


_META_MAX = 256
_meta_cache: dict = {}
_meta_lock = __import__("threading").Lock()


def _file_key(fname):
    """Identity of a file's current contents: a rewritten file (new inode,
    size or change time) gets new metadata."""
    st = os.stat(fname)
    return (os.path.realpath(fname), st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns,
            st.st_ctime_ns)


def _cached(fn):
    """Per-file memo of a metadata function (layout, chunk index, ...): a
    worker reads the same files over and over; the libhdf5 open and the
    B-tree walk are paid once per file version, not per getdata."""
    import functools

    @functools.wraps(fn)
    def wrap(fname):
        key = (fn.__name__,) + _file_key(fname)
        with _meta_lock:
            if key in _meta_cache:
                return _meta_cache[key]
        val = fn(fname)
        with _meta_lock:
            if len(_meta_cache) >= _META_MAX:
                _meta_cache.pop(next(iter(_meta_cache)))
            _meta_cache[key] = val
        return val
    return wrap


@_cached
def layout(fname) -> dict:
    """Dataset dims (C order), chunk dims and filter pipeline of ``data``."""
    H5 = h5()
    H = H5.L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            fs = H.H5Dget_space(d)
            cdims = _dims(fs)
            H.H5Sclose(fs)
            pl = _ok(H.H5Dget_create_plist(d), "create_plist")
            try:
                chunk = None
                if H.H5Pget_layout(pl) == H5D_CHUNKED:
                    cd = (hsize_t * 8)()
                    nd = H.H5Pget_chunk(pl, 8, cd)
                    chunk = tuple(int(cd[k]) for k in range(nd))
                filters = []
                for k in range(max(0, H.H5Pget_nfilters(pl))):
                    flags, nel = ctypes.c_uint(), ctypes.c_size_t(16)
                    vals = (ctypes.c_uint * 16)()
                    name = ctypes.create_string_buffer(64)
                    cfg = ctypes.c_uint()
                    fid = H.H5Pget_filter2(pl, k, ctypes.byref(flags), ctypes.byref(nel), vals,
                                           64, name, ctypes.byref(cfg))
                    filters.append(dict(id=fid, flags=flags.value,
                                        cd_values=[vals[j] for j in range(min(nel.value, 16))],
                                        name=name.value.decode(errors="replace"),
                                        available=H.H5Zfilter_avail(fid) > 0))
            finally:
                H.H5Pclose(pl)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)
    return dict(cdims=cdims, chunk=chunk, filters=filters)


H5D_CONTIGUOUS = 1
H5T_ORDER_LE = 0
HADDR_UNDEF = (1 << 64) - 1


@_cached
def raw_layout(fname):
    """(file offset, Julia shape) when ``data`` is stored as one contiguous
    block of little-endian float32 with no filter -- what
    filestream.window_to_device can read with plain preads -- else None."""
    H5 = h5()
    H = H5.L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            pl = _ok(H.H5Dget_create_plist(d), "create_plist")
            try:
                if H.H5Pget_layout(pl) != H5D_CONTIGUOUS or H.H5Pget_nfilters(pl) != 0:
                    return None
            finally:
                H.H5Pclose(pl)
            ty = _ok(H.H5Dget_type(d), "get_type")
            try:
                if (H.H5Tget_class(ty) != H5T_FLOAT or H.H5Tget_size(ty) != 4
                        or H.H5Tget_order(ty) != H5T_ORDER_LE):
                    return None
            finally:
                H.H5Tclose(ty)
            fs = H.H5Dget_space(d)
            cdims = _dims(fs)
            H.H5Sclose(fs)
            off = H.H5Dget_offset(d)
            if len(cdims) != 3 or off == HADDR_UNDEF:
                return None
            return int(off), tuple(cdims[::-1])
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)


@_cached
def raw_chunked(fname) -> bool:
    """True when ``data`` is a chunked dataset with no filter, stored as
    little-endian float32: its chunks are the elements, read like the
    compressed ones and gathered on the GPU without a decode."""
    lay = layout(fname)
    if lay["chunk"] is None or lay["filters"] or len(lay["cdims"]) != 3:
        return False
    H5 = h5()
    H = H5.L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            ty = _ok(H.H5Dget_type(d), "get_type")
            try:
                return (H.H5Tget_class(ty) == H5T_FLOAT and H.H5Tget_size(ty) == 4
                        and H.H5Tget_order(ty) == H5T_ORDER_LE)
            finally:
                H.H5Tclose(ty)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)


@_cached
def needs_bslz4(fname) -> bool:
    """True when ``data`` is bitshuffle/LZ4-compressed and libhdf5 has no
    plugin for filter 32008 (the case of this image)."""
    lay = layout(fname)
    ids = [f["id"] for f in lay["filters"]]
    if BSHUF_FILTER_ID not in ids:
        return False
    if all(f["available"] for f in lay["filters"]):
        return False
    if ids != [BSHUF_FILTER_ID]:
        raise BLDPError(-1, f"{fname}: filter pipeline {ids} not supported (only 32008 alone)")
    return True


@_cached
def chunk_index(fname):
    """The chunk index of ``data`` as dense C-order grids over the chunk grid
    [gt][gi][gc]: file offset, stored bytes (0: never written, fill value) and
    filter mask of every chunk, parsed straight from the file (h5chunks.py),
    or None outside that parser's scope."""
    from . import h5chunks

    lay = layout(fname)
    cdims, chunk = lay["cdims"], lay["chunk"]
    if chunk is None or len(cdims) != 3:
        return None
    H = h5().L
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            tab = h5chunks.chunk_table(fname, H, d)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)
    if tab is None:
        return None
    grid = tuple(-(-int(n) // int(c)) for n, c in zip(cdims, chunk))
    addr = np.zeros(grid, np.int64)
    size = np.zeros(grid, np.int64)
    mask = np.zeros(grid, np.int64)
    for key, (a, n, m) in tab["index"].items():
        g = tuple(int(k) // int(c) for k, c in zip(key, chunk))
        addr[g], size[g], mask[g] = a, n, m
    return dict(addr=addr, size=size, mask=mask, grid=grid)


def _box(win_axis, cdim):
    st, ct, sp = win_axis
    if ct == 0:
        return 0, 1
    last = st + (ct - 1) * sp
    lo, hi = min(st, last), max(st, last)
    return lo // cdim, hi // cdim - lo // cdim + 1


def read_chunks(fname, idxs, alloc=None):
    """Raw chunks covering the window, in chunk-grid order.  Returns
    (jshape, window, chunk dims (t, i, c), box origin (t, i, c), grid (t, i, c),
    chunks).  Without ``alloc`` chunks are [(filter_mask, bytes or None)].
    With ``alloc(total_bytes) -> (buffer address, keepalive)`` every chunk is
    read by libhdf5 straight into one buffer (e.g. pinned host memory) and
    chunks are [(filter_mask, offset, nbytes)] (nbytes 0: never written)."""
    lay = layout(fname)
    cdims, chunk = lay["cdims"], lay["chunk"]
    if chunk is None or len(cdims) != 3:
        raise BLDPError(-1, f"{fname}: data is not a chunked 3-D dataset")
    jshape = cdims[::-1]
    win = to_window(idxs, jshape) or [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
    for ax in range(3):
        st, ct, sp = win[3 * ax: 3 * ax + 3]
        if ct > 0:
            last = st + (ct - 1) * sp
            if min(st, last) < 0 or max(st, last) >= jshape[ax]:
                raise BoundsError(-6, f"BoundsError: axis {ax + 1} window {st + 1}:{sp}:"
                                      f"{last + 1} of {jshape[ax]}")
    # C order axes: t = Julia axis 3, i = axis 2, c = axis 1
    kt0, gt = _box(win[6:9], chunk[0])
    ki0, gi = _box(win[3:6], chunk[1])
    kc0, gc = _box(win[0:3], chunk[2])
    H5 = h5()
    H = H5.L
    out = []
    f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
    try:
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        try:
            offs, sizes = [], []
            for a in range(gt):
                for b in range(gi):
                    for c in range(gc):
                        off = _hs([(kt0 + a) * chunk[0], (ki0 + b) * chunk[1],
                                   (kc0 + c) * chunk[2]])
                        nb = hsize_t()
                        if H.H5Dget_chunk_storage_size(d, off, ctypes.byref(nb)) < 0:
                            nb.value = 0  # never written: fill value (0)
                        offs.append(off)
                        sizes.append(nb.value)
            mask = ctypes.c_uint32()
            if alloc is None:
                for off, nb in zip(offs, sizes):
                    if nb == 0:
                        out.append((0, None))
                        continue
                    buf = ctypes.create_string_buffer(nb)
                    _ok(H.H5Dread_chunk(d, H5P_DEFAULT, off, ctypes.byref(mask), buf),
                        "read_chunk")
                    out.append((mask.value, buf.raw))
            else:
                base, keep = alloc(max(1, sum(sizes)))
                pos = 0
                for off, nb in zip(offs, sizes):
                    if nb:
                        _ok(H.H5Dread_chunk(d, H5P_DEFAULT, off, ctypes.byref(mask),
                                            ctypes.c_void_p(base + pos)), "read_chunk")
                    out.append((mask.value if nb else 0, pos, nb))
                    pos += nb
                out = (out, keep)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)
    box0 = (kt0 * chunk[0], ki0 * chunk[1], kc0 * chunk[2])
    return jshape, win, tuple(chunk), box0, (gt, gi, gc), out


def read_window_bslz4(fname, idxs, device=None):
    """The window of a bitshuffle/LZ4 dataset.  device=None: decode on the
    host (C++), return a Fortran-ordered numpy array.  device="cuda:k":
    compressed bytes go to the GPU, are decoded there (bldp_bslz4_decode_dev)
    and the window is gathered on the device (bldp_unchunk_f32); returns a
    Julia-order device tensor."""
    if device is not None:
        return _read_window_bslz4_dev(fname, idxs, device)
    jshape, win, chunk, box0, grid, raw = read_chunks(fname, idxs)
    cvol = int(np.prod(chunk))
    nc, ni, nt = win[1], win[4], win[7]
    packed = np.zeros(len(raw) * cvol, np.float32)
    for k, (mask, b) in enumerate(raw):
        if b is None:
            continue
        dst = packed[k * cvol:(k + 1) * cvol]
        if mask & 1:  # filter skipped for this chunk: raw elements
            dst[:] = np.frombuffer(b, np.float32, count=cvol)
        else:
            dst[:] = bslz4_decode_host(b)[:cvol]
    if nc * ni * nt == 0:
        return np.zeros((nc, ni, nt), np.float32, order="F")
    P = packed.reshape((grid[0], grid[1], grid[2]) + chunk)  # [gt][gi][gc][ct][ci][cc]
    ax = [win[a] + win[a + 2] * np.arange(win[a + 1]) - o for a, o in zip((6, 3, 0), box0)]
    t, i, c = np.ix_(*ax)
    w = P[t // chunk[0], i // chunk[1], c // chunk[2], t % chunk[0], i % chunk[1],
          c % chunk[2]]  # [t][i][c]
    return np.asfortranarray(np.transpose(w, (2, 1, 0)))


def _chunk_sizes(H, d, chunk, kt0, ki0, kc0, grid):
    offs, sizes = [], []
    for a in range(grid[0]):
        for b in range(grid[1]):
            for c in range(grid[2]):
                off = _hs([(kt0 + a) * chunk[0], (ki0 + b) * chunk[1], (kc0 + c) * chunk[2]])
                nb = hsize_t()
                if H.H5Dget_chunk_storage_size(d, off, ctypes.byref(nb)) < 0:
                    nb.value = 0  # never written: fill value (0)
                offs.append(off)
                sizes.append(nb.value)
    return offs, sizes


_copy_streams: dict = {}


def _copy_stream(dev, priority, j=0):
    """Cached H2D streams per (device, priority)."""
    import torch

    key = (dev.index if dev.index is not None else torch.cuda.current_device(), priority, j)
    s = _copy_streams.get(key)
    if s is None:
        s = _copy_streams[key] = torch.cuda.Stream(torch.device("cuda", key[0]), priority=priority)
    return s


def _batches_of(sizes, first_bytes, batch_bytes, ramp=True):
    """Split chunk indices 0..n-1 into contiguous ranges [k0, k1) of about
    ``batch_bytes`` stored bytes.  The first holds about ``first_bytes`` so
    the first H2D copy starts early; with ``ramp`` the next ones double from
    there up to ``batch_bytes`` (the copy engine is fed while the reader pool
    gets ahead)."""
    n = len(sizes)
    if n == 0:
        return []
    cum = np.cumsum(sizes)
    out, k0, target = [], 0, first_bytes
    base = 0
    while k0 < n:
        k1 = int(np.searchsorted(cum, base + target, side="left")) + 1
        k1 = min(max(k1, k0 + 1), n)
        out.append((k0, k1))
        base = int(cum[k1 - 1])
        k0, target = k1, (min(2 * target, batch_bytes) if ramp else batch_bytes)
    return out


def _read_tasks(faddr, sizes, offsets, k0, k1, piece):
    """Preads of chunks [k0, k1): chunks adjacent in the file and in the
    buffer merge into runs, runs are cut into pieces of <= ``piece`` bytes and
    grouped into tasks of about ``piece`` bytes (one pool task each: per-chunk
    tasks are GIL-bound).  Vectorised: a batch holds hundreds of chunks."""
    fa, sz, of = faddr[k0:k1], sizes[k0:k1], offsets[k0:k1]
    keep = sz > 0
    fa, sz, of = fa[keep], sz[keep], of[keep]
    if not len(sz):
        return []
    brk = np.ones(len(sz), bool)
    brk[1:] = (fa[1:] != fa[:-1] + sz[:-1]) | (of[1:] != of[:-1] + sz[:-1])
    starts = np.flatnonzero(brk)
    ends = np.append(starts[1:], len(sz))
    run_len = np.add.reduceat(sz, starts)
    tasks, cur, cur_n = [], [], 0
    for s, n in zip(starts.tolist(), run_len.tolist()):
        fo, do = int(fa[s]), int(of[s])
        for q in range(0, n, piece):
            m = min(piece, n - q)
            cur.append((fo + q, do + q, m))
            cur_n += m
            if cur_n >= piece:
                tasks.append(cur)
                cur, cur_n = [], 0
    if cur:
        tasks.append(cur)
    del ends
    return tasks


def _read_window_bslz4_dev(fname, idxs, device, timings=None, batch_bytes=64 << 20,
                           raw_chunks=False, first_batch_bytes=16 << 20, ramp=True, dense=True):
    """Device path of a compressed window, overlapped in three stages: a
    reader thread reads batches of stored chunks straight into pinned memory
    and queues their H2D copy on a copy stream, while this thread decodes the
    previous batch on the GPU (bldp_bslz4_decode_dev_async); then the window
    is gathered (bldp_unchunk_f32).  Only compressed bytes cross PCIe.  The
    chunks are read by parallel preads at the offsets of the chunk index
    parsed from the file once per file version (``chunk_index``), or,
    outside that parser's scope, one H5Dread_chunk at a time.
    ``raw_chunks``: the dataset has no filter, every stored chunk is raw
    float32 (no decode; when every chunk is stored, the device copy of the
    chunks is the packed chunk grid itself).  ``dense=False`` returns
    (tensor, window): when the chunk box is one chunk wide in IF and channel
    (gi = gc = 1: the chunks cover the window's channel span, as in rawspec
    products) the decoded chunk grid [gt*ct][ci][cc] already is a Julia-order
    (cc, ci, gt*ct) array holding the window, so it is returned with the
    window relative to it and the gather is skipped (the reduce kernels take
    the window, steps included); otherwise (gathered tensor, None).
    ``timings`` (a dict) receives stage times."""
    import time

    import torch

    from . import _lib, engine, filestream

    dev = torch.device(device)
    t0 = time.perf_counter()
    lay = layout(fname)
    cdims, chunk = lay["cdims"], lay["chunk"]
    if chunk is None or len(cdims) != 3:
        raise BLDPError(-1, f"{fname}: data is not a chunked 3-D dataset")
    jshape = cdims[::-1]
    win = to_window(idxs, jshape) or [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
    for ax in range(3):
        st, ct, sp = win[3 * ax: 3 * ax + 3]
        if ct > 0:
            last = st + (ct - 1) * sp
            if min(st, last) < 0 or max(st, last) >= jshape[ax]:
                raise BoundsError(-6, f"BoundsError: axis {ax + 1} window {st + 1}:{sp}:"
                                      f"{last + 1} of {jshape[ax]}")
    kt0, gt = _box(win[6:9], chunk[0])
    ki0, gi = _box(win[3:6], chunk[1])
    kc0, gc = _box(win[0:3], chunk[2])
    grid, chunk = (gt, gi, gc), tuple(chunk)
    box0 = (kt0 * chunk[0], ki0 * chunk[1], kc0 * chunk[2])
    cvol = int(np.prod(chunk))
    nc, ni, nt = win[1], win[4], win[7]
    t_tab = time.perf_counter()
    tab = chunk_index(fname)  # dense index grids, cached per file version, or None
    H = d = f = None
    if tab is not None:
        sl = (slice(kt0, kt0 + gt), slice(ki0, ki0 + gi), slice(kc0, kc0 + gc))
        faddr = tab["addr"][sl].ravel()
        sizes = tab["size"][sl].ravel()
        masks = tab["mask"][sl].ravel().copy()
        coords = None
    else:  # libhdf5 one chunk at a time
        H = h5().L
        f = _ok(H.H5Fopen(os.fsencode(fname), H5F_ACC_RDONLY, H5P_DEFAULT), f"open {fname}")
        d = _ok(H.H5Dopen2(f, b"data", H5P_DEFAULT), "open dataset 'data'")
        coords, szl = _chunk_sizes(H, d, chunk, kt0, ki0, kc0, grid)
        sizes = np.array(szl, np.int64)
        faddr = np.zeros(len(sizes), np.int64)
        masks = np.zeros(len(sizes), np.int64)
    t_tab = time.perf_counter() - t_tab
    try:
        offsets = np.zeros(len(sizes), np.int64)
        if len(sizes) > 1:
            offsets[1:] = np.cumsum(sizes[:-1])
        total = int(sizes.sum())
        native = tab is not None and os.environ.get("BLDP_NATIVE_READ", "1") != "0"
        t_pin = time.perf_counter()
        if native:
            # the library's pinned slot ring stages the reads (batches no
            # larger than its slots): no pinned buffer the size of the window
            pinned = host = None
            batch_bytes = min(batch_bytes, filestream.NATIVE_BATCH_BYTES)
            first_batch_bytes = min(first_batch_bytes, batch_bytes)
        else:
            pinned = torch.empty(total + 16, dtype=torch.uint8, pin_memory=True)
            host = pinned.numpy()
        t_pin = time.perf_counter() - t_pin
        batches = _batches_of(sizes, first_batch_bytes, batch_bytes, ramp)
        with torch.cuda.device(dev):
            cdev = torch.empty(total + 16, dtype=torch.uint8, device=dev)
            dense_raw = raw_chunks and bool(np.all(sizes == 4 * cvol))
            # chunks never written read as the fill value 0; when every chunk is
            # stored each slot is written whole (decode or raw copy)
            packed = cdev[:total].view(torch.float32) if dense_raw else \
                (torch.empty if bool(np.all(sizes > 0)) else torch.zeros)(
                    len(sizes) * cvol, dtype=torch.float32, device=dev)
            # the H2D copies (the critical path) on a cached high-priority stream
            copy_streams = [_copy_stream(dev, -1)]
            if native:
                # parsed chunk index: reads, copies and decodes queued natively
                # (bldp_chunks_to_device: C++ reader threads, no interpreter lock,
                # through the device's pinned slot ring)
                t_setup = time.perf_counter() - t0
                if raw_chunks:  # no filter: stored chunks are raw elements
                    masks[:] = 1
                stats = _native_chunks(fname, faddr, sizes, offsets, masks, batches, pinned, cdev,
                                       None if dense_raw else packed, cvol, copy_streams[0],
                                       _lib, torch)
                if timings is not None:
                    timings.update(chunk_index_s=t_tab, pinned_alloc_s=t_pin, setup_s=t_setup,
                                   native_first_copy_s=stats[0] / 1e3,
                                   native_queued_s=stats[1] / 1e3, pieces=int(stats[2]),
                                   reader_threads=int(stats[3]),
                                   before_unchunk_s=time.perf_counter() - t0)
                return _window_out(dense, dev, torch, engine, _lib, nc, ni, nt, chunk, box0, grid,
                                   win, packed, timings, t0, 0.0, stats[1] / 1e3, batches, total,
                                   True)
            hostmv = memoryview(host)
            fd = os.open(fname, os.O_RDONLY) if tab is not None else None
            pool = filestream._ring(dev).pool

            # BLDP_TRACE_READ=1: host timeline of the first batch's preads too
            tr_host = [] if timings is not None and os.environ.get("BLDP_TRACE_READ") else None

            def read_task(task, b=-1):
                ts = time.perf_counter()
                for fo, do, n in task:
                    filestream._pread_into(fd, hostmv[do:do + n], fo)
                if tr_host is not None and b == 0:
                    tr_host.append((round(1e3 * (ts - t0), 3),
                                    round(1e3 * (time.perf_counter() - t0), 3)))

            # BLDP_TRACE_READ=1: GPU-event timeline of the copies (timings["trace"])
            trace = [] if timings is not None and os.environ.get("BLDP_TRACE_READ") else None
            # every batch's preads go to the pool, in batch order, so the pool
            # never idles between batches; the reader thread below only waits
            # for a batch's reads and queues its H2D copy.  The first batch is
            # submitted here and the rest by a pool task, so its copy can start
            # while the later batches are still being queued.  Batches up to
            # 32 MiB are cut into 16 pieces (the whole pool reads them), larger
            # ones into pieces of 1/8 (fewer submissions)
            t_sub = time.perf_counter()
            t_setup = t_sub - t0
            pending = rest = None
            if tab is not None:
                pending = [None] * len(batches)
                queued = [threading.Event() for _ in batches]

                def submit(b):
                    k0, k1 = batches[b]
                    bb = int(offsets[k1 - 1] + sizes[k1 - 1] - offsets[k0])
                    piece = max(256 << 10, bb // 16 if bb <= (32 << 20) else bb // 8)
                    pending[b] = [pool.submit(read_task, t, b) for t in
                                  _read_tasks(faddr, sizes, offsets, k0, k1, piece)]
                    queued[b].set()

                def submit_rest():
                    for b in range(1, len(batches)):
                        submit(b)

                submit(0)
                rest = pool.submit(submit_rest) if len(batches) > 1 else None
            t_sub = time.perf_counter() - t_sub

            def stage(b):  # reader thread: (reads landed) -> (async) device
                k0, k1 = batches[b]
                if tr_host is not None and b == 0:
                    tr_host.append(("stage0", round(1e3 * (time.perf_counter() - t0), 3)))
                if tab is not None:  # parallel preads at the parsed chunk offsets
                    if not queued[b].wait(60):
                        rest.result()  # (raises if the submitting task failed)
                        raise BLDPError(-1, f"{fname}: batch {b} reads were never queued")
                    for fu in pending[b]:
                        fu.result()
                else:
                    m = ctypes.c_uint32()
                    for k in range(k0, k1):
                        if sizes[k]:
                            _ok(H.H5Dread_chunk(d, H5P_DEFAULT, _hs(coords[k]), ctypes.byref(m),
                                                ctypes.c_void_p(pinned.data_ptr() +
                                                                int(offsets[k]))), "read_chunk")
                            masks[k] = m.value
                lo, hi = int(offsets[k0]), int(offsets[k1 - 1] + sizes[k1 - 1])
                copy_stream = copy_streams[b % len(copy_streams)]
                with torch.cuda.device(dev):
                    ev = torch.cuda.Event(enable_timing=trace is not None)
                    with torch.cuda.stream(copy_stream):
                        if trace is not None:
                            e0 = torch.cuda.Event(enable_timing=True)
                            e0.record(copy_stream)
                            trace.append(("copy", b, time.perf_counter() - t0, e0, ev, hi - lo))
                        if hi > lo:
                            cdev[lo:hi].copy_(pinned[lo:hi], non_blocking=True)
                        ev.record(copy_stream)
                return ev

            t_io = t_dec = 0.0
            try:
                if raw_chunks:  # no filter: stored chunks are raw elements
                    masks[:] = 1
                t_dec, t_io = _decode_batches(
                    batches, stage, sizes, masks, offsets, cvol,
                    None if dense_raw else packed, cdev, host, _lib, torch)
            finally:
                if pending is not None:  # (an error above: let the reads finish first)
                    if rest is not None:
                        rest.exception()  # every batch has been queued
                    for fl in pending:
                        for fu in fl or ():
                            fu.cancel() or fu.exception()
                if fd is not None:
                    os.close(fd)
    finally:
        if d is not None:
            H.H5Dclose(d)
        if f is not None:
            H.H5Fclose(f)
    if timings is not None:
        timings.update(chunk_index_s=t_tab, pinned_alloc_s=t_pin, setup_s=t_setup, submit_s=t_sub,
                       before_unchunk_s=time.perf_counter() - t0)
        if trace:
            torch.cuda.synchronize(dev)
            first = trace[0][3]
            timings["trace"] = [(b, round(1e3 * tq, 3), round(first.elapsed_time(e0), 3),
                                 round(first.elapsed_time(e1), 3), nb)
                                for _, b, tq, e0, e1, nb in trace]
            timings["trace_batch0_host_ms"] = tr_host
    return _window_out(dense, dev, torch, engine, _lib, nc, ni, nt, chunk, box0, grid, win,
                       packed, timings, t0, t_io, t_dec, batches, total, tab is not None)


def band_window_chunked_dev(fnames, idxs, device, timings=None, batch_bytes=64 << 20,
                            first_batch_bytes=16 << 20):
    """The same window of several chunked FBH5 files (a band's banks: one
    dataset shape and chunk shape, compressed with filter 32008 or stored
    without a filter) on GPU ``device`` as ONE stream of batches
    (bldp_file_chunks_to_device: the stored chunks of every file read by the
    native reader threads, copied to the device and decoded there into one
    chunk grid per bank), instead of one read call per bank
    (src/gbtworkerfunctions.jl:181-187 for each file, fanned out by
    GBT.getdata, src/gbt.jl:69-79).  Returns ``(views, rwin)``: when the
    chunk box is one chunk wide in IF and channel, each bank's decoded chunk
    grid as a Julia-order (cc, ci, gt*ct) tensor holding the window, and the
    window relative to it (the same for every bank); otherwise each bank's
    window gathered from its chunk grid (bldp_unchunk_f32) into a dense
    Julia-order tensor, and None.  None when the banks do not qualify
    (different layouts, a chunk index the parser cannot read): the caller then
    reads bank by bank.  The caller's current stream on the device is ordered
    after the decode."""
    import time

    import torch

    from . import _lib, filestream

    if not fnames:
        return None
    t0 = time.perf_counter()
    lays = [layout(f) for f in fnames]
    cdims, chunk = lays[0]["cdims"], lays[0]["chunk"]
    if chunk is None or len(cdims) != 3 or any(
            tuple(lay["cdims"]) != tuple(cdims) or tuple(lay["chunk"] or ()) != tuple(chunk)
            for lay in lays):
        return None
    comp = [needs_bslz4(f) for f in fnames]
    if not all(c or raw_chunked(f) for c, f in zip(comp, fnames)):
        return None
    jshape = cdims[::-1]
    win = to_window(idxs, jshape) or [0, jshape[0], 1, 0, jshape[1], 1, 0, jshape[2], 1]
    for ax in range(3):
        st, ct, sp = win[3 * ax: 3 * ax + 3]
        if ct > 0:
            last = st + (ct - 1) * sp
            if min(st, last) < 0 or max(st, last) >= jshape[ax]:
                raise BoundsError(-6, f"BoundsError: axis {ax + 1} window {st + 1}:{sp}:"
                                      f"{last + 1} of {jshape[ax]}")
    nc, ni, nt = win[1], win[4], win[7]
    kt0, gt = _box(win[6:9], chunk[0])
    ki0, gi = _box(win[3:6], chunk[1])
    kc0, gc = _box(win[0:3], chunk[2])
    if nc * ni * nt == 0:
        return None
    chunk = tuple(int(c) for c in chunk)
    cvol = int(np.prod(chunk))
    tabs = [chunk_index(f) for f in fnames]
    if any(t is None for t in tabs):
        return None
    sl = (slice(kt0, kt0 + gt), slice(ki0, ki0 + gi), slice(kc0, kc0 + gc))
    faddr = np.concatenate([t["addr"][sl].ravel() for t in tabs]).astype(np.int64)
    sizes = np.concatenate([t["size"][sl].ravel() for t in tabs]).astype(np.int64)
    nper = gt * gi * gc
    # unfiltered files: every stored chunk holds raw elements (filter mask bit 0)
    masks = np.concatenate([t["mask"][sl].ravel() if c else np.ones(nper, np.int64)
                            for t, c in zip(tabs, comp)]).astype(np.uint32)
    bank_of = np.repeat(np.arange(len(fnames), dtype=np.int32), nper)
    offsets = np.zeros(len(sizes), np.int64)
    if len(sizes) > 1:
        offsets[1:] = np.cumsum(sizes[:-1])
    total = int(sizes.sum())
    # reads staged through the library's pinned slot ring: batches no larger
    # than its slots, no pinned buffer the size of the band
    batch_bytes = min(batch_bytes, filestream.NATIVE_BATCH_BYTES)
    batches = _batches_of(sizes, min(first_batch_bytes, batch_bytes), batch_bytes, True)
    bend = np.array([k1 for _, k1 in batches], np.int64)
    dev = torch.device(device)
    t_setup = time.perf_counter() - t0
    with torch.cuda.device(dev):
        cdev = torch.empty(total + 16, dtype=torch.uint8, device=dev)
        # chunks never written read as the fill value 0
        packed = (torch.empty if bool(np.all(sizes > 0)) else torch.zeros)(
            len(fnames) * nper * cvol, dtype=torch.float32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        stats = (ctypes.c_double * 4)()
        L = _lib.lib()
        fds = []
        try:
            for f in fnames:
                fds.append(os.open(f, os.O_RDONLY))
            fdk = np.asarray(fds, np.int32)[bank_of]
            sp = _lib.stream_ptr()
            rc = L.bldp_file_chunks_to_device(
                len(sizes), fdk.ctypes.data, faddr.ctypes.data, sizes.ctypes.data,
                offsets.ctypes.data, masks.ctypes.data, len(bend), bend.ctypes.data,
                None, cdev.data_ptr(), total + 16, packed.data_ptr(), 4 * cvol,
                4 * packed.numel(), err.data_ptr(), _copy_stream(dev, -1).cuda_stream, sp, stats)
            # (waits for every queued copy and decode, also after a failed call)
            rc2 = L.bldp_bslz4_error(err.data_ptr(), sp)
        finally:
            for fd in fds:
                os.close(fd)
        _lib.check(rc, "bldp_file_chunks_to_device")
        _lib.check(rc2, "bslz4 decode")
    ct, ci, cc = chunk
    if gi == 1 and gc == 1:  # the chunk grid itself holds each bank's window
        views = [packed[b * nper * cvol:(b + 1) * nper * cvol].view(gt * ct, ci, cc)
                 .permute(2, 1, 0) for b in range(len(fnames))]
        rwin = [win[0] - kc0 * cc, nc, win[2], win[3] - ki0 * ci, ni, win[5], win[6] - kt0 * ct,
                nt, win[8]]
    else:  # several chunks across: each bank's window gathered dense on the device
        from . import engine

        keep = [(ctypes.c_int64 * 3)(*v) for v in (chunk, (kt0 * ct, ki0 * ci, kc0 * cc),
                                                   (gt, gi, gc))]
        w9 = (ctypes.c_int64 * 9)(*win)
        views = []
        with torch.cuda.device(dev):
            for b in range(len(fnames)):
                out = engine.fb_empty(nc, ni, nt, device=dev)
                rc = _lib.lib().bldp_unchunk_f32(packed.data_ptr() + 4 * b * nper * cvol,
                                                 keep[0], keep[1], keep[2], w9, out.data_ptr(),
                                                 _lib.stream_ptr())
                _lib.check(rc, "bldp_unchunk_f32")
                views.append(out)
        rwin = None
    if timings is not None:
        timings.update(setup_ms=t_setup * 1e3, read_decode_ms=(time.perf_counter() - t0) * 1e3,
                       first_copy_ms=stats[0], reads_ms=stats[1], pieces=int(stats[2]),
                       threads=int(stats[3]), stored_bytes=total, batches=len(batches),
                       chunks=len(sizes))
    return views, rwin


def _native_chunks(fname, faddr, sizes, offsets, masks, batches, pinned, cdev, packed, cvol,
                   copy_stream, _lib, torch):
    """bldp_chunks_to_device for the chunks of the box, then the decoder's
    error check (which also waits for the copies: a pinned buffer is free
    once this returns).  ``pinned`` None: the reads are staged through the
    library's pinned slot ring (every batch no larger than a slot).  Returns
    the call's stats (4 doubles)."""
    import ctypes as ct

    fa = np.ascontiguousarray(faddr, np.int64)
    sz = np.ascontiguousarray(sizes, np.int64)
    of = np.ascontiguousarray(offsets, np.int64)
    mk = np.ascontiguousarray(masks, np.uint32)
    bend = np.array([k1 for _, k1 in batches], np.int64)
    err = torch.zeros(1, dtype=torch.int32, device=cdev.device)
    stats = (ct.c_double * 4)()
    L = _lib.lib()
    fd = os.open(fname, os.O_RDONLY)
    try:
        rc = L.bldp_chunks_to_device(
            fd, len(sz), fa.ctypes.data, sz.ctypes.data, of.ctypes.data, mk.ctypes.data,
            len(bend), bend.ctypes.data, None if pinned is None else pinned.data_ptr(),
            cdev.data_ptr(), cdev.numel() if pinned is None else min(pinned.numel(), cdev.numel()),
            packed.data_ptr() if packed is not None else None, 4 * cvol,
            4 * packed.numel() if packed is not None else 0, err.data_ptr(),
            copy_stream.cuda_stream, _lib.stream_ptr(), stats)
        # (waits for every queued copy and decode, also after a failed call)
        rc2 = L.bldp_bslz4_error(err.data_ptr(), _lib.stream_ptr())
    finally:
        os.close(fd)
    _lib.check(rc, "bldp_chunks_to_device")
    _lib.check(rc2, "bslz4 decode")
    return list(stats)


def _window_out(dense, dev, torch, engine, _lib, nc, ni, nt, chunk, box0, grid, win, packed,
                timings, t0, t_io, t_dec, batches, total, parsed_index):
    """The window from the decoded chunk grid: with ``dense`` a gathered
    Julia-order tensor; otherwise (chunk grid, window inside it) when the box
    is one chunk wide in IF and channel, else (gathered tensor, None)."""
    import time

    gt, gi, gc = grid
    if not dense and gi == 1 and gc == 1 and nc * ni * nt > 0:
        # the packed grid [gt*ct][ci][cc] as a Julia-order array, and the
        # window relative to it
        ct, ci, cc = chunk
        grid_t = packed[:gt * ct * ci * cc].view(gt * ct, ci, cc).permute(2, 1, 0)
        rwin = [win[0] - box0[2], nc, win[2], win[3] - box0[1], ni, win[5],
                win[6] - box0[0], nt, win[8]]
        if timings is not None:
            with torch.cuda.device(dev):
                torch.cuda.synchronize()
            timings.update(total_s=time.perf_counter() - t0, wait_io_s=t_io, decode_s=t_dec,
                           batches=len(batches), compressed_bytes=total,
                           parsed_chunk_index=parsed_index, gather="window of the chunk grid")
        return grid_t, rwin
    out = _unchunk_out(dev, torch, engine, _lib, nc, ni, nt, chunk, box0, grid, win, packed,
                       timings, t0, t_io, t_dec, batches, total, parsed_index)
    return out if dense else (out, None)


def _decode_batches(batches, stage, sizes, masks, offsets, cvol, packed, cdev, host, _lib,
                    torch):
    """A reader thread runs ``stage`` over the batches (chunk ranges) ahead of
    this thread, which queues each batch's GPU decode as soon as its copy has
    landed (asynchronously; the decoder's error bits are checked once at the
    end).  Returns (decode seconds, seconds waited for reads)."""
    import time
    from concurrent.futures import ThreadPoolExecutor

    t_io = t_dec = 0.0
    err = torch.zeros(1, dtype=torch.int32, device=cdev.device)  # decoder error bits
    with ThreadPoolExecutor(max_workers=1) as reader:
        futs = [reader.submit(stage, b) for b in range(len(batches))]  # reads run ahead
        cur_stream = torch.cuda.current_stream()
        for b, (k0, k1) in enumerate(batches):
            tw = time.perf_counter()
            cur_stream.wait_event(futs[b].result())
            t_io += time.perf_counter() - tw
            td = time.perf_counter()
            sz, mk, of = sizes[k0:k1], masks[k0:k1], offsets[k0:k1]
            if packed is not None:  # stored without the filter: raw elements
                for j in np.flatnonzero((sz > 0) & ((mk & 1) == 1)).tolist():
                    k = k0 + j
                    packed.view(torch.uint8)[4 * k * cvol:4 * (k + 1) * cvol].copy_(
                        cdev[int(of[j]):int(of[j]) + 4 * cvol])
            comp = np.flatnonzero((sz > 0) & ((mk & 1) == 0))
            if len(comp):
                offs = of[comp].astype(np.uint64)
                lens = sz[comp].astype(np.uint64)
                ooff = ((comp + k0) * (4 * cvol)).astype(np.uint64)
                olen = np.full(len(comp), 4 * cvol, np.uint64)  # a whole chunk per slot
                rc = _lib.lib().bldp_bslz4_decode_dev_async(
                    len(comp), host.ctypes.data, cdev.data_ptr(), offs.ctypes.data,
                    lens.ctypes.data, 4, packed.data_ptr(), ooff.ctypes.data, olen.ctypes.data,
                    err.data_ptr(), _lib.stream_ptr())
                _lib.check(rc, "bldp_bslz4_decode_dev_async")
            t_dec += time.perf_counter() - td
    td = time.perf_counter()
    _lib.check(_lib.lib().bldp_bslz4_error(err.data_ptr(), _lib.stream_ptr()), "bslz4 decode")
    t_dec += time.perf_counter() - td
    return t_dec, t_io


def _unchunk_out(dev, torch, engine, _lib, nc, ni, nt, chunk, box0, grid, win, packed, timings,
                 t0, t_io, t_dec, batches, total, parsed_index):
    import time

    with torch.cuda.device(dev):
        out = engine.fb_empty(nc, ni, nt, device=dev)
        if out.numel():
            keep = [(ctypes.c_int64 * 3)(*v) for v in (chunk, box0, grid)]
            w9 = (ctypes.c_int64 * 9)(*win)
            rc = _lib.lib().bldp_unchunk_f32(packed.data_ptr(), keep[0], keep[1], keep[2], w9,
                                             out.data_ptr(), _lib.stream_ptr())
            _lib.check(rc, "bldp_unchunk_f32")
        if timings is not None:
            torch.cuda.synchronize()
            timings.update(total_s=time.perf_counter() - t0, wait_io_s=t_io, decode_s=t_dec,
                           batches=len(batches), compressed_bytes=total,
                           parsed_chunk_index=parsed_index)
    return out


def write_bslz4_chunks(fname, attrs: dict, jshape, chunk, chunks) -> None:
    """An FBH5 file with filter 32008 whose chunks (C-order chunk grid, each
    already encoded) are written raw with H5Dwrite_chunk.  jshape is Julia's
    (nchans, nifs, nsamps); chunk is C-order (ct, ci, cc).  An item may also
    be None (the chunk is never written: it reads as the fill value 0) or
    (filter_mask, bytes) (mask bit 0 set: stored without the filter)."""
    H5 = h5()
    H = H5.L
    cdims = tuple(jshape)[::-1]
    f = _ok(H.H5Fcreate(os.fsencode(fname), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), "create")
    try:
        sp = _ok(H.H5Screate_simple(3, _hs(cdims), None), "space")
        dcpl = _ok(H.H5Pcreate(H5.DATASET_CREATE), "dcpl")
        _ok(H.H5Pset_chunk(dcpl, 3, _hs(chunk)), "set_chunk")
        cd = (ctypes.c_uint * 5)(0, 3, 4, 0, 2)
        _ok(H.H5Pset_filter(dcpl, BSHUF_FILTER_ID, 1, 5, cd), "set_filter 32008")
        d = _ok(H.H5Dcreate2(f, b"data", H5.NATIVE_FLOAT, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT),
                "create dataset")
        H.H5Pclose(dcpl)
        H.H5Sclose(sp)
        try:
            it = iter(chunks)
            for t0 in range(0, cdims[0], chunk[0]):
                for i0 in range(0, cdims[1], chunk[1]):
                    for c0 in range(0, cdims[2], chunk[2]):
                        enc, mask = next(it), 0
                        if enc is None:
                            continue
                        if isinstance(enc, tuple):
                            mask, enc = enc
                        _ok(H.H5Dwrite_chunk(d, H5P_DEFAULT, mask, _hs([t0, i0, c0]), len(enc),
                                             enc), "write_chunk")
            for k, v in dict(attrs, DIMENSION_LABELS=["time", "feed_id", "frequency"]).items():
                _write_attr(H5, d, k, v)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)


def write_bslz4(fname, attrs: dict, data: np.ndarray, chunk, encode) -> None:
    """Test helper: an FBH5 file whose ``data`` carries filter 32008 (bitshuffle,
    LZ4) with chunks written raw through H5Dwrite_chunk; ``encode(array) ->
    bytes`` produces each chunk.  The filter is marked optional so libhdf5
    accepts the pipeline without the plugin."""
    H5 = h5()
    H = H5.L
    a = np.asfortranarray(np.asarray(data, dtype=np.float32))
    cdims = a.shape[::-1]
    c = np.ascontiguousarray(a.transpose(2, 1, 0))
    f = _ok(H.H5Fcreate(os.fsencode(fname), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), "create")
    try:
        sp = _ok(H.H5Screate_simple(3, _hs(cdims), None), "space")
        dcpl = _ok(H.H5Pcreate(H5.DATASET_CREATE), "dcpl")
        _ok(H.H5Pset_chunk(dcpl, 3, _hs(chunk)), "set_chunk")
        cd = (ctypes.c_uint * 5)(0, 3, 4, 0, 2)  # bitshuffle version, elem size, auto, LZ4
        _ok(H.H5Pset_filter(dcpl, BSHUF_FILTER_ID, 1, 5, cd), "set_filter 32008")
        d = _ok(H.H5Dcreate2(f, b"data", H5.NATIVE_FLOAT, sp, H5P_DEFAULT, dcpl, H5P_DEFAULT),
                "create dataset")
        H.H5Pclose(dcpl)
        H.H5Sclose(sp)
        try:
            for t0 in range(0, cdims[0], chunk[0]):
                for i0 in range(0, cdims[1], chunk[1]):
                    for c0 in range(0, cdims[2], chunk[2]):
                        blk = np.zeros(chunk, np.float32)  # edge chunks are padded
                        part = c[t0:t0 + chunk[0], i0:i0 + chunk[1], c0:c0 + chunk[2]]
                        blk[:part.shape[0], :part.shape[1], :part.shape[2]] = part
                        enc = encode(blk)
                        _ok(H.H5Dwrite_chunk(d, H5P_DEFAULT, 0, _hs([t0, i0, c0]), len(enc),
                                             enc), "write_chunk")
            for k, v in dict(attrs, DIMENSION_LABELS=["time", "feed_id", "frequency"]).items():
                _write_attr(H5, d, k, v)
        finally:
            H.H5Dclose(d)
    finally:
        H.H5Fclose(f)
