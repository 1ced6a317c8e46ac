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
    (src/gbtworkerfunctions.jl:181-187; whole dataset for (:,:,:))."""
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
