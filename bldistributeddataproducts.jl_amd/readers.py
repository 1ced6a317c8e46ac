"""Host-side file access and metadata for the worker functions.

* SIGPROC ``.fil`` header parse + mmap — the role of Blio's
  ``Filterbank.Header`` / ``Filterbank.mmap`` (src/gbtworkerfunctions.jl:131-139,
  171-177);
* FBH5 (``.h5``) hyperslab reads — the role of HDF5.jl (:141-155, :179-189),
  see :mod:`.fbh5`;
* ``getinventory`` — the filesystem walk + GUPPI name regexes (:35-129).

None of this is on the GPU: it is host I/O and metadata (SURVEY.md §2 C12,
C13, C15, C16) that feeds the window to the HIP reduction.
"""
from __future__ import annotations

import os
import re
import socket
import struct

import numpy as np

# --------------------------------------------------------------------------
# SIGPROC filterbank
# --------------------------------------------------------------------------
_INT_KEYS = {"telescope_id", "machine_id", "data_type", "barycentric", "pulsarcentric",
             "nbits", "nsamples", "nchans", "nifs", "nbeams", "ibeam"}
_DBL_KEYS = {"az_start", "za_start", "src_raj", "src_dej", "tstart", "tsamp", "fch1", "foff",
             "refdm", "period"}
_STR_KEYS = {"rawdatafile", "source_name"}
_DTYPES = {32: np.float32, 16: np.uint16, 8: np.uint8}


def _rd_str(f) -> str:
    (n,) = struct.unpack("<i", f.read(4))
    if not 0 < n < 256:
        raise ValueError("not a SIGPROC filterbank header")
    return f.read(n).decode("ascii")


def read_fil_header(fname) -> dict:
    """Parse a SIGPROC header into a dict (adds header_size, sample_size,
    nsamps like Blio's Filterbank.Header)."""
    hdr: dict = {}
    with open(fname, "rb") as f:
        if _rd_str(f) != "HEADER_START":
            raise ValueError(f"{fname}: missing HEADER_START")
        while True:
            key = _rd_str(f)
            if key == "HEADER_END":
                break
            if key in _INT_KEYS:
                (hdr[key],) = struct.unpack("<i", f.read(4))
            elif key in _DBL_KEYS:
                (hdr[key],) = struct.unpack("<d", f.read(8))
            elif key in _STR_KEYS:
                hdr[key] = _rd_str(f)
            else:
                raise ValueError(f"{fname}: unknown SIGPROC header key {key!r}")
        hdr["header_size"] = f.tell()
    nifs = hdr.get("nifs", 1)
    hdr.setdefault("nifs", nifs)
    hdr["sample_size"] = hdr["nchans"] * nifs * hdr["nbits"] // 8
    hdr["nsamps"] = (os.path.getsize(fname) - hdr["header_size"]) // hdr["sample_size"]
    return hdr


def write_fil(fname, hdr: dict, data: np.ndarray) -> None:
    """Write a SIGPROC filterbank; data is Julia-order (nchans, nifs, nsamps)."""
    def s(x):
        b = x.encode("ascii")
        return struct.pack("<i", len(b)) + b

    out = [s("HEADER_START")]
    for k, v in hdr.items():
        if k in ("header_size", "sample_size", "nsamps"):
            continue
        out.append(s(k))
        if k in _INT_KEYS:
            out.append(struct.pack("<i", int(v)))
        elif k in _DBL_KEYS:
            out.append(struct.pack("<d", float(v)))
        elif k in _STR_KEYS:
            out.append(s(str(v)))
        else:
            raise ValueError(f"unknown SIGPROC header key {k!r}")
    out.append(s("HEADER_END"))
    a = np.asarray(data, dtype=_DTYPES[int(hdr.get("nbits", 32))])
    with open(fname, "wb") as f:
        f.write(b"".join(out))
        f.write(np.ascontiguousarray(np.transpose(a, (2, 1, 0))).tobytes())


def fil_mmap(fname):
    """(header, data) with data a read-only memmap viewed as Julia-order
    (nchans, nifs, nsamps) — Filterbank.mmap (src/gbtworkerfunctions.jl:173)."""
    hdr = read_fil_header(fname)
    nbits = hdr["nbits"]
    if nbits not in _DTYPES:
        raise ValueError(f"unsupported nbits={nbits}")
    shape = (hdr["nsamps"], hdr["nifs"], hdr["nchans"])
    if hdr["nsamps"] == 0:
        return hdr, np.zeros(shape[::-1], dtype=_DTYPES[nbits], order="F")
    mm = np.memmap(fname, dtype=_DTYPES[nbits], mode="r", offset=hdr["header_size"], shape=shape)
    return hdr, mm.transpose(2, 1, 0)


def fil_raw_layout(fname):
    """(data offset, Julia shape) of a 32-bit SIGPROC file, whose data block
    filestream.window_to_device reads with plain preads; None otherwise."""
    hdr = read_fil_header(fname)
    if hdr.get("nbits") != 32 or hdr["nsamps"] == 0:
        return None
    return hdr["header_size"], (hdr["nchans"], hdr["nifs"], hdr["nsamps"])


def getfbheader(fbname) -> dict:
    """src/gbtworkerfunctions.jl:131-139."""
    h = read_fil_header(fbname)
    h["nfpc"] = int(np.int32(round(187.5 / 64 / abs(h["foff"]))))  # :134
    del h["header_size"]  # :136
    del h["sample_size"]  # :137
    return h


# --------------------------------------------------------------------------
# FBH5
# --------------------------------------------------------------------------
_HDF5_SIG = b"\x89HDF\r\n\x1a\n"


def ishdf5(fname) -> bool:
    """HDF5.ishdf5: superblock signature at 0, 512, 1024, 2048, ..."""
    try:
        with open(fname, "rb") as f:
            size = os.fstat(f.fileno()).st_size
            off = 0
            while off + 8 <= size:
                f.seek(off)
                if f.read(8) == _HDF5_SIG:
                    return True
                off = 512 if off == 0 else off * 2
    except OSError:
        return False
    return False


def fbh5_read(fname, idxs):
    from . import fbh5

    return fbh5.read_window(fname, idxs)


def getfbh5header(fbh5name) -> dict:
    from . import fbh5

    return fbh5.header(fbh5name)


def getheader(fname) -> dict:
    """src/gbtworkerfunctions.jl:157-159."""
    return getfbh5header(fname) if ishdf5(fname) else getfbheader(fname)


# --------------------------------------------------------------------------
# Inventory (src/gbtworkerfunctions.jl:35-129)
# --------------------------------------------------------------------------
_GUPPI_RE = re.compile(
    r"(/BLP(?P<band>[0-7])(?P<bank>[0-7])/)?([^/]*/)?((?P<host>blc..)_)?guppi_"
    r"(?P<imjd>\d+)_(?P<smjd>\d+)_(\d+_)?(?P<src>.*)_(?P<scan>\d\d\d\d)")  # :36-46
_RAWSPEC_RE = re.compile(
    r"/BLP(?P<band>[0-7])(?P<bank>[0-7])/((?P<host>blc..)_)?guppi_(?P<imjd>\d+)_"
    r"(?P<smjd>\d+)_(\d+_)?(?P<src>.*)_(?P<scan>\d\d\d\d).rawspec."
    r"(?P<product>\d\d\d\d).(h5|fil)$")  # :49-61
DEFAULT_SESSIONRE = r"[AT]GBT[12][0-9][AB]_\d+_\d+"
DEFAULT_PLAYERRE = r"^BLP([?<band>0-7])(?P<bank>[0-7])$"  # :72, quirk kept verbatim

INVENTORY_FIELDS = ("imjd", "smjd", "session", "scan", "src_name", "band", "bank", "host",
                    "file", "worker")


def parseguppiname(name):
    return _GUPPI_RE.search(name)


def parserawspecname(name):
    return _RAWSPEC_RE.search(name)


def _rx(r):
    return re.compile(r) if isinstance(r, str) else r


def _first_walk(path):
    for entry in os.walk(path):
        return entry
    raise FileNotFoundError(path)  # Julia's walkdir throws on a missing directory


def getinventory(filere=r"0002.h5$", root="/datax/dibas", sessionre=DEFAULT_SESSIONRE,
                 extra="GUPPI", playerre=DEFAULT_PLAYERRE, worker=1, warn=None):
    """List of inventory dicts (fields INVENTORY_FIELDS, src/gbtworkerfunctions.jl:63-66)."""
    filere, sessionre, playerre = _rx(filere), _rx(sessionre), _rx(playerre)
    host = socket.gethostname()
    inventory = []
    if not os.path.isdir(root):  # :79
        return inventory
    _, sessions, _ = _first_walk(root)  # :81 (symlinked dirs are listed as dirs here)
    sessions = [s for s in sessions if sessionre.search(s)]  # :85
    for session in sessions:
        _, players, _ = _first_walk(os.path.join(root, session, extra))  # :88
        players = [p for p in players if playerre.search(p)]  # :89
        for player in players:
            for d, _, files in os.walk(os.path.join(root, session, extra, player)):  # :92
                for base in (f for f in files if filere.search(f)):  # :93
                    file = os.path.join(d, base)
                    m = parseguppiname(file)
                    if m is None:
                        if warn:
                            warn(f"{host}:{file} did not match guppiname regex")
                        continue
                    if m["band"] is None or m["bank"] is None:
                        if warn:
                            warn(f"{host}:{file} did not match player regex")
                        continue
                    inventory.append(dict(
                        imjd=int(m["imjd"]), smjd=int(m["smjd"]), session=session,
                        scan=m["scan"], src_name=m["src"], band=int(m["band"]),
                        bank=int(m["bank"]), host=host, file=file, worker=worker))
    return inventory
