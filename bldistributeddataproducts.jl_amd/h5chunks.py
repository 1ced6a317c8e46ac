"""The chunk index of a chunked FBH5 ``data`` dataset, read straight from the
file: every chunk's file offset, stored size and filter mask from a handful
of small reads, instead of one libhdf5 lookup per chunk.

Why: libhdf5 1.10 (this image) has no ``H5Dchunk_iter``; ``H5Dread_chunk``
and ``H5Dget_chunk_info_by_coord`` each walk the chunk B-tree (~20-25 us per
chunk, single-threaded, not thread-safe), which bounds a compressed rawspec
product's read (src/gbtworkerfunctions.jl:181-187; H5Zbitshuffle,
Project.toml:10) at ~12 GB/s of decoded data.  With the table in hand the
compressed chunks are read by plain parallel preads (filestream.py).

Scope, checked before use (anything else returns None and the caller keeps
the libhdf5 path):
  * superblock version 0-3 with 8-byte offsets and lengths;
  * a version-1 object header for ``data`` (libver "earliest", what rawspec
    and h5py write by default), continuation blocks followed;
  * a version 1-3 data layout message of class "chunked";
  * a version-1 B-tree (node type 1) as the chunk index.
The table is cross-checked against ``H5Dget_chunk_info_by_coord`` for the
first, middle and last chunk before it is trusted.
"""
from __future__ import annotations

import ctypes
import os
import struct

_SIG = b"\x89HDF\r\n\x1a\n"
_UNDEF = (1 << 64) - 1


def _superblock(fd):
    """(base address, size of offsets, size of lengths) or None."""
    for off in [0] + [512 << k for k in range(12)]:
        b = os.pread(fd, 16, off)
        if len(b) < 16:
            return None
        if b[:8] == _SIG:
            v = b[8]
            if v in (0, 1):
                return off, b[13], b[14]
            if v in (2, 3):
                return off, b[9], b[10]
            return None
    return None


def _object_messages(fd, base, addr):
    """(type, data) of every message of a version-1 object header."""
    hdr = os.pread(fd, 16, base + addr)
    if len(hdr) < 16 or hdr[0] != 1:
        return None  # not a version-1 object header
    nmsg, size = struct.unpack_from("<H", hdr, 2)[0], struct.unpack_from("<I", hdr, 8)[0]
    blocks = [(base + addr + 16, size)]
    out = []
    while blocks and len(out) < nmsg + 64:
        start, length = blocks.pop(0)
        raw = os.pread(fd, length, start)
        pos = 0
        while pos + 8 <= len(raw):
            mtype, msize = struct.unpack_from("<HH", raw, pos)
            data = raw[pos + 8: pos + 8 + msize]
            pos += 8 + msize
            if mtype == 0x0010 and len(data) >= 16:  # continuation
                coff, clen = struct.unpack_from("<QQ", data, 0)
                blocks.append((base + coff, clen))
            else:
                out.append((mtype, data))
    return out


def _layout(msgs):
    """(B-tree address, chunk dims incl. the element-size dim) or None."""
    for mtype, d in msgs:
        if mtype != 0x0008 or not d:
            continue
        ver = d[0]
        if ver == 3:
            if d[1] != 2:
                return None  # not chunked
            nd = d[2]
            addr = struct.unpack_from("<Q", d, 3)[0]
            dims = struct.unpack_from(f"<{nd}I", d, 11)
            return addr, dims
        if ver in (1, 2):
            nd, cls = d[1], d[2]
            if cls != 2:
                return None
            addr = struct.unpack_from("<Q", d, 8)[0]
            dims = struct.unpack_from(f"<{nd}I", d, 16)
            return addr, dims
        return None
    return None


def _walk(fd, base, addr, nd, out, depth=0):
    """Leaf entries of a version-1 chunk B-tree: (offsets, addr, size, mask)."""
    if depth > 32:
        raise ValueError("B-tree too deep")
    hdr = os.pread(fd, 24, base + addr)
    if len(hdr) < 24 or hdr[:4] != b"TREE" or hdr[4] != 1:
        raise ValueError("not a chunk B-tree node")
    level, used = hdr[5], struct.unpack_from("<H", hdr, 6)[0]
    ksz = 8 + 8 * nd
    raw = os.pread(fd, used * (ksz + 8) + ksz, base + addr + 24)
    pos = 0
    for _ in range(used):
        size, mask = struct.unpack_from("<II", raw, pos)
        offs = struct.unpack_from(f"<{nd}Q", raw, pos + 8)
        child = struct.unpack_from("<Q", raw, pos + ksz)[0]
        pos += ksz + 8
        if level == 0:
            out.append((offs[:-1], child, size, mask))
        else:
            _walk(fd, base, child, nd, out, depth + 1)


def chunk_table(fname, H=None, dset=None):
    """{"base": file offset of address 0, "chunk": C-order chunk dims,
    "index": {chunk origin (t, i, c): (absolute file offset, bytes, filter
    mask)}} for ``data``, or None when the file is outside the scope above or
    the cross-check against libhdf5 fails.  ``H``/``dset``: an open libhdf5
    binding and dataset id (for the object address and the cross-check)."""
    if H is None or dset is None:
        return None
    info = (ctypes.c_uint8 * 1024)()
    if H.H5Oget_info2(dset, info, 0x0001) < 0:  # H5O_INFO_BASIC: fileno, addr, ...
        return None
    oaddr = struct.unpack_from("<Q", bytes(info), 8)[0]  # H5O_info_t.addr
    fd = os.open(fname, os.O_RDONLY)
    try:
        sb = _superblock(fd)
        if sb is None or sb[1] != 8 or sb[2] != 8:
            return None
        base = sb[0]
        msgs = _object_messages(fd, base, oaddr)
        if not msgs:
            return None
        lay = _layout(msgs)
        if lay is None or lay[0] == _UNDEF:
            return None
        baddr, cdims = lay
        entries = []
        try:
            _walk(fd, base, baddr, len(cdims), entries)
        except (ValueError, struct.error):
            return None
    finally:
        os.close(fd)
    index = {e[0]: (base + e[1], e[2], e[3]) for e in entries}
    if not index:
        return None
    # cross-check a few chunks against libhdf5
    keys = sorted(index)
    for k in {keys[0], keys[len(keys) // 2], keys[-1]}:
        off = (ctypes.c_uint64 * 3)(*k)
        mask, addr, size = ctypes.c_uint(), ctypes.c_uint64(), ctypes.c_uint64()
        if H.H5Dget_chunk_info_by_coord(dset, off, ctypes.byref(mask), ctypes.byref(addr),
                                        ctypes.byref(size)) < 0:
            return None
        if (base + addr.value, size.value, mask.value) != index[k]:
            return None
    return {"base": base, "chunk": tuple(int(x) for x in cdims[:-1]), "index": index}
