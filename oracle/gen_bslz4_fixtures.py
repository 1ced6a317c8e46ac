"""TEST INFRASTRUCTURE: golden vectors for HDF5 filter 32008 (bitshuffle +
LZ4), the codec of compressed rawspec FBH5 products (H5Zbitshuffle in the
reference, Project.toml:10).

Run with an interpreter that has imagecodecs (this image: /opt/conda/bin/python3.9,
imagecodecs 2021.8.26, which links the bitshuffle and LZ4 C libraries):

    /opt/conda/bin/python3.9 oracle/gen_bslz4_fixtures.py

Each chunk is laid out the way bitshuffle's HDF5 filter writes it
(bshuf_h5filter.c / bshuf_compress_lz4):
    uint64 BE  uncompressed bytes
    uint32 BE  block size in bytes
    per block: uint32 BE compressed size, LZ4 block of the bit-transposed block
    (blocks of `block` elements, then one block of the remainder rounded down
    to a multiple of 8 elements), then the last (n % 8) elements raw.
The bit transpose and LZ4 come from imagecodecs (i.e. the bitshuffle and
lz4 libraries themselves); every chunk is decoded back with imagecodecs and
checked before it is written.  Output: tests/golden/bslz4_v1.npz.
"""
from __future__ import annotations

import json
import os
import struct

import imagecodecs
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def encode(a: np.ndarray, block: int) -> bytes:
    es = a.itemsize
    flat = np.ascontiguousarray(a).ravel()
    n = flat.size
    parts = [struct.pack(">QI", n * es, block * es)]

    def blk(x):
        e = imagecodecs.bitshuffle_encode(x.tobytes(), itemsize=es, blocksize=x.size)
        z = imagecodecs.lz4_encode(bytes(e), header=False)
        parts.append(struct.pack(">I", len(z)) + bytes(z))

    nfull = n // block
    for b in range(nfull):
        blk(flat[b * block:(b + 1) * block])
    last = n % block
    last -= last % 8
    if last:
        blk(flat[nfull * block:nfull * block + last])
    parts.append(flat[nfull * block + last:].tobytes())
    return b"".join(parts)


def decode_check(buf: bytes, dtype, n) -> np.ndarray:
    total, bbytes = struct.unpack(">QI", buf[:12])
    es = np.dtype(dtype).itemsize
    block = bbytes // es
    pos, out = 12, []
    nfull = n // block
    sizes = [block] * nfull
    last = n % block
    last -= last % 8
    if last:
        sizes.append(last)
    for sz in sizes:
        (cl,) = struct.unpack(">I", buf[pos:pos + 4])
        raw = imagecodecs.lz4_decode(buf[pos + 4:pos + 4 + cl], header=False, out=sz * es)
        out.append(np.frombuffer(imagecodecs.bitshuffle_decode(bytes(raw), itemsize=es,
                                                                blocksize=sz), dtype))
        pos += 4 + cl
    out.append(np.frombuffer(buf[pos:], dtype))
    assert total == n * es
    return np.concatenate(out)


def main():
    rng = np.random.default_rng(32008)
    cases = {}
    # BL-like power: gamma x bandpass scallop x DC spike, one 0002-shaped chunk
    x = np.arange(4096) % 1024
    bp = (0.2 + 0.8 * np.sin(np.pi * (x + 0.5) / 1024) ** 2) * np.where(x == 512, 10, 1)
    cases["gamma_chunk"] = (rng.gamma(2.0, 5e8, (16, 1, 4096)) * bp).astype(np.float32)
    # integer-valued, highly repetitive (long and overlapping LZ4 matches)
    cases["int_runs"] = np.repeat(rng.integers(0, 8, 1200), 7).astype(np.float32)
    cases["zeros"] = np.zeros(5000, np.float32)  # offset-1 matches
    cases["noise_bits"] = rng.integers(0, 2**32, 3000, dtype=np.uint32).view(np.float32)
    cases["tiny_tail"] = (rng.random(2048 * 2 + 13) * 100).astype(np.float32)  # n % 8 == 5
    cases["lt8"] = np.array([1.5, -2.0, 3.25], np.float32)  # raw tail only
    cases["smooth"] = np.cumsum(rng.standard_normal(20000)).astype(np.float32)
    arrays, manifest = {}, []
    for name, a in cases.items():
        for block in (2048, 512):
            buf = encode(a, block)
            back = decode_check(buf, a.dtype, a.size)
            assert np.array_equal(back.view(np.uint32), a.ravel().view(np.uint32)), name
            key = f"{name}_b{block}"
            arrays[f"raw_{key}"] = a
            arrays[f"chunk_{key}"] = np.frombuffer(buf, np.uint8)
            manifest.append(dict(name=key, n=int(a.size), shape=list(a.shape), block=block,
                                 compressed_bytes=len(buf), ratio=round(a.nbytes / len(buf), 3)))
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "bslz4_v1.npz"), **arrays)
    with open(os.path.join(OUT, "bslz4_manifest.json"), "w") as f:
        json.dump(dict(generator="oracle/gen_bslz4_fixtures.py",
                       imagecodecs=imagecodecs.__version__,
                       bitshuffle=imagecodecs.bitshuffle_version(),
                       lz4=imagecodecs.lz4_version(), cases=manifest), f, indent=1)
    for m in manifest:
        print(m)


if __name__ == "__main__":
    main()
