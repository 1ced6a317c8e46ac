#!/usr/bin/env python3
"""Probe: how fast can a compressed FBH5 file's chunks get into (pinned)
host memory?  libhdf5 H5Dread_chunk one at a time vs parallel preads at the
parsed chunk index (h5chunks.py), several thread counts.  Page cache warm."""
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
fb = pkg.fbh5
z = np.load(os.path.join(REPO, "tests", "golden", "bslz4_v1.npz"), allow_pickle=False)
chunk = z["chunk_gamma_chunk_b2048"].tobytes()
nrep = 4096
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "bldp_read_probe.h5")
fb.write_bslz4_chunks(path, dict(foff=-1.0, nfpc=1024), (4096, 1, 16 * nrep), (16, 1, 4096),
                      (chunk for _ in range(nrep)))
H = fb.h5().L
fid = H.H5Fopen(path.encode(), 0, 0)
d = H.H5Dopen2(fid, b"data", 0)
t0 = time.perf_counter()
tab = pkg.h5chunks.chunk_table(path, H, d)
print(f"chunk_table: {len(tab['index'])} chunks in {1e3 * (time.perf_counter() - t0):.1f} ms")
ents = [tab["index"][k] for k in sorted(tab["index"])]
total = sum(e[1] for e in ents)
offs = np.cumsum([0] + [e[1] for e in ents[:-1]])
import torch  # noqa: E402

pinned = torch.empty(total, dtype=torch.uint8, pin_memory=True).numpy()
pageable = np.empty(total, np.uint8)
pageable[:] = 1
m = ctypes.c_uint32()
for rep in range(2):
    t0 = time.perf_counter()
    for k, key in enumerate(sorted(tab["index"])):
        H.H5Dread_chunk(d, 0, (ctypes.c_uint64 * 3)(*key), ctypes.byref(m),
                        ctypes.c_void_p(pinned.ctypes.data + int(offs[k])))
    el = time.perf_counter() - t0
print(f"H5Dread_chunk serial -> pinned: {total / el / 1e9:.2f} GB/s ({el * 1e3:.1f} ms)")
fd = os.open(path, os.O_RDONLY)


def rd(buf, k):
    mv = memoryview(buf)[int(offs[k]):int(offs[k]) + ents[k][1]]
    os.preadv(fd, [mv], ents[k][0])


for name, buf in (("pinned", pinned), ("pageable", pageable)):
    for th in (1, 4, 8, 16, 32):
        with ThreadPoolExecutor(th) as ex:
            for rep in range(2):
                t0 = time.perf_counter()
                list(ex.map(lambda k: rd(buf, k), range(len(ents))))
                el = time.perf_counter() - t0
        print(f"preadv x{th:2d} -> {name}: {total / el / 1e9:.2f} GB/s ({el * 1e3:.1f} ms)")
# batched: 16 threads, each thread a contiguous run of chunks
for th in (8, 16):
    per = (len(ents) + th - 1) // th

    def run(j, buf=pinned):
        for k in range(j * per, min(len(ents), (j + 1) * per)):
            rd(buf, k)
    with ThreadPoolExecutor(th) as ex:
        for rep in range(2):
            t0 = time.perf_counter()
            list(ex.map(run, range(th)))
            el = time.perf_counter() - t0
    print(f"preadv x{th:2d} contiguous runs -> pinned: {total / el / 1e9:.2f} GB/s")
print("cpus:", os.cpu_count(), "affinity:", len(os.sched_getaffinity(0)))
os.close(fd)
H.H5Dclose(d)
H.H5Fclose(fid)
os.remove(path)
