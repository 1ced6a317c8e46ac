#!/usr/bin/env python3
"""Probe: can two RCCL ranks share the one GPU of this box?  Runs the C-ABI
band exchange (band.NativeBand) with two processes on device 0.  Prints the
outcome; meant to be run under `timeout`."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def rank_main(rank, nid, q):
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng = pkg.engine
    torch.cuda.set_device(0)
    try:
        nb = pkg.band.NativeBand(0, 2, rank, nid)
    except Exception as e:  # noqa: BLE001
        q.put((rank, "init failed: " + str(e)))
        return
    banks = [eng.synth(4096, 1, 32, 64, seed=10 * rank + b, kind=1) for b in range(2)]
    local = eng.band_reduce(banks, 64, 8)
    got = nb.gather(local)
    torch.cuda.synchronize()
    if rank == 0:
        q.put((rank, ("ok", eng.fb_to_numpy(got).tolist())))
    else:
        q.put((rank, ("ok", eng.fb_to_numpy(local).tolist())))
    nb.close()


if __name__ == "__main__":
    import torch.multiprocessing as mp

    import __graft_entry__ as entry

    pkg = entry.load_package()
    nid = pkg.band.NativeBand.new_id()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=rank_main, args=(r, nid, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=30)
    print({r: (v if isinstance(v, str) else v[0]) for r, v in res.items()})
    if all(not isinstance(v, str) for v in res.values()):
        band = np.array(res[0][1], np.float32)
        r1 = np.array(res[1][1], np.float32)
        ok = band.shape[0] == 2 * r1.shape[0] and np.array_equal(band[r1.shape[0]:], r1)
        print("two-rank gather matches:", ok)
