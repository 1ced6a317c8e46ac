#!/usr/bin/env python3
"""What a bench step costs beyond its kernel: one prepared band reduce
(cfg1: one 0002 file, cfg2: the 8-file band, F=64 T=16, t=1:272) launched K
times back to back, ms per step from the host clock around the K launches
(barrier + synchronize as bench.py), and the kernel time its events saw.

  none    no events
  hipev   a fence-less timing HipEvent pair recorded around every launch
          (bench.py rounds 1-3)
  ext     the events carried by the kernel dispatch itself
          (bldp_reduce_launch_timed / hipExtLaunchKernel)

    python tools/gap_probe.py [--steps 20,200] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="20,200")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng, HipEvent = pkg.engine, pkg._lib.HipEvent
    w272 = [0, 65536, 1, 0, 1, 1, 0, 272, 1]
    banks = [eng.synth(65536, 1, 279, 1024, seed=10 * b + 2, kind=0) for b in range(8)]
    res = {}
    for cfg, bk in (("cfg1", banks[:1]), ("cfg2", banks)):
        prep = eng.PreparedBandReduce(bk, 64, 16, "sum", w272)
        sp = int(torch.cuda.current_stream().cuda_stream)
        for K in (int(k) for k in a.steps.split(",")):
            evs = [(HipEvent(timing=True, fence=False), HipEvent(timing=True, fence=False))
                   for _ in range(K)]
            for var in ("none", "hipev", "ext"):
                best = None
                for _ in range(a.rounds):
                    for _ in range(5):
                        prep.launch(sp)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in range(K):
                        if var == "none":
                            prep.launch(sp)
                        elif var == "hipev":
                            evs[k][0].record(sp)
                            prep.launch(sp)
                            evs[k][1].record(sp)
                        else:
                            prep.launch_timed(sp, *evs[k])
                    host = (time.perf_counter() - t0) * 1e3 / K
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) * 1e3 / K
                    kern = (sum(e0.elapsed_time(e1) for e0, e1 in evs) / K
                            if var != "none" else None)
                    r = {"ms_per_step": round(ms, 5), "kernel_ms": kern and round(kern, 5),
                         "host_ms": round(host, 5)}
                    if best is None or r["ms_per_step"] < best["ms_per_step"]:
                        best = r
                key = f"{cfg} K={K} {var}"
                res[key] = best
                print(key, best, flush=True)
        prep.close()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
