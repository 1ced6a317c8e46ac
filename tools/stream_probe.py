#!/usr/bin/env python3
"""How the per-step band exchange shares the GPU with the reduce: one rank,
one cfg3 bank (4 GiB, F=1024 T=16), K steps per variant, ms per step.

  none           reduce only (the floor)
  torch_async    band.BandPipeline as bench.py runs it: torch.distributed.gather
                 (RCCL) on the process group's stream, overlapped with the next
                 reduce
  torch_side     the same, the reduce on a fresh (non-default) stream
  native_inline  bldp_band_gather_f32 (ncclGather) on the reduce's own stream
  native_async   bldp_band_gather_f32 on a second stream, two slots, events
  native_hi      the same, the second stream at high priority
  pipe_native    band.NativeBandPipeline (high-priority stream), as bench.py
  hi_nowait      native_hi with a slot per step: the reducing stream never
                 waits for the gathers (the cost of the event record alone)
  hi_wait2       native_hi with 4 slots, the reducing stream waiting every
                 second step (for the gather two slots back)
  hi_nofence     native_hi with events recorded without the system-scope fence
  none_tev       reduce only, torch timing events around every reduce
  none_tev_nf    reduce only, fence-less HIP timing events around every reduce

    python tools/stream_probe.py [--steps 50] [--variants a,b,...]
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
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variants", default="none,torch_async,native_inline,native_hi,"
                    "pipe_native,hi_nowait,hi_nofence,none_tev,none_tev_nf")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist

    import __graft_entry__ as entry

    pkg = entry.load_package()
    eng = pkg.engine
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 1000))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    nchan, F, T = 1 << 26, 1024, 16
    bank = eng.synth(nchan, 1, 16, 1 << 20, seed=0, kind=0)
    nco = nchan // F
    torch.cuda.synchronize()
    nb = pkg.band.NativeBand(0, 1, 0, pkg.band.NativeBand.new_id())

    def run(name):
        main_s = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        comm = torch.cuda.Stream(priority=-1 if name.startswith(("native_hi", "hi_")) else 0)
        if name in ("torch_async", "torch_side", "pipe_native"):
            pipe = pkg.band.NativeBandPipeline(nco, 1, 1, device="cuda:0", comm=nb) \
                if name == "pipe_native" else \
                pkg.band.BandPipeline(nco, 1, 1, device="cuda:0", gather_single=True)
            cs = side if name == "torch_side" else main_s

            def step():
                with torch.cuda.stream(cs):
                    s = pipe.begin()
                    eng.band_reduce([bank], F, T, "sum", None, out=pipe.local(s))
                    pipe.exchange(s)

            def drain():
                pipe.drain()
        elif name in ("native_inline", "native_async", "native_hi", "hi_nowait", "hi_wait2",
                      "hi_nofence"):
            D = {"hi_nowait": a.steps + a.warmup + 1, "hi_wait2": 4}.get(name, 2)
            loc = [torch.empty((nco, 1, 1), device="cuda") for _ in range(D)]
            if name == "hi_nofence":
                HE = pkg._lib.HipEvent
                done = [HE(fence=False) for _ in range(D)]
                red = [HE(fence=False) for _ in range(D)]
            else:
                done = [torch.cuda.Event() for _ in range(D)]
                red = [torch.cuda.Event() for _ in range(D)]
            k = [0]
            res = []

            def step():
                s = k[0] % D
                k[0] += 1
                if name == "hi_wait2" and k[0] > 4 and k[0] % 2 == 1:
                    # slots s and s+1 were last gathered at steps k-4, k-3
                    main_s.wait_event(done[(s + 1) % D])
                elif D == 2 and k[0] > 2 and name == "hi_nofence":
                    done[s].wait(main_s)
                elif D == 2 and k[0] > 2 and name != "native_inline":
                    main_s.wait_event(done[s])  # the gather that last read slot s
                eng.band_reduce([bank], F, T, "sum", None, out=loc[s])
                if name == "native_inline":
                    res.append(nb.gather(loc[s], stream=main_s))
                elif name == "hi_nofence":
                    red[s].record(main_s)
                    red[s].wait(comm)
                    res.append(nb.gather(loc[s], stream=comm))
                    done[s].record(comm)
                else:
                    red[s].record(main_s)
                    comm.wait_event(red[s])
                    res.append(nb.gather(loc[s], stream=comm))
                    done[s].record(comm)
                if len(res) > 4:
                    res.pop(0)

            def drain():
                torch.cuda.current_stream().wait_stream(comm)
        else:
            out = eng.fb_empty(nco, 1, 1)
            if name == "none_tev_nf":
                tev = [pkg._lib.HipEvent(timing=True, fence=False) for _ in range(2)]
            elif name == "none_tev":
                tev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

            def step():
                if name.startswith("none_tev"):
                    tev[0].record(main_s)
                eng.band_reduce([bank], F, T, "sum", None, out=out)
                if name.startswith("none_tev"):
                    tev[1].record(main_s)

            def drain():
                pass
        for _ in range(a.warmup):
            step()
        drain()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        host = (time.perf_counter() - t0) * 1e3 / a.steps
        drain()
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) * 1e3 / a.steps
        return {"variant": name, "ms_per_step": round(el, 4), "host_ms": round(host, 4)}

    for rnd in range(2):
        for v in a.variants.split(","):
            r = run(v)
            r["round"] = rnd
            print(json.dumps(r), flush=True)
    nb.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
