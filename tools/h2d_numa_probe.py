#!/usr/bin/env python3
"""Probe: H2D and D2H copy rates from pinned host memory placed on each NUMA
node (the allocating thread's memory policy bound to the node while torch's
pinned allocator -- hipHostMalloc -- pins the pages), beside torch's default
placement.  Prints one JSON line per placement.

    python tools/h2d_numa_probe.py [--mb 1024] [--reps 10]
"""
import argparse
import ctypes
import json
import os

MPOL_DEFAULT, MPOL_BIND = 0, 2
SYS_set_mempolicy = 238  # x86-64


def set_policy(node):
    libc = ctypes.CDLL(None, use_errno=True)
    if node is None:
        return libc.syscall(SYS_set_mempolicy, MPOL_DEFAULT, None, 0) == 0
    mask = ctypes.c_ulong(1 << node)
    return libc.syscall(SYS_set_mempolicy, MPOL_BIND, ctypes.byref(mask), 64) == 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    torch.cuda.init()
    dev = torch.device("cuda", 0)
    n = a.mb << 20
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    nodes = sorted(int(x[4:]) for x in os.listdir("/sys/devices/system/node") if x.startswith("node")
                   and x[4:].isdigit())
    for node in [None] + nodes:
        ok = set_policy(node)
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        h.fill_(1)
        set_policy(None)
        res = {"placement": "default" if node is None else f"node{node}", "policy_set": ok}
        for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)),
                         ("d2h", lambda: h.copy_(d, non_blocking=True))):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            e1.synchronize()
            res[name + "_GBps"] = round(n * a.reps / (e0.elapsed_time(e1) * 1e-3) / 1e9, 2)
        print(json.dumps(res), flush=True)
        del h


if __name__ == "__main__":
    main()
