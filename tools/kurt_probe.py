#!/usr/bin/env python3
"""Kurtosis calls on short leaf windows of the 0001 band (512 channels), for a
rocprofv3 kernel trace: which launches a call makes and what each costs.

    rocprofv3 --kernel-trace --stats -d gpurun_out/kp -o run -- python tools/kurt_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__ as entry  # noqa: E402

pkg = entry.load_package()
eng = pkg.engine
b4 = [eng.synth(512, 1, 880000, 8, seed=10 * b + 1, kind=0) for b in range(8)]
torch.cuda.synchronize()
for nt in (513, 1024, 8192, 100000):
    w = [0, 512, 1, 0, 1, 1, 0, nt, 1]
    print(nt, eng.kurtosis_plan(b4[0], w), flush=True)
    for _ in range(5):
        eng.band_kurtosis(b4, w)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(20):
        eng.band_kurtosis(b4, w)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"nt={nt}: {ev[0].elapsed_time(ev[1]) / 20:.4f} ms per call", flush=True)
