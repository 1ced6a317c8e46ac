#!/usr/bin/env python3
"""Bit-exact check of a build variant against the base build on misaligned
windows (integer-valued data, so every sum is exact under any order): the
reduce paths for sum/max/min and kurtosis (leaf/regs vs mid/two-pass, within
the leaf tolerance).  Used to vet BLDP_UNALIGNED_VEC before it became the
default; run on the GPU box after `tools/ab_variants.py --build`.

    python tools/unaligned_check.py --variant unal2
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="unal2")
    ap.add_argument("--base", default="base")
    a = ap.parse_args()
    import numpy as np
    import torch

    import __graft_entry__ as entry
    from ab_variants import VDIR, load

    pkg = entry.load_package()
    eng = pkg.engine
    libs = {n: load(os.path.join(VDIR, f"libbldp_{n}.so")) for n in (a.base, a.variant)}
    sp = int(torch.cuda.current_stream().cuda_stream)
    bad = 0

    def red(L, banks, win, F, T, op):
        nchan, nif, ntime = banks[0].shape
        out = eng.fb_empty(len(banks) * (win[1] // F), nif, win[7] // T)
        ptrs = (ctypes.c_void_p * len(banks))(*[b.data_ptr() for b in banks])
        keep, wp = pkg._lib.win_arg(win)
        rc = L.bldp_band_reduce_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), nchan, nif,
                                    ntime, wp, F, T, op, out.data_ptr(), sp)
        assert rc == 0, rc
        torch.cuda.synchronize()
        del keep
        return out.cpu().numpy()

    def kurt(L, banks, win):
        nchan, nif, ntime = banks[0].shape
        out = torch.empty(len(banks) * win[1] * nif, dtype=torch.float64, device="cuda")
        ptrs = (ctypes.c_void_p * len(banks))(*[b.data_ptr() for b in banks])
        keep, wp = pkg._lib.win_arg(win)
        rc = L.bldp_band_kurtosis_f32(len(banks), ctypes.cast(ptrs, ctypes.c_void_p), nchan, nif,
                                      ntime, wp, out.data_ptr(), sp)
        assert rc == 0, rc
        torch.cuda.synchronize()
        del keep
        return out.cpu().numpy()

    # (nchan, nif, ntime), window, F, T
    red_cases = [
        ((65540, 2, 272), [1, 65536, 1, 0, 2, 1, 0, 272, 1], 64, 16),
        ((65540, 2, 272), [3, 65536, 1, 1, 1, 1, 0, 256, 1], 1024, 16),
        ((65540, 1, 272), [2, 65536, 1, 0, 1, 1, 0, 272, 1], 8, 16),
        ((65540, 1, 272), [1, 65536, 1, 0, 1, 1, 0, 272, 1], 1, 16),
        ((65540, 1, 272), [2, 65536, 1, 0, 1, 1, 0, 272, 1], 2, 16),
        ((4097, 3, 40), [1, 4096, 1, 0, 3, 1, 0, 40, 1], 4, 8),  # odd pitch: dword rows
        ((1 << 20, 1, 16), [3, (1 << 20) - 1024, 1, 0, 1, 1, 0, 16, 1], 1024, 16),
        ((515, 1, 20000), [1, 512, 1, 0, 1, 1, 0, 19456, 1], 8, 1024),
        ((515, 1, 20000), [3, 512, 1, 0, 1, 1, 0, 20000, 1], 4, 1),
        # aligned F = 1024 (interleaved / segment kernels), full and ragged rows
        ((1 << 20, 2, 32), [0, 1 << 20, 1, 0, 2, 1, 0, 32, 1], 1024, 16),
        ((1 << 20, 1, 64), [0, 1 << 20, 1, 0, 1, 1, 0, 64, 1], 1024, 4),
        ((17 * 1024, 1, 48), [0, 17 * 1024, 1, 0, 1, 1, 0, 48, 1], 1024, 48),
    ]
    for shape, win, F, T in red_cases:
        banks = [eng.synth(*shape, 64, seed=s, kind=1) for s in range(3)]
        for op in (0, 2, 3):
            r0 = red(libs[a.base], banks, win, F, T, op)
            r1 = red(libs[a.variant], banks, win, F, T, op)
            ok = np.array_equal(r0, r1)
            plan = eng.plan(banks[0], F, T, "sum", win)["path"]
            print(f"reduce {shape} win={win[:3]} F={F} T={T} op={op} base-plan={plan}: "
                  f"{'ok' if ok else 'MISMATCH'}", flush=True)
            bad += not ok
    kurt_cases = [
        ((65540, 1, 16), [1, 65536, 1, 0, 1, 1, 0, 16, 1]),
        ((65540, 2, 32), [3, 65536, 1, 0, 2, 1, 0, 32, 1]),
        ((515, 1, 5000), [1, 512, 1, 0, 1, 1, 0, 5000, 1]),
        ((4097, 1, 2048), [1, 4096, 1, 0, 1, 1, 0, 2048, 1]),
    ]
    for shape, win in kurt_cases:
        banks = [eng.synth(*shape, 64, seed=s, kind=1) for s in range(2)]
        k0 = kurt(libs[a.base], banks, win)
        k1 = kurt(libs[a.variant], banks, win)
        ok = np.allclose(k0, k1, rtol=2e-6, atol=0, equal_nan=True)
        err = float(np.nanmax(np.abs(k0 - k1) / np.maximum(np.abs(k0), 1e-300)))
        print(f"kurtosis {shape} win={win[:3]}: {'ok' if ok else 'MISMATCH'} (max rel {err:.2e})",
              flush=True)
        bad += not ok
    print("UNALIGNED CHECK", "PASS" if bad == 0 else f"FAIL ({bad})", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
