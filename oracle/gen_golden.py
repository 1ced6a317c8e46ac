"""TEST INFRASTRUCTURE: writes tests/golden/golden_v1.npz + manifest.json.

Every expected output here comes from the NumPy restatement (oracle.np_*),
written independently of the C oracle; tests check BOTH the C oracle and the
GPU against these files.  The only reference-pinned vectors are the two
fqav(range) known answers of test/runtests.jl:5-6 ("kat_range").

Integer-valued inputs (0..255) keep every float32 sum below 2^24, so their
expected outputs are exact under any summation order (bit-exact checks).
Run:  python oracle/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")
VERSION = 1


def main():
    os.makedirs(OUT, exist_ok=True)
    arrays: dict[str, np.ndarray] = {}
    cases = []

    def add_input(name, a):
        arrays[f"in_{name}"] = np.ascontiguousarray(np.transpose(a, (2, 1, 0)))  # [t][i][c]

    def add_case(kind, inp, expect, **params):
        key = f"out_{len(cases):03d}"
        e = np.asarray(expect)
        arrays[key] = np.ascontiguousarray(e.T) if e.ndim else e
        cases.append(dict(kind=kind, input=inp, output=key, ndim=int(e.ndim), **params))

    rng = np.random.default_rng(20261015)
    # (i) integer-valued, exact
    ia = np.asfortranarray(rng.integers(0, 256, (1024, 2, 48)).astype(np.float32))
    add_input("int_a", ia)
    for F, T in [(1, 16), (2, 4), (4, 1), (8, 16), (64, 1), (64, 16), (1024, 48), (16, 3)]:
        for op in ("sum", "mean", "max", "min"):
            add_case("reduce", "int_a", O.np_reduce(ia, F, T, op), fqavby=F, tavby=T, op=op,
                     win=None, exact=op != "mean" or (F * T) & (F * T - 1) == 0)
    wins = [[32, 512, 1, 1, 1, 1, 4, 32, 1],        # (33:544, 2, 5:36)
            [1020, 96, -3, 0, 2, 1, 44, 12, -3],     # (1021:-3:736, :, 45:-3:12)
            [5, 120, 8, 0, 2, 1, 0, 48, 1]]          # (6:8:957, :, :)
    for w in wins:
        for F, T in [(1, 1), (4, 4), (8, 2), (3, 6)]:
            if w[1] % F or w[7] % T:
                continue
            for op in ("sum", "max"):
                add_case("reduce", "int_a", O.np_reduce(ia, F, T, op, w), fqavby=F, tavby=T,
                         op=op, win=w, exact=True)
    ib = np.asfortranarray(rng.integers(0, 256, (96, 3, 10)).astype(np.float32))
    add_input("int_b", ib)
    for F in (3, 6, 12, 96):
        for T in (1, 2, 5, 10):
            add_case("reduce", "int_b", O.np_reduce(ib, F, T, "sum"), fqavby=F, tavby=T,
                     op="sum", win=None, exact=True)
    # (ii) gamma-distributed BL-like power, 1e-5 relative
    ga = O.gamma_bandpass(2048, 1, 64, 1024, 11)
    add_input("gamma_a", ga)
    for F, T in [(4, 1), (64, 16), (256, 4), (1024, 64), (1, 8)]:
        for op in ("sum", "mean", "max", "min"):
            add_case("reduce", "gamma_a", O.np_reduce(ga, F, T, op), fqavby=F, tavby=T, op=op,
                     win=None, exact=op in ("max", "min"))
    # signed zeros / NaN / inf: Julia max/min semantics
    sa = np.zeros((16, 1, 4), np.float32, order="F")
    sa[0:4, 0, 0] = [-0.0, -0.0, -0.0, -0.0]
    sa[4:8, 0, 0] = [-0.0, 0.0, -0.0, -0.0]
    sa[8:12, 0, 0] = [1.0, np.nan, 2.0, 3.0]
    sa[12:16, 0, 0] = [np.inf, 1.0, -np.inf, 0.0]
    sa[:, 0, 1:] = rng.integers(-3, 4, (16, 3))
    add_input("special", sa)
    for op in ("sum", "max", "min"):
        add_case("reduce", "special", O.np_reduce(sa, 4, 1, op), fqavby=4, tavby=1, op=op,
                 win=None, exact=True)
    # (iii) kurtosis
    ka = np.asfortranarray(
        (rng.standard_normal((128, 2, 600)) ** 2 + rng.standard_normal((128, 2, 600)) ** 2)
        .astype(np.float32) * 1e8)
    ka[5, 1, :] = 42.0  # constant row -> NaN
    add_input("kurt_a", ka)
    add_case("kurtosis", "kurt_a", O.np_kurtosis(ka), win=None)
    add_case("kurtosis", "kurt_a", O.np_kurtosis(ka, [8, 64, 1, 0, 2, 1, 100, 400, 1]),
             win=[8, 64, 1, 0, 2, 1, 100, 400, 1])
    # (iv) band stitch: 8 banks (64, 1, 6) -> (512, 1, 6)
    for b in range(8):
        add_input(f"bank{b}", np.asfortranarray(
            rng.integers(0, 256, (64, 1, 6)).astype(np.float32)))
    banks = [np.transpose(arrays[f"in_bank{b}"], (2, 1, 0)) for b in range(8)]
    add_case("stitch", [f"bank{b}" for b in range(8)], O.np_stitch(banks))
    add_case("band", [f"bank{b}" for b in range(8)],
             O.np_stitch([O.np_reduce(x, 8, 2, "sum") for x in banks]), fqavby=8, tavby=2,
             op="sum")
    # (v) despike
    add_case("despike", "int_a", O.np_despike(ia[:, :, :3], 16), nfpc=16, ntime=3)
    # (vi) range KATs from the reference's own tests (test/runtests.jl:5-6)
    kats = [dict(first=1, step=1, length=4, n=4, expect=[2.5, 4.0, 1]),
            dict(first=1, step=2, length=8, n=4, expect=[4.0, 8.0, 2])]
    for k in kats:
        got = O.np_fqav_range(k["first"], k["step"], k["length"], k["n"])
        assert list(got) == k["expect"], (got, k)
    np.savez_compressed(os.path.join(OUT, "golden_v1.npz"), **arrays)
    manifest = dict(version=VERSION, generator="oracle/gen_golden.py (NumPy restatement)",
                    seed=20261015, layout="arrays stored C-order [t][i][c] (Julia (c,i,t))",
                    kat_range=kats, cases=cases)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(cases)} cases, {sum(a.nbytes for a in arrays.values()) / 1e6:.2f} MB raw")


if __name__ == "__main__":
    main()
