"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu`` and run on the
MI355X box (``pytest -m gpu``); everything else runs on CPU."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import __graft_entry__ as entry  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbldp_hip)")


@pytest.fixture(scope="session")
def pkg():
    return entry.load_package()


@pytest.fixture(scope="session")
def orc():
    o = entry.load_oracle()
    o.lib()  # builds liboracle.so if needed
    return o


class Golden:
    def __init__(self):
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            self.manifest = json.load(f)
        self._z = np.load(os.path.join(GOLDEN, "golden_v1.npz"), allow_pickle=False)

    def input(self, name) -> np.ndarray:
        """Julia-order (c, i, t) Fortran array."""
        return np.asfortranarray(np.transpose(self._z[f"in_{name}"], (2, 1, 0)))

    def output(self, case) -> np.ndarray:
        a = self._z[case["output"]]
        return np.asfortranarray(a.T) if a.ndim else a

    def cases(self, kind):
        return [c for c in self.manifest["cases"] if c["kind"] == kind]


@pytest.fixture(scope="session")
def golden():
    return Golden()


# Kurtosis of windows > 512 spectra (k_kurt_leaf): the moments are exact
# Float64 about m, where StatsBase rounds z (2^-24 relative unless x - m is
# exact), z^2 and z^4 to Float32.  First order, |d cm2 / cm2| <= 3u and
# |d cm4 / cm4| <= 7u (u = 2^-24), so the ratio cm4/cm2^2 = k + 3 moves by at
# most 13u relative: |got - want| <= KURT_LEAF_TOL * |want + 3| (5% margin for
# the second-order terms).  m itself is exact on every path.
KURT_LEAF_TOL = 13 * 2.0 ** -24 * 1.05
# register-tile and two-pass paths: the recipe itself, only cm2 and cm4 (sums
# of nonnegative Float64 terms) added in another order: each within
# (nt - 1) 2^-53 relative of the exact sum, so k + 3 within 6 nt 2^-53.
def kurt_sum_tol(nt: int) -> float:
    return 6.0 * max(nt, 1) * 2.0 ** -53


# 8-bit rows (k_kurt_i8, typed.hip): exact integer power sums, re-centred
# exactly on the integer nearest the mean and finished in Float64 (within
# ~150 2^-53 of the exact ratio, typed.hip kurt_from_sums); the recipe's own
# rounding is first order (3 nt + 15) 2^-53 relative on k + 3.
KURT_INT_FINISH = 160.0 * 2.0 ** -53


def kurt_int_tol(nt: int) -> float:
    return (3.0 * max(nt, 1) + 15.0) * 2.0 ** -53 + KURT_INT_FINISH


def assert_kurtosis(got, want, path: str, nt: int, msg="") -> None:
    """GPU kurtosis against the oracle at the tolerance of the path that ran:
    bit-exact for "regs", kurt_sum_tol for "mid"/"twopass", KURT_LEAF_TOL for
    "leaf", kurt_int_tol for "int" (8-bit rows); NaN and +-Inf positions must
    match exactly everywhere."""
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    assert got.shape == want.shape, msg
    fin = np.isfinite(want)
    assert np.array_equal(np.isnan(got), np.isnan(want)), msg
    assert np.array_equal(got[~fin & ~np.isnan(want)], want[~fin & ~np.isnan(want)]), msg
    if path == "regs":
        assert same_bits(got, want), msg
        return
    tol = (KURT_LEAF_TOL if path == "leaf" else kurt_int_tol(nt) if path == "int"
           else kurt_sum_tol(nt))
    err = np.abs(got[fin] - want[fin])
    lim = tol * np.abs(want[fin] + 3.0)
    bad = err > lim
    assert not bad.any(), (msg, path, nt, float(err.max()), float((err / lim).max()))


def same_bits(a, b) -> bool:
    """Bit-exact float compare that treats every NaN as equal."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint32 if a.dtype == np.float32 else np.uint64),
                          b[~nb].view(np.uint32 if b.dtype == np.float32 else np.uint64))
