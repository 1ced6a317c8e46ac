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
