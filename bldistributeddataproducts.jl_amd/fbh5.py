"""FBH5 (filterbank-in-HDF5) window reads — placeholder until the libhdf5
binding lands."""
from __future__ import annotations

from ._lib import BLDPError


def _unavailable():
    raise BLDPError(-1, "FBH5 reader not available yet (no HDF5 backend bound)")


def read_window(fname, idxs):
    _unavailable()


def header(fname):
    _unavailable()
