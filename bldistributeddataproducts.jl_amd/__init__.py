"""MI355X engine for BLDistributedDataProducts.jl's worker-side reduction.

Layout mirrors the reference (src/BLDistributedDataProducts.jl:1-7):
``GBT`` (src/gbt.jl) with ``GBT.WorkerFunctions`` (src/gbtworkerfunctions.jl).
The arithmetic runs in libbldp_hip (HIP kernels for gfx950) behind the C ABI
of include/bldp.h; this package is the Python host side over that ABI.

The directory name is not a Python identifier; load it with
``__graft_entry__.load_package()`` (registers it as ``bldp_amd``).
"""
from . import _lib, band, engine, fbh5, filestream, gbt, h5chunks, idxs, readers, worker  # noqa: F401
from ._lib import ArgumentError, BLDPError, BoundsError, DimensionMismatch, ReadError  # noqa: F401
from .idxs import COLON, JRange, sanitizeidxs  # noqa: F401
from .worker import FRange, fqav  # noqa: F401

GBT = gbt
GBT.WorkerFunctions = worker
WorkerFunctions = worker

__all__ = ["GBT", "WorkerFunctions", "fqav", "JRange", "FRange", "COLON", "sanitizeidxs",
           "engine", "band", "DimensionMismatch", "BoundsError", "BLDPError", "ReadError"]
