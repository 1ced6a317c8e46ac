"""ctypes boundary to libbldp_hip.so (include/bldp.h).

This is the same binding a Julia ``ccall`` shim makes; the
Python host mirror calls the HIP library through it and through nothing else.
There is no CPU fallback: if the library is missing the first call raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libbldp_hip.so")
CSRC = os.path.join(PKG_DIR, "csrc")

OPS = {"sum": 0, "mean": 1, "max": 2, "min": 3}
PATHS = {0: "vector", 1: "narrow", 2: "scalar", 3: "tile", 4: "interleaved", 5: "row",
         6: "narrow_mis", 7: "lane"}
KURT_PATHS = {0: "regs", 1: "mid", 2: "leaf", 3: "twopass"}

BLDP_OK, BLDP_EINVAL, BLDP_EDIM, BLDP_EHIP, BLDP_ENOMEM, BLDP_EBOUNDS = 0, -1, -2, -3, -5, -6
BLDP_ECOMM, BLDP_EIO = -7, -8
ABI_VERSION = 5
BLDP_BAND_STAGED = 1
BLDP_BAND_PEER_STORE = 2
BLDP_COMM_ID_BYTES = 128


class BLDPError(RuntimeError):
    """Any libbldp_hip failure (ErrorException on the Julia side)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class DimensionMismatch(BLDPError, ValueError):
    """fqavby/tavby does not divide the selected axis
    (Julia reshape in fqav, src/gbtworkerfunctions.jl:18-19)."""


class BoundsError(BLDPError, IndexError):
    """Window outside the array (h5["data"][idxs...], :185)."""


class ArgumentError(BLDPError, ValueError):
    """Invalid argument (Julia AssertionError / ArgumentError analogues)."""


class ReadError(BLDPError, OSError):
    """A file read failed or ended early (truncated file, stale chunk index):
    Julia's SystemError / EOFError from the HDF5 / mmap read."""


# every symbol include/bldp.h declares, with its ctypes signature
P, I64, I, D, SZ, U64 = (ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                         ctypes.c_size_t, ctypes.c_uint64)
SIGNATURES = {
    "bldp_abi_version": ([], I),
    "bldp_last_error": ([ctypes.c_char_p, SZ], I),
    "bldp_device_count": ([P], I),
    "bldp_init": ([I, P], I),
    "bldp_finalize": ([], I),
    "bldp_host_register": ([P, SZ], I),
    "bldp_host_unregister": ([P], I),
    "bldp_plan_option": ([ctypes.c_char_p, I64, P], I),
    "bldp_reduce_shape": ([I64, I64, I64, P, I64, I64, P], I),
    "bldp_reduce_plan_f32": ([P, I64, I64, I64, P, I64, I64, I, P, P], I),
    "bldp_reduce_f32": ([P, I64, I64, I64, P, I64, I64, I, P, P], I),
    "bldp_reduce_strided_f32": ([P, I64, I64, I64, P, I64, I64, I, P, I64, I64, P], I),
    "bldp_reduce_host_f32": ([I, P, I64, I64, I64, P, I64, I64, I, P], I),
    "bldp_band_reduce_f32": ([I, P, I64, I64, I64, P, I64, I64, I, P, P], I),
    "bldp_band_reduce_prepare_f32": ([I, P, I64, I64, I64, P, I64, I64, I, P, P], I),
    "bldp_reduce_launch": ([P, P], I),
    "bldp_reduce_prepare": ([I, P, I64, I64, I64, P, I64, I64, I, P, I64, I64, P], I),
    "bldp_kurtosis_prepare": ([I, P, I64, I64, I64, P, P, P], I),
    "bldp_reduce_launch_timed": ([P, P, P, P], I),
    "bldp_reduce_release": ([P], I),
    "bldp_band_reduce_multi_f32": ([I, P, P, I64, I64, I64, P, I64, I64, I, I, P, ctypes.c_uint],
                                   I),
    "bldp_peer_access": ([I, I, P], I),
    "bldp_device_to_host": ([P, P, I64, P, P, P], I),
    "bldp_stitch_f32": ([I, P, I64, I64, I64, P, P], I),
    "bldp_despike_f32": ([P, I64, I64, I64, I64, P], I),
    "bldp_kurtosis_workspace_size": ([I64, I64, I64, P], SZ),
    "bldp_kurtosis_f32": ([P, I64, I64, I64, P, P, P, P], I),
    "bldp_kurtosis_plan_f32": ([P, I64, I64, I64, P, P], I),
    "bldp_kurtosis_host_f32": ([I, P, I64, I64, I64, P, P], I),
    "bldp_band_kurtosis_f32": ([I, P, I64, I64, I64, P, P, P], I),
    "bldp_fqav_range": ([D, D, I64, I64, P, P, P], I),
    "bldp_synth_f32": ([P, I64, I64, I64, I64, U64, I, P], I),
    "bldp_reduce_out_dtype": ([I, I], I),
    "bldp_reduce_strided": ([I, P, I64, I64, I64, P, I64, I64, I, P, I64, I64, P], I),
    "bldp_kurtosis": ([I, P, I64, I64, I64, P, P, P], I),
    "bldp_reduce_host": ([I, I, P, I64, I64, I64, P, I64, I64, I, P], I),
    "bldp_kurtosis_host": ([I, I, P, I64, I64, I64, P, P], I),
    "bldp_bslz4_info": ([P, SZ, P, P], I),
    "bldp_unchunk_f32": ([P, P, P, P, P, P, P], I),
    "bldp_bslz4_decode_host": ([P, SZ, I, P, SZ], I),
    "bldp_bslz4_decode_dev": ([I, P, P, P, P, I, P, P, P, P], I),
    "bldp_bslz4_decode_dev_async": ([I, P, P, P, P, I, P, P, P, P, P], I),
    "bldp_bslz4_error": ([P, P], I),
    "bldp_chunks_to_device": ([I, I64, P, P, P, P, I64, P, P, P, I64, P, I64, I64, P, P, P, P],
                              I),
    "bldp_file_chunks_to_device": ([I64, P, P, P, P, P, I64, P, P, P, I64, P, I64, I64, P, P, P,
                                    P], I),
    "bldp_runs_to_device": ([I, I64, P, P, P, I64, I64, I, P, P, P], I),
    "bldp_file_runs_to_device": ([I64, P, P, P, P, I64, I64, I, P, P, P], I),
    "bldp_comm_id": ([P], I),
    "bldp_comm_init": ([I, I, I, P, P], I),
    "bldp_comm_destroy": ([P], I),
    "bldp_band_gather_f32": ([P, I, P, I64, P, P], I),
}

_lib = None


def build(force: bool = False) -> str:
    """Compile libbldp_hip.so in-tree for gfx950 (hipcc, see csrc/Makefile)."""
    if force and os.path.exists(LIB_PATH):
        os.remove(LIB_PATH)
    subprocess.run(["make", "-s", "-C", CSRC], check=True)
    return LIB_PATH


def lib():
    """The loaded library.  torch is imported first so that the process has a
    single HIP runtime (libamdhip64.so.7) shared by torch and libbldp_hip."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  (HIP runtime load order, see docstring)

        if not os.path.exists(LIB_PATH):
            raise BLDPError(BLDP_EINVAL, f"{LIB_PATH} is not built; run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        if L.bldp_abi_version() != ABI_VERSION:
            raise BLDPError(BLDP_EINVAL, f"libbldp_hip ABI version {L.bldp_abi_version()}, "
                                         f"expected {ABI_VERSION}: rebuild it")
        _lib = L
    return _lib


class plan_option:
    """Context manager forcing a plan option (bldp_plan_option) and restoring
    it: ``with plan_option("row_split", 4): ...``; value -1 = the planner's
    choice.  A/B and TEST facility only: the option is process-wide (every
    thread's plans see it), so no product code path uses this."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, int(value)

    def __enter__(self):
        prev = ctypes.c_int64()
        check(lib().bldp_plan_option(self.name.encode(), self.value, ctypes.byref(prev)),
              "bldp_plan_option")
        self.prev = prev.value
        return self

    def __exit__(self, *exc):
        check(lib().bldp_plan_option(self.name.encode(), self.prev, None), "bldp_plan_option")
        return False


def last_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    lib().bldp_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int, what: str = "") -> None:
    if rc == BLDP_OK:
        return
    msg = last_error() or what
    if rc == BLDP_EDIM:
        raise DimensionMismatch(rc, msg)
    if rc == BLDP_EBOUNDS:
        raise BoundsError(rc, msg)
    if rc == BLDP_EINVAL:
        raise ArgumentError(rc, msg)
    if rc == BLDP_EIO:
        raise ReadError(rc, msg)
    raise BLDPError(rc, msg)


def win_arg(win):
    """9-int64 window -> (keepalive, pointer) or (None, None) for (:,:,:)."""
    if win is None:
        return None, None
    w = (ctypes.c_int64 * 9)(*[int(x) for x in win])
    return w, ctypes.cast(w, ctypes.c_void_p)


def stream_ptr(stream=None) -> int:
    """hipStream_t of a torch stream (default: torch's current stream); a raw
    hipStream_t (int) passes through."""
    if isinstance(stream, int):
        return stream
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


HIP_EVENT_DISABLE_TIMING = 0x2
HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000
_hip = None


def hip():
    """The HIP runtime libbldp_hip.so is linked to (its soname, so the copy
    already loaded -- torch's, when torch came first -- is the one bound)."""
    global _hip
    if _hip is None:
        lib()
        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        h.hipEventRecord.argtypes = [P, P]
        h.hipStreamWaitEvent.argtypes = [P, P, ctypes.c_uint]
        h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), P, P]
        h.hipEventSynchronize.argtypes = [P]
        h.hipEventDestroy.argtypes = [P]
        _hip = h
    return _hip


class HipEvent:
    """A HIP event with the flags torch.cuda.Event does not expose.  With
    ``fence=False`` (hipEventDisableSystemFence) recording it does no
    system-scope release (no L2 write-back to host scope), which is all a
    consumer on the same device needs: a timing event, or a stream of the same
    GPU waiting for a kernel's output (the band exchange's gather)."""

    def __init__(self, timing=False, fence=True):
        self._h = hip()
        e = ctypes.c_void_p()
        flags = (0 if timing else HIP_EVENT_DISABLE_TIMING) | \
            (0 if fence else HIP_EVENT_DISABLE_SYSTEM_FENCE)
        rc = self._h.hipEventCreateWithFlags(ctypes.byref(e), flags)
        if rc:
            raise BLDPError(BLDP_EHIP, f"hipEventCreateWithFlags(0x{flags:x}) failed: {rc}")
        self.ev = e

    def _ok(self, rc, what):
        if rc:
            raise BLDPError(BLDP_EHIP, f"{what} failed: {rc}")

    def record(self, stream=None):
        self._ok(self._h.hipEventRecord(self.ev, stream_ptr(stream)), "hipEventRecord")

    def wait(self, stream=None):
        """``stream`` (default: torch's current) waits on the GPU for it."""
        self._ok(self._h.hipStreamWaitEvent(stream_ptr(stream), self.ev, 0), "hipStreamWaitEvent")

    def synchronize(self):
        self._ok(self._h.hipEventSynchronize(self.ev), "hipEventSynchronize")

    def elapsed_time(self, end) -> float:
        ms = ctypes.c_float()
        self._ok(self._h.hipEventElapsedTime(ctypes.byref(ms), self.ev, end.ev),
                 "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        if getattr(self, "ev", None):
            self._h.hipEventDestroy(self.ev)
            self.ev = None
