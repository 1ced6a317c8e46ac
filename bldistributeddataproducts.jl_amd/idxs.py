"""Julia index tuples for the (channel, IF, time) window.

The reference takes ``idxs::Tuple`` of three Julia indices — ``Colon``,
``UnitRange``/``StepRange`` or ``Integer`` — all 1-based and inclusive
(README.md:163-168, src/gbtworkerfunctions.jl:171-195).  Here:

* ``COLON`` (or ``slice(None)``)  ≙ ``:``
* ``JRange(a, b)``                ≙ ``a:b``
* ``JRange(a, s, b)``             ≙ ``a:s:b``
* a Python ``int`` ``i``          ≙ Julia ``i`` (1-based), made ``i:i`` by
  :func:`sanitizeidxs` exactly like src/gbtworkerfunctions.jl:167-169.
"""
from __future__ import annotations

import numbers
from dataclasses import dataclass

COLON = slice(None)


@dataclass(frozen=True)
class JRange:
    """Julia ``first:step:last`` (1-based, inclusive)."""

    first: int
    step: int
    last: int

    def __init__(self, first, step_or_last, last=None):
        if last is None:
            step, last = 1, step_or_last
        else:
            step = step_or_last
        if int(step) == 0:
            raise ValueError("step cannot be zero")  # Julia ArgumentError
        object.__setattr__(self, "first", int(first))
        object.__setattr__(self, "step", int(step))
        object.__setattr__(self, "last", int(last))

    def __len__(self) -> int:
        n = (self.last - self.first) // self.step + 1
        return max(0, n)

    def __iter__(self):
        return iter(range(self.first, self.first + len(self) * self.step, self.step))

    def __repr__(self) -> str:
        if self.step == 1:
            return f"{self.first}:{self.last}"
        return f"{self.first}:{self.step}:{self.last}"


def is_colon(x) -> bool:
    return isinstance(x, slice) and x == COLON or x is Ellipsis


def sanitizeidxs(idxs: tuple) -> tuple:
    """Integers become length-1 ranges so results stay 3-D
    (src/gbtworkerfunctions.jl:167-169)."""
    return tuple(JRange(i, i) if isinstance(i, numbers.Integral) else i for i in idxs)


def to_window(idxs: tuple, shape) -> list | None:
    """Julia idxs -> the ABI's 9 int64 {start0, count, step} x 3, or None for
    (:,:,:).  Bounds are checked by the library (BoundsError)."""
    if len(idxs) != 3:  # @assert length(idxs) == 3 (:172, :180)
        raise AssertionError("idxs must have exactly three indices")
    idxs = sanitizeidxs(idxs)
    if all(is_colon(i) for i in idxs):
        return None
    win = []
    for ax, (ix, n) in enumerate(zip(idxs, shape)):
        if is_colon(ix):
            win += [0, int(n), 1]
        elif isinstance(ix, JRange):
            win += [ix.first - 1, len(ix), ix.step]
        elif isinstance(ix, range):
            raise TypeError("use JRange(a, b) for Julia a:b (Python range is 0-based)")
        else:
            raise TypeError(f"unsupported index {ix!r} on axis {ax + 1}")
    return win


def window_shape(win, shape) -> tuple:
    if win is None:
        return tuple(int(s) for s in shape)
    return (win[1], win[4], win[7])
