"""A pre-rendered last line for a process that may die in an optional phase
(native handler: ``csrc/hip/lastline.hip``).

``bench.py`` prints one JSON line after its post-headline collectives A/B,
whose result goes into the line.  :func:`arm` hands the native library a
copy of the line to write to stdout -- with write(2), from the signal
handler -- if SIGSEGV / SIGBUS / SIGABRT / SIGFPE / SIGILL / SIGTERM ends the
process first, and the status to leave with.  A ``SIGNO`` placeholder
(:data:`SIGNO`) in the text receives the signal's number.

Without the library (a CPU build that failed, or no library at all) arming
is a no-op that returns False; nothing else changes.
"""
from __future__ import annotations

import sys

SIGNO = "@@"  # two characters the handler overwrites with the signal number


def _lib():
    from ..ops import _lib

    return _lib.lib() if _lib.has("toa_lastline_arm") else None


def arm(text: str = "", code: int = 0) -> bool:
    """Arm (or re-arm) the handler.  `text` is written as is (add the
    newline); "" only sets the exit status.  Flushes Python's own stdout and
    stderr first, so the native write cannot land inside a buffered line."""
    lib = _lib()
    if lib is None:
        return False
    sys.stdout.flush()
    sys.stderr.flush()
    raw = text.encode()
    at = raw.find(SIGNO.encode())
    return lib.toa_lastline_arm(raw, len(raw), at, int(code)) == 0


def disarm() -> None:
    lib = _lib()
    if lib is not None:
        lib.toa_lastline_disarm()
