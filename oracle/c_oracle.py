"""ctypes wrapper of the C oracle (oracle/klf_oracle_c.c) — TEST INFRASTRUCTURE ONLY
(tests/ and bench.py's cpu_baseline leg)."""
from __future__ import annotations

import ctypes as C
from pathlib import Path
from typing import Sequence, Tuple

import numpy as np

_lib = C.CDLL(str(Path(__file__).resolve().parent / "_build" / "libklf_oracle.so"))


class _Counts(C.Structure):
    _fields_ = [("lines", C.c_uint64), ("parsed", C.c_uint64), ("since_ok", C.c_uint64),
                ("matched", C.c_uint64), ("selected", C.c_uint64), ("out_bytes", C.c_uint64)]


_lib.ko_filter.restype = C.c_int64
_lib.ko_filter.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.c_int32, C.c_int64, C.c_int, C.c_uint32,
                           C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p, C.c_uint64,
                           C.c_void_p, C.POINTER(_Counts)]
_lib.ko_filter_rx.restype = C.c_int64
_lib.ko_filter_rx.argtypes = [C.c_void_p, C.c_uint64, C.c_int64, C.c_int32, C.c_int64, C.c_uint32,
                              C.POINTER(C.c_char_p), C.POINTER(C.c_int32), C.POINTER(C.c_void_p),
                              C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                              C.POINTER(_Counts)]
_lib.ko_parse_ts.restype = C.c_int
_lib.ko_parse_ts.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]

GO_ZERO_TIME = (-62135596800, 0)


def parse_ts(b: bytes):
    s = C.c_int64()
    ns = C.c_int32()
    buf = C.create_string_buffer(b, len(b) or 1)
    return (s.value, ns.value) if _lib.ko_parse_ts(buf, len(b), C.byref(s), C.byref(ns)) else None


def filter_stream(data, since=GO_ZERO_TIME, tail: int = -1, grep: Sequence[bytes] = (),
                  want_lines: bool = True, want_bits: bool = True, grep_active=None):
    """Returns (out bytes, line_off uint64[L+1] or None, match bits or None, counts dict).
    `data` may be bytes or a uint8 numpy array (no copy)."""
    arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.asarray(data)
    n = arr.nbytes
    active = bool(grep) if grep_active is None else grep_active
    keep = [C.create_string_buffer(g, len(g) or 1) for g in grep]
    lits = (C.c_void_p * max(1, len(grep)))(*[C.cast(k, C.c_void_p) for k in keep])
    lens = (C.c_uint64 * max(1, len(grep)))(*[len(g) for g in grep])
    out = np.empty(max(n, 1), dtype=np.uint8)
    cap = n + 2 if want_lines else 0
    lo = np.empty(max(cap, 1), dtype=np.uint64)
    bits = np.zeros(n // 8 + 2, dtype=np.uint8) if (want_bits and active) else None
    c = _Counts()
    m = _lib.ko_filter(arr.ctypes.data if n else None, n, int(since[0]), int(since[1]), int(tail), int(active),
                       len(grep), lits, lens, out.ctypes.data, lo.ctypes.data if want_lines else None, cap,
                       bits.ctypes.data if bits is not None else None, C.byref(c))
    if m < 0:
        raise MemoryError("oracle allocation failed")
    counts = {k: int(getattr(c, k)) for k, _ in _Counts._fields_}
    L = counts["lines"]
    return (out[:m].tobytes(), lo[:L + 1].copy() if want_lines else None,
            bits[:(L + 7) // 8].tobytes() if bits is not None else None, counts)


class RegexSet:
    """A --match set translated once for ko_filter_rx (oracle/posix_re.py): POSIX ERE per
    pattern plus its required literal.  Reusable across calls and threads (each call
    compiles its own regex_t copies)."""

    def __init__(self, match: Sequence[bytes]):
        import posix_re
        tr = [posix_re.translate(m) for m in match]
        self.n = len(tr)
        self.ere = [t[0] for t in tr]
        self.req = [t[1] for t in tr]
        self._ere = (C.c_char_p * max(1, self.n))(*self.ere)
        self._icase = (C.c_int32 * max(1, self.n))(*[int(t[2]) for t in tr])
        self._keep = [C.create_string_buffer(t[1], len(t[1]) or 1) for t in tr]
        self._req = (C.c_void_p * max(1, self.n))(*[C.cast(k, C.c_void_p) for k in self._keep])
        self._req_len = (C.c_uint64 * max(1, self.n))(*[len(t[1]) for t in tr])


def filter_stream_rx(data, since=GO_ZERO_TIME, tail: int = -1, match=(), want_lines: bool = True,
                     want_bits: bool = True):
    """ko_filter_rx (glibc POSIX ERE behind the required-literal pass): the same returns as
    filter_stream.  `match` is a RegexSet or a sequence of Go-subset patterns."""
    rs = match if isinstance(match, RegexSet) else RegexSet(match)
    arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.asarray(data)
    n = arr.nbytes
    out = np.empty(max(n, 1), dtype=np.uint8)
    cap = n + 2 if want_lines else 0
    lo = np.empty(max(cap, 1), dtype=np.uint64)
    bits = np.zeros(n // 8 + 2, dtype=np.uint8) if (want_bits and rs.n) else None
    c = _Counts()
    m = _lib.ko_filter_rx(arr.ctypes.data if n else None, n, int(since[0]), int(since[1]), int(tail), rs.n,
                          rs._ere, rs._icase, rs._req, rs._req_len, out.ctypes.data,
                          lo.ctypes.data if want_lines else None, cap,
                          bits.ctypes.data if bits is not None else None, C.byref(c))
    if m == -1:
        raise MemoryError("oracle allocation failed")
    if m < -1:
        raise ValueError(f"pattern {-2 - m} does not compile as POSIX ERE: {rs.ere[-2 - m]!r}")
    counts = {k: int(getattr(c, k)) for k, _ in _Counts._fields_}
    L = counts["lines"]
    return (out[:m].tobytes(), lo[:L + 1].copy() if want_lines else None,
            bits[:(L + 7) // 8].tobytes() if bits is not None else None, counts)
