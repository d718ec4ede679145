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
                              C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_void_p, C.c_void_p, C.c_uint64,
                              C.c_void_p, C.POINTER(_Counts)]
_lib.ko_rx_error.restype = C.c_char_p
_lib.ko_rx_error.argtypes = [C.c_char_p, C.c_uint64]
_lib.ko_rx_match.restype = C.c_int
_lib.ko_rx_match.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64]
_lib.ko_rx_literal.restype = C.c_int
_lib.ko_rx_literal.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p]
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


class RegexError(ValueError):
    pass


def rx_error(pat: bytes):
    """None when `pat` is in the SPEC.md S5 subset, else the reason (Go's error text)."""
    e = _lib.ko_rx_error(pat, len(pat))
    return None if e is None else e.decode()


def rx_match(pat: bytes, s: bytes) -> bool:
    """Go regexp.Match(pat, s) restated in C (oracle/klf_oracle_rx.c)."""
    m = _lib.ko_rx_match(pat, len(pat), s, len(s))
    if m < 0:
        raise RegexError(rx_error(pat) or "allocation failed")
    return bool(m)


def rx_literal(pat: bytes) -> bytes:
    """The required literal the C leg's prefilter searches (lower case; b"" = none)."""
    buf = C.create_string_buffer(256)
    m = _lib.ko_rx_literal(pat, len(pat), buf)
    if m < 0:
        raise RegexError(rx_error(pat) or "allocation failed")
    return buf.raw[:m]


class RegexSet:
    """A --match set for ko_filter_rx: the Go-subset pattern bytes, parsed by the C leg
    itself (oracle/klf_oracle_rx.c) on every call.  Reusable across calls and threads."""

    def __init__(self, match: Sequence[bytes]):
        self.pats = [bytes(m) for m in match]
        for k, p in enumerate(self.pats):
            e = rx_error(p)
            if e is not None:
                raise RegexError(f"pattern {k} {p!r}: {e}")
        self.n = len(self.pats)
        self._keep = [C.create_string_buffer(p, len(p) or 1) for p in self.pats]
        self._pats = (C.c_void_p * max(1, self.n))(*[C.cast(k, C.c_void_p) for k in self._keep])
        self._lens = (C.c_uint64 * max(1, self.n))(*[len(p) for p in self.pats])


def filter_stream_rx(data, since=GO_ZERO_TIME, tail: int = -1, match=(), want_lines: bool = True,
                     want_bits: bool = True):
    """ko_filter_rx (the C leg's Go-regexp restatement behind its required-literal pass):
    the same returns as filter_stream.  `match` is a RegexSet or a sequence of patterns."""
    rs = match if isinstance(match, RegexSet) else RegexSet(match)
    arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.asarray(data)
    n = arr.nbytes
    out = np.empty(max(n, 1), dtype=np.uint8)
    cap = n + 2 if want_lines else 0
    lo = np.empty(max(cap, 1), dtype=np.uint64)
    bits = np.zeros(n // 8 + 2, dtype=np.uint8) if (want_bits and rs.n) else None
    c = _Counts()
    m = _lib.ko_filter_rx(arr.ctypes.data if n else None, n, int(since[0]), int(since[1]), int(tail), rs.n,
                          rs._pats, rs._lens, out.ctypes.data, lo.ctypes.data if want_lines else None, cap,
                          bits.ctypes.data if bits is not None else None, C.byref(c))
    if m == -1:
        raise MemoryError("oracle allocation failed")
    if m < -1:
        raise RegexError(f"pattern {-2 - m}: {rx_error(rs.pats[-2 - m])}")
    counts = {k: int(getattr(c, k)) for k, _ in _Counts._fields_}
    L = counts["lines"]
    return (out[:m].tobytes(), lo[:L + 1].copy() if want_lines else None,
            bits[:(L + 7) // 8].tobytes() if bits is not None else None, counts)
