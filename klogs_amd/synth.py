"""Seeded synthetic kubelet log streams (``libklf_synth.so``) — tests / bench input only."""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

TEXT, JSON, ADVERSARIAL, MIXED, LONGJSON = 0, 1, 2, 3, 4
T0 = 1729555200  # 2024-10-22T00:00:00Z (the reference snapshot date)
SPAN = 3600      # each stream spans 60 minutes
NEEDLE = b"ERR_CONN_RESET"

_lib = C.CDLL(str(Path(__file__).resolve().parent / "_lib" / "libklf_synth.so"))
_lib.ks_generate.restype = C.c_uint64
_lib.ks_generate.argtypes = [C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint64, C.c_int64, C.c_int64,
                             C.c_char_p, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_uint64, C.c_int]


_lib.ks_c4_literal.restype = C.c_uint32
_lib.ks_c4_literal.argtypes = [C.c_uint32, C.c_char_p]
_lib.ks_c5_pattern.restype = C.c_uint32
_lib.ks_c5_pattern.argtypes = [C.c_uint32, C.c_int, C.c_char_p, C.c_uint32]


def c4_literals(n: int = 1024):
    """The C4 --grep set: the first n distinct literals of the generator's vocabulary
    (MIXED streams embed literals 0..1023)."""
    out, seen, i = [], set(), 0
    buf = C.create_string_buffer(32)
    while len(out) < n:
        m = _lib.ks_c4_literal(i, buf)  # call first: buf.raw[:f(buf)] would read the stale buffer
        b = buf.raw[:m]
        if b not in seen:
            seen.add(b)
            out.append(b)
        i += 1
    return out


def c5_pattern(r: int, which: int) -> bytes:
    buf = C.create_string_buffer(128)
    m = _lib.ks_c5_pattern(r, which, buf, 128)
    return buf.raw[:m]


def c5_regexes():
    """The C5 --match set: 64 RE2-subset regexes (8 families x 8 variants)."""
    return [c5_pattern(r, 0) for r in range(64)]


def _threads():
    return max(1, min(16, os.cpu_count() or 1))


def size(kind: int, seed: int, stream: int, target: int, needle: bytes = NEEDLE, permille: int = 10,
         drop_final_nl: bool = False, t0: int = T0, span: int = SPAN) -> int:
    return int(_lib.ks_generate(kind, seed, stream, target, t0, span, needle, len(needle), permille,
                                int(drop_final_nl), None, 0, 1))


def generate_into(buf, kind: int, seed: int, stream: int, target: int, needle: bytes = NEEDLE,
                  permille: int = 10, drop_final_nl: bool = False, t0: int = T0, span: int = SPAN,
                  threads: int = 0) -> int:
    """Fills a writable numpy uint8 array (len >= size(...) + 1); returns bytes written."""
    arr = np.asarray(buf)
    assert arr.dtype == np.uint8 and arr.flags["C_CONTIGUOUS"]
    n = _lib.ks_generate(kind, seed, stream, target, t0, span, needle, len(needle), permille,
                         int(drop_final_nl), arr.ctypes.data, arr.nbytes, threads or _threads())
    return int(n)


def generate(kind: int, seed: int, stream: int, target: int, **kw) -> bytes:
    n = size(kind, seed, stream, target, **{k: v for k, v in kw.items() if k != "threads"})
    buf = np.empty(n + 1, dtype=np.uint8)  # +1: the dropped final '\n' is written first
    m = generate_into(buf, kind, seed, stream, target, **kw)
    assert m == n, (m, n)
    return buf[:n].tobytes()
