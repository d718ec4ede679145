"""ctypes binding of the host mirror of cmd/root.go (``include/klogs_host.h``,
``klogs_amd/_lib/libklogs_host.so``) and the path of the ``klogs-filter`` CLI.

Pure host logic (no GPU): Go ``time.ParseDuration``, ``getLopOpts``, the ``getPodLogs``
stream table, ``createLogFile`` and ``convertBytes``.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path
from typing import List, Optional, Sequence, Tuple

_LIB_DIR = Path(__file__).resolve().parent / "_lib"
CLI = _LIB_DIR / "klogs-filter"

KLH_OK = 0
KLH_EPARSE = -101
KLH_EIO = -102
KLH_EINVAL = -103
GO_ZERO_TIME_SEC = -62135596800


class _Time(C.Structure):
    _fields_ = [("sec", C.c_int64), ("nsec", C.c_int32), ("_reserved", C.c_int32)]


class _Filter(C.Structure):
    _fields_ = [("since", _Time), ("tail", C.c_int64), ("flags", C.c_uint32), ("_reserved", C.c_uint32)]


class _Pod(C.Structure):
    _fields_ = [("name", C.c_char_p), ("n_init", C.c_uint32), ("init", C.POINTER(C.c_char_p)),
                ("n_containers", C.c_uint32), ("containers", C.POINTER(C.c_char_p))]


class _Stream(C.Structure):
    _fields_ = [("pod", C.c_uint32), ("container", C.c_uint32), ("is_init", C.c_uint32), ("_reserved", C.c_uint32)]


_lib = C.CDLL(str(_LIB_DIR / "libklogs_host.so"))
_lib.klh_parse_duration.restype = C.c_int
_lib.klh_parse_duration.argtypes = [C.c_char_p, C.POINTER(C.c_int64), C.c_char_p, C.c_size_t]
_lib.klh_lop_opts.restype = C.c_int
_lib.klh_lop_opts.argtypes = [C.c_char_p, C.c_int64, _Time, C.POINTER(_Filter), C.POINTER(C.c_int), C.c_char_p,
                              C.c_size_t]
_lib.klh_stream_table.restype = C.c_int
_lib.klh_stream_table.argtypes = [C.POINTER(_Pod), C.c_uint32, C.c_int, C.POINTER(_Stream), C.c_uint32,
                                  C.POINTER(C.c_uint32)]
_lib.klh_log_file_name.restype = C.c_size_t
_lib.klh_log_file_name.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]
_lib.klh_create_log_file.restype = C.c_int
_lib.klh_create_log_file.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]
_lib.klh_convert_bytes.restype = C.c_size_t
_lib.klh_convert_bytes.argtypes = [C.c_int64, C.c_int, C.c_char_p, C.c_size_t]
_lib.klh_default_log_path.restype = C.c_size_t
_lib.klh_default_log_path.argtypes = [C.c_int64, C.c_char_p, C.c_size_t]

SYMBOLS = ["klh_parse_duration", "klh_lop_opts", "klh_stream_table", "klh_log_file_name", "klh_create_log_file",
           "klh_convert_bytes", "klh_default_log_path"]


class GoPanic(RuntimeError):
    """The reference panics here (e.g. an unparseable --since, cmd/root.go:207-209)."""


def parse_duration(s: str) -> int:
    ns = C.c_int64()
    err = C.create_string_buffer(256)
    rc = _lib.klh_parse_duration(s.encode(), C.byref(ns), err, 256)
    if rc != KLH_OK:
        raise ValueError(err.value.decode())
    return ns.value


def lop_opts(since: Optional[str], tail: int, now: Tuple[int, int]) -> Tuple[Tuple[int, int], int, bool]:
    """getLopOpts split for the engine: ((since_sec, since_nsec), tail, rejected)."""
    f = _Filter()
    rej = C.c_int()
    err = C.create_string_buffer(256)
    t = _Time(int(now[0]), int(now[1]), 0)
    rc = _lib.klh_lop_opts((since or "").encode(), int(tail), t, C.byref(f), C.byref(rej), err, 256)
    if rc == KLH_EPARSE:
        raise GoPanic(err.value.decode())
    if rc != KLH_OK:
        raise RuntimeError(f"klh_lop_opts: {rc}")
    return (f.since.sec, f.since.nsec), f.tail, bool(rej.value)


def stream_table(pods: Sequence[Tuple[str, Sequence[str], Sequence[str]]], init: bool) -> List[Tuple[int, int, bool]]:
    """pods: (name, init containers, containers).  Returns (pod index, container index, is_init)."""
    keep = []
    arr = (_Pod * max(1, len(pods)))()
    for i, (name, inits, conts) in enumerate(pods):
        ia = (C.c_char_p * max(1, len(inits)))(*[x.encode() for x in inits])
        ca = (C.c_char_p * max(1, len(conts)))(*[x.encode() for x in conts])
        keep += [ia, ca]
        arr[i] = _Pod(name.encode(), len(inits), ia, len(conts), ca)
    n = C.c_uint32()
    _lib.klh_stream_table(arr, len(pods), int(init), None, 0, C.byref(n))
    out = (_Stream * max(1, n.value))()
    _lib.klh_stream_table(arr, len(pods), int(init), out, n.value, C.byref(n))
    return [(out[i].pod, out[i].container, bool(out[i].is_init)) for i in range(n.value)]


def log_file_name(pod: str, container: str) -> str:
    buf = C.create_string_buffer(4096)
    _lib.klh_log_file_name(pod.encode(), container.encode(), buf, 4096)
    return buf.value.decode()


def create_log_file(logpath: str, pod: str, container: str) -> str:
    buf = C.create_string_buffer(8192)
    rc = _lib.klh_create_log_file(logpath.encode(), pod.encode(), container.encode(), buf, 8192)
    if rc != KLH_OK:
        raise OSError(f"klh_create_log_file: {rc}")
    return buf.value.decode()


def convert_bytes(n: int, color: bool = True) -> str:
    buf = C.create_string_buffer(64)
    _lib.klh_convert_bytes(int(n), int(color), buf, 64)
    return buf.value.decode()


def default_log_path(unix_sec: int) -> str:
    buf = C.create_string_buffer(128)
    _lib.klh_default_log_path(int(unix_sec), buf, 128)
    return buf.value.decode()
