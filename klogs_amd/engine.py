"""ctypes binding of the C ABI in ``include/klf.h`` (``klogs_amd/_lib/libklf.so``).

This is the same surface the Go host binds through cgo; Python uses it
for the tests and ``bench.py``.  There is deliberately no fallback: if the native
library is missing, importing this module raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_LIB_DIR = Path(os.environ.get("KLF_LIB_DIR", Path(__file__).resolve().parent / "_lib"))
_LIB_PATH = _LIB_DIR / "libklf.so"

KLF_OK = 0
KLF_EINVAL = -1
KLF_ENOMEM = -2
KLF_EHIP = -3
KLF_EPATTERN = -4
KLF_ETOOBIG = -5
KLF_ESTATE = -6
KLF_EIO = -7
KLF_PAT_LITERAL = 0
KLF_PAT_REGEX = 1
GO_ZERO_TIME = (-62135596800, 0)

MODE_NAMES = {0: "none", 1: "never", 2: "all", 3: "literal1", 4: "general"}


class KlfError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"klf error {code}: {msg}")


class _Time(C.Structure):
    _fields_ = [("sec", C.c_int64), ("nsec", C.c_int32), ("_reserved", C.c_int32)]


class _Pattern(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("len", C.c_uint32), ("kind", C.c_uint32)]


class _Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("n_patterns", C.c_uint32), ("patterns", C.POINTER(_Pattern)),
                ("hip_stream", C.c_void_p), ("staging_hint", C.c_uint64)]


class _Filter(C.Structure):
    _fields_ = [("since", _Time), ("tail", C.c_int64), ("flags", C.c_uint32), ("_reserved", C.c_uint32)]


class _Counts(C.Structure):
    _fields_ = [("lines", C.c_uint64), ("parsed", C.c_uint64), ("since_ok", C.c_uint64),
                ("matched", C.c_uint64), ("selected", C.c_uint64), ("out_bytes", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


# Every symbol include/klf.h and include/klf_debug.h declare, with its ctypes signature
# (checked by the CPU tests).
SIGNATURES = {
    "klf_open": (C.c_int, [C.POINTER(_Config), C.POINTER(C.c_void_p)]),
    "klf_close": (None, [C.c_void_p]),
    "klf_last_error": (C.c_char_p, [C.c_void_p]),
    "klf_strerror": (C.c_char_p, [C.c_int]),
    "klf_stage": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]),
    "klf_set_streams": (C.c_int, [C.c_void_p, C.c_uint32]),
    "klf_reset": (C.c_int, [C.c_void_p]),
    "klf_run": (C.c_int, [C.c_void_p, C.POINTER(_Filter), C.POINTER(C.c_void_p)]),
    "klf_layout": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "klf_run_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_uint64), C.POINTER(_Filter), C.POINTER(C.c_void_p)]),
    "klf_retail": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_void_p)]),
    "klf_result_stream": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64),
                                    C.POINTER(_Counts)]),
    "klf_result_lines": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "klf_result_match_bits": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]),
    "klf_result_pattern_counts": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64), C.c_uint32,
                                            C.POINTER(C.c_uint32)]),
    "klf_result_last_unparsed": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]),
    "klf_result_device_out": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]),
    "klf_result_write": (C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.c_uint32, C.POINTER(C.c_uint64)]),
    "klf_result_timing": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint32)]),
    "klf_result_totals": (C.c_int, [C.c_void_p, C.POINTER(_Counts)]),
    "klf_result_index_mode": (C.c_int, [C.c_void_p]),
    "klf_result_compaction": (C.c_int, [C.c_void_p]),
    "klf_result_free": (None, [C.c_void_p]),
    "klf_follow_open": (C.c_int, [C.c_void_p, C.POINTER(_Filter), C.POINTER(C.c_void_p)]),
    "klf_follow_feed": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_size_t]),
    "klf_follow_flush": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "klf_follow_open_bytes": (C.c_uint64, [C.c_void_p, C.c_uint32]),
    "klf_follow_close": (None, [C.c_void_p]),
    "klf_parse_rfc3339nano": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(_Time)]),
    "klf_debug_compile": (C.c_int, [C.POINTER(_Pattern), C.c_uint32, C.POINTER(C.c_uint32), C.c_char_p,
                                    C.c_size_t]),
    "klf_debug_match": (C.c_int, [C.POINTER(_Pattern), C.c_uint32, C.c_void_p, C.c_size_t,
                                  C.POINTER(C.c_int)]),
    "klf_debug_since_digits": (C.c_int, [C.c_int64, C.c_int32, C.c_void_p]),
    "klf_debug_clock": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32, C.c_void_p]),
    "klf_debug_factors": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_char_p, C.c_size_t,
                                    C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    "klf_debug_prefilter": (C.c_int, [C.POINTER(_Pattern), C.c_uint32, C.c_void_p, C.c_size_t, C.c_uint32,
                                      C.POINTER(C.c_int), C.POINTER(C.c_uint32)]),
    "klf_debug_prefilter_hits": (C.c_int, [C.POINTER(_Pattern), C.c_uint32, C.c_void_p, C.c_size_t, C.c_void_p,
                                           C.c_size_t, C.POINTER(C.c_uint64), C.c_char_p, C.c_size_t]),
}


def _load():
    # One HIP runtime per process: when PyTorch is present its bundled libamdhip64.so.7
    # must be the one libklf.so binds to (same SONAME), so device pointers and streams
    # from torch are valid here.  Loading libklf first would pull /opt/rocm's runtime
    # in beside torch's, and whichever initialises second sees no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not _LIB_PATH.exists():
        raise ImportError(f"{_LIB_PATH} is missing: build it with `python -m klogs_amd._build` "
                          "(the filter has no CPU fallback)")
    lib = C.CDLL(str(_LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = _load()


def lib():
    return _lib


def _check(rc: int, eng=None):
    if rc != KLF_OK:
        msg = _lib.klf_strerror(rc).decode()
        if eng is not None:
            detail = _lib.klf_last_error(eng).decode()
            if detail:
                msg += ": " + detail
        raise KlfError(rc, msg)


def _patterns(grep: Sequence[bytes], match: Sequence[bytes]):
    """The klf_pattern array (16 B each: bytes pointer, len, kind) over ONE buffer holding
    every pattern's bytes, filled with numpy (a 1,024-literal set costs microseconds, not the
    milliseconds of a ctypes object per pattern)."""
    items = [bytes(g) for g in grep] + [bytes(m) for m in match]
    n = len(items)
    lens = np.fromiter((len(b) for b in items), dtype=np.uint64, count=n)
    blob = np.frombuffer(b"".join(items) + b"\0", dtype=np.uint8).copy()  # +1: never a zero-size buffer
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        np.cumsum(lens[:-1], out=offs[1:])
    rec = np.zeros(max(1, n), dtype=np.dtype([("p", "<u8"), ("len", "<u4"), ("kind", "<u4")]))
    rec["p"][:n] = np.uint64(blob.ctypes.data) + offs
    rec["len"][:n] = lens.astype(np.uint32)
    rec["kind"][:len(grep)] = KLF_PAT_LITERAL
    rec["kind"][len(grep):n] = KLF_PAT_REGEX
    arr = (_Pattern * max(1, n)).from_buffer(rec)
    return arr, n, (blob, rec)


KLF_FILTER_STAGE_TIMES = 1
KLF_FILTER_PATTERN_COUNTS = 2
KLF_FILTER_FULL_INDEX = 4
KLF_FILTER_NO_TIMING = 8
INDEX_MODES = {0: "full", 1: "windowed", 2: "on_demand"}  # klf_result_index_mode
COMPACTIONS = {0: "gather", 1: "tiles", 2: "one_pass"}  # klf_result_compaction


def _filter(since: Optional[Tuple[int, int]], tail: int, stage_times: bool = False,
            pattern_counts: bool = False, full_index: bool = False, timing: bool = True) -> _Filter:
    f = _Filter()
    s = GO_ZERO_TIME if since is None else since
    f.since.sec, f.since.nsec = int(s[0]), int(s[1])
    f.tail = int(tail)
    f.flags = ((KLF_FILTER_STAGE_TIMES if stage_times else 0) | (KLF_FILTER_PATTERN_COUNTS if pattern_counts else 0)
               | (KLF_FILTER_FULL_INDEX if full_index else 0) | (0 if timing else KLF_FILTER_NO_TIMING))
    return f


def layout(lens: Sequence[int]) -> Tuple[np.ndarray, int]:
    n = len(lens)
    L = (C.c_uint64 * max(1, n))(*[int(x) for x in lens])
    B = (C.c_uint64 * max(1, n))()
    tot = C.c_uint64()
    _check(_lib.klf_layout(n, L, B, C.byref(tot)))
    return np.array(B[:n], dtype=np.uint64), int(tot.value)


def parse_rfc3339nano(b: bytes) -> Optional[Tuple[int, int]]:
    t = _Time()
    buf = C.create_string_buffer(b, len(b) or 1)
    rc = _lib.klf_parse_rfc3339nano(buf, len(b), C.byref(t))
    return (t.sec, t.nsec) if rc == KLF_OK else None


def debug_compile(grep=(), match=()) -> Tuple[int, str, str]:
    arr, n, keep = _patterns(grep, match)
    mode = C.c_uint32()
    err = C.create_string_buffer(512)
    rc = _lib.klf_debug_compile(arr, n, C.byref(mode), err, 512)
    return rc, MODE_NAMES.get(mode.value, "?"), err.value.decode()


def debug_match(content: bytes, grep=(), match=()) -> bool:
    arr, n, keep = _patterns(grep, match)
    m = C.c_int()
    buf = C.create_string_buffer(content, len(content) or 1)
    _check(_lib.klf_debug_match(arr, n, buf, len(content), C.byref(m)))
    return bool(m.value)


def debug_prefilter(content: bytes, grep=(), match=(), phase: int = 0):
    """(match, {on, q, stride, needles, anchor}) of the prefiltered general matcher on the host
    (anchor: the short needles' anchor byte, None when every needle is probed)."""
    arr, n, keep = _patterns(grep, match)
    m = C.c_int()
    info = (C.c_uint32 * 5)()
    buf = C.create_string_buffer(content, len(content) or 1)
    _check(_lib.klf_debug_prefilter(arr, n, buf, len(content), phase, C.byref(m), info))
    return bool(m.value), dict(on=bool(info[0]), q=info[1], stride=info[2], needles=info[3],
                               anchor=(info[4] & 0xFF) if info[4] else None)


def debug_prefilter_hits(sample: bytes, data: bytes, grep=(), match=()):
    """The prefilter layout chosen on `sample`'s statistics and its work over `data` (host):
    {stride, q, k, anchor, probes, bitmap_hits, anchor_hits, verified, pair_pass, layout}."""
    arr, n, keep = _patterns(grep, match)
    out = (C.c_uint64 * 9)()
    lay = C.create_string_buffer(256)
    sb = C.create_string_buffer(sample, len(sample) or 1)
    db = C.create_string_buffer(data, len(data) or 1)
    _check(_lib.klf_debug_prefilter_hits(arr, n, sb, len(sample), db, len(data), out, lay, 256))
    return dict(stride=out[0], q=out[1], k=out[2], anchor=(out[3] & 0xFF) if out[3] else None, probes=out[4],
                bitmap_hits=out[5], anchor_hits=out[6], verified=out[7], pair_pass=out[8],
                layout=lay.value.decode())


def debug_factors(pattern: bytes, want: int = 0):
    """(factor strings, pre bound or None, loose) of one regex, or None without a factor."""
    buf = C.create_string_buffer(4096)
    n, pre, loose = C.c_uint32(), C.c_uint32(), C.c_uint32()
    p = C.create_string_buffer(pattern, len(pattern) or 1)
    rc = _lib.klf_debug_factors(p, len(pattern), want, buf, 4096, C.byref(n), C.byref(pre), C.byref(loose))
    if rc == KLF_EINVAL:
        return None
    _check(rc)
    alts = buf.raw.split(b"\0")[: n.value]
    return alts, (None if pre.value == 0xFFFFFFFF else pre.value), bool(loose.value)


def debug_since_digits(sec: int, nsec: int = 0):
    """The since cutoff's packed digits as the scan's fast timestamp path compares them
    (six u32, klf_debug_since_digits)."""
    out = (C.c_uint32 * 6)()
    _check(_lib.klf_debug_since_digits(sec, nsec, out))
    return list(out)


def debug_clock(device: int = 0, iters: int = 200_000, reps: int = 20):
    """{median, min, max} MHz that a VALU loop holds on the device (needs a GPU)."""
    out = (C.c_double * 3)()
    _check(_lib.klf_debug_clock(device, iters, reps, out))
    return {"median_mhz": round(out[0], 1), "min_mhz": round(out[1], 1), "max_mhz": round(out[2], 1)}


@dataclass
class StreamOut:
    out: bytes
    counts: dict


class Result:
    def __init__(self, ptr: int, n_streams: int, eng):
        self._p = C.c_void_p(ptr)
        self.n_streams = n_streams
        self._eng = eng

    def stream(self, i: int) -> StreamOut:
        p = C.c_void_p()
        n = C.c_uint64()
        c = _Counts()
        _check(_lib.klf_result_stream(self._p, i, C.byref(p), C.byref(n), C.byref(c)))
        data = C.string_at(p.value, n.value) if n.value else b""
        return StreamOut(data, c.as_dict())

    def lines(self, i: int) -> np.ndarray:
        p = C.c_void_p()
        n = C.c_uint64()
        _check(_lib.klf_result_lines(self._p, i, C.byref(p), C.byref(n)))
        cnt = n.value + 1
        if n.value == 0:
            return np.zeros(1, dtype=np.uint64) if p.value is None else np.frombuffer(
                C.string_at(p.value, 8), dtype=np.uint64).copy()
        return np.frombuffer(C.string_at(p.value, 8 * cnt), dtype=np.uint64).copy()

    def match_bits(self, i: int) -> bytes:
        p = C.c_void_p()
        n = C.c_uint64()
        _check(_lib.klf_result_match_bits(self._p, i, C.byref(p), C.byref(n)))
        return C.string_at(p.value, n.value) if n.value else b""

    def pattern_counts(self, i: int) -> List[int]:
        """klf_result_pattern_counts: matching lines of stream i per pattern (the run needs
        pattern_counts=True)."""
        n = C.c_uint32()
        _check(_lib.klf_result_pattern_counts(self._p, i, None, 0, C.byref(n)), self._eng._h)
        buf = (C.c_uint64 * max(1, n.value))()
        _check(_lib.klf_result_pattern_counts(self._p, i, buf, n.value, C.byref(n)), self._eng._h)
        return [int(x) for x in buf[: n.value]]

    def last_unparsed(self, i: int) -> int:
        """klf_result_last_unparsed: rank from the end (over newline-terminated lines) of the
        stream's last unparseable terminated line, 0 = none."""
        v = C.c_uint64()
        _check(_lib.klf_result_last_unparsed(self._p, i, C.byref(v)))
        return int(v.value)

    def device_out(self, i: int) -> Tuple[int, int, int]:
        p = C.c_void_p()
        off = C.c_uint64()
        n = C.c_uint64()
        _check(_lib.klf_result_device_out(self._p, i, C.byref(p), C.byref(off), C.byref(n)))
        return p.value or 0, off.value, n.value

    def write_fds(self, fds: Sequence[int]) -> int:
        """klf_result_write: append stream i's selected bytes to fds[i] (< 0 skips it);
        returns the bytes written.  writeLogToDisk (cmd/root.go:359-374)."""
        arr = (C.c_int * len(fds))(*[int(f) for f in fds])
        n = C.c_uint64()
        _check(_lib.klf_result_write(self._p, arr, len(fds), C.byref(n)), self._eng._h)
        return n.value

    def write_files(self, paths: Sequence[Optional[str]]) -> int:
        """Create (truncate) paths[i] and write stream i into it (None skips the stream)."""
        fds = []
        try:
            for pth in paths:
                fds.append(-1 if pth is None else os.open(pth, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644))
            return self.write_fds(fds)
        finally:
            for f in fds:
                if f >= 0:
                    os.close(f)

    def timing(self) -> List[float]:
        ms = (C.c_double * 8)()
        k = C.c_uint32()
        _check(_lib.klf_result_timing(self._p, ms, 8, C.byref(k)))
        return list(ms[: k.value])

    def stream_counts(self, i: int) -> dict:
        """The stream's counts alone (klf_result_stream with bytes NULL: no output D2H)."""
        n = C.c_uint64()
        c = _Counts()
        _check(_lib.klf_result_stream(self._p, i, None, C.byref(n), C.byref(c)))
        return c.as_dict()

    def index_mode(self) -> str:
        """klf_result_index_mode: "full" (the run wrote every line's u64 offset), "windowed"
        (the --tail windows' lines only) or "on_demand" (none; klf_result_lines builds it)."""
        m = _lib.klf_result_index_mode(self._p)
        if m < 0:
            _check(m)
        return INDEX_MODES[m]

    def compaction(self) -> str:
        """klf_result_compaction: "gather" (the selected lines gathered), "tiles" (tile copy
        after the scan) or "one_pass" (compacted in the scan, range by range)."""
        m = _lib.klf_result_compaction(self._p)
        if m < 0:
            _check(m)
        return COMPACTIONS[m]

    def totals(self) -> dict:
        c = _Counts()
        _check(_lib.klf_result_totals(self._p, C.byref(c)))
        return c.as_dict()

    def retail(self, tail: int) -> "Result":
        """The same run with --tail N re-applied (klf_retail): counts, tail window and
        compaction only.  This result is stale afterwards (its output buffer is reused)."""
        r = C.c_void_p()
        _check(_lib.klf_retail(self._eng._h, self._p, int(tail), C.byref(r)), self._eng._h)
        return Result(r.value or 0, self.n_streams, self._eng)

    def free(self):
        if self._p:
            _lib.klf_result_free(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """One engine = one GPU (klf_open).  grep: literals (Go bytes.Contains); match: Go
    regexp subset (SPEC.md S5)."""

    def __init__(self, device: int = 0, grep: Iterable[bytes] = (), match: Iterable[bytes] = (),
                 hip_stream: Optional[int] = None):
        arr, n, self._keep = _patterns(list(grep), list(match))
        cfg = _Config()
        cfg.device = device
        cfg.n_patterns = n
        cfg.patterns = arr
        cfg.hip_stream = hip_stream
        h = C.c_void_p()
        rc = _lib.klf_open(C.byref(cfg), C.byref(h))
        self._h = h
        if rc != KLF_OK:
            msg = _lib.klf_strerror(rc).decode()
            if h.value:
                msg += ": " + _lib.klf_last_error(h).decode()
                _lib.klf_close(h)
                self._h = C.c_void_p()
            raise KlfError(rc, msg)

    def set_streams(self, n: int):
        _check(_lib.klf_set_streams(self._h, n), self._h)

    def stage_array(self, stream_id: int, arr: np.ndarray):
        """klf_stage straight from a contiguous uint8 numpy array (no intermediate copy)."""
        a = np.ascontiguousarray(arr, dtype=np.uint8)
        _check(_lib.klf_stage(self._h, stream_id, C.c_void_p(a.ctypes.data if a.size else 0), a.size), self._h)

    def stage(self, stream_id: int, data: bytes):
        buf = C.create_string_buffer(data, len(data) or 1)
        _check(_lib.klf_stage(self._h, stream_id, buf, len(data)), self._h)

    def reset(self):
        _check(_lib.klf_reset(self._h), self._h)

    def run(self, since=None, tail: int = -1, n_streams: Optional[int] = None, stage_times: bool = False,
            pattern_counts: bool = False, full_index: bool = False, timing: bool = True) -> Result:
        f = _filter(since, tail, stage_times, pattern_counts, full_index, timing)
        r = C.c_void_p()
        _check(_lib.klf_run(self._h, C.byref(f), C.byref(r)), self._h)
        return Result(r.value or 0, n_streams if n_streams is not None else 0, self)

    def run_device(self, d_ptr: int, seg_base: Sequence[int], lens: Sequence[int], since=None,
                   tail: int = -1, stage_times: bool = False, pattern_counts: bool = False,
                   full_index: bool = False, timing: bool = True) -> Result:
        n = len(lens)
        B = (C.c_uint64 * max(1, n))(*[int(x) for x in seg_base])
        L = (C.c_uint64 * max(1, n))(*[int(x) for x in lens])
        f = _filter(since, tail, stage_times, pattern_counts, full_index, timing)
        r = C.c_void_p()
        _check(_lib.klf_run_device(self._h, C.c_void_p(d_ptr), n, B, L, C.byref(f), C.byref(r)), self._h)
        return Result(r.value or 0, n, self)

    def close(self):
        if self._h:
            _lib.klf_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
