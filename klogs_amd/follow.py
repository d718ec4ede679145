"""Follow mode (`-f`): the filter over log streams that keep growing.

The reference sets `PodLogOptions.Follow` (cmd/root.go:217-218) and `io.Copy`s each
stream until it ends (`streamLog`, cmd/root.go:312-339; the "ended prematurely" warning at
:314-318).  kubelet applies `--since` / `--tail` to the backlog it holds when the request
arrives and then streams every new line (since-filtered; tail no longer applies).  The
client side cannot tell backlog bytes from new ones, so in follow mode the server keeps
`SinceSeconds` / `TailLines` (getLopOpts, :201-221, plus `Timestamps`), and the engine
applies what is per line: the since cutoff (idempotent with the server's) and the grep
set, prefix strip included (SPEC.md S1/S2/S5).

`Follow` is a thin wrapper over the C ABI's follow session (klf_follow_open / feed /
flush / close, include/klf.h), which carries each stream's open (unterminated) line
across reads and stages complete ones on the engine as they arrive; every flush runs ONE
engine pass over what all streams completed since the previous flush (tail -1, per-line
rules only), and a final flush also emits each stream's last unterminated line, as
kubelet does at end of stream.  Concatenated flush outputs equal the filter of the whole
stream with tail -1 (tests/test_follow.py).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple


class Follow:
    """A follow session on one Engine (klf_follow_*): feed(stream, chunk) from any thread
    (different streams concurrently), flush(final) -> {stream_id: output bytes} for the
    streams that received input since the previous flush."""

    def __init__(self, engine, since: Optional[Tuple[int, int]] = None):
        from . import engine as E
        self._E = E
        self._eng = engine
        f = E._filter(since, -1)
        h = C.c_void_p()
        E._check(E._lib.klf_follow_open(engine._h, C.byref(f), C.byref(h)), engine._h)
        self._h = h

    def feed(self, stream_id: int, chunk: bytes) -> None:
        E = self._E
        buf = C.create_string_buffer(chunk, len(chunk) or 1)
        E._check(E._lib.klf_follow_feed(self._h, stream_id, buf, len(chunk)), self._eng._h)

    def open_bytes(self, stream_id: int) -> int:
        return int(self._E._lib.klf_follow_open_bytes(self._h, stream_id))

    def flush(self, final: bool = False) -> Dict[int, bytes]:
        E = self._E
        r = C.c_void_p()
        E._check(E._lib.klf_follow_flush(self._h, 1 if final else 0, C.byref(r)), self._eng._h)
        res = E.Result(r.value or 0, 0, self._eng)
        try:
            out = {}
            i = 0
            while True:  # the result covers ids [0, max id fed]
                p, n, c = C.c_void_p(), C.c_uint64(), E._Counts()
                rc = E._lib.klf_result_stream(res._p, i, C.byref(p), C.byref(n), C.byref(c))
                if rc == E.KLF_EINVAL:  # past the last stream id of the result
                    break
                E._check(rc, self._eng._h)  # a D2H / HIP failure is an error, not the end
                if c.lines:
                    out[i] = C.string_at(p.value, n.value) if n.value else b""
                i += 1
            return out
        finally:
            res.free()

    def close(self) -> None:
        if self._h:
            self._E._lib.klf_follow_close(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
