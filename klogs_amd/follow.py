"""Follow mode (`-f`): the filter over log streams that keep growing.

The reference sets `PodLogOptions.Follow` (cmd/root.go:217-218) and `io.Copy`s each
stream until it ends (`streamLog`, cmd/root.go:312-339; the "ended prematurely" warning at
:314-318).  kubelet applies `--since` / `--tail` to the backlog it holds when the request
arrives and then streams every new line (since-filtered; tail no longer applies).  The
client side cannot tell backlog bytes from new ones, so in follow mode the server keeps
`SinceSeconds` / `TailLines` (getLopOpts, :201-221, plus `Timestamps`), and the engine
applies what is per line: the since cutoff (idempotent with the server's) and the grep
set, prefix strip included (SPEC.md S1/S2/S5).

`Follow` is the product path: a thin wrapper over the C ABI's follow session
(klf_follow_open / feed / flush / close, include/klf.h), which carries the open lines and
stages complete ones on the engine as they arrive.  `FollowBatch` restates the same
carry rules in Python over any batch runner (the CPU tests drive it with the oracle).

`FollowBatch` is the incremental chunked engine: `feed(stream, chunk)` carries each
stream's open (unterminated) line across chunks; `flush()` runs ONE engine pass over the
complete lines every stream has received since the last flush (one device batch for all
streams: tail -1, per-line rules only), and `flush(final=True)` also closes the streams,
emitting their last unterminated line as kubelet does at end of stream.  Concatenated
flush outputs equal the filter of the whole stream with tail -1 (tests/test_follow.py).
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Dict, List, Optional, Sequence, Tuple


class FollowBatch:
    def __init__(self, runner: Callable[[List[bytes]], List[bytes]]):
        """runner(list of stream bytes) -> list of output bytes, tail -1 and the run's since
        / grep (`engine_runner` over a klogs_amd.engine.Engine; the CPU tests pass the
        oracle)."""
        self._run = runner
        self._carry: Dict[int, bytes] = {}
        self._pending: Dict[int, List[bytes]] = {}

    def feed(self, stream_id: int, chunk: bytes) -> None:
        """Appends bytes read from a stream (any split: partial lines are carried)."""
        if not chunk:
            return
        buf = self._carry.get(stream_id, b"") + chunk
        cut = buf.rfind(b"\n") + 1
        if cut:
            self._pending.setdefault(stream_id, []).append(buf[:cut])
        self._carry[stream_id] = buf[cut:]

    def open_bytes(self, stream_id: int) -> int:
        """Bytes of the stream's open line (received, not yet filtered)."""
        return len(self._carry.get(stream_id, b""))

    def flush(self, final: bool = False) -> Dict[int, bytes]:
        """Filters what is complete (with final=True also the open lines, closing every
        stream) -> {stream_id: output bytes} for the streams that had input."""
        ids = set(self._pending)
        if final:
            ids |= {s for s, c in self._carry.items() if c}
        order = sorted(ids)
        if not order:
            if final:
                self._carry.clear()
            return {}
        data = [b"".join(self._pending.get(s, ())) + (self._carry.get(s, b"") if final else b"") for s in order]
        outs = self._run(data)
        self._pending.clear()
        if final:
            self._carry.clear()
        return dict(zip(order, outs))


def engine_runner(engine, since=None) -> Callable[[Sequence[bytes]], List[bytes]]:
    """FollowBatch runner over a klogs_amd.engine.Engine: one batch run per flush."""
    def run(streams: Sequence[bytes]) -> List[bytes]:
        engine.reset()
        engine.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                engine.stage(i, s)
        r = engine.run(since=since, tail=-1, n_streams=len(streams))
        try:
            return [r.stream(i).out for i in range(len(streams))]
        finally:
            r.free()
    return run


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
                if E._lib.klf_result_stream(res._p, i, C.byref(p), C.byref(n), C.byref(c)):
                    break
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
