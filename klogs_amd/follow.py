"""Follow mode (`-f`): the filter over log streams that keep growing.

The reference sets `PodLogOptions.Follow` (cmd/root.go:217-218) and `io.Copy`s each
stream until it ends (`streamLog`, cmd/root.go:312-339; the "ended prematurely" warning at
:314-318).  kubelet applies `--since` / `--tail` to the backlog it holds when the request
arrives and then streams every new line (since-filtered; tail no longer applies).  The
client side cannot tell backlog bytes from new ones, so in follow mode the server keeps
`SinceSeconds` / `TailLines` (getLopOpts, :201-221, plus `Timestamps`), and the engine
applies what is per line: the since cutoff (idempotent with the server's) and the grep
set, prefix strip included (SPEC.md S1/S2/S5).

`FollowBatch` is the incremental chunked engine: `feed(stream, chunk)` carries each
stream's open (unterminated) line across chunks; `flush()` runs ONE engine pass over the
complete lines every stream has received since the last flush (one device batch for all
streams: tail -1, per-line rules only), and `flush(final=True)` also closes the streams,
emitting their last unterminated line as kubelet does at end of stream.  Concatenated
flush outputs equal the filter of the whole stream with tail -1 (tests/test_follow.py).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence


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
