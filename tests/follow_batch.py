"""Test scaffolding for follow mode: a Python restatement of the carry rules of the C
follow session (klf_follow_feed / klf_follow_flush, klogs_amd/csrc/klf_engine.cpp) over
any batch runner.  The CPU tests drive it with the C oracle; the GPU tests compare it,
over the batch API (`engine_runner`), with the C session.  Not part of the product path.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence


class FollowBatch:
    def __init__(self, runner: Callable[[List[bytes]], List[bytes]]):
        """runner(list of stream bytes) -> list of output bytes, tail -1 and the run's since
        / grep (`engine_runner` over a klogs_amd.engine.Engine, or the oracle)."""
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
