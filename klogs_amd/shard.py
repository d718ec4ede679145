"""Multi-GPU stream sharding: one process per GPU, streams never split.

The reference fans out one goroutine per (pod, container) stream (cmd/root.go:248-249,
260-261) and every stream is filtered independently (since / tail are per stream,
kubelet logs.go).  Here the streams of the stream table (getPodLogs order,
cmd/root.go:224-277) are assigned to ranks by size-balanced greedy (LPT), each rank runs
the whole filter path on its own device batch, and the only collective is one
all-gather of fixed-size per-stream count records (RCCL over xGMI on the GPU box, gloo
in the CPU tests).  Output bytes never cross GPUs: each rank writes its own streams'
files.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence

import numpy as np

# record layout of the gathered per-stream counts (int64 each)
RECORD_FIELDS = ("stream_id", "lines", "parsed", "since_ok", "matched", "selected", "out_bytes")
NREC = len(RECORD_FIELDS)


def assign(lens: Sequence[int], world: int) -> List[int]:
    """Rank of every stream: longest processing time first (ties by stream-table index),
    each onto the least-loaded rank (ties to the lowest rank).  Deterministic, so every
    rank computes the same table without communicating."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(lens)), key=lambda i: (-int(lens[i]), i))
    load = [0] * world
    owner = [0] * len(lens)
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += int(lens[i])
    return owner


def local_streams(lens: Sequence[int], world: int, rank: int) -> List[int]:
    """Stream ids owned by `rank`, in stream-table order (the order of the rank's batch)."""
    own = assign(lens, world)
    return [i for i, r in enumerate(own) if r == rank]


def pack_records(counts: Dict[int, dict], cap: int, n_patterns: int = 0) -> np.ndarray:
    """Fixed-size [cap, NREC + n_patterns] int64 block of this rank's records (stream_id -1
    = padding).  With n_patterns > 0 every counts dict also holds "patterns": the lines of
    the stream each --grep/--match pattern matches (klf_result_pattern_counts)."""
    rec = np.zeros((cap, NREC + n_patterns), dtype=np.int64)
    rec[:, 0] = -1
    for j, (sid, c) in enumerate(sorted(counts.items())):
        rec[j, 0] = sid
        for k, f in enumerate(RECORD_FIELDS[1:], start=1):
            rec[j, k] = int(c[f])
        if n_patterns:
            rec[j, NREC:] = np.asarray(c["patterns"], dtype=np.int64)
    return rec


def unpack_records(blocks: np.ndarray, n_streams: int, n_patterns: int = 0) -> np.ndarray:
    """[world * cap, NREC + n_patterns] gathered blocks -> dense [n_streams, NREC - 1 +
    n_patterns] count table."""
    w = NREC + n_patterns
    out = np.zeros((n_streams, w - 1), dtype=np.int64)
    seen = np.zeros(n_streams, dtype=bool)
    for row in blocks.reshape(-1, w):
        sid = int(row[0])
        if sid < 0:
            continue
        if seen[sid]:
            raise RuntimeError(f"stream {sid} reported by two ranks")
        seen[sid] = True
        out[sid] = row[1:]
    if not seen.all():
        raise RuntimeError(f"streams {np.flatnonzero(~seen).tolist()} reported by no rank")
    return out


def gather_counts(counts: Dict[int, dict], lens: Sequence[int], world: int, device=None,
                  allgather=None, n_patterns: int = 0) -> np.ndarray:
    """All-gathers every rank's per-stream records (one collective) -> [n_streams, 6 +
    n_patterns].  allgather(block [cap, width] int64) -> [world * cap, width] replaces the
    collective (the in-process simulations of several ranks)."""
    cap = max(len(local_streams(lens, world, r)) for r in range(world)) or 1
    if allgather is not None:
        return unpack_records(np.asarray(allgather(pack_records(counts, cap, n_patterns))), len(lens), n_patterns)
    import torch
    import torch.distributed as dist

    rec = torch.from_numpy(pack_records(counts, cap, n_patterns))
    if device is not None:
        rec = rec.to(device)
    if world > 1:
        out = torch.empty(world * cap, NREC + n_patterns, dtype=torch.int64, device=rec.device)
        dist.all_gather_into_tensor(out, rec)
    else:
        out = rec
    return unpack_records(out.cpu().numpy(), len(lens), n_patterns)


class PendingGather:
    """An all-gather of count records in flight (gather_counts_async); wait() -> table."""

    def __init__(self, work, out, n_streams: int, n_patterns: int, table=None):
        self._work, self._out, self._n, self._np, self._table = work, out, n_streams, n_patterns, table

    def wait(self) -> np.ndarray:
        if self._table is None:
            if self._work is not None:
                self._work.wait()
            self._table = unpack_records(self._out.cpu().numpy(), self._n, self._np)
        return self._table


def gather_counts_async(counts: Dict[int, dict], lens: Sequence[int], world: int, device=None,
                        n_patterns: int = 0) -> PendingGather:
    """gather_counts with the collective left in flight (async_op): the caller overlaps it
    with the next batch's filter and waits later -- the bench's steps at N > 1."""
    cap = max(len(local_streams(lens, world, r)) for r in range(world)) or 1
    rec = pack_records(counts, cap, n_patterns)
    if world == 1:
        return PendingGather(None, None, len(lens), n_patterns, unpack_records(rec, len(lens), n_patterns))
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(rec)
    if device is not None:
        t = t.to(device, non_blocking=True)
    out = torch.empty(world * cap, NREC + n_patterns, dtype=torch.int64, device=t.device)
    work = dist.all_gather_into_tensor(out, t, async_op=True)
    return PendingGather(work, out, len(lens), n_patterns)


def run_shard(lens: Sequence[int], fetch: Callable[[int], bytes], runner, world: int, rank: int,
              device=None, allgather=None, n_patterns: int = 0):
    """Filters this rank's streams and gathers every stream's counts.

    fetch(stream_id) -> the stream's captured bytes; runner(list of bytes) -> list of
    (out bytes, counts dict) in the same order (the engine on a GPU; the CPU tests pass
    a checker).  With n_patterns the counts carry per-pattern line counts ("patterns").
    Returns ({stream_id: out bytes} for the local streams, count table)."""
    mine = local_streams(lens, world, rank)
    res = runner([fetch(i) for i in mine]) if mine else []
    outs = {sid: r[0] for sid, r in zip(mine, res)}
    counts = {sid: r[1] for sid, r in zip(mine, res)}
    return outs, gather_counts(counts, lens, world, device, allgather, n_patterns)


def engine_runner(engine, since=None, tail: int = -1, pattern_counts: bool = False):
    """runner for run_shard over a klogs_amd.engine.Engine (one GPU per process)."""
    def run(streams: List[bytes]):
        engine.reset()
        engine.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                engine.stage(i, s)
        r = engine.run(since=since, tail=tail, n_streams=len(streams), pattern_counts=pattern_counts)
        try:
            out = []
            for i in range(len(streams)):
                so = r.stream(i)
                c = dict(so.counts)
                if pattern_counts:
                    c["patterns"] = r.pattern_counts(i)
                out.append((so.out, c))
            return out
        finally:
            r.free()
    return run


# ---------------------------------------------------------------------------------------
# One huge stream split by byte range (SURVEY.md §8e, C2 at more than one GPU).
#
# Rank r owns the lines whose first byte lies in its byte range; the ranges are cut just
# after a newline, so every shard but the last ends with '\n' and only the last can hold
# the unterminated final fragment (kubelet tail.go: the fragment is emitted, not counted).
# since and grep are per line; --tail is the only cross-shard rule.  Every rank filters its
# shard with the global N (a superset of its share: the global window is a suffix of the
# stream, so a shard's part of it is a suffix of the shard's own last-N window), then ONE
# exchange of each shard's count of newline-terminated G lines (G = matching lines, every
# line without patterns: the set kubelet's tail counts, SPEC.md S3/S4) gives every rank its
# share n_r = clamp(N - sum of later shards' counts, 0, own count).  At most two shards
# re-apply the tail rule (the one the window's first line falls in, and the end shard when
# the fragment must be cut although its own count is below N); they re-run only the tail
# and compaction stages on the line index already in HBM (klf_retail).
# Output bytes never cross GPUs: the stream's file is the shards' outputs in rank order.
# ---------------------------------------------------------------------------------------

def split_bounds(n: int, world: int, find_nl: Callable[[int], int]) -> List[int]:
    """Shard boundaries [b_0 = 0, ..., b_world = n] of an n-byte stream: b_r is just past
    the first '\\n' at or after byte r*n//world - 1 (n when there is none), so a line
    belongs to the shard its first byte is in.  find_nl(pos) -> index of the first '\\n'
    at index >= pos, or -1."""
    if world < 1:
        raise ValueError("world must be >= 1")
    b = [0]
    for r in range(1, world):
        c = r * n // world
        p = find_nl(max(c - 1, 0)) if c > 0 else -1
        cut = n if p < 0 else p + 1
        b.append(max(cut, b[-1]))
    b.append(n)
    return b


def end_shard(bounds: Sequence[int]) -> int:
    """The shard holding the stream's last byte (the last non-empty one; the shards after
    it are empty).  Every other non-empty shard ends with '\n'."""
    w = len(bounds) - 1
    ne = [r for r in range(w) if bounds[r] < bounds[r + 1]]
    return ne[-1] if ne else w - 1


def tail_shares(g_term: Sequence[int], tail: int, last: int = -1, unparsed=None) -> List[int]:
    """Each shard's share of the global --tail N (-1 = all lines: every shard -1).  An
    earlier shard gets N minus the newline-terminated G lines of the shards after it,
    clamped to [0, its own count].  The end shard `last` (default: the final one) holds
    the fragment.  kubelet (SPEC.md S4) reads from G-rank max(0, T - N), counts parsed lines
    only and stops after N of them, so the fragment is emitted iff the window's terminated
    lines hold fewer than N parsed ones: when T < N, or when some terminated line of the
    window is unparseable.  The end shard applies that rule to its own part of the window
    with its share; an unparseable line in an EARLIER shard's part is visible to it only
    through unparsed[r] (rank from the end of shard r's last unparseable terminated line,
    0 = none; klf_result_last_unparsed): when one lies inside shard r's share, the end
    shard gets share N, which keeps all of its terminated lines (its share was its whole
    count anyway) and makes its own rule emit the fragment."""
    w = len(g_term)
    last = w - 1 if last < 0 else last
    if tail < 0:
        return [-1] * w
    total = sum(int(x) for x in g_term)
    out = [0] * w
    later = 0
    for r in reversed(range(w)):
        if r == last:
            out[r] = tail if total < tail else min(tail, int(g_term[r]))
        else:
            out[r] = max(0, min(int(g_term[r]), tail - later))
        later += int(g_term[r])
    if unparsed is not None and any(r != last and 0 < int(unparsed[r]) <= out[r] for r in range(w)):
        out[last] = tail
    return out


COUNT_FIELDS = ("lines", "parsed", "since_ok", "matched", "selected", "out_bytes")


def _allgather_ints(vec: Sequence[int], world: int, device=None) -> np.ndarray:
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(x) for x in vec], dtype=torch.int64)
    if device is not None:
        t = t.to(device)
    if world == 1:
        return t.cpu().numpy().reshape(1, -1)
    out = torch.empty(world * t.numel(), dtype=torch.int64, device=t.device)
    dist.all_gather_into_tensor(out, t)
    return out.cpu().numpy().reshape(world, -1)


def run_split(n: int, find_nl: Callable[[int], int], runner, world: int, rank: int, tail: int,
              allgather=None, device=None):
    """Filters this rank's byte range of one stream; returns (this shard's output bytes,
    whole-stream counts).  runner(lo, hi, tail) -> a shard handle with .out (bytes),
    .counts (dict of COUNT_FIELDS), .g_term (newline-terminated G lines), .u_rank (rank
    from the end of its last unparseable terminated G line, 0 = none) and .retail(n) ->
    handle (the same shard with the tail rule re-applied).
    allgather(list of ints) -> [world, k] array (default: torch.distributed, RCCL on the
    GPU box, gloo in the CPU tests)."""
    ag = allgather or (lambda v: _allgather_ints(v, world, device))
    b = split_bounds(n, world, find_nl)
    h = runner(b[rank], b[rank + 1], tail)
    ex = ag([h.g_term, h.u_rank])                        # the one exchange step
    g_term, u_rank = ex[:, 0], ex[:, 1]
    last = end_shard(b)
    share = tail_shares(g_term, tail, last, u_rank)[rank]
    ran_as = tail if rank == last else min(tail, int(g_term[rank]))  # what the first run selected
    if tail >= 0 and share != ran_as:
        h = h.retail(share)
    counts = ag([int(h.counts[f]) for f in COUNT_FIELDS])  # whole-stream counts (reporting)
    return h.out, {f: int(counts[:, k].sum()) for k, f in enumerate(COUNT_FIELDS)}


class EngineShard:
    """runner handle over klogs_amd.engine.Engine (host-staged shard bytes)."""

    def __init__(self, engine, data: bytes, since, tail: int, has_patterns: bool, result=None):
        self._eng, self._data, self._since, self._pat = engine, data, since, has_patterns
        if result is None:
            engine.reset()
            engine.set_streams(1)
            if data:
                engine.stage(0, data)
            result = engine.run(since=since, tail=tail, n_streams=1)
        self._r = result
        so = result.stream(0)
        self.out, self.counts = so.out, so.counts
        frag = bool(data) and not data.endswith(b"\n")
        frag_in_g = frag and (not has_patterns or self._last_bit())
        self.g_term = int(self.counts["matched"]) - (1 if frag_in_g else 0)
        # with patterns every G line is parsed; without, G is every line
        self.u_rank = 0 if has_patterns else result.last_unparsed(0)

    def _last_bit(self) -> bool:
        lines = int(self.counts["lines"])
        bits = self._r.match_bits(0)
        return lines > 0 and bool((bits[(lines - 1) >> 3] >> ((lines - 1) & 7)) & 1)

    def retail(self, tail: int) -> "EngineShard":
        r = self._r.retail(tail)
        self._r.free()
        return EngineShard(self._eng, self._data, self._since, tail, self._pat, result=r)

    def free(self):
        self._r.free()


def engine_split_runner(engine, data: bytes, since=None, has_patterns: bool = False):
    """runner for run_split: the engine on the shard data[lo:hi] (one GPU per process)."""
    def run(lo: int, hi: int, tail: int):
        return EngineShard(engine, data[lo:hi], since, tail, has_patterns)
    return run
