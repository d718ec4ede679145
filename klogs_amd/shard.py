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


def pack_records(counts: Dict[int, dict], cap: int) -> np.ndarray:
    """Fixed-size [cap, NREC] int64 block of this rank's records (stream_id -1 = padding)."""
    rec = np.zeros((cap, NREC), dtype=np.int64)
    rec[:, 0] = -1
    for j, (sid, c) in enumerate(sorted(counts.items())):
        rec[j, 0] = sid
        for k, f in enumerate(RECORD_FIELDS[1:], start=1):
            rec[j, k] = int(c[f])
    return rec


def unpack_records(blocks: np.ndarray, n_streams: int) -> np.ndarray:
    """[world * cap, NREC] gathered blocks -> dense [n_streams, NREC - 1] count table."""
    out = np.zeros((n_streams, NREC - 1), dtype=np.int64)
    seen = np.zeros(n_streams, dtype=bool)
    for row in blocks.reshape(-1, NREC):
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


def gather_counts(counts: Dict[int, dict], lens: Sequence[int], world: int, device=None) -> np.ndarray:
    """All-gathers every rank's per-stream records (one collective) -> [n_streams, 6]."""
    import torch
    import torch.distributed as dist

    cap = max(len(local_streams(lens, world, r)) for r in range(world)) or 1
    rec = torch.from_numpy(pack_records(counts, cap))
    if device is not None:
        rec = rec.to(device)
    if world > 1:
        out = torch.empty(world * cap, NREC, dtype=torch.int64, device=rec.device)
        dist.all_gather_into_tensor(out, rec)
    else:
        out = rec
    return unpack_records(out.cpu().numpy(), len(lens))


def run_shard(lens: Sequence[int], fetch: Callable[[int], bytes], runner, world: int, rank: int,
              device=None):
    """Filters this rank's streams and gathers every stream's counts.

    fetch(stream_id) -> the stream's captured bytes; runner(list of bytes) -> list of
    (out bytes, counts dict) in the same order (the engine on a GPU; the CPU tests pass
    a checker).  Returns ({stream_id: out bytes} for the local streams, count table)."""
    mine = local_streams(lens, world, rank)
    res = runner([fetch(i) for i in mine]) if mine else []
    outs = {sid: r[0] for sid, r in zip(mine, res)}
    counts = {sid: r[1] for sid, r in zip(mine, res)}
    return outs, gather_counts(counts, lens, world, device)


def engine_runner(engine, since=None, tail: int = -1):
    """runner for run_shard over a klogs_amd.engine.Engine (one GPU per process)."""
    def run(streams: List[bytes]):
        engine.reset()
        engine.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                engine.stage(i, s)
        r = engine.run(since=since, tail=tail, n_streams=len(streams))
        try:
            out = []
            for i in range(len(streams)):
                so = r.stream(i)
                out.append((so.out, so.counts))
            return out
        finally:
            r.free()
    return run
