"""Stream sharding across ranks (klogs_amd/shard.py): LPT table and the count gather,
over a world_size-2 gloo group on the CPU (the GPU box runs the same code over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import c_oracle as co
from klogs_amd import shard, synth

SINCE = (synth.T0 + 1800, 0)
TAIL = 25


def test_assign_is_balanced_and_deterministic():
    lens = [64, 1, 1, 1, 32, 32, 0, 16, 16, 16, 16]
    own = shard.assign(lens, 2)
    assert own == shard.assign(lens, 2)
    load = [sum(l for l, r in zip(lens, own) if r == k) for k in range(2)]
    assert abs(load[0] - load[1]) <= 1
    # every stream (empty ones included) has exactly one owner
    assert sorted(i for k in range(2) for i in shard.local_streams(lens, 2, k)) == list(range(len(lens)))
    assert shard.assign(lens, 1) == [0] * len(lens)
    with pytest.raises(ValueError):
        shard.assign(lens, 0)


def test_lpt_equal_streams_round_robin():
    # 1,024 equal streams over 8 ranks (BASELINE config 3): 128 each, table order kept per rank
    own = shard.assign([64 << 20] * 1024, 8)
    for r in range(8):
        mine = shard.local_streams([64 << 20] * 1024, 8, r)
        assert len(mine) == 128 and mine == sorted(mine)
    assert own[:8] == list(range(8))


def test_records_roundtrip_and_duplicates():
    counts = {3: dict(lines=5, parsed=4, since_ok=3, matched=2, selected=1, out_bytes=9),
              0: dict(lines=1, parsed=1, since_ok=1, matched=1, selected=1, out_bytes=2)}
    rec = shard.pack_records(counts, 3)
    assert rec.shape == (3, shard.NREC) and rec[2, 0] == -1
    other = shard.pack_records({1: counts[0], 2: counts[3]}, 3)
    table = shard.unpack_records(np.concatenate([rec, other]), 4)
    assert table[3].tolist() == [5, 4, 3, 2, 1, 9]
    with pytest.raises(RuntimeError):
        shard.unpack_records(np.concatenate([rec, rec]), 4)
    with pytest.raises(RuntimeError):
        shard.unpack_records(rec, 4)


def _streams():
    return [synth.generate(synth.TEXT, 31, i, 20_000 + 9_000 * (i % 5)) if i % 7 else b"" for i in range(13)]


def _oracle_runner(streams):
    res = []
    for s in streams:
        out, _, _, c = co.filter_stream(s, SINCE, TAIL, [b"pod"], want_lines=False, want_bits=False)
        res.append((out, c))
    return res


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        streams = _streams()
        lens = [len(s) for s in streams]
        outs, table = shard.run_shard(lens, lambda i: streams[i], _oracle_runner, world, rank)
        q.put((rank, {k: v for k, v in outs.items()}, table))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_gather_matches_serial():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    streams = _streams()
    serial = _oracle_runner(streams)
    tables = [t for _, _, t in got]
    assert np.array_equal(tables[0], tables[1])
    outs = {}
    for _, o, _ in got:
        assert not (set(o) & set(outs)), "a stream was filtered on two ranks"
        outs.update(o)
    assert sorted(outs) == list(range(len(streams)))
    for i, (out, c) in enumerate(serial):
        assert outs[i] == out
        assert tables[0][i].tolist() == [c[k] for k in shard.RECORD_FIELDS[1:]]
