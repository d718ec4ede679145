"""Stream sharding with the ENGINE as each rank's filter: a
world-size-2 gloo group of two processes that both drive cuda:0 through the C ABI
(shard.run_shard + shard.engine_runner; the driver's 8-GPU runs use the same code with
RCCL and one GPU per rank), checked against the C oracle (literal) and the Python oracle
(per-pattern counts of a regex set)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import c_oracle as co
from klogs_amd import shard, synth

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + 1800, 0)
TAIL = 25
GREP = [b"pod"]
MATCH = [rb"took \d+ms", rb"(?i)POD-\d"]


def _streams():
    return [synth.generate(synth.TEXT, 41, i, 30_000 + 11_000 * (i % 5)) if i % 6 else b"" for i in range(15)]


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from klogs_amd import engine as E
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        streams = _streams()
        lens = [len(s) for s in streams]
        res = {}
        for name, pats in (("grep", dict(grep=GREP)), ("mixed", dict(grep=GREP, match=MATCH))):
            with E.Engine(0, **pats) as eng:
                npat = len(pats.get("grep", [])) + len(pats.get("match", []))
                run = shard.engine_runner(eng, since=SINCE, tail=TAIL, pattern_counts=True)
                outs, table = shard.run_shard(lens, lambda i: streams[i], run, world, rank, n_patterns=npat)
                res[name] = (outs, table)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_engine_shards_equal_oracles():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    from oracle import klf_oracle as ko
    streams = _streams()
    for name, grep, match in (("grep", GREP, []), ("mixed", GREP, MATCH)):
        t0, t1 = got[0][name][1], got[1][name][1]
        assert np.array_equal(t0, t1), "the two ranks gathered different tables"
        outs = {}
        for r in range(world):
            o = got[r][name][0]
            assert not (set(o) & set(outs)), "a stream was filtered on two ranks"
            outs.update(o)
        assert sorted(outs) == list(range(len(streams)))
        pats = ko.compile_patterns(grep=grep, match=match)
        for i, s in enumerate(streams):
            ref = ko.filter_stream(s, SINCE, TAIL, pats)
            assert outs[i] == ref.out, (name, i)
            row = t0[i].tolist()
            assert row[:6] == [ref.n_lines, ref.n_parsed, ref.n_since, ref.n_matched, ref.n_selected, len(ref.out)]
            assert row[6:] == ko.pattern_counts(s, pats), (name, i)
            if not match:  # the literal path also against the C oracle
                out, _, _, c = co.filter_stream(s, SINCE, TAIL, grep, want_lines=False, want_bits=False)
                assert out == outs[i] and c["matched"] == row[3]
