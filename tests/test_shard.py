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
    # per-pattern columns ride after the fixed fields
    pc = {k: dict(v, patterns=[k, 7]) for k, v in counts.items()}
    rec = shard.pack_records(pc, 2, n_patterns=2)
    assert rec.shape == (2, shard.NREC + 2)
    table = shard.unpack_records(np.concatenate([rec, shard.pack_records({1: pc[0], 2: pc[3]}, 2, 2)]), 4, 2)
    assert table[3].tolist() == [5, 4, 3, 2, 1, 9, 3, 7] and table[1].tolist()[-2:] == [0, 7]


def _streams():
    return [synth.generate(synth.TEXT, 31, i, 20_000 + 9_000 * (i % 5)) if i % 7 else b"" for i in range(13)]


def _oracle_runner(streams):
    from oracle import klf_oracle as ko
    pats = ko.compile_patterns([b"pod"])
    res = []
    for s in streams:
        out, _, _, c = co.filter_stream(s, SINCE, TAIL, [b"pod"], want_lines=False, want_bits=False)
        c = dict(c, patterns=ko.pattern_counts(s, pats))
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
        outs, table = shard.run_shard(lens, lambda i: streams[i], _oracle_runner, world, rank, n_patterns=1)
        # the bench's asynchronous form, two gathers in flight at once, gives the same table
        mine = shard.local_streams(lens, world, rank)
        res = _oracle_runner([streams[i] for i in mine])
        counts = {sid: r[1] for sid, r in zip(mine, res)}
        p1 = shard.gather_counts_async(counts, lens, world, n_patterns=1)
        p2 = shard.gather_counts_async(counts, lens, world, n_patterns=1)
        assert np.array_equal(p1.wait(), table) and np.array_equal(p2.wait(), table)
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
        assert tables[0][i].tolist() == [c[k] for k in shard.RECORD_FIELDS[1:]] + c["patterns"]
        assert c["patterns"][0] == c["matched"]  # one literal: its count is `matched`


# ---- one stream split by byte range (shard.run_split) ---------------------------------

class _OracleShard:
    """run_split handle over the C oracle (the CPU stand-in for one rank's engine)."""

    def __init__(self, data, since, tail, grep):
        self.data, self.since, self.grep = data, since, grep
        self.out, _, bits, self.counts = co.filter_stream(data, since, tail, grep, want_lines=False, want_bits=True)
        frag = bool(data) and not data.endswith(b"\n")
        L = self.counts["lines"]
        in_g = (not grep) or (L > 0 and (bits[(L - 1) >> 3] >> ((L - 1) & 7)) & 1)
        self.g_term = self.counts["matched"] - (1 if frag and in_g else 0)
        self.u_rank = 0 if grep else _last_unparsed(data)

    def retail(self, tail):
        return _OracleShard(self.data, self.since, tail, self.grep)


def _last_unparsed(data):
    """Rank from the end (over newline-terminated lines) of the last unparseable one, 0 = none
    (SPEC.md S2: no space, or a prefix Go time.Parse rejects)."""
    lines = data.split(b"\n")[:-1]  # the terminated lines (the last piece is the fragment or b"")
    for k, ln in enumerate(reversed(lines), start=1):
        sp = ln.find(b" ")
        if sp < 0 or co.parse_ts(ln[:sp]) is None:
            return k
    return 0


def _split_case(data, world, tail, grep):
    """run_split over `world` simulated ranks (all-gather by direct exchange) -> output."""
    find_nl = lambda p: data.find(b"\n", p)
    handles = {}
    stage = {}

    # run every rank's first phase, then the exchange, then the second phase
    b = shard.split_bounds(len(data), world, find_nl)
    for r in range(world):
        handles[r] = _OracleShard(data[b[r]:b[r + 1]], SINCE, tail, grep)
    g = np.array([[handles[r].g_term, handles[r].u_rank] for r in range(world)])
    outs, totals = [], {}
    for r in range(world):
        it = iter([g, np.array([[int(handles[k].counts[f]) for f in shard.COUNT_FIELDS] for k in range(world)])])

        def ag(vec, _it=it, _r=r):
            m = next(_it)
            return m

        runner = lambda lo, hi, t, _r=r: handles[_r]
        out, tot = shard.run_split(len(data), find_nl, runner, world, r, tail, allgather=ag)
        outs.append(out)
        totals = tot
    return b"".join(outs), totals


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("tail", [-1, 0, 1, 7, 40, 10_000])
@pytest.mark.parametrize("grep", [(), (b"pod",)])
@pytest.mark.parametrize("frag", [False, True])
def test_split_stream_equals_unsplit(world, tail, grep, frag):
    data = synth.generate(synth.TEXT, 77, 3, 60_000)
    if frag:
        data = data + b"2024-10-22T00:59:59.000000000Z frag pod no newline"
    want, _, _, wc = co.filter_stream(data, SINCE, tail, list(grep), want_lines=False, want_bits=False)
    got, totals = _split_case(data, world, tail, list(grep))
    # counts that do not depend on the tail rule add up across shards (selected / out_bytes
    # are summed from the shards' own runs before any re-tail in this simulation)
    for f in ("lines", "parsed", "since_ok", "matched"):
        assert totals[f] == wc[f], f
    assert got == want


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("tail", [1, 2, 3, 5, 8, 13])
@pytest.mark.parametrize("where", ["early", "late", "none", "many"])
def test_split_unparseable_in_window_emits_fragment(world, tail, where):
    """kubelet emits the fragment when the tail window holds an unparseable terminated line
    (SPEC.md S4); that line may sit in an earlier shard than the fragment (advisor r01)."""
    good = [b"2024-10-22T00:%02d:00.000000000Z line %d\n" % (40 + i // 10, i) for i in range(12)]
    bad = b"garbage-without-a-timestamp\n"
    lines = list(good)
    if where == "early":
        lines.insert(3, bad)
    elif where == "late":
        lines.insert(10, bad)
    elif where == "many":
        for p in (2, 6, 11):
            lines.insert(p, bad)
    data = b"".join(lines) + b"2024-10-22T00:59:59Z the fragment"
    for grep in ((), (b"line",)):
        want, _, _, _ = co.filter_stream(data, SINCE, tail, list(grep), want_lines=False, want_bits=False)
        got, _ = _split_case(data, world, tail, list(grep))
        assert got == want, (grep, got, want)


def test_tail_shares_unparsed():
    # shard 0's last unparseable line is 2 lines from its end, inside its share of 3
    assert shard.tail_shares([5, 2], 5, unparsed=[2, 0]) == [3, 5]
    # outside its share: no fragment from it
    assert shard.tail_shares([5, 2], 5, unparsed=[4, 0]) == [3, 2]
    # the end shard's own unparseable lines are its own rule's business
    assert shard.tail_shares([5, 2], 5, unparsed=[0, 1]) == [3, 2]


def test_split_bounds_edges():
    data = b"a\nbb\nccc\n" * 3 + b"tail"
    fn = lambda p: data.find(b"\n", p)
    for w in (1, 2, 3, 4, 7, 50):
        b = shard.split_bounds(len(data), w, fn)
        assert b[0] == 0 and b[-1] == len(data) and all(x <= y for x, y in zip(b, b[1:]))
        last = shard.end_shard(b)
        for r in range(w):
            if b[r] < b[r + 1] and r != last:
                assert data[b[r + 1] - 1:b[r + 1]] == b"\n"
    assert shard.split_bounds(0, 3, lambda p: -1) == [0, 0, 0, 0]
    assert shard.tail_shares([5, 5, 5], 7) == [0, 2, 5]
    assert shard.tail_shares([5, 5, 5], 3) == [0, 0, 3]
    assert shard.tail_shares([1, 1, 1], 7) == [1, 1, 7]
    assert shard.tail_shares([5, 5, 5], -1) == [-1, -1, -1]
    assert shard.tail_shares([5, 5, 0], 7, last=1) == [2, 5, 0]


def _split_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = synth.generate(synth.TEXT, 78, 1, 80_000) + b"2024-10-22T00:59:59.5Z pod fragment"
        find_nl = lambda p: data.find(b"\n", p)
        runner = lambda lo, hi, t: _OracleShard(data[lo:hi], SINCE, t, [b"pod"])
        out, tot = shard.run_split(len(data), find_nl, runner, world, rank, 33)
        q.put((rank, out, tot))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_split_stream():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (o, t)) for r, o, t in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = synth.generate(synth.TEXT, 78, 1, 80_000) + b"2024-10-22T00:59:59.5Z pod fragment"
    want, _, _, wc = co.filter_stream(data, SINCE, 33, [b"pod"], want_lines=False, want_bits=False)
    assert got[0][0] + got[1][0] == want
    assert got[0][1] == got[1][1]
    assert got[0][1]["selected"] == wc["selected"] and got[0][1]["out_bytes"] == wc["out_bytes"]
    assert got[0][1]["matched"] == wc["matched"]
