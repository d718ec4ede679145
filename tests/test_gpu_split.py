"""One stream split by byte range across ranks (shard.run_split) and klf_retail, on the GPU.

Each simulated rank has its own Engine (its own HBM workspace, as one process per GPU
would); the exchange is done in-process.  The concatenated shard outputs must equal the
C oracle's single-stream result byte for byte."""
import numpy as np
import pytest

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import shard, synth

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + 1800, 0)


def _split_on_engines(data, world, tail, grep):
    find_nl = lambda p: data.find(b"\n", p)
    engines = [E.Engine(0, grep=grep) for _ in range(world)]
    try:
        b = shard.split_bounds(len(data), world, find_nl)
        hs = [shard.EngineShard(engines[r], data[b[r]:b[r + 1]], SINCE, tail, bool(grep)) for r in range(world)]
        g = np.array([[h.g_term, h.u_rank] for h in hs])
        outs, counts = [], []
        for r in range(world):
            calls = iter([g])

            def ag(vec, _c=calls, _r=r):
                try:
                    return next(_c)
                except StopIteration:  # the reporting gather: this rank's counts only
                    return np.array([vec])
            out, tot = shard.run_split(len(data), find_nl, lambda lo, hi, t, _r=r: hs[_r], world, r, tail,
                                       allgather=ag)
            outs.append(out)
            counts.append(tot)
        return b"".join(outs), counts
    finally:
        for e in engines:
            e.close()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("tail", [-1, 0, 5, 300, 10**9])
@pytest.mark.parametrize("grep", [[], [b"pod"], [synth.NEEDLE]])
@pytest.mark.parametrize("frag", [False, True])
def test_split_equals_single_stream(gpu, world, tail, grep, frag):
    data = synth.generate(synth.TEXT, 91, 2, 400_000)
    if frag:
        data += b"2024-10-22T00:59:59.000000001Z pod tail fragment " + synth.NEEDLE
    want, _, _, wc = co.filter_stream(data, SINCE, tail, grep, want_lines=False, want_bits=False)
    got, counts = _split_on_engines(data, world, tail, grep)
    assert got == want
    assert sum(c["selected"] for c in counts) == wc["selected"]
    assert sum(c["out_bytes"] for c in counts) == wc["out_bytes"]
    assert sum(c["lines"] for c in counts) == wc["lines"]


@pytest.mark.parametrize("grep", [[], [b"pod"]])
def test_retail_equals_fresh_run(gpu, grep):
    data = synth.generate(synth.TEXT, 92, 0, 600_000) + b"2024-10-22T00:59:59Z pod frag"
    with E.Engine(0, grep=grep) as eng:
        eng.set_streams(1)
        eng.stage(0, data)
        r = eng.run(since=SINCE, tail=100, n_streams=1)
        for t in (7, 0, -1, 100, 5000):
            r2 = r.retail(t)
            want, _, _, wc = co.filter_stream(data, SINCE, t, grep, want_lines=False, want_bits=False)
            so = r2.stream(0)
            assert so.out == want, t
            for k in ("lines", "parsed", "since_ok", "selected", "out_bytes"):
                assert so.counts[k] == wc[k], (t, k)
            with pytest.raises(E.KlfError):  # the previous result's workspace was reused
                r.stream(0)
            r.free()
            r = r2
        r.free()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("tail", [1, 3, 8, 13])
@pytest.mark.parametrize("where", ["early", "late", "many"])
def test_split_unparseable_in_window_on_engines(gpu, world, tail, where):
    """An unparseable terminated line in an earlier shard's part of the tail window makes
    kubelet emit the trailing fragment (SPEC.md S4): klf_result_last_unparsed carries it."""
    good = [b"2024-10-22T00:%02d:00.000000000Z line %d\n" % (40 + i // 10, i) for i in range(12)]
    bad = b"garbage-without-a-timestamp\n"
    lines = list(good)
    for p in {"early": (3,), "late": (10,), "many": (2, 6, 11)}[where]:
        lines.insert(p, bad)
    data = b"".join(lines) + b"2024-10-22T00:59:59Z the fragment"
    for grep in ([], [b"line"]):
        want, _, _, _ = co.filter_stream(data, SINCE, tail, grep, want_lines=False, want_bits=False)
        got, _ = _split_on_engines(data, world, tail, grep)
        assert got == want, (grep, got, want)
