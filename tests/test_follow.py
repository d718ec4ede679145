"""Follow mode (klogs_amd/follow.py; tests/follow_batch.py restates its carry rules): chunked feeding with carried partial lines equals
the filter of the whole stream with tail -1 (C oracle on the CPU; the engine on the GPU)."""
import random

import pytest

import c_oracle as co
from follow_batch import FollowBatch, engine_runner
from klogs_amd import follow, synth

SINCE = (synth.T0 + 1200, 0)
GREP = [b"pod"]


def _streams():
    s = [synth.generate(synth.TEXT, 40 + i, i, 30_000 + 7_000 * i) for i in range(4)]
    s[1] += b"2024-10-22T00:59:59.9Z pod unterminated tail"
    s[2] = b""
    s.append(synth.generate(synth.ADVERSARIAL, 5, 0, 6_000, drop_final_nl=True, permille=40))
    return s


def _oracle_runner(streams):
    return [co.filter_stream(x, SINCE, -1, GREP, want_lines=False, want_bits=False)[0] for x in streams]


def _drive(runner, streams, seed, fb=None):
    rng = random.Random(seed)
    fb = fb or FollowBatch(runner)
    pos = [0] * len(streams)
    got = [b""] * len(streams)
    while any(p < len(s) for p, s in zip(pos, streams)):
        for i, s in enumerate(streams):
            if pos[i] < len(s) and rng.random() < 0.7:
                k = rng.choice([1, 2, 17, 300, 4096, 20_000])
                fb.feed(i, s[pos[i]:pos[i] + k])
                pos[i] += k
        if rng.random() < 0.3:
            for sid, out in fb.flush().items():
                got[sid] += out
    for sid, out in fb.flush(final=True).items():
        got[sid] += out
    return got


@pytest.mark.parametrize("seed", range(6))
def test_follow_equals_whole_stream(seed):
    streams = _streams()
    got = _drive(_oracle_runner, streams, seed)
    want = _oracle_runner(streams)
    assert got == want


def test_follow_carry_and_empty_flush():
    fb = FollowBatch(_oracle_runner)
    assert fb.flush() == {} and fb.flush(final=True) == {}
    fb.feed(3, b"2024-10-22T00:59:00Z pod a")
    assert fb.open_bytes(3) == len(b"2024-10-22T00:59:00Z pod a") and fb.flush() == {}
    fb.feed(3, b"bc\n2024-10-22T00:59:01Z pod d")
    assert fb.flush() == {3: b"pod abc\n"}
    assert fb.flush(final=True) == {3: b"pod d"}


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_follow_on_engine(gpu, seed):
    """The C follow session (klf_follow_open / feed / flush / close) against the oracle."""
    from klogs_amd import engine as E
    streams = _streams()
    with E.Engine(0, grep=GREP) as eng, follow.Follow(eng, since=SINCE) as fw:
        got = _drive(None, streams, seed, fb=fw)
    assert got == _oracle_runner(streams)


@pytest.mark.gpu
def test_follow_on_engine_carry_and_empty_flush(gpu):
    from klogs_amd import engine as E
    with E.Engine(0, grep=GREP) as eng, follow.Follow(eng, since=SINCE) as fw:
        assert fw.flush() == {} and fw.flush(final=True) == {}
        fw.feed(3, b"2024-10-22T00:59:00Z pod a")
        assert fw.open_bytes(3) == len(b"2024-10-22T00:59:00Z pod a") and fw.flush() == {}
        fw.feed(3, b"bc\n2024-10-22T00:59:01Z pod d")
        assert fw.flush() == {3: b"pod abc\n"}
        assert fw.flush(final=True) == {3: b"pod d"}
        fw.feed(0, b"x\n")  # a session continues after a final flush
        assert fw.flush() == {0: b""}


@pytest.mark.gpu
def test_follow_on_engine_concurrent_feeds(gpu):
    """One reader thread per stream (cmd/root.go:249) feeding the same session."""
    import threading
    from klogs_amd import engine as E
    streams = [synth.generate(synth.TEXT, 60 + i, i, 400_000 + 1_000 * i) for i in range(12)]
    with E.Engine(0, grep=GREP) as eng, follow.Follow(eng, since=SINCE) as fw:
        def reader(i):
            rng = random.Random(i)
            s, p = streams[i], 0
            while p < len(s):
                k = rng.choice([5, 999, 65_536, 300_000])
                fw.feed(i, s[p:p + k])
                p += k
        th = [threading.Thread(target=reader, args=(i,)) for i in range(len(streams))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        got = fw.flush(final=True)
    assert sorted(got) == list(range(len(streams)))
    assert [got[i] for i in range(len(streams))] == _oracle_runner(streams)


@pytest.mark.gpu
def test_follow_engine_runner(gpu):
    """FollowBatch over the batch API (engine_runner) agrees too."""
    from klogs_amd import engine as E
    streams = _streams()
    with E.Engine(0, grep=GREP) as eng:
        got = _drive(engine_runner(eng, since=SINCE), streams, 11)
    assert got == _oracle_runner(streams)
