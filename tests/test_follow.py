"""Follow mode (klogs_amd/follow.py): chunked feeding with carried partial lines equals
the filter of the whole stream with tail -1 (C oracle on the CPU; the engine on the GPU)."""
import random

import pytest

import c_oracle as co
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


def _drive(runner, streams, seed):
    rng = random.Random(seed)
    fb = follow.FollowBatch(runner)
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
    fb = follow.FollowBatch(_oracle_runner)
    assert fb.flush() == {} and fb.flush(final=True) == {}
    fb.feed(3, b"2024-10-22T00:59:00Z pod a")
    assert fb.open_bytes(3) == len(b"2024-10-22T00:59:00Z pod a") and fb.flush() == {}
    fb.feed(3, b"bc\n2024-10-22T00:59:01Z pod d")
    assert fb.flush() == {3: b"pod abc\n"}
    assert fb.flush(final=True) == {3: b"pod d"}


@pytest.mark.gpu
def test_follow_on_engine(gpu):
    from klogs_amd import engine as E
    streams = _streams()
    with E.Engine(0, grep=GREP) as eng:
        got = _drive(follow.engine_runner(eng, since=SINCE), streams, 11)
    assert got == _oracle_runner(streams)
