"""The host staging path (klf_stage / klf_run, SURVEY.md §8b threading contract and §8f-2
capture) and the run's error paths, on the GPU."""
import random
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + 1500, 0)


def test_16_threads_stage_1024_streams_interleaved(gpu):
    """One goroutine per container stream (cmd/root.go:249, :261): 16 threads stage 1,024
    streams in random pieces and random order, with no klf_set_streams (the table grows
    while other threads copy into their streams), three streams large enough to ship
    several 64 MiB chunks early.  Every stream bit-exact against the C oracle."""
    n = 1024
    big = {5: 150 << 20, 600: 70 << 20, 1023: 129 << 20}
    streams = [synth.generate(synth.TEXT, 17, i, big.get(i, 4000 + 61 * (i % 97))) for i in range(n)]
    owner = [i % 16 for i in range(n)]
    eng = E.Engine(0, grep=[b"pod"])
    errors = []

    def worker(t):
        rng = random.Random(t)
        mine = [i for i in range(n) if owner[i] == t]
        pos = {i: 0 for i in mine}
        try:
            while pos:
                i = rng.choice(list(pos))
                step = rng.choice([1, 100, 4096, 1 << 20, 9_000_001])
                s = streams[i]
                eng.stage_array(i, np.frombuffer(s, dtype=np.uint8)[pos[i]:pos[i] + step])
                pos[i] += step
                if pos[i] >= len(s):
                    del pos[i]
        except Exception as ex:  # surfaced below
            errors.append(ex)
    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    r = eng.run(since=SINCE, tail=200, n_streams=n)
    got = [r.stream(i) for i in range(n)]
    r.free()
    eng.close()

    def check(i):
        out, _, _, c = co.filter_stream(streams[i], SINCE, 200, [b"pod"], want_lines=False, want_bits=False)
        return got[i].out == out and got[i].counts["lines"] == c["lines"] and got[i].counts["matched"] == c["matched"]
    with ThreadPoolExecutor(8) as ex:
        bad = [i for i, ok in enumerate(ex.map(check, range(n))) if not ok]
    assert not bad, bad[:10]


def test_stage_after_run_is_estate(gpu):
    d = synth.generate(synth.TEXT, 3, 0, 50_000)
    with E.Engine(0) as eng:
        eng.stage(0, d)
        r = eng.run(n_streams=1)
        assert r.stream(0).out == co.filter_stream(d, want_lines=False, want_bits=False)[0]
        with pytest.raises(E.KlfError) as ei:
            eng.stage(0, b"more")
        assert ei.value.code == E.KLF_ESTATE
        with pytest.raises(E.KlfError) as ei:
            eng.set_streams(3)
        assert ei.value.code == E.KLF_ESTATE
        r2 = eng.run(n_streams=1)  # a second run over the same staging is fine
        assert r2.stream(0).out == co.filter_stream(d, want_lines=False, want_bits=False)[0]
        r2.free()
        eng.reset()
        eng.stage(0, d[:1000])
        r3 = eng.run(n_streams=1)
        assert r3.stream(0).out == co.filter_stream(d[:1000], want_lines=False, want_bits=False)[0]
        r3.free()
        r.free()


def test_double_overflow_is_an_error(gpu, monkeypatch):
    """The line capacity is estimated, then re-sized exactly once; a second overflow (here
    forced by a clamp on the capacity) must fail the run, never return the aborted run's
    records (advisor r01)."""
    d = synth.generate(synth.TEXT, 4, 0, 400_000)
    monkeypatch.setenv("KLF_DEBUG_CAP_CLAMP", "500")
    with E.Engine(0) as eng:
        eng.stage(0, d)
        with pytest.raises(E.KlfError) as ei:
            eng.run(n_streams=1)
        assert ei.value.code == E.KLF_ENOMEM
        monkeypatch.delenv("KLF_DEBUG_CAP_CLAMP")
        r = eng.run(n_streams=1)  # the engine stays usable
        assert r.stream(0).out == co.filter_stream(d, want_lines=False, want_bits=False)[0]
        r.free()


def test_last_unparsed_matches_host(gpu):
    """klf_result_last_unparsed against a host walk of the same stream."""
    from test_shard import _last_unparsed
    for seed in range(4):
        d = synth.generate(synth.ADVERSARIAL, 90 + seed, 0, 3000, drop_final_nl=bool(seed & 1), permille=40)
        for cut in (len(d), len(d) // 2, 100):
            s = d[:cut]
            with E.Engine(0) as eng:
                eng.stage(0, s)
                r = eng.run(n_streams=1)
                assert r.last_unparsed(0) == _last_unparsed(s), (seed, cut)
                r.free()
    with E.Engine(0) as eng:  # every line parses
        eng.stage(0, synth.generate(synth.TEXT, 1, 0, 20_000))
        r = eng.run(n_streams=1)
        assert r.last_unparsed(0) == 0
        r.free()
