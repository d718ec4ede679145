"""The fused compaction (k_scan<plain, fused>: --tail -1 without patterns, the copy done by
the scan through a look-back over workgroup turns; opt-in with KLF_FUSE=1, which every test
here sets) against the C oracle and against the two-pass compaction (the default) on the
same batches: tiles whose carried-in line starts
many tiles back, prefixes that straddle tile boundaries, non-canonical timestamps parsed in
the scan, unparseable lines, dense tiles, fragments, streams shorter than a turn, and the
since cutoff.  Anchor: the per-stream output of writeLogToDisk (cmd/root.go:359-374) under
kubelet's rules with no --tail (SPEC.md S3/S4)."""
import random

import numpy as np
import pytest

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def fused_on(monkeypatch):
    monkeypatch.setenv("KLF_FUSE", "1")


def run(streams, since=None, tail=-1):
    with E.Engine(0) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                eng.stage(i, s)
        r = eng.run(since=since, tail=tail, n_streams=len(streams))
        out = [(r.stream(i).out, r.stream(i).counts) for i in range(len(streams))]
        r.free()
    return out


def check(streams, since=None, monkeypatch=None):
    got = run(streams, since)
    for i, s in enumerate(streams):
        out, _, _, c = co.filter_stream(s, since or co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)
        assert got[i][0] == out, f"stream {i}: output differs ({len(got[i][0])} vs {len(out)})"
        for k in ("lines", "parsed", "since_ok", "selected", "out_bytes"):
            assert got[i][1][k] == c[k], (i, k, got[i][1], c)
    if monkeypatch is not None:  # the two-pass compaction agrees
        monkeypatch.setenv("KLF_FUSE", "0")
        two = run(streams, since)
        monkeypatch.setenv("KLF_FUSE", "1")
        for i in range(len(streams)):
            if two[i][1] != got[i][1]:
                raise AssertionError(f"stream {i}: counts fused {got[i][1]} two-pass {two[i][1]}")
            if two[i][0] != got[i][0]:
                a, b = two[i][0], got[i][0]
                k = next((j for j in range(min(len(a), len(b))) if a[j] != b[j]), min(len(a), len(b)))
                raise AssertionError(f"stream {i}: output fused {len(b)} B two-pass {len(a)} B, first diff at {k}: "
                                     f"{b[max(0, k - 20):k + 20]!r} vs {a[max(0, k - 20):k + 20]!r}")
    return got


def test_c3_shape(gpu, monkeypatch):
    """C3's shape at test size: TEXT streams of 2-3 MiB, every line out."""
    check([synth.generate(synth.TEXT, 42, i, 2_000_000 + 77_777 * i) for i in range(6)], monkeypatch=monkeypatch)


@pytest.mark.parametrize("since", [None, (synth.T0 + 1800, 0)])
def test_long_lines_and_since(gpu, monkeypatch, since):
    """1-32 KiB lines: the carried-in line of most tiles started tiles back."""
    check([synth.generate(synth.LONGJSON, 5, i, 3_000_000, permille=20) for i in range(2)], since, monkeypatch)


@pytest.mark.parametrize("seed", range(3))
def test_adversarial(gpu, monkeypatch, seed):
    """Non-canonical timestamps (the general parse inside the scan), unparseable lines,
    CRLF, fragments, mixed with large text streams."""
    streams = [synth.generate(synth.ADVERSARIAL, 70 + seed, 0, 20_000, drop_final_nl=bool(seed & 1), permille=40),
               synth.generate(synth.TEXT, 71 + seed, 0, 500_000),
               synth.generate(synth.ADVERSARIAL, 72 + seed, 1, 3_000, permille=200),
               b"", b"no newline at all", b"\n\n\n", b"2024-10-22T00:00:00Z x"]
    for since in [None, (synth.T0 + 1800, 0), (synth.T0 + 600, 123)]:
        check(streams, since, monkeypatch if since is None else None)


def test_many_tiny_streams(gpu, monkeypatch):
    """Streams of a few hundred bytes to two tiles: turns that hold several streams."""
    rng = random.Random(5)
    streams = [synth.generate(synth.TEXT, 90, i, rng.choice([300, 1000, 5000, 9000, 17000])) for i in range(257)]
    check(streams, monkeypatch=monkeypatch)


def test_prefix_across_tile_boundaries(gpu, monkeypatch):
    """Lines sized so that timestamp prefixes straddle every 8 KiB boundary in turn, and
    lines whose content starts exactly at a boundary."""
    parts = []
    pos = 0
    k = 0
    while pos < 600_000:
        ts = b"2024-10-22T00:%02d:%02d.%09dZ " % (k // 60 % 60, k % 60, k)
        # content length chosen so that the next prefix starts 0..40 bytes before a boundary
        nxt = (pos // 8192 + 1) * 8192 - (k % 41) - pos - len(ts) - 1
        body = b"x" * max(1, nxt if 0 < nxt < 9000 else 37 + k % 300)
        line = ts + body + b"\n"
        parts.append(line)
        pos += len(line)
        k += 1
    d = b"".join(parts)
    check([d, d[:8192 * 7 + 5], d[:8192 * 3 - 31]], monkeypatch=monkeypatch)


def test_dense_tiles(gpu, monkeypatch):
    """Tiles with more line starts than staged slots (lines < 32 B): the pool path."""
    rng = random.Random(7)
    parts = []
    for i in range(60000):
        k = rng.random()
        if k < 0.5:
            parts.append(b"\n")
        elif k < 0.8:
            parts.append(b"x%d\n" % i)
        else:
            parts.append(b"2024-10-22T00:00:%02dZ %s\n" % (i % 60, b"ok"))
    d = b"".join(parts)
    check([d, synth.generate(synth.TEXT, 1, 0, 100_000), d[:70001]], monkeypatch=monkeypatch)


def test_c1_64mib(gpu):
    check([synth.generate(synth.TEXT, 3, 0, 64 << 20)])
