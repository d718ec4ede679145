"""The one-pass compaction (klf_result_compaction "one_pass": no patterns, --tail -1; the
scan compacts each wave's tile range in place, k_fcarry fills the bytes a range's first
line start leaves to the line carried into it) against the C oracle, through the C ABI.
KLF_DEBUG_FUSE_RANGE shortens the ranges to a few tiles so that every seam case occurs:
lines straddling range seams, a prefix cut by a seam, lines longer than whole ranges (a
chain of ranges without a line start), ranges covering several streams, since cutoffs and
unparseable lines at seams."""
import random

import numpy as np
import pytest

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu

TS = b"2024-10-22T00:%02d:%02d.%09dZ "


def _line(i, n, bad=False):
    body = (b"x%d-" % i + bytes(random.Random(i).choices(b"abcdefghij ", k=max(0, n))))[:max(0, n)]
    if bad:
        return b"not-a-timestamp " + body + b"\n"
    return TS % ((i // 60) % 60, i % 60, (i * 7919) % 10**9) + body + b"\n"


def _run(streams, since=None, **kw):
    with E.Engine(0) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                eng.stage(i, s)
        r = eng.run(since=since, tail=-1, n_streams=len(streams), **kw)
        res = dict(mode=r.compaction(), index=r.index_mode(),
                   outs=[r.stream(i).out for i in range(len(streams))],
                   counts=[r.stream(i).counts for i in range(len(streams))],
                   lines=[r.lines(i) for i in range(len(streams))])
        r.free()
        return res


def check(streams, since=None, want_mode="one_pass"):
    got = _run(streams, since)
    assert got["mode"] in want_mode.split("|"), got["mode"]
    for i, s in enumerate(streams):
        out, lo, _, c = co.filter_stream(s, since or co.GO_ZERO_TIME, -1, [])
        assert got["outs"][i] == out, f"stream {i}: out differs ({len(got['outs'][i])} vs {len(out)})"
        assert np.array_equal(got["lines"][i], lo), f"stream {i}: line offsets differ"
        for k in ("lines", "parsed", "since_ok", "selected", "out_bytes"):
            assert got["counts"][i][k] == c[k], (i, k, got["counts"][i], c)
    return got


@pytest.mark.parametrize("rng_tiles", ["", "8", "16"])
def test_text_streams(gpu, monkeypatch, rng_tiles):
    if rng_tiles:
        monkeypatch.setenv("KLF_DEBUG_FUSE_RANGE", rng_tiles)
    streams = [synth.generate(synth.TEXT, 31, i, 300_000 + 77_777 * i) for i in range(5)]
    g = check(streams)
    assert g["index"] == "on_demand"
    check(streams, since=(synth.T0 + 1800, 0))


def test_seams_long_lines_and_prefix_cuts(gpu, monkeypatch):
    """8-tile ranges (64 KiB): lines of up to 300 KiB span whole ranges (chains of ranges
    without a line start), and short lines put line starts, prefixes and unparseable lines
    at every offset of the range seams."""
    monkeypatch.setenv("KLF_DEBUG_FUSE_RANGE", "8")
    rnd = random.Random(5)
    parts, n, i = [], 0, 0
    while n < 1_500_000:
        k = rnd.random()
        ln = _line(i, rnd.randint(200_000, 300_000)) if k < 0.01 else _line(i, rnd.randint(0, 90), bad=k > 0.97)
        parts.append(ln)
        n += len(ln)
        i += 1
    d = b"".join(parts)
    check([d])
    check([d, d[:700_001], b"", d[5:65_536 * 3 + 17]])
    check([d], since=(synth.T0 + 1200, 0))


def test_prefix_across_every_seam_offset(gpu, monkeypatch):
    """A line start placed 0..40 bytes before a range seam (its 31-B prefix cut there) and
    right after it, for each offset."""
    monkeypatch.setenv("KLF_DEBUG_FUSE_RANGE", "8")
    seam = 8 * 8192
    for off in list(range(0, 41)) + [8191, 8192, 8193]:
        pre = seam - off
        head = b"2024-10-22T00:00:00.000000000Z " + b"h" * (pre - 32) + b"\n"  # ends at pre
        assert len(head) == pre
        tail_lines = b"".join(_line(j, 50) for j in range(2000))
        check([head + tail_lines])


def test_many_small_streams_in_one_range(gpu):
    streams = [synth.generate(synth.TEXT, 32, i, 1 + (i * 977) % 20_000) for i in range(300)]
    streams[7] = b""
    streams[8] = b"no newline"
    streams[9] = b"\n\n\n"
    check(streams)


def test_write_and_device_views(gpu, tmp_path):
    streams = [synth.generate(synth.TEXT, 33, i, 2_000_000) for i in range(6)]
    with E.Engine(0) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            eng.stage(i, s)
        r = eng.run(tail=-1, n_streams=len(streams))
        assert r.compaction() == "one_pass"
        paths = [str(tmp_path / f"s{i}.log") for i in range(len(streams))]
        n = r.write_files(paths)  # straight from the extents (no host view yet)
        want = [co.filter_stream(s, co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)[0] for s in streams]
        assert n == sum(len(w) for w in want)
        for p, w in zip(paths, want):
            assert open(p, "rb").read() == w
        import ctypes as C
        hip = C.CDLL("libamdhip64.so.7")  # (the runtime libklf.so and torch share)
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        for i, w in enumerate(want):  # the contiguous device copy
            p, off, ln = r.device_out(i)
            assert ln == len(w)
            buf = C.create_string_buffer(max(ln, 1))
            if ln:
                assert hip.hipMemcpy(buf, C.c_void_p(p + off), ln, 2) == 0  # hipMemcpyDeviceToHost
            assert buf.raw[:ln] == w
        assert [r.stream(i).out for i in range(len(streams))] == want
        r.free()


def test_general_prefixes_decided_in_the_scan(gpu):
    """Non-canonical prefixes (offsets, 1-9 fraction digits, ',' fractions) and unparseable
    lines go through Go's time.Parse restated inside the one-pass scan."""
    odd = b"".join(b"2024-10-22T00:00:%02d.5+01:00 off by an hour %d\n" % (i % 60, i) for i in range(3000))
    frac = b"".join(b"2024-10-22T00:%02d:00%s-00:30 f %d\n" % (i % 60, [b"", b".1", b",123456789", b".0000000001"][i % 4], i)
                    for i in range(3000))
    bad = b"".join(b"garbage line %d\n" % i if i % 5 == 0 else b"2024-10-22T00:01:00.000000000Z ok %d\n" % i
                   for i in range(3000))
    check([synth.generate(synth.TEXT, 34, 0, 200_000), odd, frac, bad])
    check([odd, frac, bad], since=(synth.T0 - 3600 + 1, 0))


def test_dense_tiles_rerun_two_pass(gpu):
    """A tile with more line starts than its slots (lines < 32 B) voids the one pass: the
    run redoes the two-pass compaction, equal to the oracle."""
    dense = b"".join(b"\n" if i % 3 else b"2024-10-22T00:00:00Z x\n" for i in range(30000))
    check([dense], want_mode="tiles|gather")
    check([synth.generate(synth.TEXT, 34, 1, 200_000)])


def test_extent_table_follows_the_layout(gpu, monkeypatch):
    """One engine: a one-pass run on layout A, a --tail run on layout B (the same tile count,
    other stream boundaries: more streams per range), then a one-pass run on B.  The third
    run must rebuild the per-range extent table for B (the advisor's round-5 finding: it was
    keyed on the last run's layout, which the --tail run had moved to B, so A's extent counts
    were reused: writes past a range's extents and streams' bytes swapped)."""
    monkeypatch.setenv("KLF_DEBUG_FUSE_RANGE", "8")
    b = [synth.generate(synth.TEXT, 36, 1 + i, n) for i, n in enumerate((300_000, 300_000, 400_000))]
    ntiles = lambda ss: sum((len(s) + 8191) // 8192 for s in ss)  # noqa: E731
    nt = ntiles(b)
    big = synth.generate(synth.TEXT, 36, 0, nt * 8192 + 100_000)
    a = [big[:big.rindex(b"\n", 0, nt * 8192) + 1]]  # whole lines, the same tile count as b
    assert ntiles(a) == nt
    with E.Engine(0) as eng:
        for streams, tail in ((a, -1), (b, 5), (b, -1), (a, -1)):
            eng.reset()
            eng.set_streams(len(streams))
            for i, s in enumerate(streams):
                eng.stage(i, s)
            r = eng.run(tail=tail, n_streams=len(streams))
            if tail < 0:
                assert r.compaction() == "one_pass"
            for i, s in enumerate(streams):
                want = co.filter_stream(s, co.GO_ZERO_TIME, tail, [], want_lines=False, want_bits=False)[0]
                assert r.stream(i).out == want, (tail, i)
            r.free()


def test_disabled_by_env(gpu, monkeypatch):
    monkeypatch.setenv("KLF_FUSE", "0")
    check([synth.generate(synth.TEXT, 35, 0, 500_000)], want_mode="tiles|gather")
