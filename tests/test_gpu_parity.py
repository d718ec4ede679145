"""HIP engine vs the oracles, through the C ABI (libklf.so) on the GPU."""
import random

import numpy as np
import pytest

import c_oracle as co
import klf_oracle as po
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu

GZ = po.GO_ZERO_TIME


def run_engine(streams, since=None, tail=-1, grep=(), match=()):
    with E.Engine(0, grep=grep, match=match) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                eng.stage(i, s)
        r = eng.run(since=since, tail=tail, n_streams=len(streams))
        res = []
        for i in range(len(streams)):
            so = r.stream(i)
            bits = r.match_bits(i) if (grep or match) else None
            res.append((so.out, r.lines(i), bits, so.counts))
        r.free()
        return res


def check_against_c(streams, since, tail, grep):
    got = run_engine(streams, since=since, tail=tail, grep=grep)
    for i, s in enumerate(streams):
        out, lo, bits, c = co.filter_stream(s, since or GZ, tail, list(grep))
        g_out, g_lo, g_bits, g_c = got[i]
        assert g_out == out, f"stream {i}: out differs ({len(g_out)} vs {len(out)})"
        assert np.array_equal(g_lo, lo), f"stream {i}: line offsets differ"
        if grep:
            assert g_bits == bits, f"stream {i}: match bits differ"
        for k in ("lines", "parsed", "since_ok", "selected", "out_bytes"):
            assert g_c[k] == c[k], (i, k, g_c, c)
        if grep:
            assert g_c["matched"] == c["matched"], (i, g_c, c)


@pytest.mark.parametrize("kind", [synth.TEXT, synth.JSON])
@pytest.mark.parametrize("tail", [-1, 0, 1, 100])
def test_single_stream_synthetic(gpu, kind, tail):
    d = synth.generate(kind, 11, 0, 3_000_000)
    check_against_c([d], (synth.T0 + 3300, 0), tail, [])
    check_against_c([d], (synth.T0 + 3300, 0), tail, [synth.NEEDLE])


@pytest.mark.parametrize("seed", range(4))
def test_adversarial(gpu, seed):
    rng = random.Random(seed)
    d = synth.generate(synth.ADVERSARIAL, seed, 0, 4000, drop_final_nl=bool(seed & 1), permille=30)
    for _ in range(6):
        since = rng.choice([None, (synth.T0 + 1800, 0), (synth.T0 + 600, 123)])
        tail = rng.choice([-1, 0, 1, 7, 3999, 10000])
        grep = rng.choice([[], [synth.NEEDLE], [b"ms"], [b"Z "]])
        check_against_c([d], since, tail, grep)


def test_multi_stream_and_empty(gpu):
    streams = [synth.generate(synth.TEXT, 5, i, 50_000 * (i % 4)) for i in range(9)]
    streams.append(b"")
    streams.append(b"no newline at all")
    streams.append(b"\n\n\n")
    streams.append(synth.generate(synth.ADVERSARIAL, 9, 2, 500, drop_final_nl=True))
    for since, tail, grep in [(None, -1, []), ((synth.T0 + 1200, 0), 10, []), (None, 5, [synth.NEEDLE]),
                              (None, 3, [b"pod"])]:
        check_against_c(streams, since, tail, grep)


def test_dense_tiles(gpu):
    """Tiles with more line starts than staged slots (lines < 32 B) take the pool path."""
    import random as _r
    rng = _r.Random(7)
    parts = []
    for i in range(60000):
        k = rng.random()
        if k < 0.5:
            parts.append(b"\n")
        elif k < 0.8:
            parts.append(b"x%d\n" % i)
        else:
            parts.append(b"2024-10-22T00:00:%02dZ %s\n" % (i % 60, b"ERR_CONN_RESET" if i % 7 == 0 else b"ok"))
    d = b"".join(parts)
    for since, tail, grep in [(None, -1, []), ((synth.T0 + 30, 0), 100, []), (None, 50, [synth.NEEDLE]),
                              (None, -1, [synth.NEEDLE])]:
        check_against_c([d, synth.generate(synth.TEXT, 1, 0, 100_000), d[:70001]], since, tail, grep)


def _date_edge_lines(n, seed):
    """Canonical prefixes around every rule of the scan's fast path (digits compared against
    the cutoff's digits; the month's length only for days 29..31): years 1969/1970/2099/2100,
    Feb 29 in leap / non-leap years (2000, 2024, 2023, 2100), day 00 / 31 of 30-day months,
    hour 24, minute / second 60, fraction digits at both ends, and a corrupted byte."""
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        y = rnd.choice([1969, 1970, 1971, 2000, 2023, 2024, 2099, 2100, rnd.randint(1965, 2105)])
        mo = rnd.choice([0, 1, 2, 2, 2, 4, 6, 9, 11, 12, 13, rnd.randint(1, 12)])
        d = rnd.choice([0, 1, 28, 29, 29, 30, 31, 32, rnd.randint(1, 31)])
        h, mi, s = rnd.choice([0, 23, 24, 12]), rnd.choice([0, 59, 60, 30]), rnd.choice([0, 59, 60, 30])
        ns = rnd.choice([0, 999_999_999, rnd.randint(0, 999_999_999)])
        t = b"%04d-%02d-%02dT%02d:%02d:%02d.%09dZ " % (y, mo, d, h, mi, s, ns)
        if rnd.random() < 0.05:
            k = rnd.randrange(31)
            t = t[:k] + bytes([rnd.choice(b"0123456789:-TZ. /a")]) + t[k + 1:]
        out.append(t + b"line %d ERR_CONN_RESET\n" % i if i % 3 == 0 else t + b"line %d\n" % i)
    return b"".join(out)


@pytest.mark.parametrize("grep", [[], [synth.NEEDLE], [b"ERR_CONN"] + [b"lit%03d" % i for i in range(20)]])
def test_fast_timestamp_date_edges(gpu, grep):
    d = _date_edge_lines(40_000, 17)
    cuts = [None, (951_782_400, 0), (951_868_799, 999_999_999), (1_709_164_800, 1),  # 2000-02-29, 2024-02-29
            (-1, 999_999_999), (0, 0), (4_102_444_799, 999_999_999), (4_102_444_800, 0), (1_729_555_200 + 7, 5)]
    for since in cuts:
        for tail in ([-1, 100] if not grep else [-1]):
            check_against_c([d, d[:100_001]], since, tail, grep)


def _golden():
    import json
    from pathlib import Path
    g = Path(__file__).resolve().parent / "golden"
    return g, json.loads((g / "manifest.json").read_text())["cases"]


@pytest.mark.parametrize("idx", range(len(_golden()[1])))
def test_golden_fixtures(gpu, idx):
    g, cases = _golden()
    c = cases[idx]
    data = (g / c["input"]).read_bytes()
    grep = [bytes.fromhex(x) for x in c["grep"]]
    match = [bytes.fromhex(x) for x in c["match"]]
    out, lo, bits, cnt = run_engine([data], since=tuple(c["since"]), tail=c["tail"], grep=grep, match=match)[0]
    assert out == (g / c["expect_out"]).read_bytes(), c["name"]
    assert lo.tolist() == np.load(g / c["expect_lines"]).tolist(), c["name"]
    if c["expect_bits"] is not None:
        assert bits.hex() == c["expect_bits"], c["name"]
    assert [cnt["lines"], cnt["parsed"], cnt["since_ok"], cnt["matched"], cnt["selected"]] == c["expect_counts"]


@pytest.mark.parametrize("since,tail", [((synth.T0 + synth.SPAN + 1 - 300, 0), 100), (None, -1),
                                        ((synth.T0 + 1800, 0), -1)])
def test_c1_64mib(gpu, since, tail):
    """BASELINE config 1 shape (one 64 MiB stream, --since 5m --tail 100) and the
    all-lines case that makes the compaction copy the whole stream."""
    d = synth.generate(synth.TEXT, 3, 0, 64 << 20)
    check_against_c([d], since, tail, [])


def test_many_small_streams_all_selected(gpu):
    """Many streams, every line selected: output ranges of adjacent streams share 16-B
    chunks at every boundary (bytewise edge stores)."""
    streams = [synth.generate(synth.TEXT, 21, i, 1000 + 37 * i) for i in range(300)]
    check_against_c(streams, None, -1, [])
    check_against_c(streams, None, 3, [])


# ---- general pattern sets: fused q-gram prefilter + Glushkov NFA on candidates -----------
def check_against_py(streams, since, tail, grep=(), match=()):
    got = run_engine(streams, since=since, tail=tail, grep=grep, match=match)
    pats = po.compile_patterns(grep, match)
    for i, s in enumerate(streams):
        ref = po.filter_stream(s, since or GZ, tail, pats)
        g_out, g_lo, g_bits, g_c = got[i]
        assert g_out == ref.out, f"stream {i}: out differs ({len(g_out)} vs {len(ref.out)})"
        assert g_lo.tolist() == ref.line_off, f"stream {i}: line offsets differ"
        assert g_bits == ref.match_bits, f"stream {i}: match bits differ"
        assert [g_c[k] for k in ("lines", "parsed", "since_ok", "matched", "selected")] == \
            [ref.n_lines, ref.n_parsed, ref.n_since, ref.n_matched, ref.n_selected], (i, g_c)


@pytest.mark.parametrize("two", [True, False])
@pytest.mark.parametrize("since,tail", [(None, -1), ((synth.T0 + 1800, 0), 50)])
def test_c4_literal_set_mixed_lines(gpu, monkeypatch, since, tail, two):
    """BASELINE config 4 shape at test size: 1,024 literals over mixed-length lines, through
    the two-level probe (exact 2-gram stage, then 4 Bloom bits; the default for such sets)
    and the one-level 3-bit probe (KLF_QF_TWO=0)."""
    if not two:
        monkeypatch.setenv("KLF_QF_TWO", "0")
    lits = synth.c4_literals(1024)
    assert E.debug_prefilter(b"", grep=lits)[1]["on"]
    d = synth.generate(synth.MIXED, 4, 0, 3_000_000, permille=5)
    assert E.debug_prefilter_hits(d[:1 << 20], d[:1 << 16], grep=lits)["k"] == (5 if two else 3)
    check_against_c([d, synth.generate(synth.MIXED, 4, 1, 700_000, permille=50)], since, tail, lits)


def test_two_level_folded(gpu, monkeypatch):
    """The two-level probe of a case-folded set: the pair stage tests the data's raw bytes
    against a bitmap that lists every case variant of the needles' pairs (p with p | 0x2020
    in the folded set).  The C5 regexes (loose factors) and case-insensitive literals whose
    occurrences in the data are re-cased."""
    monkeypatch.setenv("KLF_QF_TWO", "force")
    rx = synth.c5_regexes()
    streams = [synth.generate(synth.LONGJSON, 7, i, 1_000_000, permille=30) for i in range(2)]
    assert E.debug_prefilter_hits(streams[0][:1 << 16], streams[0][:1 << 16], match=rx)["k"] == 5
    check_against_py(streams, None, -1, match=rx)
    lits = [l for l in synth.c4_literals(1024) if len(l) >= 6][:40]
    pats = [b"(?i)" + b"".join(b"\\%c" % c if c in b".^$*+?()[]{}|\\" else b"%c" % c for c in l) for l in lits]
    rng = random.Random(3)
    recase = lambda b: bytes(c ^ 0x20 if (65 <= c <= 90 or 97 <= c <= 122) and rng.random() < 0.5 else c
                             for c in b)
    d = _with_inserts(synth.generate(synth.MIXED, 13, 0, 600_000, permille=5), [recase(l) for l in lits], 5, 40)
    assert E.debug_prefilter_hits(d[:1 << 16], d[:1 << 16], match=pats)["k"] == 5
    check_against_py([d], None, -1, match=pats)
    check_against_py([d], (synth.T0 + 1800, 0), 30, match=pats)


@pytest.mark.parametrize("since,tail", [(None, -1), ((synth.T0 + 1800, 0), 50)])
def test_grid6_needles(gpu, since, tail):
    """Literal sets whose shortest needle is 8-9 bytes: the 3-per-16-B sampling grid
    (stride 6, k_scan<gen, 6>), each needle's window spanning 8 bytes."""
    lits = [l for l in synth.c4_literals(1024) if 8 <= len(l) <= 9][:200]
    d = synth.generate(synth.MIXED, 12, 0, 3_000_000, permille=20)
    assert E.debug_prefilter_hits(d[:1 << 16], d[:1 << 16], grep=lits)["stride"] == 6
    check_against_c([d, synth.generate(synth.MIXED, 12, 1, 700_000, permille=80)], since, tail, lits)


@pytest.mark.parametrize("since,tail", [(None, -1), ((synth.T0 + 1800, 0), 50)])
def test_long_needles_stride8(gpu, since, tail):
    """Literal sets whose shortest needle allows an 8-byte sampling stride (k_scan<gen, 8>)."""
    lits = [l for l in synth.c4_literals(1024) if len(l) >= 12][:300]
    info = E.debug_prefilter(b"", grep=lits)[1]
    assert info["on"] and info["stride"] == 8
    d = synth.generate(synth.MIXED, 9, 0, 3_000_000, permille=20)
    check_against_c([d, synth.generate(synth.MIXED, 9, 1, 700_000, permille=80)], since, tail, lits)


@pytest.mark.parametrize("since,tail", [(None, -1), ((synth.T0 + 1800, 0), 20)])
def test_c5_regex_set_long_json(gpu, since, tail):
    """BASELINE config 5 shape at test size: 64 regexes over 1-32 KiB JSON lines (events
    and near misses that hold the factor but not the match)."""
    rx = synth.c5_regexes()
    assert E.debug_prefilter(b"", match=rx)[1]["on"]
    streams = [synth.generate(synth.LONGJSON, 5, i, 2_000_000, permille=20) for i in range(3)]
    check_against_py(streams, since, tail, match=rx)


def _with_inserts(data: bytes, parts, seed: int, every: int) -> bytes:
    """`data` with one of `parts` inserted after every `every`-th line's timestamp prefix."""
    rng = random.Random(seed)
    lines = data.split(b"\n")
    for i in range(0, len(lines), every):
        ln = lines[i]
        if len(ln) > 31:
            k = rng.randint(31, len(ln))
            lines[i] = ln[:k] + rng.choice(parts) + ln[k:]
    return b"\n".join(lines)


ANC_PARTS = [b"tx-0123abcd-commit5", b"tx-0123abc-commit5", b"-commit", b"tx--commit1", b"user3_id=u12345 login",
             b"a-b", b"K_EY=value", b"k_ey=", b"AB_CD7", b"ab_cd", b"x_y_z", b"deadline exceeded after 3s"]


@pytest.mark.parametrize("which", ["c5", "loose"])
@pytest.mark.parametrize("since,tail", [(None, -1), ((synth.T0 + 1800, 0), 30)])
def test_anchored_short_needles(gpu, monkeypatch, which, since, tail):
    """Short needles anchored on one byte beside stride-8 probes (forced, so that every
    data shape runs it): the C5 set (`-commitN` on '-') and a loose set (anchor '_' tested
    OR 0x20), over JSON / text / adversarial streams with the needles and look-alikes
    inserted, tile-crossing ones included."""
    monkeypatch.setenv("KLF_QF_ANCHOR", "force")
    if which == "c5":
        grep, match = [], synth.c5_regexes()
    else:
        grep, match = [b"longer needle here"], [rb"(?i)k_ey=\w+", rb"(?i)ab_cd\d", rb"(?i)x_y_z", rb"deadline exceeded after \d+s"]
    info = E.debug_prefilter(b"", grep=grep, match=match)[1]
    assert info["stride"] == 8 and info["anchor"] is not None, info
    streams = [_with_inserts(synth.generate(synth.LONGJSON, 7, 0, 1_500_000, permille=20), ANC_PARTS, 1, 3),
               _with_inserts(synth.generate(synth.TEXT, 8, 0, 600_000), ANC_PARTS, 2, 5),
               synth.generate(synth.ADVERSARIAL, 9, 0, 3000, permille=40), b""]
    check_against_py(streams, since, tail, grep, match)


GEN_SETS = [
    ([synth.NEEDLE, b"volume", b"x" * 80], [rb"(?i)took \d+ms", rb"status=(200|5\d\d)"]),
    ([b"pod", b"ready"], []),
    ([], [rb"(?i)ERR_CONN_\w+", rb"user= ?\w+ took"]),
    ([b"ab"], [rb"\d+"]),  # prefilter off: k_match decides every line
    ([b"READY_X"], [rb"a\nb", rb"took \d+ms"]),  # a factor holding "\n" never occurs in content
]


@pytest.mark.parametrize("idx", range(len(GEN_SETS)))
@pytest.mark.parametrize("seed", range(2))
def test_general_sets_adversarial(gpu, idx, seed):
    grep, match = GEN_SETS[idx]
    d = synth.generate(synth.ADVERSARIAL, 50 + seed, 0, 3000, drop_final_nl=bool(seed), permille=40)
    t = synth.generate(synth.TEXT, 60 + seed, 0, 400_000)
    # long literal across tile boundaries
    t = t.replace(b"volume", b"volume" + b"x" * 80, 50)
    for since, tail in [(None, -1), ((synth.T0 + 1800, 0), 7), (None, 0)]:
        check_against_py([d, t, b"", b"2024-10-22T00:00:00Z pod ready\n"], since, tail, grep, match)


def test_general_set_dense_tiles(gpu):
    rng = random.Random(3)
    parts = []
    for i in range(40000):
        k = rng.random()
        if k < 0.4:
            parts.append(b"\n")
        else:
            parts.append(b"2024-10-22T00:00:%02dZ %s\n" % (i % 60, rng.choice([b"ok", b"took 12ms", b"pod x", b"q"])))
    d = b"".join(parts)
    check_against_py([d], None, -1, [b"pod x"], [rb"took \d+ms"])
    check_against_py([d], None, 100, [b"pod x"], [rb"took \d+ms"])


def test_candidate_queue_overflow_falls_back(gpu, monkeypatch):
    """More NFA candidates than the queue holds: k_match decides every line (exact)."""
    monkeypatch.setenv("KLF_CAND_CAP", "16")
    d = synth.generate(synth.LONGJSON, 9, 0, 1_500_000, permille=100)
    check_against_py([d], None, -1, match=synth.c5_regexes()[:16])


def test_hit_list_overflow_falls_back(gpu, monkeypatch):
    """More prefilter bitmap hits than the list holds: k_match decides every line."""
    monkeypatch.setenv("KLF_HITS_CAP", "16")
    d = synth.generate(synth.TEXT, 8, 0, 1_000_000)  # "pod" / "took": tens of hits per tile -> spills
    check_against_c([d], None, 10, [b"pod", b"ready"])
    check_against_py([d], None, -1, grep=[b"ERR_"], match=[rb"(?i)took \d+ms"])


@pytest.mark.parametrize("since,tail", [(None, -1), (None, 100), ((synth.T0 + 3000, 0), -1)])
def test_long_lines_copy_chunks(gpu, since, tail):
    """Selected output of 1-32 KiB lines: one compaction block spans many 64 KiB copy chunks."""
    streams = [synth.generate(synth.LONGJSON, 12, i, 3_000_000 + 777 * i, permille=5) for i in range(3)]
    check_against_c(streams, since, tail, [])


def test_stream_over_4gib_offsets(gpu):
    """one stream longer than 2^32 bytes (u64 line offsets past 4 GiB),
    device-resident, since + tail + one literal: output, counts and every line offset
    against the C oracle."""
    import torch
    target = (4 << 30) + (96 << 20)
    n = synth.size(synth.JSON, 7, 0, target, permille=10)
    assert n > (1 << 32)
    host = np.empty(n + 1, dtype=np.uint8)
    synth.generate_into(host, synth.JSON, 7, 0, target, permille=10)
    host = host[:n]
    base, total = E.layout([n])
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    dev[:n].copy_(torch.from_numpy(host))
    torch.cuda.synchronize()
    since = (synth.T0 + synth.SPAN - 240, 0)
    with E.Engine(0, grep=[synth.NEEDLE]) as eng:
        r = eng.run_device(dev.data_ptr(), base, [n], since=since, tail=1000)
        so = r.stream(0)
        lo = r.lines(0)
        r.free()
    del dev
    want, want_lo, _, wc = co.filter_stream(host, since, 1000, [synth.NEEDLE], want_lines=True, want_bits=False)
    assert so.out == want
    for k in ("lines", "parsed", "since_ok", "matched", "selected", "out_bytes"):
        assert so.counts[k] == wc[k], k
    assert lo.shape == want_lo.shape and int(lo[-1]) == n
    assert np.array_equal(lo, want_lo)
    assert int(np.count_nonzero(lo > (1 << 32))) > 0


def test_staging_across_pinned_chunks(gpu):
    """klf_stage in odd-sized pieces that straddle the 64 MiB pinned staging chunks, two
    streams interleaved, then klf_run: bit-exact with the C oracle."""
    a = synth.generate(synth.JSON, 21, 0, 150 << 20, permille=10)
    b = synth.generate(synth.TEXT, 22, 1, 70 << 20)
    since = (synth.T0 + 3000, 0)
    with E.Engine(0, grep=[synth.NEEDLE]) as eng:
        for rep in range(2):  # the second run reuses the pooled chunks
            eng.reset()
            eng.set_streams(2)
            pa = pb = 0
            step = 7_777_777 + rep
            while pa < len(a) or pb < len(b):
                if pa < len(a):
                    eng.stage_array(0, np.frombuffer(a, dtype=np.uint8)[pa:pa + step])
                    pa += step
                if pb < len(b):
                    eng.stage(1, b[pb:pb + step // 3])
                    pb += step // 3
            r = eng.run(since=since, tail=5000, n_streams=2)
            for i, s in enumerate((a, b)):
                so = r.stream(i)
                want, _, _, wc = co.filter_stream(s, since, 5000, [synth.NEEDLE], want_lines=False, want_bits=False)
                assert so.out == want, (rep, i)
                assert so.counts["lines"] == wc["lines"] and so.counts["selected"] == wc["selected"]
            r.free()


def test_short_lines_regex_set_first_attempt_overflows(gpu):
    """Lines averaging under 32 B overflow the first attempt's line capacity (estimated at
    one line per 32 B).  With a regex set k_verify runs beside k_scatter (side stream), so
    the overflow must be raised before either indexes the match bitmap by line (the r03a
    fault: k_verify wrote bits[] past cap_lines); a fresh engine per case, so every run
    starts from the estimate.  Output equal to the Python oracle."""
    rng = random.Random(17)
    parts = []
    for i in range(60000):
        k = rng.random()
        parts.append(b"\n" if k < 0.55 else b"x\n" if k < 0.7 else
                     b"2024-10-22T00:00:%02dZ %s\n" % (i % 60, rng.choice([b"pod x", b"took 7ms", b"q"])))
    d = b"".join(parts)
    assert len(d) / d.count(b"\n") < 32
    for grep, match in [([b"pod x"], [rb"took \d+ms"]), ([], [rb"took \d+ms", rb"(?i)POD"])]:
        check_against_py([d, d[:9000], b""], None, -1, grep, match)
        check_against_py([d], (synth.T0 + 30, 0), 25, grep, match)


def test_clamped_capacity_with_regex_set_fails_cleanly(gpu, monkeypatch):
    """A line capacity clamped on every attempt (KLF_DEBUG_CAP_CLAMP) with a regex set:
    the run fails with KLF_ENOMEM, nothing past the arrays is touched, and the engine
    stays usable (advisor r02)."""
    d = synth.generate(synth.TEXT, 8, 0, 300_000)
    rx = [rb"pod=\d+", rb"(?i)TIMEOUT \w+", rb"took \d+ms"]
    monkeypatch.setenv("KLF_DEBUG_CAP_CLAMP", "40")
    with E.Engine(0, match=rx) as eng:
        eng.stage(0, d)
        with pytest.raises(E.KlfError) as ei:
            eng.run(n_streams=1)
        assert ei.value.code == E.KLF_ENOMEM
        monkeypatch.delenv("KLF_DEBUG_CAP_CLAMP")
        r = eng.run(n_streams=1)
        ref = po.filter_stream(d, GZ, -1, po.compile_patterns([], rx))
        assert r.stream(0).out == ref.out
        r.free()


@pytest.mark.parametrize("win", ["1", "0"])
def test_windowed_line_index(gpu, monkeypatch, win):
    """Literal patterns (a set without regexes, or one literal) build the global line index
    after the tail rule, for the tail windows' lines only (k_scatter mode 2; tiles with deferred lines before the counts,
    mode 1).  Against the C oracle with KLF_WIN_INDEX on and off: tails from none to all
    lines, non-canonical prefixes (deferred lines that match), both compaction paths; the
    whole index on demand (line offsets, klf_retail); and the hit-list overflow, whose
    k_match fallback needs every line (the run is redone with the whole index)."""
    monkeypatch.setenv("KLF_WIN_INDEX", win)
    lits = [l for l in synth.c4_literals(1024)][:300] + [b"ms"]
    streams = [synth.generate(synth.MIXED, 21, 0, 600_000, permille=30),
               synth.generate(synth.ADVERSARIAL, 22, 1, 80_000, drop_final_nl=True, permille=40), b"",
               synth.generate(synth.MIXED, 23, 3, 300_000, permille=5)]
    for grep in (lits, [synth.NEEDLE], [b"ms"]):  # a set; one literal (k_scan<lit>: hit tiles flagged)
        for tail in (-1, 0, 1, 100, 10**9):
            check_against_c(streams, None, tail, grep)
        check_against_c(streams, (synth.T0 + 1800, 0), 25, grep)
    monkeypatch.setenv("KLF_HITS_CAP", "16")
    check_against_c(streams, None, 50, lits)


@pytest.mark.parametrize("win", ["1", "0"])
def test_windowed_index_regex_sets(gpu, monkeypatch, win):
    """Regex sets index only their tail windows too (round 6): k_verify writes each NFA
    candidate line's start, end and meta -- the end from this tile's next slot or the first
    later tile that lists a line start (1-32 KiB lines span several tiles) -- for k_nfa_win /
    k_nfa, and the whole index is built on demand (r.lines).  Against the Python oracle with
    KLF_WIN_INDEX_RX on and off: tails from none to all lines, since, deferred lines
    (adversarial prefixes), unbounded regexes (k_nfa), mixed literal + regex sets, klf_retail
    to other tails, and the candidate-queue overflow (k_match needs every line: the run is
    redone with the whole index)."""
    monkeypatch.setenv("KLF_WIN_INDEX_RX", win)
    rx = synth.c5_regexes()
    streams = [synth.generate(synth.LONGJSON, 41, 0, 1_200_000, permille=30),
               synth.generate(synth.ADVERSARIAL, 42, 1, 3000, drop_final_nl=True, permille=40), b"",
               synth.generate(synth.LONGJSON, 43, 3, 700_000, drop_final_nl=True, permille=30)]
    for tail in (-1, 0, 1, 7, 10**9):
        check_against_py(streams, None, tail, match=rx)
    check_against_py(streams, (synth.T0 + 1800, 0), 25, match=rx)
    for grep, match in (GEN_SETS[0], GEN_SETS[2], GEN_SETS[4]):
        check_against_py(streams, None, 9, grep, match)
    # klf_retail on the windowed run: the tail stage again over the index and bitmap in HBM
    pats = po.compile_patterns([], rx)
    with E.Engine(0, match=rx) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                eng.stage(i, s)
        r = eng.run(tail=3, n_streams=len(streams))
        for t2 in (50, 1, -1):
            r2 = r.retail(t2)
            for i, s in enumerate(streams):
                assert r2.stream(i).out == po.filter_stream(s, GZ, t2, pats).out, (t2, i)
            r = r2
        r.free()
    monkeypatch.setenv("KLF_CAND_CAP", "16")
    check_against_py(streams[:1], None, 5, match=rx)


@pytest.mark.parametrize("mode", ["sample", "underestimate", "two_phase"])
def test_first_run_line_sample(gpu, monkeypatch, mode):
    """A fresh engine's first run (literal or no patterns) sizes its line arrays from a
    newline count over 64 tiles spread over the batch (k_nlsample, read back before the
    scan) instead of reading the line count back between the scan and the rest.  An
    estimate far too low (KLF_DEBUG_NL_SCALE) overflows and reruns with the exact count;
    KLF_TWO_PHASE keeps the two-phase first run.  Dense and sparse parts in one batch,
    against the C oracle (run_engine opens a fresh engine per call)."""
    if mode == "underestimate":
        monkeypatch.setenv("KLF_DEBUG_NL_SCALE", "0.0001")
    if mode == "two_phase":
        monkeypatch.setenv("KLF_TWO_PHASE", "1")
    long = synth.generate(synth.LONGJSON, 81, 0, 3_000_000)
    dense = b"".join(b"2024-10-22T00:00:%02d.000000000Z x\n" % (i % 60) for i in range(60_000)) + b"\n" * 40_000
    streams = [long, dense, b"", synth.generate(synth.TEXT, 82, 3, 500_000)]
    for tail in (-1, 50):
        check_against_c(streams, None, tail, [])
    check_against_c(streams, (synth.T0 + 1800, 0), 30, [b"x"])
    check_against_c(streams, None, 20, synth.c4_literals(1024)[:100] + [b" x"])


@pytest.mark.parametrize("mode", ["pool", "records", "overflow"])
def test_line_slot_storage(gpu, monkeypatch, mode):
    """Where the scan keeps each tile's line slots (round 6): one line start in the tile's
    TileStat, two or more appended to the wave's chunk of the pool (the default), or the
    per-tile record regions of earlier rounds (KLF_WAVE_POOL=0); a first attempt whose pool
    is far too small (KLF_DEBUG_POOL_CAP) overflows and is redone.  Every reader of the
    slots runs: the whole index, windows, deferred lines, literal and regex verification,
    the dense compaction and the one-pass compaction, against the oracles."""
    if mode == "records":
        monkeypatch.setenv("KLF_WAVE_POOL", "0")
    if mode == "overflow":
        monkeypatch.setenv("KLF_DEBUG_POOL_CAP", "64")
    streams = [synth.generate(synth.LONGJSON, 91, 0, 2_000_000, permille=30),
               synth.generate(synth.ADVERSARIAL, 92, 1, 3000, drop_final_nl=True, permille=40), b"",
               synth.generate(synth.TEXT, 93, 3, 1_500_000)]
    for tail in (-1, 40):
        check_against_c(streams, None, tail, [])
        check_against_c(streams, (synth.T0 + 1800, 0), tail, [synth.NEEDLE])
    check_against_c(streams, None, 25, synth.c4_literals(1024)[:300])
    check_against_py(streams, (synth.T0 + 1800, 0), 15, match=synth.c5_regexes())


@pytest.mark.parametrize("split", ["3", "8"])
def test_scatter_split(gpu, monkeypatch, split):
    """k_scatter with each 64-tile group's lines split over several waves (small batches
    such as C1 pick the split from the grid; forced here on every shape): the whole index,
    the window pass, the pre-count pass, on-demand indexes."""
    monkeypatch.setenv("KLF_SCATTER_SPLIT", split)
    streams = [synth.generate(synth.TEXT, 71, 0, 3_000_000),
               synth.generate(synth.ADVERSARIAL, 72, 1, 3000, drop_final_nl=True, permille=40), b"",
               synth.generate(synth.JSON, 73, 2, 900_000, permille=20)]
    for tail in (-1, 100):
        check_against_c(streams, None, tail, [])
    check_against_c(streams, (synth.T0 + 1800, 0), 40, [synth.NEEDLE])
    check_against_c(streams, None, 30, synth.c4_literals(1024)[:200])
    check_against_py(streams[:2], None, 12, match=synth.c5_regexes())


def _long_window_stream(pre_bytes, long_len, after, lit=b"ms"):
    """Short lines up to `pre_bytes`, then one line of `long_len` content bytes holding `lit`,
    then `after` short lines holding it: a --tail after+1 window starts at the long line."""
    ts = b"2024-10-22T00:59:00.000000000Z "
    parts, n, i = [], 0, 0
    while n < pre_bytes:
        ln = ts + b"short line %d %s\n" % (i, lit if i % 3 == 0 else b"--")
        parts.append(ln)
        n += len(ln)
        i += 1
    parts.append(ts + b"L" * (long_len // 2) + lit + b"x" * (long_len - long_len // 2 - len(lit)) + b"\n")
    for j in range(after):
        parts.append(ts + b"after %d %s\n" % (j, lit))
    return b"".join(parts)


@pytest.mark.parametrize("win", ["1", "0"])
def test_windowed_index_long_first_line(gpu, monkeypatch, win):
    """The first line of a tail window is longer than 16 KiB and straddles a 64-tile
    (512 KiB) scatter-group boundary: the window pass must visit the tile that holds that
    line's start slot (the tile of the newline before it), not a tile found from the
    window's line index minus one tile.  Several tiles after that
    one carry no line start at all."""
    monkeypatch.setenv("KLF_WIN_INDEX", win)
    lits = synth.c4_literals(1024)[:200] + [b"ms"]
    for pre, long_len in ((500_000, 40_000), (520_000, 20_000), (300_000, 600_000), (0, 70_000)):
        d = _long_window_stream(pre, long_len, 20)
        lead = synth.generate(synth.TEXT, 3, 0, 200_000)  # moves the global tile numbering
        for grep in ([b"ms"], lits):
            for tail in (21, 22, 20, 1):
                check_against_c([d], None, tail, grep)
                check_against_c([lead, d], None, tail, grep)
            check_against_c([d, lead], (synth.T0 + 1800, 0), 21, grep)


def test_literal_automaton_thread(gpu, monkeypatch):
    """A literal set's Aho-Corasick automaton is built and uploaded by a host thread that
    klf_open starts and the first run joins: engines closed before any run (the thread
    joined by klf_close), runs right after open, and runs whose matcher is the automaton
    itself (the prefilter's hit list forced to overflow: k_match over every line)."""
    lits = synth.c4_literals(1024)[:500]
    for _ in range(8):
        E.Engine(0, grep=lits).close()
    d = synth.generate(synth.MIXED, 31, 0, 400_000, permille=20)
    check_against_c([d], None, 40, lits)
    monkeypatch.setenv("KLF_HITS_CAP", "1")
    check_against_c([d, synth.generate(synth.ADVERSARIAL, 32, 1, 30_000, permille=40)], (synth.T0 + 1800, 0), -1, lits)


@pytest.mark.parametrize("pats", ["none", "literal", "regex"])
def test_graph_replay(gpu, monkeypatch, pats):
    """Small batches replay their launch sequence as a HIP graph (round 6): captured the
    second time the same arguments run, replayed from the third, recaptured when they
    change.  Every run of an alternating sequence against the C / Python oracle, and the
    replays carry no scan dispatch events (the mark that the graph ran, not eager launches)."""
    import torch
    monkeypatch.setenv("KLF_GRAPH", "1")
    streams = [synth.generate(synth.TEXT, 81, 0, 2_000_000), b"",
               synth.generate(synth.JSON, 82, 1, 700_000, permille=20),
               synth.generate(synth.ADVERSARIAL, 83, 2, 2000, drop_final_nl=True, permille=40)]
    lens = [len(s) for s in streams]
    base, total = E.layout(lens)
    host = np.zeros(total, dtype=np.uint8)
    for b, s in zip(base, streams):
        host[b:b + len(s)] = np.frombuffer(s, dtype=np.uint8)
    dev = torch.from_numpy(host).to("cuda")
    torch.cuda.synchronize()
    kw = {"none": {}, "literal": {"grep": [synth.NEEDLE, b"ms"]},
          "regex": {"grep": [synth.NEEDLE], "match": synth.c5_regexes()[:8]}}[pats]
    A = ((synth.T0 + 1800, 0), 100)
    B = (None, -1)
    seq = [A, A, A, A, B, B, B, A, A, B]
    replays = 0
    pp = po.compile_patterns(kw.get("grep", []), kw.get("match", [])) if pats == "regex" else None
    with E.Engine(0, **kw) as eng:
        for since, tail in seq:
            r = eng.run_device(dev.data_ptr(), base, lens, since=since, tail=tail)
            tm = r.timing()
            replays += tm[6] == 0
            for i, s in enumerate(streams):
                so = r.stream(i)
                if pats == "regex":
                    ref = po.filter_stream(s, since or GZ, tail, pp)
                    assert so.out == ref.out, (i, since, tail)
                    assert so.counts["matched"] == ref.n_matched, (i, since, tail)
                else:
                    out, lo, bits, c = co.filter_stream(s, since or GZ, tail, list(kw.get("grep", [])))
                    assert so.out == out, (i, since, tail)
                    assert np.array_equal(r.lines(i), lo), (i, since, tail)
                    for k in ("lines", "parsed", "since_ok", "selected", "out_bytes"):
                        assert so.counts[k] == c[k], (i, k, since, tail)
            r.free()
    # replays: runs 3, 4 (A), 7 (B), 9 (A) -- each the third or later sighting in a row
    assert replays >= 4, replays


@pytest.mark.parametrize("plan", ["0", "1", "2"])
def test_gather_plan_modes(gpu, monkeypatch, plan):
    """A --tail run's line gather with its block sums and prefix in k_cplan / k_cmid (0), in
    k_cplan's last block (1) or in k_tailw's last block (2; runs whose line index precedes
    k_tailw, i.e. no patterns): selections of one to many compaction blocks, empty streams,
    windows with a fragment, literal and regex sets (which fall back to 1)."""
    monkeypatch.setenv("KLF_PLAN_MODE", plan)
    streams = [synth.generate(synth.TEXT, 91, 0, 2_000_000), b"",
               synth.generate(synth.ADVERSARIAL, 92, 1, 3000, drop_final_nl=True, permille=40),
               synth.generate(synth.JSON, 93, 2, 900_000, permille=20),
               synth.generate(synth.LONGJSON, 94, 3, 1_500_000, permille=5)]
    for since, tail in ((None, 0), (None, 1), ((synth.T0 + 1800, 0), 100), (None, 999), (None, 5000)):
        check_against_c(streams, since, tail, [])
    check_against_c(streams, (synth.T0 + 1800, 0), 100, [synth.NEEDLE])
    check_against_c(streams, None, 3000, synth.c4_literals(1024)[:100])
    check_against_py(streams[:3], None, 50, match=synth.c5_regexes()[:16])
