"""The q-gram prefilter of general pattern sets (klf_patterns.cpp build_prefilter /
regex_factors) on the host: the prefiltered decision (samples at every phase of the
stride, bitmap, bucket verification, literal hits final, regex factor hits -> Glushkov
NFA) must equal the full matcher's and Python re / bytes.Contains on every content."""
import random

import pytest

import klf_oracle as po
from klogs_amd import engine as E
from klogs_amd import synth

ALPH = b"abcdeERO0123456789_-= .:\"{}tiumo"


def _text(rng, n):
    return bytes(rng.choice(ALPH) for _ in range(n))


def _want(s, grep, match):
    return any(g in s for g in grep) or any(po.Pattern("regex", m).matches(s) for m in match)


def _check(grep, match, contents):
    info = None
    for s in contents:
        want = _want(s, grep, match)
        assert E.debug_match(s, grep=grep, match=match) == want, s
        got, info = E.debug_prefilter(s, grep=grep, match=match, phase=0)
        assert got == want, (s, 0, info)
        for ph in range(1, 16 if info["stride"] >= 6 else 4):  # (the grid of stride 6 repeats every 16)
            got, info = E.debug_prefilter(s, grep=grep, match=match, phase=ph)
            assert got == want, (s, ph, info)
    return info


@pytest.mark.parametrize("seed", range(6))
def test_literal_sets(seed):
    rng = random.Random(seed)
    lits = [_text(rng, rng.randint(3, 12)) for _ in range(rng.randint(2, 60))]
    contents = []
    for _ in range(200):
        s = _text(rng, rng.randint(0, 60))
        if rng.random() < 0.3:
            lit = rng.choice(lits)
            k = rng.randint(0, len(s))
            s = s[:k] + lit + s[k:]
        contents.append(s)
    info = _check(lits, [], contents)
    assert info["on"] and info["needles"] == len(set(lits))


RX_SETS = [
    [rb"timeout after \d+ms", rb"(?i)panic: [a-z]+", rb"status=(500|502|503)"],
    [rb"user_id=u\d{4,6}", rb"(?i)OOM(killed|_score)", rb"tx-[0-9a-f]{4}-done"],
    [rb"abc(de|fg)*hij", rb"^start.*end$", rb"x{3}y+"],
    [rb"(?i)error: (disk|net)\w* full", rb"\Qa.b*c\E", rb"abc.def"],
]


@pytest.mark.parametrize("idx", range(len(RX_SETS)))
def test_regex_sets(idx):
    rng = random.Random(100 + idx)
    match = RX_SETS[idx]
    inserts = [b"timeout after 123ms", b"timeout after ms", b"PANIC: xyz", b"panic: 1", b"status=502",
               b"user_id=u12345", b"user_id=u12", b"oomKILLED", b"tx-0a9f-done", b"abcdefghij", b"abchij",
               b"start mid end", b"xxxyy", b"ERROR: disk0 full", b"a.b*c", b"abcXdef", b"Error: Network full"]
    contents = []
    for _ in range(300):
        s = _text(rng, rng.randint(0, 40))
        if rng.random() < 0.5:
            k = rng.randint(0, len(s))
            s = s[:k] + rng.choice(inserts) + s[k:]
        contents.append(s)
    info = _check([], match, contents + inserts)
    assert info["on"], info


def test_mixed_literals_and_regexes_prefiltered():
    rng = random.Random(7)
    grep = [b"ERR_CONN_RESET", b"segfault"]
    match = [rb"user=\w+ took \d{3,}ms", rb"(?i)deadline exceeded"]
    extra = [b"user=bob took 1234ms", b"user=bob took 12ms", b"DEADLINE Exceeded", b"ERR_CONN_RESET", b"segfault"]
    contents = [_text(rng, rng.randint(0, 50)) + (rng.choice(extra) if rng.random() < 0.5 else b"")
                for _ in range(300)]
    info = _check(grep, match, contents)
    assert info["on"] and info["stride"] >= 2


@pytest.mark.parametrize("grep,match,why", [
    ([b"ab", b"xyz"], [], "short literal"),
    ([], [rb"\d+"], "regex without a factor"),
    ([], [rb"a.b"], "1-byte factors"),
])
def test_prefilter_off_falls_back(grep, match, why):
    _, info = E.debug_prefilter(b"x", grep=grep, match=match)
    assert not info["on"], why
    rng = random.Random(1)
    _check(grep, match, [_text(rng, rng.randint(0, 20)) for _ in range(100)])


@pytest.mark.parametrize("grep,match,q,stride", [
    ([b"abcdefg", b"0123456789"], [], 4, 4),
    ([b"abcdef", b"0123456789"], [], 3, 4),
    ([b"abcde", b"0123456789"], [], 4, 2),
    ([b"abcd", b"0123456789"], [], 3, 2),
    ([b"abc", b"0123456789"], [], 3, 1),
    ([], [rb"(?i)timeout"], 4, 4),
    ([b"abcdefghij", b"0123456789AB"], [], 3, 8),
    ([b"abcdefghijk"], [rb"x+connection reset"], 4, 8),
    ([b"abcdefghi", b"0123456789AB"], [], 4, 6),
    ([b"abcdefgh", b"0123456789AB"], [], 3, 6),
])
def test_gram_and_stride_choice(grep, match, q, stride):
    _, info = E.debug_prefilter(b"", grep=grep, match=match)
    assert info["on"] and (info["q"], info["stride"]) == (q, stride), info


def test_short_needles_anchored():
    """Needles shorter than the stride-8 window (10 bytes) that share a rare byte ('_'):
    anchored at it, the rest probed at stride 8; the decision still equals the full
    matcher's on contents that hold the needles, their look-alikes and the anchor alone."""
    rng = random.Random(11)
    grep = [b"ab_cd1", b"xy_z9", b"q_rst", b"0123456789AB", b"longer needle here"]
    match = [rb"tx=[0-9]{3}_end\d", rb"(?i)deadline exceeded after \d+s"]
    _, info = E.debug_prefilter(b"", grep=grep, match=match)
    assert info["on"] and info["stride"] == 8 and info["anchor"] == ord("_"), info
    extra = [b"ab_cd1", b"xy_z9", b"q_rst", b"ab_cd", b"y_z9", b"_rst", b"0123456789AB", b"tx=123_end4",
             b"tx=12_end4", b"_end7", b"DEADLINE exceeded after 5s", b"longer needle here", b"___", b"_"]
    contents = []
    for _ in range(400):
        s = _text(rng, rng.randint(0, 50))
        for _ in range(rng.randint(0, 3)):
            k = rng.randint(0, len(s))
            s = s[:k] + rng.choice(extra) + s[k:]
        contents.append(s)
    _check(grep, match, contents + extra)


def test_c5_set_anchored(monkeypatch):
    """The C5 regex set with its short factor family (`-commitN`, 8 bytes) anchored on
    '-' (forced: without data statistics '-' counts as common): stride 8, equal decisions
    on C5-shaped content."""
    monkeypatch.setenv("KLF_QF_ANCHOR", "force")
    rx = synth.c5_regexes()
    _, info = E.debug_prefilter(b"", match=rx)
    assert info["on"] and info["stride"] == 8 and info["q"] == 3 and info["anchor"] == ord("-"), info
    rng = random.Random(12)
    parts = [b"tx-0123abcd-commit5", b"tx-0123abc-commit5", b"-commit", b"tx--commit1", b"user3_id=u12345 login",
             b"status=503 path=/api/v3/x", b"PANIC: foo error in mod3", b"shard2 deadline exceeded after 1.5s",
             b"GET /v2/items/7 404", b"conn reset by peer3", b"OOMkilled for pid5=9", b"2024-10-22", b"a-b-c"]
    contents = []
    for _ in range(300):
        s = _text(rng, rng.randint(0, 60))
        for _ in range(rng.randint(0, 3)):
            k = rng.randint(0, len(s))
            s = s[:k] + rng.choice(parts) + s[k:]
        contents.append(s)
    _check([], rx, contents + parts)


def test_c4_c5_sets_are_prefiltered():
    lits = synth.c4_literals(1024)
    assert len(lits) == 1024 and min(map(len, lits)) >= 6 and max(map(len, lits)) <= 24
    _, info = E.debug_prefilter(b"", grep=lits)
    assert info["on"] and info["stride"] >= 2, info
    rx = synth.c5_regexes()
    assert len(rx) == 64
    _, info = E.debug_prefilter(b"", match=rx)
    assert info["on"], info


# ---- the NFA window around each factor occurrence (rx_pre) ------------------------------
WINDOW_SETS = [
    [rb"ab{2,3}cd\d+xyz", rb"(?i)k(ey|ay)=v\d{1,3}:done"],
    [rb"p[qr]{0,4}STARTtail\w+", rb"(x|yy|zzz)marker\d"],
    [rb"(?i)panic: \w+ error in mod\d", rb"tx-[0-9a-f]{8}-commit\d"],
    [rb"^headFACTOR\d", rb"FACTOR2x$", rb"a*FACTOR3"],  # anchors; an unbounded prefix
]


@pytest.mark.parametrize("idx", range(len(WINDOW_SETS)))
def test_nfa_windows_equal_full_search(idx):
    """Matches whose factor occurs several times, lookalike prefixes before it, a match
    right at the content's start or end: the windowed NFA equals the full search."""
    rng = random.Random(300 + idx)
    match = WINDOW_SETS[idx]
    parts = [b"abbcd12xyz", b"abbbbcd1xyz", b"abcd1xyz", b"KAY=v12:done", b"key=v1234:done", b"pqqSTARTtailx",
             b"prrrrrSTARTtail", b"zzzmarker7", b"yymarker", b"PANIC: foo error in mod3", b"panic: error in mod3",
             b"tx-0123abcd-commit5", b"tx-0123abc-commit5", b"headFACTOR1", b"xheadFACTOR1", b"FACTOR2x",
             b"FACTOR2xy", b"aaaFACTOR3", b"FACTOR", b"cd1xyz", b":done", b"-commit"]
    contents = []
    for _ in range(400):
        s = _text(rng, rng.randint(0, 30))
        for _ in range(rng.randint(0, 3)):
            k = rng.randint(0, len(s))
            s = s[:k] + rng.choice(parts) + s[k:]
        contents.append(s)
    _check([], match, contents + parts)


@pytest.mark.parametrize("pat,want,pre", [
    (rb"status=5\d\d path=/api/v0/\w+", 0, 10),
    (rb"tx-[0-9a-f]{8}-commit0", 0, 11),
    (rb"(?i)panic: \w+ error in mod0", 0, None),  # the longest factor follows \w+
    (rb"(?i)panic: \w+ error in mod0", 6, 0),     # a bounded one long enough for stride 4
    (rb"x(ab|cde)+y", 0, 1),
    (rb"a{2,5}bcd", 0, 5),                        # "bcd" after up to five a
])
def test_factor_prefix_bounds(pat, want, pre):
    alts, got_pre, _ = E.debug_factors(pat, want)
    assert got_pre == pre, (pat, alts, got_pre)
