"""Pins the oracles (CPU): known-answer vectors, stdlib cross-checks, the two
independent restatements against each other, and the committed golden fixtures."""
import datetime as dt
import json
import random
import re
from pathlib import Path

import numpy as np
import pytest

import c_oracle as co
import klf_oracle as po
from klogs_amd import synth

GOLDEN = Path(__file__).resolve().parent / "golden"


# ---- Go time.Parse(RFC3339Nano) -----------------------------------------------------
# Known answers: Go's documented RFC3339 examples plus the parse rules of format.go.
TS_KAT = [
    (b"2006-01-02T15:04:05Z", (1136214245, 0)),                 # Go's reference time
    (b"2006-01-02T15:04:05+07:00", (1136189045, 0)),            # time.RFC3339 example
    (b"2006-01-02T15:04:05.999999999Z", (1136214245, 999999999)),
    (b"1970-01-01T00:00:00Z", (0, 0)),
    (b"2024-10-22T00:00:00.000000000Z", (1729555200, 0)),
    (b"2024-10-22T00:00:00.5Z", (1729555200, 500000000)),       # 1 fraction digit
    (b"2024-10-22T00:00:00,25Z", (1729555200, 250000000)),      # comma separator (Go >= 1.17)
    (b"2024-10-22T00:00:00.1234567891234Z", (1729555200, 123456789)),  # >9 digits truncated
    (b"2024-10-22T5:00:00Z", (1729573200, 0)),                  # stdHour accepts one digit
    (b"2024-02-29T12:00:00Z", (1709208000, 0)),                 # leap day
    (b"2024-10-22T00:00:00-00:00", (1729555200, 0)),
    (b"2024-10-22T00:00:00+24:00", (1729468800, 0)),            # hh <= 24 accepted
    (b"2024-10-22T00:00:00+01:60", (1729548000, 0)),            # mm <= 60 accepted
    (b"0001-01-01T00:00:00Z", (-62135596800, 0)),               # Go zero time
    (b"0000-01-01T00:00:00Z", (-62167219200, 0)),               # year 0 (proleptic, leap)
    (b"9999-12-31T23:59:59.999999999Z", (253402300799, 999999999)),
]
TS_BAD = [
    b"", b"2024", b"2024-10-22", b"2024-10-22T00:00:00", b"2024-10-22 00:00:00Z",
    b"2024-13-01T00:00:00Z", b"2024-00-01T00:00:00Z", b"2023-02-29T00:00:00Z", b"2024-04-31T00:00:00Z",
    b"2024-10-22T24:00:00Z", b"2024-10-22T00:60:00Z", b"2024-10-22T00:00:60Z", b"2024-1-22T00:00:00Z",
    b"2024-10-2T00:00:00Z", b"2024-10-22T00:0:00Z", b"2024-10-22T00:00:0Z", b"2024-10-22T00:00:00.Z",
    b"2024-10-22T00:00:00Zx", b"2024-10-22T00:00:00+25:00", b"2024-10-22T00:00:00+01:61",
    b"2024-10-22T00:00:00+1:00", b"2024-10-22T00:00:00+0100", b"2024-10-22T00:00:00z",
    b"2024-10-22t00:00:00Z", b"+024-10-22T00:00:00Z", b"2024-10-22T123:00:00Z",
    b"2024-10-22T00:00:00.5", b"2024-10-22T00:00:00 Z",
]


@pytest.mark.parametrize("s,want", TS_KAT)
def test_ts_known_answers(s, want):
    assert po.go_parse_rfc3339nano(s) == want
    assert co.parse_ts(s) == want


@pytest.mark.parametrize("s", TS_BAD)
def test_ts_rejects(s):
    assert po.go_parse_rfc3339nano(s) is None
    assert co.parse_ts(s) is None


def test_ts_vs_python_datetime():
    rng = random.Random(0)
    for _ in range(3000):
        y = rng.randint(1, 9999)
        mo = rng.randint(1, 12)
        d = rng.randint(1, 31)
        h, mi, s = rng.randint(0, 23), rng.randint(0, 59), rng.randint(0, 59)
        nd = rng.randint(0, 9)
        frac = "".join(rng.choice("0123456789") for _ in range(nd))
        oh, om = rng.randint(0, 23), rng.randint(0, 59)
        sign = rng.choice("+-Z")
        tz = "Z" if sign == "Z" else f"{sign}{oh:02d}:{om:02d}"
        txt = f"{y:04d}-{mo:02d}-{d:02d}T{h:02d}:{mi:02d}:{s:02d}" + (f".{frac}" if nd else "") + tz
        try:
            off = dt.timedelta(0) if sign == "Z" else (1 if sign == "+" else -1) * dt.timedelta(hours=oh, minutes=om)
            ref = dt.datetime(y, mo, d, h, mi, s, tzinfo=dt.timezone(off))
            want = (int((ref - dt.datetime(1970, 1, 1, tzinfo=dt.timezone.utc)).total_seconds()),
                    int((frac + "000000000")[:9]) if nd else 0)
        except ValueError:
            want = None
        got = po.go_parse_rfc3339nano(txt.encode())
        assert got == want, txt
        assert co.parse_ts(txt.encode()) == want, txt


# ---- kubelet tail ------------------------------------------------------------------
def test_find_tail_line_start_index_upstream_vector():
    """k8s pkg/util/tail/tail_test.go (recalled): 4 full lines of blockSize bytes + an
    incomplete half line."""
    line = b"a" * po.TAIL_BLOCK_SIZE
    buf = line + b"\n" + line + b"\n" + line + b"\n" + line + b"\n" + line[po.TAIL_BLOCK_SIZE // 2:]
    for n, start in [(-1, 0), (0, (len(line) + 1) * 4), (1, (len(line) + 1) * 3), (9999, 0)]:
        assert po.find_tail_line_start_index(buf, n) == start


def test_read_logs_tail_edges():
    mk = lambda i, c: b"2024-10-22T00:00:%02dZ %s" % (i, c)
    # terminated lines + fragment
    buf = mk(1, b"a\n") + mk(2, b"b\n") + mk(3, b"c\n") + mk(4, b"frag")
    assert po.read_logs(buf, -1, po.GO_ZERO_TIME) == b"a\nb\nc\nfrag"
    assert po.read_logs(buf, 0, po.GO_ZERO_TIME) == b""            # limitedNum == 0: nothing
    assert po.read_logs(buf, 1, po.GO_ZERO_TIME) == b"c\n"         # fragment not emitted
    assert po.read_logs(buf, 2, po.GO_ZERO_TIME) == b"b\nc\n"
    # an unparseable line inside the window does not count -> the fragment is emitted
    buf2 = mk(1, b"a\n") + b"garbage\n" + mk(3, b"c\n") + mk(4, b"frag")
    assert po.read_logs(buf2, 2, po.GO_ZERO_TIME) == b"c\nfrag"
    # since drops a line but it still counts toward tail
    assert po.read_logs(buf, 2, (1729555200 + 3, 0)) == b"c\n"
    # since == a timestamp keeps it (not Before)
    assert po.read_logs(buf, -1, (1729555200 + 2, 0)) == b"b\nc\nfrag"
    # zero-time default drops year-0000 lines
    assert po.read_logs(b"0000-01-01T00:00:00Z x\n0001-01-01T00:00:00Z y\n", -1, po.GO_ZERO_TIME) == b"y\n"


# ---- Go ParseDuration ----------------------------------------------------------------
DUR_KAT = [(b"5m", 300 * 10**9), (b"1h2m3.5s", 3723500000000), (b"-1.5h", -5400 * 10**9), (b"0", 0),
           (b"+0", 0), (b"1.5s", 1500000000), (b".5s", 500000000), (b"1ns", 1), (b"1us", 1000),
           ("1µs".encode(), 1000), (b"300ms", 300000000), (b"2562047h47m16.854775807s", (1 << 63) - 1)]
DUR_BAD = [b"", b"1", b"5x", b"s", b".s", b"-", b"1.5", b"9223372036854775808ns", b"2562048h"]


@pytest.mark.parametrize("s,want", DUR_KAT)
def test_duration(s, want):
    assert po.go_parse_duration(s) == want


@pytest.mark.parametrize("s", DUR_BAD)
def test_duration_bad(s):
    assert po.go_parse_duration(s) is None


def test_duration_seconds_trunc():
    assert po.duration_seconds_trunc(1500000000) == 1
    assert po.duration_seconds_trunc(999999999) == 0
    assert po.duration_seconds_trunc(-1500000000) == -1
    # float64 rounding of Seconds(): 2^33 s + 999999999 ns rounds up before truncation
    assert po.duration_seconds_trunc((1 << 33) * 10**9 + 999999999) == (1 << 33) + 1


# ---- Go regexp subset: the Python re translation and the C leg ------------------------
RX_KAT_GO = [  # regexp/syntax parse.go rules the two legs were written to (round 5)
    (rb"a{01}", b"a{01}", True), (rb"a{01}", b"a", False),          # parseInt: no leading zeros -> literal '{'
    (rb"a{1,02}", b"a{1,02}", True), (rb"x{0}y", b"y", True),
    (rb"\Qab\E*", b"a", True), (rb"^\Qab\E*$", b"abbb", True),   # the repetition takes the last byte
    (rb"^\Qab\E*$", b"abab", False), (rb"\Q(a|b\E", b"x(a|b", True), (rb"\Qa.b", b"a.b", True),
    (rb"^a(?i)*$", b"aaa", True), (rb"^a*(?i)*$", b"aaa", True),    # (?flags) pushes nothing
    (rb"(?i)[[:^upper:]]", b"aB", False), (rb"(?i)[[:^upper:]]", b"a1", True),  # fold, then negate
    (rb"(?i)[^A-Z]", b"q", False), (rb"(?i)\W", b"K", False), (rb"[[:word:]]", b"_", True),
    (rb"a(?i)b|c", b"C", True), (rb"(?i:a)b", b"AB", False), (rb"(?i)a(?-i)b", b"AB", False),
    (rb"(?s).", b"\n", True), (rb".", b"\n", False), (rb"[^a]", b"\n", True),
    (rb"(?P<x>ab)+$", b"abab", True), (rb"(?<x>a)", b"a", True), (rb"\x{41}", b"A", True),
    (rb"\0", b"\x00", True), (rb"\x7f", b"\x7f", True), (rb"[]a]", b"]", True), (rb"[^]a]", b"]", False),
    (rb"[a-]", b"-", True), (rb"[]-a]", b"^", True), (rb"\_", b"_", True), (rb"x{2}{", b"xx{", True),
    (rb"^$", b"", True), (rb"$^", b"", True), (rb"a$^", b"a", False), (rb"(a|)+b", b"b", True),
    (rb"(a*)*$", b"bbb", True), (rb"((a*)*|b)+c", b"abac", True), (rb"[[:alpha:]-]{3}", b"a-b", True), (rb"[\d-z]", b"-", True),
]
RX_KAT = [
    (rb"a.c", b"xabc", True), (rb"a.c", b"ac", False), (rb"^abc", b"abcd", True), (rb"^abc", b"xabc", False),
    (rb"abc$", b"xabc", True), (rb"abc$", b"abcx", False), (rb"(?i)error", b"an ERROR here", True),
    (rb"err(?i:OR)", b"errOr", True), (rb"err(?i:OR)", b"ERRor", False), (rb"\d{3}-\d{4}", b"call 555-1234", True),
    (rb"\s", b"a\x0bb", False), (rb"[[:alpha:]]+\d", b"abc1", True), (rb"a{,2}", b"a{,2}", True),
    (rb"a|b|", b"zzz", True), (rb"x*", b"", True), (rb"^$", b"", True), (rb"^$", b"a", False),
    (rb"\Qa.b\E", b"axb", False), (rb"\Qa.b\E", b"a.b", True), (rb"[^a]", b"a", False), (rb"\x41", b"A", True),
    (rb"\101", b"A", True), (rb"(?:ab)+c", b"ababc", True), (rb"user=\w+ took \d+ms", b"user=bob took 12ms", True),
]


@pytest.mark.parametrize("pat,s,want", RX_KAT + RX_KAT_GO)
def test_regex_known_answers(pat, s, want):
    """Both regex legs: the Python oracle (Python re) and the C oracle's own parser + lazy DFA."""
    assert po.Pattern("regex", pat).matches(s) is want
    assert co.rx_match(pat, s) is want


@pytest.mark.parametrize("pat", [rb"a**", rb"(", rb"a)", rb"[a", rb"\b", rb"\pL", rb"\1", rb"*a", rb"a{2,1}",
                                 rb"x{1001}", "é".encode(), rb"(?P<n", rb"\8", rb"(?i-)"])
def test_regex_rejects(pat):
    with pytest.raises((po.PatternError, re.error)):
        po.Pattern("regex", pat)
    assert co.rx_error(pat) is not None


@pytest.mark.parametrize("pat", [rb"[[:foo:]]", rb"a{2}{3}", rb"a*?+", rb"(?i)*", rb"\Q\E*", rb"[z-a]",
                                 rb"\C", rb"a{1001,}", rb"(?P=x)", rb"(?x)", rb"\x{}", rb"\xg1"])
def test_regex_rejects_go_rules(pat):
    with pytest.raises((po.PatternError, re.error)):
        po.Pattern("regex", pat)
    assert co.rx_error(pat) is not None


def _random_regex(rng, depth=0):
    """A random pattern of the SPEC.md S5 subset over a small alphabet."""
    atoms = ["a", "b", "B", "-", ".", r"\d", r"\w", r"\s", r"\W", "[a-c]", "[^ab]", "[[:upper:]]", "[[:^alpha:]]",
             r"\.", r"\x41", "[-b]", "^", "$"]
    out = []
    for _ in range(rng.randint(1, 4)):
        k = rng.random()
        if k < 0.15 and depth < 2:
            inner = "|".join(_random_regex(rng, depth + 1) for _ in range(rng.randint(1, 3)))
            a = rng.choice(["(", "(?:", "(?i:", "(?P<g>"]) + inner + ")"
        elif k < 0.2:
            a = r"\Q" + rng.choice(["a.", "b*", "ab"]) + r"\E"
        else:
            a = rng.choice(atoms)
        if a not in ("^", "$") or rng.random() < 0.3:
            a += rng.choice(["", "", "", "*", "+", "?", "{2}", "{1,3}", "{0,}", "*?", "{01}"])
        out.append(a)
        if rng.random() < 0.1:
            out.append(rng.choice(["(?i)", "(?-i)", "(?s)"]))
    return "".join(out)


@pytest.mark.parametrize("seed", range(4))
def test_regex_legs_agree_random(seed):
    """The two regex legs (Python re over the Python oracle's translation; the C leg's own
    parser, Thompson NFA and lazy DFA) decide random subset patterns the same way, and
    accept / reject the same patterns."""
    rng = random.Random(1000 + seed)
    alphabet = "abAB-.1 _\tzC"
    n_ok = 0
    for _ in range(400):
        pat = _random_regex(rng).encode()
        try:
            py = po.Pattern("regex", pat)
        except (po.PatternError, re.error):
            assert co.rx_error(pat) is not None, pat
            continue
        assert co.rx_error(pat) is None, pat
        n_ok += 1
        for _ in range(12):
            s = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 9))).encode()
            assert co.rx_match(pat, s) is py.matches(s), (pat, s)
    assert n_ok > 250


# ---- the two restatements agree -----------------------------------------------------
@pytest.mark.parametrize("seed", range(5))
def test_python_and_c_oracles_agree(seed):
    rng = random.Random(seed)
    d = synth.generate(synth.ADVERSARIAL, seed, 1, 1500, drop_final_nl=bool(seed & 1), permille=40)
    ts = [p[0] for p in (po.parse_line(d[s:e]) for s, e in po.split_lines(d)) if p]
    for _ in range(10):
        since = rng.choice([po.GO_ZERO_TIME, rng.choice(ts), (synth.T0 + 1800, 0)])
        tail = rng.choice([-1, 0, 1, 3, 50, 1499, 4000])
        grep = rng.choice([[], [synth.NEEDLE], [b"ms", b"pod"], [b""], [b"\n"]])
        r = po.filter_stream(d, since, tail, po.compile_patterns(grep=grep))
        out, lo, bits, c = co.filter_stream(d, since, tail, grep)
        assert out == r.out
        assert list(lo) == r.line_off
        assert bits == r.match_bits
        assert (c["lines"], c["parsed"], c["since_ok"], c["matched"], c["selected"]) == \
            (r.n_lines, r.n_parsed, r.n_since, r.n_matched, r.n_selected)


# ---- committed golden fixtures ------------------------------------------------------
def _golden_cases():
    man = GOLDEN / "manifest.json"
    if not man.exists():
        return []
    return json.loads(man.read_text())["cases"]


@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_golden_python_oracle(case):
    data = (GOLDEN / case["input"]).read_bytes()
    pats = po.compile_patterns(grep=[bytes.fromhex(g) for g in case["grep"]],
                               match=[bytes.fromhex(m) for m in case["match"]])
    r = po.filter_stream(data, tuple(case["since"]), case["tail"], pats)
    assert r.out == (GOLDEN / case["expect_out"]).read_bytes()
    assert r.line_off == np.load(GOLDEN / case["expect_lines"]).tolist()
    if r.match_bits is not None:
        assert r.match_bits.hex() == case["expect_bits"]
    assert [r.n_lines, r.n_parsed, r.n_since, r.n_matched, r.n_selected] == case["expect_counts"]


@pytest.mark.parametrize("case", [c for c in _golden_cases() if not c["match"]], ids=lambda c: c["name"])
def test_golden_c_oracle(case):
    data = (GOLDEN / case["input"]).read_bytes()
    grep = [bytes.fromhex(g) for g in case["grep"]]
    out, lo, bits, c = co.filter_stream(data, tuple(case["since"]), case["tail"], grep)
    assert out == (GOLDEN / case["expect_out"]).read_bytes()
    assert lo.tolist() == np.load(GOLDEN / case["expect_lines"]).tolist()
    if grep:
        assert bits.hex() == case["expect_bits"]


@pytest.mark.parametrize("seed", range(3))
def test_c_oracle_aho_corasick_equals_memmem(seed):
    """Sets of more than 8 literals go through the C oracle's Aho-Corasick DFA; the same set
    split into groups of <= 8 (memmem) must give the same match bits, OR-ed."""
    import numpy as np
    rng = random.Random(seed)
    lits = rng.sample(synth.c4_literals(1024), 200) + [b"pod", b"took 1", b"=0h"]  # overlapping / common ones too
    d = synth.generate(synth.MIXED, 40 + seed, 0, 1_500_000, permille=40)
    whole = co.filter_stream(d, co.GO_ZERO_TIME, 30, lits)
    bits = None
    for k in range(0, len(lits), 8):
        b = np.frombuffer(co.filter_stream(d, co.GO_ZERO_TIME, -1, lits[k:k + 8])[2], np.uint8)
        bits = b.copy() if bits is None else bits | b
    assert whole[2] == bits.tobytes()
    assert whole[3]["matched"] == int(np.unpackbits(bits).sum()) > 0


def test_big_check_helpers_equal_the_whole_stream_oracle():
    """tests/big_check.py (the >8 GiB parity checks): the forked per-line table equals
    filter_stream's counts and bits, and the oracle on the tail suffix gives the whole
    stream's output."""
    import big_check as bc
    rx = synth.c5_regexes()
    d = synth.generate(synth.LONGJSON, 21, 0, 1_200_000, permille=300)
    arr = np.frombuffer(d, np.uint8)
    since = (synth.T0 + 1800, 0)
    pats = po.compile_patterns(match=rx)
    ref = po.filter_stream(d, since, 5, pats)
    hit, parsed, since_ok = bc.py_line_table(arr, since, match=rx, procs=4)
    assert (hit.size, parsed, since_ok, int(hit.sum())) == (ref.n_lines, ref.n_parsed, ref.n_since, ref.n_matched)
    assert np.array_equal(bc.unpack_bits(ref.match_bits, ref.n_lines), hit)
    starts = np.array(ref.line_off, dtype=np.uint64)
    a = bc.tail_suffix(arr, starts, hit, 5)
    assert a > 0 and po.filter_stream(d[a:], since, 5, pats).out == ref.out


def test_c_oracle_aho_corasick_every_byte_value():
    """Literals covering all 256 byte values (the class counter must not wrap):
    the Aho-Corasick path equals memmem groups of <= 8."""
    lits = [bytes([b, (b * 7 + 3) & 0xFF, (b * 13 + 5) & 0xFF]) for b in range(256)]
    lits = [x for x in lits if 0x0A not in x]
    d = bytearray(synth.generate(synth.ADVERSARIAL, 3, 0, 400_000, permille=40))
    rng = random.Random(5)
    for _ in range(300):  # plant some of the literals inside line contents
        lit = rng.choice(lits)
        at = rng.randrange(40, len(d) - 8)
        if 0x0A not in d[at - 1:at + len(lit) + 1]:
            d[at:at + len(lit)] = lit
    d = bytes(d)
    whole = co.filter_stream(d, co.GO_ZERO_TIME, -1, lits)
    bits = None
    for k in range(0, len(lits), 8):
        b = np.frombuffer(co.filter_stream(d, co.GO_ZERO_TIME, -1, lits[k:k + 8])[2], np.uint8)
        bits = b.copy() if bits is None else bits | b
    assert whole[2] == bits.tobytes()
    assert whole[3]["matched"] == int(np.unpackbits(bits).sum()) > 0


# ---- the C regex leg over whole streams equals the Python oracle ---------------------------
RX_SETS = [
    synth.c5_regexes(),
    [rb"ms$", rb"^\S+ \d", rb"(?i)POD", rb"a.b|c[^x]d", rb"\w{3,5}-\d+", rb"x*", rb"\.\*"],
    [rb"[]^-]", rb"[-^a]z", rb"q\+?", rb"(ab|cd)+e", rb"\A\d", rb"[[:alpha:]]{4}\z"],
]


@pytest.mark.parametrize("k", range(len(RX_SETS)))
@pytest.mark.parametrize("kind", [synth.LONGJSON, synth.ADVERSARIAL, synth.TEXT])
def test_c_regex_leg_equals_python_oracle(k, kind):
    rx = RX_SETS[k]
    d = synth.generate(kind, 60 + k, 0, 300_000 if kind == synth.LONGJSON else 120_000, permille=150)
    since = (synth.T0 + 1800, 0)
    for tail in (-1, 7):
        r = po.filter_stream(d, since, tail, po.compile_patterns(match=rx))
        out, lo, bits, c = co.filter_stream_rx(d, since, tail, rx)
        assert bits == r.match_bits
        assert out == r.out
        assert list(lo) == r.line_off
        assert (c["lines"], c["parsed"], c["since_ok"], c["matched"], c["selected"]) == \
            (r.n_lines, r.n_parsed, r.n_since, r.n_matched, r.n_selected)
