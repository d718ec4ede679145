"""The C-ABI library on CPU: loads, exports every symbol include/*.h declares, and the
host-side pieces (timestamp parse, pattern compiler tables) agree with the oracles.
No compute call touches a GPU here."""
import ctypes as C
import random
import re
from pathlib import Path

import pytest

import klf_oracle as po
from klogs_amd import engine as E

ROOT = Path(__file__).resolve().parent.parent


def _declared(header: Path):
    txt = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(klf_[a-z0-9_]+|klh_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported():
    names = _declared(ROOT / "include" / "klf.h") + _declared(ROOT / "include" / "klf_debug.h")
    assert len(names) >= 20
    assert not [n for n in _declared(ROOT / "include" / "klf.h") if n.startswith("klf_debug")]
    lib = C.CDLL(str(ROOT / "klogs_amd" / "_lib" / "libklf.so"))
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(E.SIGNATURES), set(names) ^ set(E.SIGNATURES)


def test_every_host_symbol_is_exported():
    from klogs_amd import host as H
    names = _declared(ROOT / "include" / "klogs_host.h")
    lib = C.CDLL(str(ROOT / "klogs_amd" / "_lib" / "libklogs_host.so"))
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(H.SYMBOLS), set(names) ^ set(H.SYMBOLS)


def test_strerror_and_layout():
    assert E.lib().klf_strerror(E.KLF_EPATTERN).decode().startswith("pattern")
    base, total = E.layout([10, 0, 300, 1])
    assert list(base) == [0, 256, 256, 768]
    assert total >= 1024 + 8192 + 64  # scan read-ahead: one 8 KiB wave-tile + halo past the end


@pytest.mark.parametrize("s,want", [(b"2024-10-22T00:00:00.123Z", (1729555200, 123000000)),
                                    (b"2024-10-22T00:00:00+01:00", (1729551600, 0)),
                                    (b"2023-02-29T00:00:00Z", None), (b"2024-10-22T00:00:00Z ", None)])
def test_host_ts_parse(s, want):
    assert E.parse_rfc3339nano(s) == want


def test_host_ts_parse_matches_oracle_random():
    rng = random.Random(3)
    alphabet = b"0123456789-T:.,Z+ "
    for _ in range(20000):
        base = bytearray(b"2024-10-22T12:34:56.789Z")
        for _ in range(rng.randint(0, 3)):
            i = rng.randrange(len(base))
            op = rng.randrange(3)
            if op == 0:
                base[i] = rng.choice(alphabet)
            elif op == 1:
                del base[i]
            else:
                base.insert(i, rng.choice(alphabet))
        s = bytes(base)
        assert E.parse_rfc3339nano(s) == po.go_parse_rfc3339nano(s), s


def test_open_rejects_bad_regex_before_touching_a_device():
    with pytest.raises(E.KlfError) as ei:
        E.Engine(0, match=[rb"a(b"])
    assert ei.value.code == E.KLF_EPATTERN
    with pytest.raises(E.KlfError) as ei:
        E.Engine(0, match=[rb"\bword"])
    assert ei.value.code == E.KLF_EPATTERN


@pytest.mark.parametrize("grep,match,mode", [
    ([], [], "none"), ([b"x"], [], "literal1"), ([b""], [], "all"), ([b"a\nb"], [], "never"),
    ([b"a", b"b"], [], "general"), ([], [rb"a+b"], "general"), ([], [rb"x*"], "all"),
    ([b"x", b"x"], [], "literal1"), ([b"x" * 300], [], "general"),
])
def test_compile_modes(grep, match, mode):
    rc, m, err = E.debug_compile(grep, match)
    assert rc == 0 and m == mode, (rc, m, err)


def test_compile_too_many_positions():
    rc, m, err = E.debug_compile([], [rb"a{65}"])
    assert rc == E.KLF_ETOOBIG, err
    rc, m, err = E.debug_compile([], [rb"a{64}"])
    assert rc == 0


# ---- the GPU matcher's tables, run on the host, vs Python re (independent engine) -------
RX = [rb"a.c", rb"^abc", rb"abc$", rb"(?i)error", rb"err(?i:OR)", rb"\d{3}-\d{4}", rb"\s", rb"[[:alpha:]]+\d",
      rb"a{,2}", rb"a|b|", rb"x*y", rb"^$", rb"^", rb"$", rb"\Qa.b\E", rb"[^a]", rb"\x41", rb"(?:ab)+c",
      rb"user=\w+ took \d+ms", rb"(a|ab)(c|bcd)(d*)", rb"(^|x)y", rb"y($|x)", rb"a^b", rb"a$b", rb"(?:^)*a",
      rb"(a*)*b", rb"[a-c]{2,4}d?", rb"(?s).", rb"\.\*\+", rb"[\d\s]+x", rb"(?i)[a-f]{3}", rb"a?b?c?$",
      rb"((a|b)*c){2}", rb"\A[0-9]+\z", rb"(?m)^x$", rb"status=(200|404|5\d\d)", rb"[]a]+", rb"[a-]+z"]
ALPH = b"abcdxyzABCERO0123456789-= .*+\tq"


def _rand_text(rng, n):
    return bytes(rng.choice(ALPH) for _ in range(n))


@pytest.mark.parametrize("pat", RX)
def test_glushkov_tables_vs_python_re(pat):
    rng = random.Random(hash(pat) & 0xFFFF)
    ref = po.Pattern("regex", pat)
    samples = [b"", b"a", b"abc", b"xabc", b"ERROR", b"555-1234", b"acd", b"abcd", b"y", b"xy", b"a.b", b"x"]
    samples += [_rand_text(rng, rng.randint(0, 12)) for _ in range(300)]
    for s in samples:
        assert E.debug_match(s, match=[pat]) == ref.matches(s), (pat, s)


def test_aho_corasick_tables_vs_contains():
    rng = random.Random(5)
    for trial in range(40):
        lits = [_rand_text(rng, rng.randint(1, 4)) for _ in range(rng.randint(2, 30))]
        for _ in range(40):
            s = _rand_text(rng, rng.randint(0, 30))
            want = any(l in s for l in lits)
            assert E.debug_match(s, grep=lits) == want, (lits, s)


def test_mixed_literals_and_regexes():
    rng = random.Random(9)
    pats = [rb"user=\w+ took \d{3,}ms"]
    lits = [b"ERR_CONN_RESET", b"panic:"]
    for _ in range(300):
        s = _rand_text(rng, rng.randint(0, 40))
        if rng.random() < 0.2:
            s += rng.choice([b"user=bob took 1234ms", b"panic: x", b"ERR_CONN_RESET"])
        want = any(l in s for l in lits) or any(po.Pattern("regex", p).matches(s) for p in pats)
        assert E.debug_match(s, grep=lits, match=pats) == want, s
