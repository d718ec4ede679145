"""Go RE2 subset (SPEC.md S5) -> glibc POSIX ERE, for the compiled CPU baseline of regex
sets (oracle/klf_oracle_c.c ko_filter_rx).  TEST INFRASTRUCTURE ONLY (bench.py's
cpu_baseline leg and tests/); the product never imports it.

The translation goes through the Python oracle's own reader (klf_oracle._GoRegexToPy),
whose output uses a small fixed vocabulary: non-capturing groups, alternation, the
repetition operators, \\A / \\Z and explicit byte classes ([\\xHH-\\xHH...]: Go's \\d \\w \\s,
`.` and (?i) are already expanded into byte sets there).  That text is rewritten token by
token into POSIX ERE: groups become plain groups, \\A / \\Z become ^ / $ (matched per line
content with REG_STARTEND), and every byte class becomes a bracket expression of raw bytes
(C locale: ranges are byte ranges).  No case flag is needed: case folding is in the sets.

Each pattern also gets its required literal: the longest run of single bytes (or ASCII
case pairs) at the top level that every match contains, searched lower-cased when the run
holds a case pair.  ko_filter_rx skips a line that holds no pattern's required literal.
NUL cannot appear in a regcomp string, so 0x00 is dropped from byte classes (the synthetic
logs hold no NUL; the translation is validated against the Python oracle in
tests/test_oracle.py)."""
from __future__ import annotations

import re
from typing import List, Optional, Tuple

from klf_oracle import PatternError, go_regex_to_python

_ERE_SPECIAL = set(b".[]()*+?{}|^$\\")


class Unsupported(ValueError):
    pass


def _tokens(py: str):
    """Tokens of the oracle's Python-regex text: ('open',) ('close',) ('never',) ('bol',)
    ('eol',) ('set', frozenset) ('op', text)."""
    i, n = 0, len(py)
    while i < n:
        if py.startswith("(?!)", i):
            yield ("never",)
            i += 4
        elif py.startswith("(?:", i):
            yield ("open",)
            i += 3
        elif py[i] == ")":
            yield ("close",)
            i += 1
        elif py.startswith("\\A", i):
            yield ("bol",)
            i += 2
        elif py.startswith("\\Z", i):
            yield ("eol",)
            i += 2
        elif py[i] == "[":
            j = py.index("]", i)
            s = set()
            for m in re.finditer(r"\\x([0-9a-f]{2})(?:-\\x([0-9a-f]{2}))?", py[i + 1:j]):
                lo = int(m.group(1), 16)
                hi = int(m.group(2), 16) if m.group(2) else lo
                s.update(range(lo, hi + 1))
            yield ("set", frozenset(s))
            i = j + 1
        elif py[i] == "{":
            j = py.index("}", i)
            yield ("op", py[i:j + 1])
            i = j + 1
        elif py[i] in "|*+?":
            yield ("op", py[i])
            i += 1
        else:
            raise Unsupported(f"unexpected {py[i]!r} in the oracle's translation")


def _bracket(s: frozenset) -> bytes:
    s = set(s) - {0}
    if not s:
        raise Unsupported("a byte class that holds only NUL (or nothing)")
    if len(s) == 1:
        (c,) = s
        return (b"\\" if c in _ERE_SPECIAL else b"") + bytes([c])
    special = {ord("]"), ord("-"), ord("^"), ord("["), ord("\\")}
    head, tail, body = b"", b"", []
    xs = sorted(s)
    i = 0
    while i < len(xs):
        j = i
        while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
            j += 1
        lo, hi = xs[i], xs[j]
        if hi - lo >= 2 and lo not in special and hi not in special:
            body.append(bytes([lo, ord("-"), hi]))
        else:
            for c in range(lo, hi + 1):
                if c == ord("]"):
                    head = b"]"
                elif c == ord("-"):
                    tail = b"-"
                else:
                    body.append(bytes([c]))
        i = j + 1
    if body and body[0] == b"^" and not head:  # '^' first would negate: move it behind
        body = body[1:] + [b"^"] if len(body) > 1 else body
    if body == [b"^"] and not head:  # the set is {'^', '-'}: a leading '-' is literal
        return b"[-^]"
    inner = head + b"".join(body) + tail
    return b"[" + inner + b"]"


def _optional(op: str) -> bool:
    return op in ("*", "?") or (op.startswith("{") and op[1:].split(",")[0].strip("}") == "0")


def translate(pat: bytes) -> Tuple[bytes, bytes, bool]:
    """(POSIX ERE, required literal or b"", literal searched lower-cased)."""
    try:
        py = go_regex_to_python(pat).decode("latin-1")
    except PatternError as e:
        raise Unsupported(str(e))
    toks = list(_tokens(py))
    out: List[bytes] = []
    depth = 0
    # required literal: runs of single bytes / case pairs at depth 0
    best: Tuple[bytes, bool] = (b"", False)
    run: List[Tuple[int, bool]] = []
    no_literal = False

    def flush():
        nonlocal best, run
        if run:
            loose = any(l for _, l in run)
            lit = bytes((c | 0x20) if (loose and 0x41 <= c <= 0x5A) else c for c, _ in run)
            if len(lit) > len(best[0]):
                best = (lit, loose)
        run = []

    for k, t in enumerate(toks):
        nxt = toks[k + 1] if k + 1 < len(toks) else None
        quant = nxt[1] if nxt and nxt[0] == "op" and nxt[1] != "|" else None
        if t[0] == "never":
            raise Unsupported("a class that matches nothing")
        if t[0] == "open":
            if depth == 0:
                flush()
            depth += 1
            out.append(b"(")
        elif t[0] == "close":
            depth -= 1
            out.append(b")")
        elif t[0] == "bol":
            out.append(b"^")
        elif t[0] == "eol":
            out.append(b"$")
        elif t[0] == "op":
            if t[1] == "|" and depth == 0:  # (the reader wraps alternations in groups)
                no_literal = True
            out.append(t[1].encode())
        else:  # set
            out.append(_bracket(t[1]))
            if depth:
                continue
            s = t[1]
            ch: Optional[Tuple[int, bool]] = None
            if len(s) == 1:
                (c,) = s
                ch = (c, False)
            elif len(s) == 2:
                a, b = sorted(s)
                if 0x41 <= a <= 0x5A and b == a + 32:
                    ch = (b, True)
            if ch is None or (quant and _optional(quant)):
                flush()
                continue
            run.append(ch)
            if quant:  # + or {n,m} n >= 1: the byte is there once, then repetition
                flush()
    flush()
    if no_literal:
        best = (b"", False)
    return b"".join(out), best[0], best[1]
