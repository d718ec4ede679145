"""CPU oracle for the klogs log-filter hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as the *checker*.  The product path
(``klogs_amd`` + ``libklf.so``) never routes through it.

What it restates (see SPEC.md for the frozen rules S1-S7):

* klogs today asks the API server for ``PodLogOptions{SinceSeconds, TailLines}``
  (``/root/reference/cmd/root.go:201-221``) and ``io.Copy``s the filtered body
  into ``<logpath>/<pod>__<container>.log`` (``cmd/root.go:341-374``).  The
  filtering itself happens in the kubelet, which is *not* in ``/root/reference``
  nor in its go.mod graph: ``k8s.io/kubernetes`` v1.30.3 (the release matching
  ``k8s.io/client-go v0.30.3``, ``/root/reference/go.mod:13``)
  ``pkg/kubelet/kuberuntime/logs/logs.go`` (``NewLogOptions``, ``ReadLogs``,
  ``parseCRILog``, ``logWriter.write``) and ``pkg/util/tail/tail.go``
  (``FindTailLineStartIndex``).  Those algorithms are restated here from their
  published source, function by function (``find_tail_line_start_index``,
  ``read_logs``).
* Timestamps are parsed with Go 1.22 ``time.Parse(time.RFC3339Nano, s)`` semantics
  (``go_parse_rfc3339nano``), restated from Go's ``time/format.go``.
* ``--grep`` is Go ``bytes.Contains``; ``--match`` is Go ``regexp.Match`` over the
  RE2 subset of SPEC.md S5, translated here to Python ``re`` (an independent engine
  from the engine's Glushkov NFA).

Parity pinning: the reference's own tests (``cmd/root_test.go``) cover only
``convertBytes`` — nothing on this path.  So for this path parity is anchored on
the call sites above plus known-answer vectors recalled from the upstream tests
(kubernetes ``pkg/util/tail/tail_test.go``; Go ``time`` docs) and stdlib
cross-checks (Python ``datetime``/``re``).  "Parity unpinned" against reference
fixtures: none exist.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

# Go's zero time.Time (0001-01-01T00:00:00Z) as Unix seconds.  kubelet's LogOptions.since
# defaults to it (logs.go NewLogOptions), and logWriter.write drops ts.Before(since).
GO_ZERO_TIME = (-62135596800, 0)
TAIL_BLOCK_SIZE = 1024  # pkg/util/tail/tail.go blockSize


# ----------------------------------------------------------------------------------
# Go time.Parse(RFC3339Nano) restated  (Go 1.22 src/time/format.go: Parse/parse,
# getnum, skip, parseNanoseconds, stdISO8601ColonTZ; date validation via daysIn)
# ----------------------------------------------------------------------------------

def _is_digit(s: bytes, i: int) -> bool:
    return i < len(s) and 0x30 <= s[i] <= 0x39


def _getnum(s: bytes, fixed: bool):
    """format.go getnum: one or two digits (two required when fixed)."""
    if not _is_digit(s, 0):
        return None
    if not _is_digit(s, 1):
        if fixed:
            return None
        return s[0] - 0x30, s[1:]
    return (s[0] - 0x30) * 10 + (s[1] - 0x30), s[2:]


def is_leap(y: int) -> bool:
    return y % 4 == 0 and (y % 100 != 0 or y % 400 == 0)


def days_in(month: int, year: int) -> int:
    if month == 2:
        return 29 if is_leap(year) else 28
    return 30 if month in (4, 6, 9, 11) else 31


def days_from_civil(y: int, m: int, d: int) -> int:
    """Days since 1970-01-01 of the proleptic Gregorian date (H. Hinnant's algorithm)."""
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    mp = (m + 9) % 12
    doy = (153 * mp + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def go_parse_rfc3339nano(v: bytes) -> Optional[Tuple[int, int]]:
    """time.Parse("2006-01-02T15:04:05.999999999Z07:00", v) -> (unix_sec, nsec) or None.

    Layout chunks: stdLongYear '-' stdZeroMonth '-' stdZeroDay 'T' stdHour ':'
    stdZeroMinute ':' stdZeroSecond stdFracSecond9 stdISO8601ColonTZ.
    """
    # stdLongYear: 4 bytes, first must be a digit, atoi of all four
    if len(v) < 4 or not _is_digit(v, 0):
        return None
    ys = v[:4]
    if not all(0x30 <= c <= 0x39 for c in ys):
        return None
    year = int(ys)
    v = v[4:]
    if v[:1] != b"-":
        return None
    r = _getnum(v[1:], True)  # stdZeroMonth
    if r is None:
        return None
    month, v = r
    if month <= 0 or month > 12:
        return None
    if v[:1] != b"-":
        return None
    r = _getnum(v[1:], True)  # stdZeroDay (validated after the loop)
    if r is None:
        return None
    day, v = r
    if v[:1] != b"T":
        return None
    r = _getnum(v[1:], False)  # stdHour: NOT fixed -> one digit allowed
    if r is None:
        return None
    hour, v = r
    if hour >= 24:
        return None
    if v[:1] != b":":
        return None
    r = _getnum(v[1:], True)  # stdZeroMinute
    if r is None:
        return None
    minute, v = r
    if minute >= 60:
        return None
    if v[:1] != b":":
        return None
    r = _getnum(v[1:], True)  # stdZeroSecond
    if r is None:
        return None
    sec, v = r
    if sec >= 60:
        return None
    nsec = 0
    # stdFracSecond9: optional; '.' or ',' followed by a digit; any number of digits.
    if len(v) >= 2 and v[0] in (0x2E, 0x2C) and _is_digit(v, 1):
        i = 0
        while i + 1 < len(v) and _is_digit(v, i + 1):
            i += 1
        nbytes = 1 + i
        digits = v[1:min(nbytes, 10)]  # parseNanoseconds: at most 9 digits
        ns = int(digits)
        for _ in range(10 - min(nbytes, 10)):
            ns *= 10
        nsec = ns
        v = v[nbytes:]
    # stdISO8601ColonTZ
    if len(v) >= 1 and v[0] == 0x5A:  # 'Z'
        v = v[1:]
        off = 0
    else:
        if len(v) < 6 or v[3] != 0x3A:
            return None
        sign, hh, mm = v[0], v[1:3], v[4:6]
        v = v[6:]
        r1 = _getnum(hh, True)
        r2 = _getnum(mm, True)
        if r1 is None or r2 is None:
            return None
        hr, m2 = r1[0], r2[0]
        if hr > 24 or m2 > 60:
            return None
        off = (hr * 60 + m2) * 60
        if sign == 0x2D:
            off = -off
        elif sign != 0x2B:
            return None
    if len(v) != 0:  # "extra text"
        return None
    if day < 1 or day > days_in(month, year):
        return None
    secs = days_from_civil(year, month, day) * 86400 + hour * 3600 + minute * 60 + sec - off
    return secs, nsec


def time_before(a: Tuple[int, int], b: Tuple[int, int]) -> bool:
    return a < b


# ----------------------------------------------------------------------------------
# Line model
# ----------------------------------------------------------------------------------

def split_lines(data: bytes) -> List[Tuple[int, int]]:
    """(start, end) of every line; a line includes its '\\n'; a final piece without
    '\\n' is the unterminated fragment (bufio.Reader.ReadBytes('\\n') loop)."""
    out = []
    pos = 0
    n = len(data)
    while pos < n:
        nl = data.find(b"\n", pos)
        if nl < 0:
            out.append((pos, n))
            break
        out.append((pos, nl + 1))
        pos = nl + 1
    return out


def parse_line(line: bytes):
    """Timestamped-line parse, as kubelet parseCRILog splits at the first ' ' delimiter
    and time.Parse(RFC3339Nano)s the head (logs.go parseCRILog).
    Returns ((sec, nsec), content) with content = bytes after the first space
    (terminating '\\n' kept), or None when unparseable."""
    idx = line.find(b" ")
    if idx < 0:
        return None
    ts = go_parse_rfc3339nano(line[:idx])
    if ts is None:
        return None
    return ts, line[idx + 1:]


def content_for_match(content: bytes) -> bytes:
    """S5: patterns see the content without its terminating '\\n'."""
    return content[:-1] if content.endswith(b"\n") else content


# ----------------------------------------------------------------------------------
# Patterns: Go bytes.Contains literals and a Go-regexp (RE2) subset -> Python re
# ----------------------------------------------------------------------------------

class PatternError(ValueError):
    pass


_PERL = {
    "d": set(range(0x30, 0x3A)),
    "w": set(range(0x30, 0x3A)) | set(range(0x41, 0x5B)) | set(range(0x61, 0x7B)) | {0x5F},
    "s": {0x09, 0x0A, 0x0C, 0x0D, 0x20},  # Go \s = [\t\n\f\r ] (no \v)
}
_POSIX = {
    "alnum": set(range(0x30, 0x3A)) | set(range(0x41, 0x5B)) | set(range(0x61, 0x7B)),
    "alpha": set(range(0x41, 0x5B)) | set(range(0x61, 0x7B)),
    "ascii": set(range(0x00, 0x80)),
    "blank": {0x09, 0x20},
    "cntrl": set(range(0x00, 0x20)) | {0x7F},
    "digit": set(range(0x30, 0x3A)),
    "graph": set(range(0x21, 0x7F)),
    "lower": set(range(0x61, 0x7B)),
    "print": set(range(0x20, 0x7F)),
    "punct": set(range(0x21, 0x30)) | set(range(0x3A, 0x41)) | set(range(0x5B, 0x61)) | set(range(0x7B, 0x7F)),
    "space": {0x09, 0x0A, 0x0B, 0x0C, 0x0D, 0x20},
    "upper": set(range(0x41, 0x5B)),
    "word": _PERL["w"],
    "xdigit": set(range(0x30, 0x3A)) | set(range(0x41, 0x47)) | set(range(0x61, 0x67)),
}
_ALL = set(range(256))


def _fold(s: set) -> set:
    out = set(s)
    for c in s:
        if 0x41 <= c <= 0x5A:
            out.add(c + 32)
        elif 0x61 <= c <= 0x7A:
            out.add(c - 32)
    return out


class _GoRegexToPy:
    """Recursive-descent reader of the Go RE2 subset (SPEC.md S5) emitting an
    equivalent Python ``re`` bytes pattern.  Character sets are emitted as explicit
    byte classes so Python's own flag semantics never apply."""

    def __init__(self, pat: bytes):
        if any(c >= 0x80 for c in pat):
            raise PatternError("non-ASCII pattern bytes are outside the supported subset")
        self.p = pat
        self.i = 0
        self.quoted = []  # bytes of a \Q...\E still to push

    def peek(self, k=0):
        j = self.i + k
        return self.p[j] if j < len(self.p) else None

    def eof(self):
        return self.i >= len(self.p)

    @staticmethod
    def emit_set(s: set) -> str:
        if not s:
            return "(?!)"
        if s == _ALL:
            return "[\\x00-\\xff]"
        parts = []
        xs = sorted(s)
        i = 0
        while i < len(xs):
            j = i
            while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
                j += 1
            parts.append("\\x%02x" % xs[i] if i == j else "\\x%02x-\\x%02x" % (xs[i], xs[j]))
            i = j + 1
        return "[" + "".join(parts) + "]"

    def parse(self) -> str:
        flags = {"i": False, "s": False}
        out = self.alt(flags)
        if not self.eof():
            raise PatternError("unexpected ')'")
        return out

    def alt(self, flags) -> str:
        branches = [self.concat(flags)]
        while self.peek() == 0x7C:  # '|'
            self.i += 1
            branches.append(self.concat(flags))
        return branches[0] if len(branches) == 1 else "(?:" + "|".join(branches) + ")"

    def concat(self, flags) -> str:
        items = []
        after_none = False  # the last step pushed nothing ((?flags) or an empty \Q\E)
        while self.quoted or (not self.eof() and self.peek() not in (0x7C, 0x29)):
            if self.quoted:  # \Q...\E: one literal per byte; a repetition after \E takes the last
                b = self.quoted.pop(0)
                atom = self.emit_set(_fold({b}) if flags["i"] else {b})
                items.append(self.repeat(atom) if not self.quoted else atom)
                after_none = False
                continue
            if after_none and items and self.at_repeat():
                # Go parse.go: (?flags) pushes nothing, so a repetition right after it
                # applies to the item before it (and is not a nested repetition)
                items[-1] = self.repeat(items[-1])
                after_none = False
                continue
            atom = self.atom(flags)
            if atom is None:  # flag group that only changed flags
                after_none = True
                continue
            after_none = False
            if self.quoted:  # (the \Q text's first byte came back as this atom)
                items.append(atom)
                continue
            atom = self.repeat(atom)
            items.append(atom)
        return "".join(items)

    def at_repeat(self) -> bool:
        c = self.peek()
        return c in (0x2A, 0x2B, 0x3F) or (c == 0x7B and _BRACES.match(self.p, self.i) is not None)

    def repeat(self, atom: str) -> str:
        seen = False
        while True:
            c = self.peek()
            if c in (0x2A, 0x2B, 0x3F):  # * + ?
                if seen:
                    raise PatternError("invalid nested repetition operator")
                self.i += 1
                atom = "(?:%s)%s" % (atom, chr(c))
            elif c == 0x7B:  # {
                r = self.try_braces()
                if r is None:
                    return atom
                if seen:
                    raise PatternError("invalid nested repetition operator")
                lo, hi = r
                atom = "(?:%s){%d,%s}" % (atom, lo, "" if hi is None else str(hi))
            else:
                return atom
            seen = True
            if self.peek() == 0x3F:  # lazy marker: irrelevant for boolean match
                self.i += 1

    def try_braces(self):
        m = _BRACES.match(self.p, self.i)
        if not m:
            return None  # Go: literal '{' (parseInt takes no leading zeros)
        lo = int(m.group(1))
        hi = lo if m.group(2) is None else (None if m.group(3) is None else int(m.group(3)))
        if lo > 1000 or (hi is not None and (hi > 1000 or hi < lo)):
            raise PatternError("invalid repeat count")
        self.i = m.end()
        return lo, hi

    def atom(self, flags):
        c = self.peek()
        if c in (0x2A, 0x2B, 0x3F) or (c == 0x7B and _BRACES.match(self.p, self.i)):
            raise PatternError("missing argument to repetition operator")
        if c == 0x28:  # (
            return self.group(flags)
        if c == 0x5B:  # [
            return self.emit_set(self.bracket(flags))
        if c == 0x2E:  # .
            self.i += 1
            return self.emit_set(_ALL if flags["s"] else _ALL - {0x0A})
        if c == 0x5E:  # ^  (no '\n' in matched content: ^ == \A with or without (?m))
            self.i += 1
            return "\\A"
        if c == 0x24:  # $
            self.i += 1
            return "\\Z"
        if c == 0x5C:  # backslash
            return self.escape(flags)
        self.i += 1
        s = {c}
        return self.emit_set(_fold(s) if flags["i"] else s)

    def group(self, flags):
        self.i += 1
        if self.peek() == 0x3F:  # (?
            m = re.match(rb"\?P?<([A-Za-z0-9_]+)>", self.p[self.i:])
            if m:
                self.i += m.end()
                inner = self.alt(dict(flags))
                self.expect_close()
                return "(?:" + inner + ")"
            m = re.match(rb"\?([imsU]*)(?:-([imsU]*))?(:|\))", self.p[self.i:])
            if not m or (m.group(1) == b"" and m.group(2) is None and m.group(3) == b")") \
                    or m.group(2) == b"":
                raise PatternError("invalid or unsupported Perl syntax")
            newf = dict(flags)
            for ch in m.group(1).decode():
                if ch in "is":
                    newf[ch] = True
            for ch in (m.group(2) or b"").decode():
                if ch in "is":
                    newf[ch] = False
            self.i += m.end()
            if m.group(3) == b")":  # (?flags) applies to the rest of the current group
                flags.update(newf)
                return None
            inner = self.alt(newf)
            self.expect_close()
            return "(?:" + inner + ")"
        inner = self.alt(dict(flags))
        self.expect_close()
        return "(?:" + inner + ")"

    def expect_close(self):
        if self.peek() != 0x29:
            raise PatternError("missing closing )")
        self.i += 1

    def escape_byte(self, in_class: bool):
        """Returns ('set', set) or ('assert', str)."""
        self.i += 1
        c = self.peek()
        if c is None:
            raise PatternError("trailing backslash at end of expression")
        self.i += 1
        ch = chr(c)
        if ch in "dws":
            return "set", set(_PERL[ch])
        if ch in "DWS":
            return "set", _ALL - _PERL[ch.lower()]
        simple = {"t": 0x09, "n": 0x0A, "r": 0x0D, "f": 0x0C, "v": 0x0B, "a": 0x07}
        if ch in simple:
            return "char", simple[ch]
        if ch == "x":
            if self.peek() == 0x7B:
                m = re.match(rb"\{([0-9A-Fa-f]{1,8})\}", self.p[self.i:])
                if not m:
                    raise PatternError("invalid escape sequence")
                v = int(m.group(1), 16)
                self.i += m.end()
            else:
                m = re.match(rb"[0-9A-Fa-f]{2}", self.p[self.i:])
                if not m:
                    raise PatternError("invalid escape sequence")
                v = int(m.group(0), 16)
                self.i += 2
            if v >= 0x80:
                raise PatternError("non-ASCII escapes are outside the supported subset")
            return "char", v
        if ch in "01234567":
            # Go syntax/parse.go parseEscape: a single non-zero digit would be a backreference
            # (unsupported); '0' or a digit followed by an octal digit reads up to 3 digits.
            if ch != "0" and not (self.i < len(self.p) and 0x30 <= self.p[self.i] <= 0x37):
                raise PatternError("invalid escape sequence")
            v = c - 0x30
            for _ in range(2):
                if self.i < len(self.p) and 0x30 <= self.p[self.i] <= 0x37:
                    v = v * 8 + self.p[self.i] - 0x30
                    self.i += 1
                else:
                    break
            if v >= 0x80:
                raise PatternError("non-ASCII escapes are outside the supported subset")
            return "char", v
        if not in_class:
            if ch == "A":
                return "assert", "\\A"
            if ch == "z":
                return "assert", "\\Z"
        if not ch.isalnum():  # punctuation (and '_') escapes itself
            return "char", c
        raise PatternError("invalid or unsupported escape \\" + ch)

    def escape(self, flags):
        if self.p[self.i:self.i + 2] == b"\\Q":
            end = self.p.find(b"\\E", self.i + 2)
            lit = self.p[self.i + 2:] if end < 0 else self.p[self.i + 2:end]
            self.i = len(self.p) if end < 0 else end + 2
            if not lit:
                return None
            self.quoted = list(lit[1:])
            return self.emit_set(_fold({lit[0]}) if flags["i"] else {lit[0]})
        kind, v = self.escape_byte(False)
        if kind == "assert":
            return v
        if kind == "char":
            v = {v}
        return self.emit_set(_fold(v) if flags["i"] else v)

    def bracket(self, flags) -> set:
        self.i += 1
        neg = False
        if self.peek() == 0x5E:
            neg = True
            self.i += 1
        s = set()
        first = True
        while True:
            c = self.peek()
            if c is None:
                raise PatternError("missing closing ]")
            if c == 0x5D and not first:
                self.i += 1
                break
            first = False
            if c == 0x5B and self.peek(1) == 0x3A:  # [:name:]
                m = re.match(rb"\[:(\^?)([a-z]+):\]", self.p[self.i:])
                if m:
                    if m.group(2).decode() not in _POSIX:
                        raise PatternError("invalid character class range")
                    cls = _POSIX[m.group(2).decode()]
                    if flags["i"]:  # appendGroup: fold the group, then negate it
                        cls = _fold(cls)
                    s |= (_ALL - cls) if m.group(1) else cls
                    self.i += m.end()
                    continue
            lo = self.class_char()
            if isinstance(lo, set):
                s |= lo
                continue
            if self.peek() == 0x2D and self.peek(1) not in (0x5D, None):  # range
                self.i += 1
                hi = self.class_char()
                if isinstance(hi, set) or hi < lo:
                    raise PatternError("invalid character class range")
                s |= set(range(lo, hi + 1))
            else:
                s.add(lo)
        if flags["i"]:
            s = _fold(s)
        if neg:
            s = _ALL - s
            if not flags["s"]:
                pass  # Go: negated classes DO match '\n' unless... ([^a] matches \n); no \n in content
        return s

    def class_char(self):
        c = self.peek()
        if c == 0x5C:
            kind, v = self.escape_byte(True)
            return v  # int for a single byte, set for \d \w \s \D \W \S
        self.i += 1
        return c


_BRACES = re.compile(rb"\{(0|[1-9][0-9]*)(,(0|[1-9][0-9]*)?)?\}")


def go_regex_to_python(pat: bytes) -> bytes:
    return _GoRegexToPy(pat).parse().encode("latin-1")


@dataclass
class Pattern:
    kind: str  # "literal" | "regex"
    text: bytes
    _rx: Optional[re.Pattern] = field(default=None, repr=False)

    def __post_init__(self):
        if self.kind == "regex":
            self._rx = re.compile(go_regex_to_python(self.text), re.DOTALL)
        elif self.kind != "literal":
            raise ValueError(self.kind)

    def matches(self, content: bytes) -> bool:
        if self.kind == "literal":
            return self.text in content  # bytes.Contains
        return self._rx.search(content) is not None  # regexp.Match (unanchored)


def compile_patterns(grep: Sequence[bytes] = (), match: Sequence[bytes] = ()) -> List[Pattern]:
    return [Pattern("literal", g) for g in grep] + [Pattern("regex", m) for m in match]


def pattern_counts(data: bytes, pats: Sequence[Pattern]) -> List[int]:
    """Per-pattern match counts of one stream (klf_result_pattern_counts; SURVEY.md §8a
    K4/K5 `count[stream][pattern]`): parsed lines whose content, without its '\\n'
    (SPEC.md S5), matches pattern p -- a line matching several patterns counts for each,
    since and tail play no part (like the `matched` count, SPEC.md S6)."""
    counts = [0] * len(pats)
    for lo, hi in split_lines(data):
        p = parse_line(data[lo:hi])
        if p is None:
            continue
        c = content_for_match(p[1])
        for k, pat in enumerate(pats):
            if pat.matches(c):
                counts[k] += 1
    return counts


# ----------------------------------------------------------------------------------
# kubelet restated
# ----------------------------------------------------------------------------------

def find_tail_line_start_index(buf: bytes, n: int) -> int:
    """pkg/util/tail/tail.go FindTailLineStartIndex: start of the last n lines; an
    unterminated final line is not counted as a line."""
    if n < 0:
        return 0
    size = len(buf)
    left = 0
    cnt = 0
    blk = b""
    right = size
    while right > 0 and cnt <= n:
        left = right - TAIL_BLOCK_SIZE
        if left < 0:
            left = 0
        blk = buf[left:right]
        cnt += blk.count(b"\n")
        right -= TAIL_BLOCK_SIZE
    while cnt > n:
        idx = blk.find(b"\n") + 1
        blk = blk[idx:]
        left += idx
        cnt -= 1
    return left


def read_logs(buf: bytes, tail: int, since: Tuple[int, int]) -> bytes:
    """pkg/kubelet/kuberuntime/logs/logs.go ReadLogs (follow=false, timestamps=false,
    no LimitBytes) over a file of timestamped lines.  limitedNum decrements for every
    parsed line, including lines logWriter.write drops for being before `since`;
    unparseable lines are skipped without decrementing."""
    start = find_tail_line_start_index(buf, tail)
    limited = tail >= 0
    limited_num = tail
    out = bytearray()
    pos = start
    stop = False
    while True:
        if stop or (limited and limited_num == 0):
            return bytes(out)
        nl = buf.find(b"\n", pos)
        if nl < 0:
            line = buf[pos:]
            pos = len(buf)
            stop = True
            if len(line) == 0:
                continue
        else:
            line = buf[pos:nl + 1]
            pos = nl + 1
        p = parse_line(line)
        if p is None:
            continue
        ts, content = p
        if not time_before(ts, since):  # logWriter.write
            out += content
        if limited:
            limited_num -= 1


# ----------------------------------------------------------------------------------
# The engine contract: one stream
# ----------------------------------------------------------------------------------

@dataclass
class StreamResult:
    out: bytes
    line_off: List[int]            # len = n_lines + 1 (sentinel = stream length)
    match_bits: Optional[bytes]    # packed little-endian bitmap (bit l of byte l>>3); None w/o patterns
    n_lines: int
    n_parsed: int
    n_since: int
    n_matched: int
    n_selected: int

    @property
    def out_bytes(self) -> int:
        return len(self.out)


def filter_stream(data: bytes, since: Tuple[int, int] = GO_ZERO_TIME, tail: int = -1,
                  patterns: Sequence[Pattern] = ()) -> StreamResult:
    """SPEC.md S4: grep acts as a source filter (G = matching parseable lines; every
    line when no pattern is given), then kubelet's exact tail+since over G."""
    lines = split_lines(data)
    line_off = [s for s, _ in lines] + [len(data)]
    n_parsed = n_since = 0
    gfile = bytearray()
    bits = bytearray((len(lines) + 7) // 8) if patterns else None
    n_matched = 0
    for li, (s, e) in enumerate(lines):
        ln = data[s:e]
        p = parse_line(ln)
        if p is not None:
            n_parsed += 1
            if not time_before(p[0], since):
                n_since += 1
        if patterns:
            hit = p is not None and any(pt.matches(content_for_match(p[1])) for pt in patterns)
            if hit:
                bits[li >> 3] |= 1 << (li & 7)
                n_matched += 1
                gfile += ln
        else:
            n_matched += 1
            gfile += ln
    out = read_logs(bytes(gfile), tail, since)
    # n_selected: the number of emitted lines (recount by replaying the selection)
    n_sel = _count_selected(bytes(gfile), tail, since)
    return StreamResult(out, line_off, bytes(bits) if bits is not None else None,
                        len(lines), n_parsed, n_since, n_matched, n_sel)


def _count_selected(buf: bytes, tail: int, since) -> int:
    start = find_tail_line_start_index(buf, tail)
    n = 0
    left = tail
    for s, e in split_lines(buf[start:]):
        if tail >= 0 and left == 0:
            break
        p = parse_line(buf[start + s:start + e])
        if p is None:
            continue
        if not time_before(p[0], since):
            n += 1
        left -= 1
    return n


# ----------------------------------------------------------------------------------
# Go time.ParseDuration restated (src/time/format.go ParseDuration, Go 1.22) — used by
# the host-mirror tests of getLopOpts (cmd/root.go:204-211)
# ----------------------------------------------------------------------------------

_UNIT = {b"ns": 1, b"us": 1000, "µs".encode(): 1000, "μs".encode(): 1000,
         b"ms": 10**6, b"s": 10**9, b"m": 60 * 10**9, b"h": 3600 * 10**9}
_I64MAX = (1 << 63) - 1


def go_parse_duration(s: bytes) -> Optional[int]:
    """Returns nanoseconds, or None for an error (ParseDuration's err != nil)."""
    orig = s
    d = 0
    neg = False
    if s[:1] in (b"-", b"+"):
        neg = s[:1] == b"-"
        s = s[1:]
    if s == b"0":
        return 0
    if s == b"":
        return None
    while s:
        if not (s[:1] == b"." or (b"0" <= s[:1] <= b"9")):
            return None
        # leadingInt
        i = 0
        v = 0
        while i < len(s) and 0x30 <= s[i] <= 0x39:
            if v > (1 << 63) // 10:
                return None
            v = v * 10 + (s[i] - 0x30)
            if v > 1 << 63:
                return None
            i += 1
        pre = i != 0
        s = s[i:]
        f, scale, post = 0, 1.0, False
        if s[:1] == b".":
            s = s[1:]
            # leadingFraction
            i = 0
            overflow = False
            while i < len(s) and 0x30 <= s[i] <= 0x39:
                if not overflow:
                    if f > _I64MAX // 10:
                        overflow = True
                    else:
                        y = f * 10 + (s[i] - 0x30)
                        if y > 1 << 63:
                            overflow = True
                        else:
                            f = y
                            scale *= 10
                i += 1
            post = i != 0
            s = s[i:]
        if not pre and not post:
            return None
        i = 0
        while i < len(s) and not (s[i] == 0x2E or 0x30 <= s[i] <= 0x39):
            i += 1
        if i == 0:
            return None  # missing unit
        u = s[:i]
        s = s[i:]
        unit = _UNIT.get(u)
        if unit is None:
            return None
        if v > (1 << 63) // unit:
            return None
        v *= unit
        if f > 0:
            v += int(float(f) * (float(unit) / scale))
            if v > 1 << 63:
                return None
        d += v
        if d > 1 << 63:
            return None
    if neg:
        return -d
    if d > _I64MAX:
        return None
    return d


def duration_seconds_trunc(d_ns: int) -> int:
    """int64(time.Duration(d).Seconds()) as in cmd/root.go:210 (float64 then truncate)."""
    sec = d_ns // 10**9 if d_ns >= 0 else -((-d_ns) // 10**9)  # Go '/' truncates
    nsec = d_ns - sec * 10**9
    f = float(sec) + float(nsec) / 1e9
    return int(f)  # float64 -> int64 truncates toward zero
