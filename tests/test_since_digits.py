"""The since cutoff as the scan's fast timestamp path compares it (klf_debug_since_digits,
host only): the 23 digits of the cutoff's canonical UTC prefix, big-endian per dword, against
Python's own calendar (datetime), with the clamps below 1970 and from 2100 on.  The GPU side
of the comparison is tests/test_gpu_parity.py::test_fast_timestamp_date_edges."""
import datetime
import random

import pytest

from klogs_amd import engine as E

GO_ZERO = -62135596800  # 0001-01-01T00:00:00Z


def want(sec, nsec):
    if sec < 0:
        d = "19700101000000000000000"
    elif sec >= 4102444800:
        d = "9" * 23
    else:
        t = datetime.datetime(1970, 1, 1) + datetime.timedelta(seconds=sec)
        d = t.strftime("%Y%m%d%H%M%S") + "%09d" % nsec
    be = lambda s: int.from_bytes(s.encode(), "big")  # noqa: E731
    return [be(d[0:4]), be(d[4:8]), be(d[8:12]), be(d[12:16]), be(d[16:20]), be(d[20:22] + "0" + d[22])]


@pytest.mark.parametrize("sec,nsec", [
    (GO_ZERO, 0), (-1, 999_999_999), (0, 0), (0, 1), (59, 999_999_999),
    (951_782_400, 0),          # 2000-02-29 (a leap day of a century year)
    (951_868_799, 999_999_999),
    (1_709_164_800, 123_456_789),  # 2024-02-29
    (1_729_555_200 + 3300, 0),     # the synthetic streams' since cutoff
    (4_102_444_799, 999_999_999), (4_102_444_800, 0), (1 << 40, 5)])
def test_fixed_instants(sec, nsec):
    assert E.debug_since_digits(sec, nsec) == want(sec, nsec)


def test_random_instants():
    rnd = random.Random(11)
    for _ in range(20_000):
        sec = rnd.randint(-100_000, 4_102_444_800 + 100_000)
        nsec = rnd.choice([0, 999_999_999, rnd.randint(0, 999_999_999)])
        assert E.debug_since_digits(sec, nsec) == want(sec, nsec), (sec, nsec)


def test_digits_order_like_instants():
    """Lexicographic order of the packed digits is the order of the instants (1970..2099)."""
    rnd = random.Random(12)
    pts = sorted((rnd.randint(0, 4_102_444_799), rnd.randint(0, 999_999_999)) for _ in range(5_000))
    digs = [E.debug_since_digits(s, n) for s, n in pts]
    assert all(a <= b for a, b in zip(digs, digs[1:]))
