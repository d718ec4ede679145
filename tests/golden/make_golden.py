"""Writes the golden fixtures under tests/golden/ from the Python oracle (SPEC.md).

Run from the repo root:  python tests/golden/make_golden.py
Inputs are hand-written edge cases plus small seeded synthetic streams; each case stores
the input, the expected output bytes, the expected line offsets (.npy, u64, L+1), the
match bitmap (hex, LSB-first) and the counts [lines, parsed, since_ok, matched, selected].
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import klf_oracle as po  # noqa: E402
from klogs_amd import synth  # noqa: E402

T0 = synth.T0
GZ = list(po.GO_ZERO_TIME)


def ts(sec, frac="000000000", tz="Z"):
    import datetime as dt
    d = dt.datetime.fromtimestamp(sec, dt.timezone.utc)
    return (d.strftime("%Y-%m-%dT%H:%M:%S") + ("." + frac if frac else "") + tz).encode()


def lines(*items):
    return b"".join(items)


HAND = {
    "empty": b"",
    "fragment_only": ts(T0) + b" no newline",
    "basic": lines(*[ts(T0 + i) + b" line %d\n" % i for i in range(10)]) + ts(T0 + 10) + b" frag",
    "fractions": lines(*[ts(T0 + i, "123456789"[:k]) + b" f%d\n" % k for i, k in enumerate(range(0, 10))],
                       ts(T0 + 20, "1234567891234") + b" long fraction\n",
                       ts(T0 + 21).replace(b".", b",") + b" comma\n"),
    "offsets": lines(b"2024-10-22T01:30:00+01:30 a\n", b"2024-10-21T17:00:00-07:00 b\n",
                     b"2024-10-23T00:00:00+24:00 c\n", b"2024-10-22T00:00:00-00:00 d\n",
                     b"2024-10-22T00:00:00+25:00 bad\n", b"2024-10-22T00:00:00+1:00 bad\n"),
    "unparseable": lines(ts(T0) + b" ok1\n", b"garbage line\n", b"\n", b"   \n",
                         b"2024-02-30T00:00:00Z bad date\n", ts(T0 + 1) + b"\n", ts(T0 + 2) + b"  two spaces\n",
                         b"0000-01-01T00:00:00Z year zero\n", b"2024-10-22T5:00:00Z one digit hour\n",
                         ts(T0 + 3) + b" ok2\n", b"2024-10-22T00:00:00.Z bad frac\n", ts(T0 + 4) + b" last"),
    "crlf": lines(*[ts(T0 + i) + b" crlf %d\r\n" % i for i in range(6)], b"\r\n", ts(T0 + 9) + b" end\r\n"),
    "nonmonotonic": lines(*[ts(T0 + (i * 37) % 11) + b" nm%d ERR_CONN_RESET\n" % i if i % 3 == 0 else
                            ts(T0 + (i * 37) % 11) + b" nm%d\n" % i for i in range(30)]),
    "prefix_lookalike": lines(ts(T0) + b" x\n", ts(T0 + 1) + b" Z y\n", ts(T0 + 2) + b" z\n",
                              b"ERR_CONN_RESET 2024 no ts\n", ts(T0 + 3) + b" ERR_CONN_RESET\n"),
}

CASES = []


def add(name, data, since=GZ, tail=-1, grep=(), match=()):
    fn = f"{name}.log"
    (HERE / fn).write_bytes(data)
    r = po.filter_stream(data, tuple(since), tail, po.compile_patterns(grep=grep, match=match))
    tag = f"{name}__s{since[0] - T0 if since != GZ else 'Z'}_{since[1]}_t{tail}_g{len(grep)}_m{len(match)}"
    (HERE / f"{tag}.out").write_bytes(r.out)
    np.save(HERE / f"{tag}.lines.npy", np.array(r.line_off, dtype=np.uint64))
    CASES.append({
        "name": tag, "input": fn, "since": list(since), "tail": tail,
        "grep": [g.hex() for g in grep], "match": [m.hex() for m in match],
        "expect_out": f"{tag}.out", "expect_lines": f"{tag}.lines.npy",
        "expect_bits": r.match_bits.hex() if r.match_bits is not None else None,
        "expect_counts": [r.n_lines, r.n_parsed, r.n_since, r.n_matched, r.n_selected],
    })


def main():
    for old in HERE.glob("*"):
        if old.suffix in (".log", ".out", ".npy") or old.name == "manifest.json":
            old.unlink()
    for name, data in HAND.items():
        for tail in (-1, 0, 1, 3, 100):
            add(name, data, GZ, tail)
        add(name, data, [T0 + 3, 0], -1)            # cutoff == a timestamp
        add(name, data, [T0 + 3, 1], 2)
        add(name, data, GZ, 2, grep=[b"ERR_CONN_RESET"])
        add(name, data, GZ, -1, grep=[b"Z "])        # must not match inside the prefix
        add(name, data, GZ, 4, match=[rb"(?i)^(ok|line)\s*\d?", rb"nm\d+$"])
    text = synth.generate(synth.TEXT, 1, 0, 40_000)
    js = synth.generate(synth.JSON, 2, 0, 60_000, permille=50)
    adv = synth.generate(synth.ADVERSARIAL, 3, 0, 300, drop_final_nl=True, permille=40)
    for name, data in (("text", text), ("json", js), ("adv", adv)):
        add(name, data, [T0 + 1800, 0], 25)
        add(name, data, [T0 + 3000, 0], -1)
        add(name, data, GZ, 7, grep=[synth.NEEDLE])
        add(name, data, GZ, -1, grep=[b"took", b"pod"])
        add(name, data, [T0 + 600, 0], 50, match=[rb"user=\w+", rb"status [0-9]{2,3}\b?".replace(b"\\b?", b"")])
    (HERE / "manifest.json").write_text(json.dumps({"generator": "tests/golden/make_golden.py",
                                                    "oracle": "oracle/klf_oracle.py", "cases": CASES}, indent=1))
    print(len(CASES), "cases")


if __name__ == "__main__":
    main()
