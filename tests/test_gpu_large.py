"""BASELINE configs 4 and 5 past 8 GiB on one batch (the large-batch tile index
k_tindex<16, *> with the prefilter's hit flattening, unforced), checked in full against the
oracles: C4's 1,024 literals against the C oracle (Aho-Corasick, a thread per stream), C5's
64 regexes against the Python oracle (a pool of forked workers), plus every line offset
against numpy's newline positions.  Anchors: the per-stream output of writeLogToDisk
(/root/reference/cmd/root.go:359-374) under kubelet's since/tail (SPEC.md S3/S4)."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import big_check as bc
import c_oracle as co
import klf_oracle as po
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + synth.SPAN + 1 - 300, 0)  # --since 5m
TAIL = 100


def _batch(kind, sizes, permille):
    """Generate the streams into one pinned-free host buffer per stream, upload them into
    one device batch (klf_layout), return (host arrays, device tensor, seg_base, lens)."""
    import torch
    lens = [synth.size(kind, 77, i, sz, permille=permille) for i, sz in enumerate(sizes)]
    seg_base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    host = []
    for i, (sz, n) in enumerate(zip(sizes, lens)):
        h = np.empty(n + 1, dtype=np.uint8)
        synth.generate_into(h, kind, 77, i, sz, permille=permille)
        dev[int(seg_base[i]):int(seg_base[i]) + n].copy_(torch.from_numpy(h[:n]))
        host.append(h[:n])
    torch.cuda.synchronize()
    return host, dev, seg_base, lens


def _line_starts(h: np.ndarray) -> np.ndarray:
    nl = np.flatnonzero(h == 10).astype(np.uint64) + 1
    starts = np.concatenate([np.zeros(1, np.uint64), nl])
    if len(h) and h[-1] == 10:  # a final '\n' opens no line
        starts = starts[:-1]
    return np.concatenate([starts, np.array([len(h)], np.uint64)])


def test_c4_literal_set_9gib(gpu):
    lits = synth.c4_literals(1024)
    host, dev, seg_base, lens = _batch(synth.MIXED, [3200 << 20] * 3, 5)
    assert sum(lens) > (9 << 30) - (512 << 20)
    with E.Engine(0, grep=lits) as eng:
        r = eng.run_device(dev.data_ptr(), seg_base, lens, since=SINCE, tail=TAIL)
        got = [(r.stream(i), r.lines(i), r.match_bits(i)) for i in range(len(lens))]
        r.free()
    with ThreadPoolExecutor(len(host)) as ex:  # ctypes releases the GIL: one oracle thread per stream
        ref = list(ex.map(lambda h: co.filter_stream(h, SINCE, TAIL, lits, want_lines=False), host))
    for i, h in enumerate(host):
        so, lo, bits = got[i]
        out, _, rbits, c = ref[i]
        assert so.out == out, f"stream {i}: output differs"
        assert so.counts == c | {"out_bytes": len(out)} or all(so.counts[k] == c[k] for k in c), (i, so.counts, c)
        assert bits == rbits, f"stream {i}: match bits differ"
        assert np.array_equal(lo, _line_starts(h)), f"stream {i}: line offsets differ"
        assert c["selected"] == TAIL and c["matched"] > 1000


def test_c5_regex_set_9gib(gpu):
    rx = synth.c5_regexes()
    host, dev, seg_base, lens = _batch(synth.LONGJSON, [3150 << 20] * 3, 5)
    assert sum(lens) > (9 << 30) - (512 << 20)
    with E.Engine(0, match=rx) as eng:
        r = eng.run_device(dev.data_ptr(), seg_base, lens, since=SINCE, tail=TAIL)
        got = [(r.stream(i), r.lines(i), r.match_bits(i)) for i in range(len(lens))]
        r.free()
    del dev
    pats = po.compile_patterns(match=rx)
    for i, h in enumerate(host):
        so, lo, bits = got[i]
        starts = _line_starts(h)
        assert np.array_equal(lo, starts), f"stream {i}: line offsets differ"
        hit, parsed, since_ok = bc.py_line_table(h, SINCE, match=rx)
        L = len(starts) - 1
        assert hit.size == L and so.counts["lines"] == L
        assert np.array_equal(bc.unpack_bits(bits, L), hit), f"stream {i}: match bits differ"
        assert (so.counts["parsed"], so.counts["since_ok"], so.counts["matched"]) == (parsed, since_ok, int(hit.sum()))
        # the tail window: the oracle on the shortest suffix that holds the last TAIL + 2 G lines
        a = bc.tail_suffix(h, starts, hit, TAIL)
        ref = po.filter_stream(bytes(h[a:]), SINCE, TAIL, pats)
        assert so.out == ref.out and so.counts["selected"] == ref.n_selected == TAIL, f"stream {i}: output differs"
