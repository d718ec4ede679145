"""Both compaction paths and BASELINE config 3 on the GPU.

k_wprefix picks the path per run: the tile copy (k_tkeep / k_ksum / k_kbase / k_tcopy) when
at least a quarter of the lines can be selected, else the line gather (k_csum / k_cscan /
k_cgather).  KLF_COMPACT=dense|sparse forces one, so every shape below runs through both,
bit-exact against the C oracle."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import shard, synth
from test_gpu_parity import check_against_c, check_against_py

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + 1800, 0)


@pytest.fixture(params=["dense", "sparse"])
def compact(request, monkeypatch):
    monkeypatch.setenv("KLF_COMPACT", request.param)
    return request.param


@pytest.mark.parametrize("since,tail,grep", [(None, -1, []), (SINCE, -1, []), (None, 37, []),
                                             (SINCE, -1, [synth.NEEDLE]), (None, 0, []), (None, 10**9, [b"pod"])])
def test_forced_paths_text_json(gpu, compact, since, tail, grep):
    streams = [synth.generate(synth.TEXT, 41, 0, 700_000), synth.generate(synth.JSON, 42, 1, 900_000),
               b"", synth.generate(synth.TEXT, 43, 3, 9_000, drop_final_nl=True)]
    check_against_c(streams, since, tail, grep)


@pytest.mark.parametrize("tail", [-1, 0, 1, 3])
def test_empty_content_fragment(gpu, compact, tail):
    """A stream ending in a parsed fragment whose content is empty ("<ts> "): kubelet emits
    it (no bytes) and it counts as a selected line, on both paths (and fused)."""
    base = synth.generate(synth.TEXT, 44, 0, 30_000)
    streams = [base + b"2024-10-22T00:59:59.5Z ", b"2024-10-22T00:00:01Z ", base + b"2024-10-22T00:59:59.5Z x\n"]
    check_against_c(streams, None, tail, [])
    check_against_c(streams, None, tail, [b""])


@pytest.mark.parametrize("seed", range(3))
def test_forced_paths_adversarial(gpu, compact, seed):
    """Unparseable lines, odd prefixes, CRLF, fragments, empty contents."""
    d = synth.generate(synth.ADVERSARIAL, 70 + seed, 0, 6000, drop_final_nl=bool(seed & 1), permille=40)
    for since, tail, grep in [(None, -1, []), (SINCE, -1, []), (None, 11, [b"ms"]), (None, -1, [b"Z "])]:
        check_against_c([d, d[: len(d) // 3]], since, tail, grep)


def test_forced_paths_long_lines(gpu, compact):
    """1-32 KiB lines: one line spans several tiles (its kept run is cut at every tile edge)."""
    streams = [synth.generate(synth.LONGJSON, 13, i, 2_000_000 + 999 * i, permille=5) for i in range(3)]
    check_against_c(streams, None, -1, [])
    check_against_c(streams, SINCE, 30, [])


def test_forced_paths_tiny_lines(gpu, compact):
    """Lines of a few bytes (dense line slots) and 0-byte contents."""
    parts = []
    for i in range(30000):
        parts.append(b"2024-10-22T00:00:%02dZ \n" % (i % 60) if i % 3 == 0 else
                     b"2024-10-22T00:00:%02dZ %d\n" % (i % 60, i) if i % 3 == 1 else b"x\n")
    d = b"".join(parts)
    check_against_c([d, d[:4097], d[:8193]], None, -1, [])
    check_against_c([d], (synth.T0 + 20, 0), -1, [])


def test_forced_paths_regex_set(gpu, compact):
    rx = synth.c5_regexes()[:16]
    streams = [synth.generate(synth.LONGJSON, 6, i, 1_000_000, permille=50) for i in range(2)]
    check_against_py(streams, None, -1, match=rx)


def test_many_streams_all_selected_both(gpu, compact):
    """Adjacent streams' outputs share 16-B chunks at every boundary."""
    streams = [synth.generate(synth.TEXT, 21, i, 1000 + 37 * i) for i in range(300)]
    check_against_c(streams, None, -1, [])


# ---- BASELINE config 3: 1,024 streams selected by -l, sharded over 8 GPUs -------------------
def _c3_streams(n, size):
    return [synth.generate(synth.TEXT, 42, i, size) for i in range(n)]


def test_c3_sharded_over_8_ranks(gpu):
    """C3 at test size: 1,024 TEXT streams, -l only (every line out), LPT-sharded over 8
    simulated ranks (one Engine each, as one process per GPU would hold), each rank's
    batch through shard.engine_runner, the count records through run_shard's all-gather.
    Every stream's output and every gathered record against the C oracle."""
    world = 8
    streams = _c3_streams(1024, 24_000)
    lens = [len(s) for s in streams]
    engines = [E.Engine(0) for _ in range(world)]
    try:
        # phase 1: every rank filters its streams; phase 2: run_shard with the exchange
        results = {}
        for r in range(world):
            mine = shard.local_streams(lens, world, r)
            assert len(mine) == 128
            results[r] = shard.engine_runner(engines[r])([streams[i] for i in mine])
        cap = 128
        blocks = np.concatenate([shard.pack_records(
            {sid: res[1] for sid, res in zip(shard.local_streams(lens, world, r), results[r])}, cap)
            for r in range(world)])
        outs, tables = {}, []
        for r in range(world):
            o, t = shard.run_shard(lens, lambda i: streams[i], lambda _s, _r=r: results[_r], world, r,
                                   allgather=lambda blk: blocks)
            assert not (set(o) & set(outs))
            outs.update(o)
            tables.append(t)
    finally:
        for e in engines:
            e.close()
    assert sorted(outs) == list(range(1024))
    for t in tables[1:]:
        assert np.array_equal(t, tables[0])

    def want(i):
        out, _, _, c = co.filter_stream(streams[i], co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)
        return out, c
    with ThreadPoolExecutor(8) as ex:
        for i, (out, c) in enumerate(ex.map(want, range(1024))):
            assert outs[i] == out, i
            assert tables[0][i].tolist() == [c[k] for k in shard.RECORD_FIELDS[1:]], i


def test_c3_full_per_gpu_batch(gpu):
    """One GPU's full C3 share (128 x 64 MiB = 8 GiB), device-resident as the bench runs it:
    every stream's output and counts against the C oracle."""
    import torch
    n_streams, size = 128, 64 << 20
    lens = [synth.size(synth.TEXT, 42, i, size) for i in range(n_streams)]
    base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    h = np.empty(max(lens) + 1, dtype=np.uint8)
    for i, n in enumerate(lens):
        synth.generate_into(h, synth.TEXT, 42, i, size)
        dev[int(base[i]):int(base[i]) + n].copy_(torch.from_numpy(h[:n]))
    torch.cuda.synchronize()
    with E.Engine(0) as eng:
        r = eng.run_device(dev.data_ptr(), base, lens)
        got = [r.stream(i) for i in range(n_streams)]
        r.free()
    del dev

    def check(i):
        buf = np.empty(lens[i] + 1, dtype=np.uint8)
        synth.generate_into(buf, synth.TEXT, 42, i, size, threads=2)
        out, _, _, c = co.filter_stream(buf[:lens[i]], co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)
        ok = got[i].out == out and all(got[i].counts[k] == c[k] for k in ("lines", "parsed", "selected", "out_bytes"))
        return i, ok
    with ThreadPoolExecutor(8) as ex:
        bad = [i for i, ok in ex.map(check, range(n_streams)) if not ok]
    assert not bad, f"streams differ from the oracle: {bad[:10]}"


@pytest.mark.parametrize("tails", [(100, -1, 10**9), (0, 5, -1), (10**9, 3, -1)])
def test_output_buffer_grown_on_demand(gpu, compact, tails, monkeypatch):
    """A --tail run sizes the output buffer to its output (the copy that would not fit is
    skipped, the buffer grown, the tail stage rerun); a fresh engine's first run (its
    initial buffer forced down to 4 KiB) and a re-tail to a larger window (klf_retail) both
    take that path, bit-exact."""
    monkeypatch.setenv("KLF_DEBUG_OUT_INIT", "4096")
    streams = [synth.generate(synth.TEXT, 61, i, 400_000 + 50_000 * i) for i in range(5)]
    with E.Engine(0, grep=[]) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            eng.stage(i, s)
        r = eng.run(tail=tails[0], n_streams=len(streams))
        for k, tail in enumerate(tails):
            if k:
                r2 = r.retail(tail)
                r.free()
                r = r2
            for i, s in enumerate(streams):
                out, _, _, c = co.filter_stream(s, co.GO_ZERO_TIME, tail, [], want_lines=False, want_bits=False)
                g = r.stream(i)
                assert g.out == out, (tail, i, len(g.out), len(out))
                assert g.counts["selected"] == c["selected"], (tail, i)
        r.free()


def test_long_timestamp_prefix(gpu, compact):
    """Go's RFC3339Nano parse takes any number of fraction digits: a prefix past the meta
    word's 14-bit content offset (kPlenEscape) is found again from the bytes, also for a line
    that spans tiles and one carried into the next tile."""
    base = synth.generate(synth.TEXT, 51, 0, 20_000)
    frac = b"1" * 20_000
    streams = [base + b"2024-10-22T00:59:59." + frac + b"Z long prefix\n" + base,
               b"2024-10-22T00:59:59." + frac[:9000] + b"Z x\n" + base + b"2024-10-22T00:00:01." + frac + b"Z",
               base[:5000] + b"2024-10-22T00:59:59." + frac[:8170] + b"Z tile edge\n"]
    for since, tail in [(None, -1), (SINCE, -1), (None, 2)]:
        check_against_c(streams, since, tail, [])
    check_against_c(streams, None, -1, [b"prefix"])


@pytest.mark.parametrize("lazy", ["1", "0"])
def test_lazy_line_index(gpu, monkeypatch, lazy):
    """Runs without patterns and --tail -1 leave the global line index out when the dense
    path copies (its runs come from the scan's line slots); the index is built on demand by
    klf_result_lines / klf_retail / klf_result_last_unparsed.  Either way (KLF_LAZY_INDEX=0:
    always built) outputs, line offsets, re-tails and the last unparsed line equal the C
    oracle, over deferred (non-canonical) prefixes, long lines carried across tiles, dense
    tiles, fragments and empty streams."""
    monkeypatch.setenv("KLF_LAZY_INDEX", lazy)
    streams = [synth.generate(synth.ADVERSARIAL, 5, 0, 120_000, drop_final_nl=True, permille=40),
               synth.generate(synth.LONGJSON, 6, 1, 700_000, permille=5), b"",
               b"".join(b"2024-10-22T00:00:%02dZ %d\n" % (i % 60, i) for i in range(20000)),
               synth.generate(synth.TEXT, 7, 4, 300_000)]
    from test_shard import _last_unparsed
    with E.Engine(0, grep=[]) as eng:
        for since in (None, SINCE):
            eng.reset()
            eng.set_streams(len(streams))
            for i, s in enumerate(streams):
                if s:
                    eng.stage(i, s)
            r = eng.run(since=since, n_streams=len(streams))
            want = [co.filter_stream(s, since or co.GO_ZERO_TIME, -1, []) for s in streams]
            for i, s in enumerate(streams):
                assert r.stream(i).out == want[i][0], i
                assert r.stream(i).counts["selected"] == want[i][3]["selected"], i
            if since is None:  # the index built by klf_retail first, then read
                r2 = r.retail(7)
                r.free()
                r = r2
                for i, s in enumerate(streams):
                    out, lo, _, _ = co.filter_stream(s, co.GO_ZERO_TIME, 7, [])
                    assert r.stream(i).out == out, i
                    assert np.array_equal(r.lines(i), lo), i
            else:  # built by klf_result_last_unparsed, then by klf_result_lines (no-op)
                for i, s in enumerate(streams):
                    if s:
                        assert r.last_unparsed(i) == _last_unparsed(s), i
                    assert np.array_equal(r.lines(i), want[i][1]), i
            r.free()


@pytest.mark.parametrize("plan", ["1", "0"])
def test_planned_runs(gpu, monkeypatch, plan):
    """Runs without patterns and --tail -1 take the dense copy from the scan's own plans (each
    tile's kept runs and aggregate; k_cmid / k_cmove scan the aggregates for the output
    offsets and carried-in runs, no listing pass).  Over lines spanning several tiles, tiles
    of more than 128 lines (runs listed by k_tcopy), a prefix straddling a tile edge, empty
    contents, fragments and empty streams, since on and off, KLF_PLAN_RUNS=0 (k_tkeep lists
    every tile) and 1 equal the C oracle; a re-tail of the result lists the runs again."""
    monkeypatch.setenv("KLF_PLAN_RUNS", plan)
    monkeypatch.setenv("KLF_COMPACT", "dense")
    edge = synth.generate(synth.TEXT, 3, 0, 8180)
    edge = edge[:edge.rfind(b"\n") + 1]
    edge = edge + b"x" * (8192 - 10 - len(edge)) + b"\n" + b"2024-10-22T00:59:59.123456789Z straddles\n"
    streams = [synth.generate(synth.LONGJSON, 8, 0, 900_000, permille=5), b"",
               b"".join(b"2024-10-22T00:00:%02dZ %d\n" % (i % 60, i % 7) for i in range(30000)),
               synth.generate(synth.TEXT, 9, 3, 500_000, drop_final_nl=True), edge,
               b"2024-10-22T00:00:01Z \n2024-10-22T00:00:02Z \n2024-10-22T00:00:03Z"]
    with E.Engine(0, grep=[]) as eng:
        for since in (None, SINCE):
            eng.reset()
            eng.set_streams(len(streams))
            for i, s in enumerate(streams):
                if s:
                    eng.stage(i, s)
            r = eng.run(since=since, n_streams=len(streams))
            for i, s in enumerate(streams):
                out, _, _, c = co.filter_stream(s, since or co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)
                assert r.stream(i).out == out, (since, i)
                assert r.stream(i).counts["selected"] == c["selected"], (since, i)
            r2 = r.retail(40)
            r.free()
            for i, s in enumerate(streams):
                out, _, _, _ = co.filter_stream(s, since or co.GO_ZERO_TIME, 40, [], want_lines=False, want_bits=False)
                assert r2.stream(i).out == out, (since, i)
            r2.free()
