"""Per-pattern match counts (klf_result_pattern_counts, SURVEY.md §8a K4/K5 and the §8e
per-stream record) on the GPU, against the Python oracle's pattern_counts (parsed lines
whose content matches each pattern), on every matcher path: the fused prefilter with
k_verify / k_nfa_win / k_nfa, the fix-up of non-canonical timestamps, the k_match fallback
(prefilter off or overflowed lists), the single fused literal, and the special sets."""
import pytest

import klf_oracle as po
from klogs_amd import engine as E
from klogs_amd import synth
from test_gpu_parity import GEN_SETS

pytestmark = pytest.mark.gpu


def run_counts(streams, grep=(), match=(), since=None, tail=-1):
    with E.Engine(0, grep=grep, match=match) as eng:
        eng.set_streams(len(streams))
        for i, s in enumerate(streams):
            if s:
                eng.stage(i, s)
        r = eng.run(since=since, tail=tail, n_streams=len(streams), pattern_counts=True)
        try:
            return [r.pattern_counts(i) for i in range(len(streams))], [r.stream(i).counts for i in range(len(streams))]
        finally:
            r.free()


def check(streams, grep=(), match=(), since=None, tail=-1):
    got, cnt = run_counts(streams, grep, match, since, tail)
    pats = po.compile_patterns(grep, match)
    for i, s in enumerate(streams):
        assert got[i] == po.pattern_counts(s, pats), f"stream {i}"
    return got, cnt


def test_c4_literal_set(gpu):
    lits = synth.c4_literals(1024)
    streams = [synth.generate(synth.MIXED, 4, 0, 2_000_000, permille=20), synth.generate(synth.MIXED, 4, 1, 500_000, permille=80)]
    got, _ = check(streams, grep=lits, since=(synth.T0 + 1800, 0), tail=50)
    assert sum(got[0]) > 0


def test_c5_regex_set(gpu):
    rx = synth.c5_regexes()
    streams = [synth.generate(synth.LONGJSON, 5, i, 1_500_000, permille=30) for i in range(3)]
    got, _ = check(streams, match=rx)
    assert sum(map(sum, got)) > 0


@pytest.mark.parametrize("idx", range(len(GEN_SETS)))
def test_general_sets_adversarial(gpu, idx):
    """Mixed literal / regex sets (one with the prefilter off) over adversarial lines:
    non-canonical timestamps go through k_fixup (then k_fixcount), unparseable lines
    count nowhere."""
    grep, match = GEN_SETS[idx]
    d = synth.generate(synth.ADVERSARIAL, 61, 0, 4000, permille=40)
    t = synth.generate(synth.TEXT, 62, 0, 300_000).replace(b"volume", b"volume" + b"x" * 80, 50)
    check([d, t, b"", b"2024-10-22T00:00:00Z pod ready\n"], grep, match)


def test_overflowed_lists_fall_back(gpu, monkeypatch):
    monkeypatch.setenv("KLF_HITS_CAP", "16")
    monkeypatch.setenv("KLF_CAND_CAP", "16")
    d = synth.generate(synth.TEXT, 8, 0, 600_000)
    check([d], grep=[b"ERR_", b"pod"], match=[rb"(?i)took \d+ms", rb"status=\w+"])


def test_pair_set_grows(gpu, monkeypatch):
    monkeypatch.setenv("KLF_PAIRS_LOG2", "4")  # 16 entries: overflows, the run repeats larger
    d = synth.generate(synth.TEXT, 9, 0, 200_000)
    check([d], grep=[b"pod", b"ready", b"took"], match=[rb"sync\w*"])


def test_single_literal_duplicates_and_never(gpu):
    d = synth.generate(synth.JSON, 3, 0, 800_000, permille=30)
    got, cnt = check([d, b""], grep=[synth.NEEDLE, synth.NEEDLE, b"a\nb"])
    assert got[0][0] == got[0][1] == cnt[0]["matched"] and got[0][2] == 0 and got[1] == [0, 0, 0]


def test_always_pattern(gpu):
    d = synth.generate(synth.ADVERSARIAL, 5, 0, 2000, permille=40)
    got, cnt = check([d], grep=[b""], match=[rb"x*"])
    assert got[0] == [cnt[0]["parsed"]] * 2


@pytest.mark.parametrize("grep,match", [([b"", b"pod"], []), ([b"", b"pod", b"ready"], [rb"took \d+ms"]),
                                        ([b"pod"], [rb"x*"]), ([b""], [rb"(?i)ERR_\w+"])])
def test_always_pattern_beside_others(gpu, grep, match):
    """`--grep ""` (bytes.Contains(x, "") is true) next to real patterns: every parsed line
    is selected, and each other pattern still gets its own count; same output as the
    always-set without counts."""
    d = synth.generate(synth.ADVERSARIAL, 5, 0, 3000, permille=40)
    t = synth.generate(synth.TEXT, 6, 0, 200_000)
    got, cnt = check([d, t, b""], grep, match)
    for i in range(2):
        assert cnt[i]["matched"] == cnt[i]["parsed"]
    always = [k for k, p in enumerate(list(grep) + list(match)) if p in (b"", rb"x*")]
    assert all(got[0][k] == cnt[0]["parsed"] for k in always)
    with E.Engine(0, grep=grep, match=match) as eng:  # the same selection without counts
        for i, s in enumerate([d, t]):
            eng.stage(i, s)
        r = eng.run(since=(synth.T0 + 1800, 0), tail=40, n_streams=2)
        plain = [r.stream(i).out for i in range(2)]
        r.free()
    with E.Engine(0, grep=[b""]) as eng:
        for i, s in enumerate([d, t]):
            eng.stage(i, s)
        r = eng.run(since=(synth.T0 + 1800, 0), tail=40, n_streams=2)
        assert [r.stream(i).out for i in range(2)] == plain
        r.free()


def test_counts_on_all_empty_batch(gpu):
    """Per-pattern counts asked for on a batch whose streams are all empty: zeros."""
    got, cnt = run_counts([b"", b""], grep=[b"pod", b"ready"], match=[rb"took \d+ms"])
    assert got == [[0, 0, 0], [0, 0, 0]]


def test_counts_need_the_flag(gpu):
    with E.Engine(0, grep=[b"pod", b"ready"]) as eng:
        eng.stage(0, synth.generate(synth.TEXT, 1, 0, 10_000))
        r = eng.run(n_streams=1)
        with pytest.raises(E.KlfError) as ei:
            r.pattern_counts(0)
        assert ei.value.code == E.KLF_ESTATE
        r.free()
