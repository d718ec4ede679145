"""The large-batch tile index (k_tindex with 4,096 tiles per block), which the engine uses
above 8 GiB (kScanSmallTiles tiles): KLF_DEBUG_TINDEX_WIDE=1 runs it on test-sized
batches.  Each batch spans several of its blocks (> 4,096 tiles of 8 KiB), and the
streams cross block boundaries, so the block totals, the earlier blocks' prefix, the
streams' line / count ranges, the deferred-line fix-up (adversarial prefixes) and the
flattened prefilter hit list (literal sets) are all exercised, byte-exact against the
C oracle."""
import pytest

from klogs_amd import synth
from test_gpu_parity import check_against_c, check_against_py

pytestmark = pytest.mark.gpu

SINCE = (synth.T0 + 1800, 0)


@pytest.fixture(autouse=True)
def wide(monkeypatch):
    monkeypatch.setenv("KLF_DEBUG_TINDEX_WIDE", "1")


def _streams():
    # ~88 MiB in 6 streams (~11,000 tiles: three 4,096-tile blocks), one of them
    # adversarial (non-canonical prefixes -> deferred lines), one empty, one tiny
    return [synth.generate(synth.JSON, 51, 0, 30_000_000),
            synth.generate(synth.ADVERSARIAL, 52, 1, 9_000_000),
            b"",
            synth.generate(synth.TEXT, 53, 3, 27_000_000),
            synth.generate(synth.TEXT, 54, 4, 3_000),
            synth.generate(synth.MIXED, 55, 5, 26_000_000)]


@pytest.mark.parametrize("since,tail,grep", [(None, -1, []), (SINCE, 100, [synth.NEEDLE]), (SINCE, -1, [])])
def test_wide_index_plain_and_literal(gpu, since, tail, grep):
    check_against_c(_streams(), since, tail, grep)


def test_wide_index_literal_set(gpu):
    """A literal set: the q-gram prefilter's hits flattened by the wide index."""
    check_against_c(_streams(), SINCE, 50, synth.c4_literals(64) + [synth.NEEDLE])


def test_wide_index_regex_set(gpu):
    """A regex set over long JSON lines (carried-in lines across tiles), side-stream
    scatter beside the verification, against the Python oracle."""
    streams = [synth.generate(synth.LONGJSON, 56, i, 12_000_000, permille=20) for i in range(3)]
    check_against_py(streams, SINCE, 40, match=synth.c5_regexes()[:24])
