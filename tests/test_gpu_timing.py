"""klf_result_timing through the C ABI: which device times a run reports, and that a run
without dispatch events (KLF_SCAN_EVENTS=0) followed by a stage-times run on the SAME
engine neither fails nor reports stale times (round-4 review: an event pair a run never
recorded left a sticky HIP error that the next launch check reported).  These runs launch
eagerly (KLF_GRAPH=0): a small batch's graph replay records only the run's bracket [4]
(test_gpu_parity.py::test_graph_replay)."""
import numpy as np
import pytest
import torch

import c_oracle as co
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu


def _device_batch(streams):
    lens = [len(s) for s in streams]
    seg_base, total = E.layout(lens)
    dev = torch.zeros(total, dtype=torch.uint8, device="cuda:0")
    for b, s in zip(seg_base, streams):
        dev[int(b):int(b) + len(s)].copy_(torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()))
    torch.cuda.synchronize()
    return dev, seg_base, lens


@pytest.mark.parametrize("grep", [[], [synth.NEEDLE]])
def test_events_off_then_stage_times_same_engine(gpu, monkeypatch, grep):
    monkeypatch.setenv("KLF_GRAPH", "0")
    streams = [synth.generate(synth.TEXT, 21, i, 2_000_000) for i in range(3)]
    dev, seg_base, lens = _device_batch(streams)
    since = (synth.T0 + 1800, 0)
    want = [co.filter_stream(s, since, 50, grep, want_lines=False, want_bits=False)[0] for s in streams]
    with E.Engine(0, grep=grep, hip_stream=torch.cuda.current_stream().cuda_stream) as eng:
        for rnd in range(2):
            monkeypatch.setenv("KLF_SCAN_EVENTS", "0")
            r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=50)
            tm = r.timing()
            assert len(tm) == 8
            assert tm[6] == 0.0 and tm[7] == 0.0, tm  # no dispatch events recorded
            assert tm[4] > 0.0, tm                     # the run's bracket still is
            assert [r.stream(i).out for i in range(3)] == want
            r.free()
            monkeypatch.delenv("KLF_SCAN_EVENTS")
            r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=50, stage_times=True)
            tm = r.timing()
            assert all(x > 0.0 for x in (tm[0], tm[3], tm[4], tm[6])), tm
            assert tm[6] <= tm[0] + 1e-3, tm  # the scan is part of the scan stage
            assert [r.stream(i).out for i in range(3)] == want
            r.free()
            r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=50)
            tm = r.timing()
            assert tm[0] == 0.0 and tm[6] > 0.0 and tm[4] >= tm[6], tm
            r.free()


def test_dense_copy_kernel_timed(gpu, monkeypatch):
    """With the one-pass compaction off, a run without patterns and --tail -1 takes the
    dense copy (k_tcopy): timing [7] is its dispatch alone, inside the compaction stage [3];
    on a --tail run (the sparse gather) k_tcopy exits at once.  The one-pass run has no
    k_tcopy."""
    monkeypatch.setenv("KLF_GRAPH", "0")
    streams = [synth.generate(synth.TEXT, 22, i, 16_000_000) for i in range(4)]
    dev, seg_base, lens = _device_batch(streams)
    with E.Engine(0, hip_stream=torch.cuda.current_stream().cuda_stream) as eng:
        r = eng.run_device(dev.data_ptr(), seg_base, lens, stage_times=True)
        assert r.compaction() == "one_pass" and r.timing()[7] == 0.0 and r.timing()[6] > 0.0, r.timing()
        r.free()
    monkeypatch.setenv("KLF_FUSE", "0")
    with E.Engine(0, hip_stream=torch.cuda.current_stream().cuda_stream) as eng:
        r = eng.run_device(dev.data_ptr(), seg_base, lens, stage_times=True)
        tm = r.timing()
        assert tm[7] > 0.0 and tm[7] <= tm[3] + 1e-3, tm
        dense_ms = tm[7]
        want = co.filter_stream(streams[2], co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)[0]
        assert r.stream(2).out == want
        r.free()
        r = eng.run_device(dev.data_ptr(), seg_base, lens, tail=10)
        assert r.timing()[7] < dense_ms, (r.timing(), dense_ms)
        r.free()


def test_no_timing_flag(gpu, monkeypatch):
    """KLF_FILTER_NO_TIMING: the run records no event (timing all zeros, even with stage
    times asked for) and its output is the same; the next default run times again."""
    monkeypatch.setenv("KLF_GRAPH", "0")
    streams = [synth.generate(synth.TEXT, 23, i, 2_000_000) for i in range(2)]
    dev, seg_base, lens = _device_batch(streams)
    since = (synth.T0 + 1800, 0)
    for grep in ([], [synth.NEEDLE]):
        want = [co.filter_stream(s, since, 50, grep, want_lines=False, want_bits=False)[0] for s in streams]
        with E.Engine(0, grep=grep, hip_stream=torch.cuda.current_stream().cuda_stream) as eng:
            for stage in (False, True):
                r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=50, stage_times=stage, timing=False)
                assert r.timing() == [0.0] * 8, r.timing()
                assert [r.stream(i).out for i in range(2)] == want
                r.free()
            r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=50)
            tm = r.timing()
            assert tm[4] > 0.0 and tm[6] > 0.0, tm
            assert [r.stream(i).out for i in range(2)] == want
            r.free()
