"""Output write path: klf_result_write, the replacement of
writeLogToDisk's io.Copy (cmd/root.go:359-374), checked byte-exact against the C oracle
and against the host view of the same result (klf_result_stream)."""
import os

import pytest

import c_oracle as co
import klf_oracle as po
from klogs_amd import engine as E
from klogs_amd import synth

pytestmark = pytest.mark.gpu


def _run(eng, streams, since=None, tail=-1):
    eng.set_streams(len(streams))
    for i, s in enumerate(streams):
        if s:
            eng.stage(i, s)
    return eng.run(since=since, tail=tail, n_streams=len(streams))


def _read(p):
    with open(p, "rb") as f:
        return f.read()


@pytest.mark.parametrize("since,tail,grep", [(None, -1, []), ((synth.T0 + 1200, 0), 10, []),
                                             (None, 5, [synth.NEEDLE])])
def test_write_files_matches_oracle(gpu, tmp_path, since, tail, grep):
    streams = [synth.generate(synth.TEXT, 21, i, 40_000 * (i % 4)) for i in range(7)]
    streams += [b"", b"no newline at all", b"\n\n\n",
                synth.generate(synth.ADVERSARIAL, 4, 1, 400, drop_final_nl=True)]
    paths = [str(tmp_path / f"s{i}.log") for i in range(len(streams))]
    with E.Engine(0, grep=grep) as eng:
        r = _run(eng, streams, since, tail)
        n = r.write_files(paths)
        r.free()
    total = 0
    for i, s in enumerate(streams):
        out = co.filter_stream(s, since or po.GO_ZERO_TIME, tail, list(grep))[0]
        assert _read(paths[i]) == out, f"stream {i}"
        total += len(out)
    assert n == total


def test_write_crosses_pinned_chunks(gpu, tmp_path):
    """~190 MiB of output: three 64 MiB bounce chunks, stream boundaries inside them."""
    streams = [synth.generate(synth.JSON, 3, i, (17 + 13 * i) << 20) for i in range(5)]
    paths = [str(tmp_path / f"s{i}.log") for i in range(len(streams))]
    with E.Engine(0) as eng:
        r = _run(eng, streams)
        n = r.write_files(paths)
        host = [r.stream(i).out for i in range(len(streams))]  # klf_result_stream's D2H
        r.free()
    assert n == sum(len(h) for h in host) > (128 << 20)
    for i in range(len(streams)):
        got = _read(paths[i])
        assert got == host[i], f"stream {i}"
    # spot check one stream against the oracle (the host view is checked elsewhere)
    assert _read(paths[1]) == co.filter_stream(streams[1], po.GO_ZERO_TIME, -1, [])[0]


def test_write_appends_and_skips(gpu, tmp_path):
    """Bytes go at the descriptor's offset (io.Copy into an open file); fd < 0 skips."""
    streams = [synth.generate(synth.TEXT, 8, i, 30_000) for i in range(3)]
    p0, p2 = tmp_path / "a.log", tmp_path / "c.log"
    with E.Engine(0) as eng:
        r = _run(eng, streams, tail=4)
        fd0 = os.open(p0, os.O_WRONLY | os.O_CREAT, 0o644)
        os.write(fd0, b"HEAD\n")
        fd2 = os.open(p2, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            n = r.write_fds([fd0, -1, fd2])
        finally:
            os.close(fd0)
            os.close(fd2)
        h = [r.stream(i).out for i in range(3)]
        # after klf_result_stream the host copy is reused: same bytes again
        p2b = tmp_path / "c2.log"
        assert r.write_files([None, None, str(p2b)]) == len(h[2])
        r.free()
    assert n == len(h[0]) + len(h[2])
    assert _read(p0) == b"HEAD\n" + h[0]
    assert _read(p2) == h[2] == _read(p2b)


def test_write_errors(gpu, tmp_path):
    streams = [synth.generate(synth.TEXT, 2, 0, 20_000)]
    p = tmp_path / "ro.log"
    p.write_bytes(b"")
    with E.Engine(0) as eng:
        r = _run(eng, streams)
        with pytest.raises(E.KlfError) as ei:
            r.write_fds([0, 1])  # wrong stream count
        assert ei.value.code == E.KLF_EINVAL
        fd = os.open(p, os.O_RDONLY)
        try:
            with pytest.raises(E.KlfError) as ei:
                r.write_fds([fd])
            assert ei.value.code == E.KLF_EIO and "stream 0" in str(ei.value)
        finally:
            os.close(fd)
        r2 = r.retail(1)  # the first result is stale now
        with pytest.raises(E.KlfError) as ei:
            r.write_files([str(tmp_path / "x.log")])
        assert ei.value.code == E.KLF_ESTATE
        assert r2.write_files([str(tmp_path / "y.log")]) == len(r2.stream(0).out)
        r2.free()
        r.free()


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_write_threads_offsets_and_fallbacks(gpu, tmp_path, monkeypatch, threads):
    """The threaded path (>= 8 MiB out, distinct descriptors: one worker per file) writes
    at each descriptor's offset and leaves it where write(2) would; O_APPEND works the
    same; a descriptor shared by every stream gets them in stream order.  Same bytes
    every way."""
    monkeypatch.setenv("KLF_WRITE_THREADS", threads)
    streams = [synth.generate(synth.TEXT, 31, i, (3 + 2 * i) << 20) for i in range(4)]
    with E.Engine(0) as eng:
        r = _run(eng, streams)
        n = r.write_files([str(tmp_path / f"p{i}.log") for i in range(4)])
        h = [_read(tmp_path / f"p{i}.log") for i in range(4)]
        assert n == sum(map(len, h)) > (8 << 20)
        assert h[2] == co.filter_stream(streams[2], po.GO_ZERO_TIME, -1, [])[0]
        # headers already in the files, then a second write after the first
        fds = []
        for i in range(4):
            fd = os.open(tmp_path / f"q{i}.log", os.O_WRONLY | os.O_CREAT, 0o644)
            os.write(fd, b"#%d\n" % i)
            fds.append(fd)
        try:
            r.write_fds(fds)
            for fd in fds:
                os.write(fd, b"END\n")
        finally:
            for fd in fds:
                os.close(fd)
        for i in range(4):
            assert _read(tmp_path / f"q{i}.log") == b"#%d\n" % i + h[i] + b"END\n"
        # O_APPEND descriptors
        fds = [os.open(tmp_path / f"a{i}.log", os.O_WRONLY | os.O_CREAT | os.O_APPEND, 0o644) for i in range(4)]
        try:
            r.write_fds(fds)
        finally:
            for fd in fds:
                os.close(fd)
        for i in range(4):
            assert _read(tmp_path / f"a{i}.log") == h[i]
        # one descriptor for every stream: concatenation in stream order
        fd = os.open(tmp_path / "all.log", os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            r.write_fds([fd] * 4)
        finally:
            os.close(fd)
        assert _read(tmp_path / "all.log") == b"".join(h)
        r.free()
