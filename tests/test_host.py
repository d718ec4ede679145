"""Host mirror of cmd/root.go (libklogs_host.so + the klogs-filter CLI), no GPU needed."""
import os
import subprocess

import pytest

from klogs_amd import host as H

# /root/reference/cmd/root_test.go:17-23 — the reference's own TestConvertBytes table
# (pterm.Red("0 B") is the ANSI red escape around the text).
CONVERT_BYTES_CASES = [
    ("Zero bytes", 0, "\x1b[31m0 B\x1b[0m"),
    ("Less than 1 KB", 512, "512 B"),
    ("Exactly 1 KB", 1024, "1 KB"),
    ("1.5 KB", 1536, "1 KB"),
    ("Less than 1 MB", 1024 * 512, "512 KB"),
    ("Exactly 1 MB", 1024 * 1024, "1 MB"),
    ("1.5 MB", int(1024 * 1024 * 1.5), "1 MB"),
]


@pytest.mark.parametrize("name,inp,want", CONVERT_BYTES_CASES)
def test_convert_bytes_reference_table(name, inp, want):
    assert H.convert_bytes(inp) == want, name


def test_convert_bytes_no_color():
    assert H.convert_bytes(0, color=False) == "0 B"
    assert H.convert_bytes(5 << 30, color=False) == "5120 MB"


# Go time.ParseDuration known answers (Go src/time/time_test.go parseDurationTests,
# recalled; the reference calls ParseDuration at cmd/root.go:206).
MS, S, M, H_ = 10**6, 10**9, 60 * 10**9, 3600 * 10**9
GOOD_DURATIONS = [
    ("0", 0), ("5s", 5 * S), ("30s", 30 * S), ("1478s", 1478 * S), ("-5s", -5 * S), ("+5s", 5 * S),
    ("-0", 0), ("+0", 0), ("5.0s", 5 * S), ("5.6s", 5 * S + 600 * MS), ("5.s", 5 * S), (".5s", 500 * MS),
    ("1.0s", S), ("1.00s", S), ("1.004s", S + 4 * MS), ("1.0040s", S + 4 * MS), ("100.00100s", 100 * S + 1 * MS),
    ("10ns", 10), ("11us", 11 * 1000), ("12µs", 12 * 1000), ("12μs", 12 * 1000), ("13ms", 13 * MS), ("14s", 14 * S),
    ("15m", 15 * M), ("16h", 16 * H_), ("3h30m", 3 * H_ + 30 * M), ("10.5s4m", 4 * M + 10 * S + 500 * MS),
    ("-2m3.4s", -(2 * M + 3 * S + 400 * MS)), ("1h2m3s4ms5us6ns", H_ + 2 * M + 3 * S + 4 * MS + 5 * 1000 + 6),
    ("39h9m14.425s", 39 * H_ + 9 * M + 14 * S + 425 * MS), ("52763797000ns", 52763797000),
    ("0.3333333333333333333h", 20 * M), ("9007199254740993ns", (1 << 53) + 1),
    ("9223372036854775807ns", (1 << 63) - 1), ("9223372036854775.807us", (1 << 63) - 1),
    ("9223372036s854ms775us807ns", (1 << 63) - 1), ("-9223372036854775808ns", -(1 << 63)),
    ("-9223372036854775.808us", -(1 << 63)), ("-9223372036s854ms775us808ns", -(1 << 63)),
    ("0.100000000000000000000h", 6 * M), ("0.830103483285477580700h", 49 * M + 48 * S + 372539827),
]
BAD_DURATIONS = ["", "3", "-", "s", ".", "-.", ".s", "+.s", "1d", "\x85\x85", "\xffff", "hello \xffff world",
                 "9223372036854775808ns", "9223372036854775.808us", "9223372036854ms775us808ns",
                 "-9223372036854775809ns"]


@pytest.mark.parametrize("s,ns", GOOD_DURATIONS)
def test_parse_duration_good(s, ns):
    assert H.parse_duration(s) == ns


@pytest.mark.parametrize("s", BAD_DURATIONS)
def test_parse_duration_bad(s):
    with pytest.raises(ValueError, match="time: "):
        H.parse_duration(s)


def test_parse_duration_messages():
    with pytest.raises(ValueError, match='time: missing unit in duration "3"'):
        H.parse_duration("3")
    with pytest.raises(ValueError, match='time: unknown unit "d" in duration "1d"'):
        H.parse_duration("1d")


NOW = (1729558801, 250)


def test_lop_opts_since_and_tail():
    # int64(duration.Seconds()) truncates (cmd/root.go:210); since = now - since_s
    assert H.lop_opts("5m", 100, NOW) == ((NOW[0] - 300, 250), 100, False)
    assert H.lop_opts("1.9s", -1, NOW) == ((NOW[0] - 1, 250), -1, False)
    assert H.lop_opts("90m30.5s", 0, NOW) == ((NOW[0] - 5430, 250), 0, False)
    # unset: kubelet's zero-time since, tail -1 (not sent)
    assert H.lop_opts(None, -1, NOW) == ((H.GO_ZERO_TIME_SEC, 0), -1, False)
    assert H.lop_opts("", -1, NOW)[2] is False


def test_lop_opts_server_rejections():
    # ValidatePodLogOptions: sinceSeconds < 1, tailLines < 0 -> stream error, empty file
    assert H.lop_opts("500ms", -1, NOW)[2] is True
    assert H.lop_opts("-5m", -1, NOW)[2] is True
    assert H.lop_opts("0", -1, NOW)[2] is True
    assert H.lop_opts(None, -2, NOW)[2] is True
    assert H.lop_opts(None, -1, NOW)[2] is False


def test_lop_opts_panics_on_bad_duration():
    with pytest.raises(H.GoPanic, match="invalid duration"):
        H.lop_opts("five minutes", -1, NOW)


def test_stream_table_order_init_and_dedupe():
    pods = [("web-1", ["migrate", "warm"], ["app", "sidecar"]),
            ("web-2", [], ["app"]),
            ("web-1", ["migrate"], ["app", "sidecar"])]  # second -l selector hit the same pod
    assert H.stream_table(pods, init=False) == [(0, 0, False), (0, 1, False), (1, 0, False)]
    assert H.stream_table(pods, init=True) == [(0, 0, True), (0, 1, True), (0, 0, False), (0, 1, False),
                                               (1, 0, False)]
    assert H.stream_table([], init=True) == []


def test_file_layout(tmp_path):
    assert H.log_file_name("web-1", "app") == "web-1__app.log"
    lp = tmp_path / "logs" / "2024-10-22T00-00"
    p = H.create_log_file(str(lp), "web-1", "app")
    assert p == str(lp / "web-1__app.log")
    assert os.path.getsize(p) == 0
    assert (os.stat(lp).st_mode & 0o777) == (0o755 & ~_umask())
    # os.Create truncates
    with open(p, "wb") as f:
        f.write(b"old")
    H.create_log_file(str(lp), "web-1", "app")
    assert os.path.getsize(p) == 0


def _umask():
    m = os.umask(0)
    os.umask(m)
    return m


def test_default_log_path_layout():
    p = H.default_log_path(1729555200)
    assert p.startswith("logs/") and len(p) == len("logs/2024-10-22T00-00") and p[15] == "T" and p[18] == "-"


def _manifest(tmp_path, rows):
    m = tmp_path / "manifest.tsv"
    m.write_text("".join("\t".join(r) + "\n" for r in rows))
    return m


def test_cli_rejected_request_leaves_empty_files(tmp_path):
    """--since 500ms: the server rejects every request -> files exist, empty (no GPU used)."""
    body = tmp_path / "b.log"
    body.write_bytes(b"2024-10-22T00:00:00.000000000Z hello\n")
    m = _manifest(tmp_path, [("p1", "container", "app", str(body)), ("p1", "init", "setup", str(body))])
    out = tmp_path / "out"
    r = subprocess.run([str(H.CLI), "-p", str(out), "-s", "500ms", "--no-color", str(m)], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert sorted(os.listdir(out)) == ["p1__app.log"]  # init containers only with -i
    assert os.path.getsize(out / "p1__app.log") == 0
    assert "Error getting logs for container app" in r.stderr
    assert "p1\tapp\t0 B" in r.stdout


def test_cli_bad_since_panics_before_files(tmp_path):
    m = _manifest(tmp_path, [("p1", "container", "app", "-")])
    out = tmp_path / "out"
    r = subprocess.run([str(H.CLI), "-p", str(out), "-s", "soon", str(m)], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 2 and "panic: time: invalid duration" in r.stderr
    assert not out.exists()
