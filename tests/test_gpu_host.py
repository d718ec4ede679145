"""klogs-filter CLI end to end on the GPU: the files it writes equal the C oracle's bytes."""
import os
import subprocess

import pytest

import c_oracle as co
from klogs_amd import host as H
from klogs_amd import synth

pytestmark = pytest.mark.gpu


def test_cli_end_to_end(gpu, tmp_path):
    bodies = {}
    rows = []
    for p in range(3):
        for kind, cname in (("init", "setup"), ("container", "app"), ("container", "sidecar")):
            data = synth.generate(synth.TEXT if p % 2 else synth.JSON, 77, p * 3 + len(cname), 200_000 + 5000 * p)
            f = tmp_path / f"body_{p}_{cname}.log"
            f.write_bytes(data)
            bodies[(f"pod-{p}", cname)] = data
            rows.append((f"pod-{p}", kind, cname, str(f)))
    rows.append(("pod-1", "container", "broken", "-"))  # Stream() failed: empty file
    rows.append(("pod-0", "container", "app", rows[1][3]))  # duplicate from a second -l
    m = tmp_path / "manifest.tsv"
    m.write_text("".join("\t".join(r) + "\n" for r in rows))
    now = synth.T0 + synth.SPAN + 1
    out = tmp_path / "logs"
    r = subprocess.run([str(H.CLI), "-p", str(out), "-s", "20m", "-t", "50", "-i", "--grep", synth.NEEDLE.decode(),
                        "--now", str(now), "--no-color", str(m)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    since, tail, rej = H.lop_opts("20m", 50, (now, 0))
    assert not rej
    names = sorted(os.listdir(out))
    assert names == sorted({H.log_file_name(p, c) for p, c in bodies} | {"pod-1__broken.log"})
    for (p, c), data in bodies.items():
        want, _, _, _ = co.filter_stream(data, since, tail, [synth.NEEDLE], want_lines=False, want_bits=False)
        assert (out / H.log_file_name(p, c)).read_bytes() == want, (p, c)
    assert (out / "pod-1__broken.log").read_bytes() == b""
    assert "Error getting logs for container broken" in r.stderr
    assert "pod-1\tbroken\t0 B" in r.stdout
