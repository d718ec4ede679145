"""Host-side native pieces under the sanitizers (CPU only): the staging copy workers of
klf_stage (klogs_amd/csrc/klf_copypool.hpp) stressed from 8 caller threads under TSAN."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_copypool_tsan(tmp_path):
    exe = tmp_path / "cps"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-pthread",
                    str(ROOT / "tests" / "native" / "copypool_stress.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-2000:]
    assert "copypool: ok" in r.stdout
