"""In-tree build of the native pieces (no JIT cache: the .so files travel to the GPU box).

* ``klogs_amd/_lib/libklf.so``       — the engine: HIP kernels for gfx950 + the C ABI
  of ``include/klf.h`` + the pattern compiler.
* ``klogs_amd/_lib/libklogs_host.so`` and ``klogs_amd/_lib/klogs-filter`` — the C++ host
  mirror of ``cmd/root.go`` (flags, stream table, file layout) over the C ABI.
* ``klogs_amd/_lib/libklf_synth.so``  — seeded synthetic log generator (tests / bench).
* ``oracle/_build/libklf_oracle.so``  — the C oracle (test infrastructure only).
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "klogs_amd" / "csrc"
LIB = ROOT / "klogs_amd" / "_lib"
ORACLE = ROOT / "oracle"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("KLF_OFFLOAD_ARCH", "gfx950")

ENGINE_SRCS = ["klf_kernels.hip", "klf_engine.cpp", "klf_patterns.cpp"]
ENGINE_HDRS = ["klf_kernels.hpp", "klf_patterns.hpp", "klf_ts.hpp", "klf_copypool.hpp"]


def _stale(out: Path, deps) -> bool:
    if not out.exists():
        return True
    t = out.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, quiet):
    if not quiet:
        print("+", " ".join(map(str, cmd)), file=sys.stderr)
    subprocess.run([str(c) for c in cmd], check=True)


def build_engine(force=False, quiet=True) -> Path:
    LIB.mkdir(parents=True, exist_ok=True)
    out = LIB / "libklf.so"
    hdrs = [CSRC / h for h in ENGINE_HDRS] + [ROOT / "include" / "klf.h", ROOT / "include" / "klf_debug.h"]
    objs = []
    for src in ENGINE_SRCS:
        s = CSRC / src
        o = LIB / (src.replace(".", "_") + ".o")
        if force or _stale(o, [s] + hdrs):
            if src.endswith(".cpp"):  # host code: plain C++ against the HIP runtime headers
                cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__",
                       "-I/opt/rocm/include", "-c", s, "-o", o]
            else:
                cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                       "-Wno-unused-function", "-c", s, "-o", o]
            _run(cmd, quiet)
        objs.append(o)
    if force or _stale(out, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out], quiet)
    return out


def build_synth(force=False, quiet=True) -> Path:
    LIB.mkdir(parents=True, exist_ok=True)
    out = LIB / "libklf_synth.so"
    src = CSRC / "klf_synth.c"
    if force or _stale(out, [src]):
        _run(["gcc", "-O2", "-shared", "-fPIC", "-pthread", src, "-o", out, "-lm"], quiet)
    return out


def build_host(force=False, quiet=True):
    src = CSRC / "klogs_host.cpp"
    if not src.exists():
        return None
    LIB.mkdir(parents=True, exist_ok=True)
    so = LIB / "libklogs_host.so"
    exe = LIB / "klogs-filter"
    deps = [src, ROOT / "include" / "klogs_host.h", ROOT / "include" / "klf.h", LIB / "libklf.so"]
    deps = [d for d in deps if Path(d).exists()]
    if force or _stale(so, deps):
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-shared", "-fPIC", src, "-o", so], quiet)
    cli = CSRC / "klogs_filter_main.cpp"
    if cli.exists() and (force or _stale(exe, deps + [cli, so])):
        _run(["g++", "-O2", "-std=c++17", "-Wall", cli, "-o", exe, f"-L{LIB}", "-lklogs_host", "-lklf",
              "-Wl,-rpath,$ORIGIN"], quiet)
    return so


def build_oracle(force=False, quiet=True) -> Path:
    out_dir = ORACLE / "_build"
    out_dir.mkdir(parents=True, exist_ok=True)
    out = out_dir / "libklf_oracle.so"
    srcs = [ORACLE / "klf_oracle_c.c", ORACLE / "klf_oracle_rx.c"]
    if force or _stale(out, srcs):
        _run(["gcc", "-O2", "-Wall", "-shared", "-fPIC", *srcs, "-o", out], quiet)
    return out


def build_all(force=False, quiet=True):
    build_engine(force, quiet)
    build_synth(force, quiet)
    build_host(force, quiet)
    build_oracle(force, quiet)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, quiet=False)
