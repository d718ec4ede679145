#!/usr/bin/env python3
"""Prefilter false hits on the GPU against the host emulation of the same layout (C4 shape).

For each layout source (KLF_QF_TUNE=0: placed at open from byte-class estimates; 1: from
the first batch's GPU statistics, as the bench runs) a child process runs C4's generator
(MIXED lines, the 1,024 literals) on 8 streams of --mb MiB each with KLF_DIAG and reports
the scan's bitmap hits (k_verify's walked count) and the layout line; the parent runs the
host emulation (klf_debug_prefilter_hits) on the same bytes, untuned and tuned on a sample
of 64 KiB per stream.  Hits are per 8 KiB tile.

    python scripts/qf_check.py [--mb 32]
"""
import argparse
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def data(mb):
    from klogs_amd import synth
    return [synth.generate(synth.MIXED, 42, i, mb << 20, permille=5) for i in range(8)]


def child(mb):
    from klogs_amd import engine as E
    from klogs_amd import synth
    streams = data(mb)
    with E.Engine(0, grep=synth.c4_literals(1024)) as eng:
        for _ in range(2):
            eng.reset()
            eng.set_streams(len(streams))
            for i, s in enumerate(streams):
                eng.stage(i, s)
            eng.run(n_streams=len(streams)).free()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=32)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.mb)
        return
    from klogs_amd import engine as E
    from klogs_amd import synth
    streams = data(a.mb)
    tiles = sum(len(s) for s in streams) / 8192
    lits = synth.c4_literals(1024)
    sample = b"".join(s[:1 << 16] for s in streams)
    for two in ("1", "0"):
        os.environ["KLF_QF_TWO"] = two
        for name, smp in (("untuned", b""), ("tuned", sample)):
            hb = vb = 0
            for s in streams:
                h = E.debug_prefilter_hits(smp, s, grep=lits)
                hb += h["bitmap_hits"]
                vb += h["verified"]
            print(f"host two={two} {name}: bitmap hits/tile {hb / tiles:.3f} verified/tile {vb / tiles:.3f} "
                  f"[{h['layout']} k={h['k']}]", flush=True)
        for tune in ("0", "1"):
            env = dict(os.environ, KLF_DIAG="1", KLF_QF_TUNE=tune, KLF_QF_TWO=two)
            p = subprocess.run([sys.executable, __file__, "--child", "--mb", str(a.mb)], env=env,
                               capture_output=True, text=True, timeout=300)
            hits = [int(x) for x in re.findall(r"hits=(\d+)", p.stderr)]
            lay = re.findall(r"prefilter layout[^\n]*", p.stderr)
            print(f"gpu  two={two} tune={tune}: rc {p.returncode} hits/tile "
                  f"{[round(x / tiles, 3) for x in hits]} {lay[-1] if lay else ''}", flush=True)
            if p.returncode:
                print(p.stderr[-2000:])
                sys.exit(1)


if __name__ == "__main__":
    main()
