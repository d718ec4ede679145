#!/usr/bin/env python3
"""Runs one BASELINE config's device-resident filter a few times (profiling driver).

    python scripts/run_config.py c1|c2|c3|c4|c5 [--steps K] [--warmup W]

bench.run_config without the checks, the CPU baseline, the write and capture paths.
Prints the result dict as one JSON line."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--probe", action="store_true", help="add bench.box_probe (the box's copy / read rates)")
    a = ap.parse_args()
    ns = argparse.Namespace(steps=a.steps, warmup=a.warmup, no_verify=True, no_write=True, no_capture=True,
                            no_cpu_baseline=True, capture_piece=4 << 20)
    now = bench.synth.T0 + bench.synth.SPAN + 1
    probe = bench.box_probe(0) if a.probe else None
    out = bench.run_config(a.config, ns, 0, now)
    if probe:
        out["box_probe"] = probe
    print(json.dumps(out))


if __name__ == "__main__":
    main()
