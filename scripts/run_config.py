#!/usr/bin/env python3
"""Runs one BASELINE config's device-resident filter a few times (profiling driver).

    python scripts/run_config.py c2|c3|c4|c5 [--steps K] [--bytes B]

c2 is bench.py's headline workload (one 4 GiB JSON stream, --since 5m --tail 100 --grep);
c3/c4/c5 are bench.run_extra's.  Prints the result dict as one JSON line."""
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
    ap.add_argument("--bytes", type=int, default=32 << 30, help="total bytes of c4 / c5")
    a = ap.parse_args()
    ns = argparse.Namespace(steps=a.steps, warmup=a.warmup, extra_bytes=a.bytes, no_verify=True, no_write=True)
    now = bench.synth.T0 + bench.synth.SPAN + 1
    out = bench.run_extra(a.config, ns, 0, now)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
