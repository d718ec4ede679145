#!/usr/bin/env python3
"""Does C3's copy read its input from the Infinity Cache (MALL, 256 MiB) when the batch is
small?  Runs the C3 pipeline (TEXT streams of 64 MiB, -l only: every line out, dense
compaction) on batches of 1 .. 128 streams and prints per-GB stage times (scan stage,
compaction stage) -- a small batch's k_tcopy re-reads bytes k_scan has just streamed.

    python scripts/mall_probe.py [--streams 1,2,4,8,16,128]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from klogs_amd import engine as E  # noqa: E402
from klogs_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", default="1,2,4,8,16,128")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    ns = [int(x) for x in a.streams.split(",")]
    size = 64 << 20
    lens_all = [synth.size(synth.TEXT, 42, i, size) for i in range(max(ns))]
    seg_base, total = E.layout(lens_all)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda:0")
    h = np.empty(max(lens_all) + 1, dtype=np.uint8)
    for i, n in enumerate(lens_all):
        synth.generate_into(h, synth.TEXT, 42, i, size)
        dev[int(seg_base[i]):int(seg_base[i]) + n].copy_(torch.from_numpy(h[:n]))
    torch.cuda.synchronize()
    eng = E.Engine(0, hip_stream=torch.cuda.current_stream().cuda_stream)
    for n in ns:
        lens = lens_all[:n]
        sb, _ = E.layout(lens)
        out = []
        for r in range(a.reps + 1):
            res = eng.run_device(dev.data_ptr(), sb, lens, stage_times=True)
            if r:
                out.append(res.timing())
            res.free()
        t = np.mean(np.array(out), axis=0)
        gb = sum(lens) / 1e9
        print(json.dumps({"streams": n, "GB": round(gb, 3), "scan_ms_per_GB": round(t[0] / gb, 4),
                          "compaction_ms_per_GB": round(t[3] / gb, 4), "total_ms_per_GB": round(t[4] / gb, 4),
                          "stage_ms": [round(x, 4) for x in t]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
