#!/usr/bin/env python3
"""k_verify's phases from a KLF_TIMELINE build (diagnostic): runs a config's filter twice
with the timeline dumped after each run, then prints per-phase cycle quantiles over the hit
threads of the second run (s_memtime stamps; KLF_VSTAMP in klf_kernels.hip).
    KLF_LIB_DIR=klogs_amd/_lib_vtl python3 scripts/vtl.py c5 OUT.bin"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from klogs_amd import engine as E  # noqa: E402

cfg, out = sys.argv[1], sys.argv[2]
sizes, kind, pats, permille, mode, _ = bench.config_table(cfg)
dev, seg_base, lens = bench.load_batch(sizes, kind, permille, list(range(len(sizes))), 0)
now = bench.synth.T0 + bench.synth.SPAN + 1
since, tail = ((None, -1) if mode == "-l" else ((now - bench.SINCE_S, 0), bench.TAIL))
os.environ["KLF_TIMELINE_OUT"] = out
with E.Engine(0, **pats) as eng:
    for _ in range(2):
        eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
t = np.fromfile(out, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
t = t[t[:, 0] > 0]
names = ["start", "loaded", "entry match", "line search", "walk back", "bitmap", "bounds written", "end"]
print(f"{len(t)} threads stamped")
t0 = t[:, 0]
print("phase        reached   cycles from start: p50 / p90 / p99 / max")
for k in range(1, 8):
    m = t[:, k] > 0
    if not m.any():
        continue
    d = t[m, k] - t0[m]
    print(f"{names[k]:14s} {int(m.sum()):8d}   {np.percentile(d, 50):9.0f} {np.percentile(d, 90):9.0f} "
          f"{np.percentile(d, 99):9.0f} {d.max():9.0f}")
span = t[:, 7].max() - t0.min()
print(f"kernel span of stamped threads: {span} cycles")
