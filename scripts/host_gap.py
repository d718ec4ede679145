#!/usr/bin/env python3
"""Host-side cost of one C2-shaped step (diagnostic): wall time of run_device + timing()
+ free() against the device time of the run, over N steps on one 256 MiB JSON stream."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from klogs_amd import engine as E  # noqa: E402
from klogs_amd import synth  # noqa: E402

n = 256 << 20
ln = synth.size(synth.JSON, 42, 0, n)
h = np.empty(ln + 1, dtype=np.uint8)
synth.generate_into(h, synth.JSON, 42, 0, n)
seg_base, total = E.layout([ln])
dev = torch.empty(total, dtype=torch.uint8, device="cuda:0")
dev[:ln].copy_(torch.from_numpy(h[:ln]))
torch.cuda.synchronize()
eng = E.Engine(0, grep=[synth.NEEDLE], hip_stream=torch.cuda.current_stream().cuda_stream)
since = (synth.T0 + synth.SPAN - 300, 0)
for _ in range(5):
    eng.run_device(dev.data_ptr(), seg_base, [ln], since=since, tail=100).free()
K = 200
t_run = t_tm = t_free = 0.0
dev_ms = 0.0
t0 = time.perf_counter()
for _ in range(K):
    a = time.perf_counter()
    r = eng.run_device(dev.data_ptr(), seg_base, [ln], since=since, tail=100)
    b = time.perf_counter()
    tm = r.timing()
    c = time.perf_counter()
    r.free()
    d = time.perf_counter()
    t_run += b - a
    t_tm += c - b
    t_free += d - c
    dev_ms += tm[4]
wall = time.perf_counter() - t0
print(f"per step: wall {wall / K * 1e6:.1f} us, run_device {t_run / K * 1e6:.1f} us, device {dev_ms / K * 1e3:.1f} us, "
      f"timing() {t_tm / K * 1e6:.1f} us, free() {t_free / K * 1e6:.1f} us")
