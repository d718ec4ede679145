#!/usr/bin/env python3
"""HBM bounds on this MI355X for the byte-moving kernels' rooflines: device-to-device copy
(hipMemcpyAsync through torch), write-only (fill) and read-only (int64 sum) over the C3
per-GPU share's size (8 GiB), HIP events, best of 5.

    python3 scripts/copy_bound.py > profiles/<round>/copy_bound.json"""
import json

import torch

N = 8 << 30


def timed(f, reps=5):
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        f()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / 1e3)
    return best


src = torch.empty(N, dtype=torch.uint8, device="cuda")
dst = torch.empty(N, dtype=torch.uint8, device="cuda")
src.fill_(7)
torch.cuda.synchronize()
t_copy = timed(lambda: dst.copy_(src))
t_fill = timed(lambda: dst.fill_(1))
v = src.view(torch.int64)
t_read = timed(lambda: v.sum())
half = N // 2
t_copy_off = timed(lambda: dst[5:5 + half].copy_(src[0:half]))  # byte-misaligned destination
print(json.dumps({
    "bytes": N,
    "d2d_copy_GBps_read_plus_write": round(2 * N / t_copy / 1e9, 1),
    "fill_write_GBps": round(N / t_fill / 1e9, 1),
    "int64_sum_read_GBps": round(N / t_read / 1e9, 1),
    "misaligned_copy_GBps_read_plus_write": round(2 * half / t_copy_off / 1e9, 1),
    "how": "torch copy_ / fill_ / sum on cuda:0, HIP events, best of 5",
}))
