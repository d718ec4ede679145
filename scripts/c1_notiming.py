#!/usr/bin/env python3
"""C1's step with and without the run's timing events (KLF_FILTER_NO_TIMING), same engine,
alternating blocks of steps (diagnostic).    python3 scripts/c1_notiming.py [cfg]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
import torch  # noqa: E402
from klogs_amd import engine as E  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
sizes, kind, pats, permille, mode, _ = bench.config_table(cfg)
dev, seg_base, lens = bench.load_batch(sizes, kind, permille, list(range(len(sizes))), 0)
now = bench.synth.T0 + bench.synth.SPAN + 1
since, tail = (now - bench.SINCE_S, 0), bench.TAIL
with E.Engine(0, hip_stream=torch.cuda.current_stream().cuda_stream, **pats) as eng:
    for _ in range(10):
        eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
    res = {True: [], False: []}
    for rnd in range(6):
        for timing in (True, False):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(100):
                eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail, timing=timing).free()
            torch.cuda.synchronize()
            res[timing].append((time.perf_counter() - t0) / 100 * 1e3)
    for k, v in res.items():
        print(f"{cfg} timing={k}: ms per step {sorted(v)}", flush=True)
