#!/usr/bin/env python3
"""The bench's one-shot measurement (bench.cold_run: a fresh engine, its first run, its
second run) with KLF_DIAG's marks, after a warm-up engine has loaded the code objects:
    KLF_DIAG=1 python scripts/cold_diag.py c5|c2|c4|c3
The marks of the cold engine's runs go to stderr after the line '== cold engine'."""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import torch  # noqa: E402

import bench  # noqa: E402
from klogs_amd import engine as E  # noqa: E402


def main():
    name = sys.argv[1]
    sizes, kind, pats, permille, mode, _ = bench.config_table(name)
    dev, seg_base, lens = bench.load_batch(sizes, kind, permille, list(range(len(sizes))), 0)
    now = bench.synth.T0 + bench.synth.SPAN + 1
    since, tail = ((None, -1) if mode == "-l" else ((now - bench.SINCE_S, 0), bench.TAIL))
    st = torch.cuda.current_stream().cuda_stream
    with E.Engine(0, hip_stream=st, **pats) as w:  # the code objects, the allocator
        for _ in range(3):
            w.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
    torch.cuda.synchronize()
    time.sleep(0.2)
    # the same warm engine after an idle gap: what a one-shot run pays for the board's state
    with E.Engine(0, hip_stream=st, **pats) as w:
        for _ in range(3):
            w.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
        torch.cuda.synchronize()
        res = {}
        for gap_ms in (0, 1, 3, 10, 30):
            ts = []
            for _ in range(3):
                time.sleep(gap_ms / 1e3)
                t0 = time.perf_counter()
                w.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
                ts.append((time.perf_counter() - t0) * 1e3)
            res[gap_ms] = round(min(ts), 3), round(sum(ts) / len(ts), 3)
        print({"warm_run_after_idle_gap_ms": res}, flush=True)
    print("== cold engine", file=sys.stderr, flush=True)
    print(bench.cold_run(0, pats, dev.data_ptr(), seg_base, lens, since, tail), flush=True)
    print(bench.cold_run(0, pats, dev.data_ptr(), seg_base, lens, since, tail), flush=True)


if __name__ == "__main__":
    main()
