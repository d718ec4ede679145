#!/usr/bin/env python3
"""C1's one-shot cost on fresh engines in a warm process (diagnostic): bench.cold_run
repeated, per KLF_PLAN_MODE, with the first run's KLF_DIAG marks on stderr.
    python3 scripts/cold_probe.py c1"""
import os
import sys
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
# warm the process as the bench does before its C1 line (another engine's runs)
with E.Engine(0, **pats) as eng:
    for _ in range(5):
        eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
for pm in ("0", "2", "0", "2"):
    os.environ["KLF_PLAN_MODE"] = pm
    res = [bench.cold_run(0, pats, dev.data_ptr(), seg_base, lens, since, tail) for _ in range(4)]
    print(f"plan {pm}: first_run_ms {[r['first_run_ms'] for r in res]} second {[r['second_run_ms'] for r in res]}",
          flush=True)
