#!/bin/bash
# Round 6: where a graph-replayed C1 step spends its host time
set -e
cd "$(dirname "$0")/.."
o=gpurun_out/r6r; mkdir -p $o
KLF_DIAG=1 timeout -k 10 120 python scripts/run_config.py c1 --steps 10 --warmup 3 > $o/c1_diag.json 2> $o/c1_diag.err
python3 - <<'P' > $o/steps.txt 2>&1
import time, os, sys
sys.path.insert(0, ".")
import bench, torch
from klogs_amd import engine as E
sizes, kind, pats, permille, mode, _ = bench.config_table("c1")
dev, seg_base, lens = bench.load_batch(sizes, kind, permille, [0], 0)
now = bench.synth.T0 + bench.synth.SPAN + 1
since, tail = (now - bench.SINCE_S, 0), bench.TAIL
for g in ("0", "1"):
    os.environ["KLF_GRAPH"] = g
    with E.Engine(0, **pats) as eng:
        for _ in range(5):
            eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail).free()
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            r = eng.run_device(dev.data_ptr(), seg_base, lens, since=since, tail=tail)
            t1 = time.perf_counter()
            tm = r.timing()
            r.free()
            t2 = time.perf_counter()
            ts.append((t1 - t0, t2 - t1, tm[4]))
        import numpy as np
        a = np.array(ts)
        print(f"KLF_GRAPH={g}: run {np.median(a[:,0])*1e6:.1f} us, timing+free {np.median(a[:,1])*1e6:.1f} us, device {np.median(a[:,2])*1e3:.1f} us; mean run {a[:,0].mean()*1e6:.1f}")
P
cat $o/steps.txt
echo "r6r done"
