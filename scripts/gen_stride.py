"""k_scan<gen> time by sampling stride on one 4 GiB mixed-line stream: a long-needle literal
set (stride 8), the same set plus one 9-byte literal (stride 4), and no patterns."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from klogs_amd import engine as E, synth
n = synth.size(synth.MIXED, 42, 0, 4 << 30, permille=5)
host = np.empty(n + 1, np.uint8); synth.generate_into(host, synth.MIXED, 42, 0, 4 << 30, permille=5)
base, total = E.layout([n])
dev = torch.empty(total, dtype=torch.uint8, device="cuda"); dev[:n].copy_(torch.from_numpy(host[:n])); torch.cuda.synchronize()
lits = [l for l in synth.c4_literals(1024) if len(l) >= 12][:300]
res = {}
for name, g in (("stride8", lits), ("stride4", lits + [b"zq_9bytes"]), ("plain", [])):
    info = E.debug_prefilter(b"", grep=g)[1] if g else {}
    eng = E.Engine(0, grep=g)
    ts = []
    for i in range(8):
        r = eng.run_device(dev.data_ptr(), base, [n], since=(synth.T0 + 3301, 0), tail=100)
        ts.append(r.timing()); r.free()
    ts = np.array(ts[2:])
    res[name] = {"stride": info.get("stride"), "k_scan_ms": round(float(np.median(ts[:, 6])), 4),
                 "total_ms": round(float(np.median(ts[:, 4])), 4)}
    eng.close()
print(json.dumps(res))
