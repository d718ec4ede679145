"""Times the scan stage of libklf variants (KLF_LIB_DIR) on the bench stream: with and
without the literal, median of 10 runs.  Timing-only; ablated builds give wrong output."""
import json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from klogs_amd import engine as E, synth
n = synth.size(synth.JSON, 42, 0, 4 << 30)
host = np.empty(n + 1, np.uint8); synth.generate_into(host, synth.JSON, 42, 0, 4 << 30)
base, total = E.layout([n])
dev = torch.empty(total, dtype=torch.uint8, device="cuda"); dev[:n].copy_(torch.from_numpy(host[:n])); torch.cuda.synchronize()
res = {"lib": os.environ.get("KLF_LIB_DIR", "default")}
for name, grep in (("nogrep", []), ("lit", [synth.NEEDLE])):
    eng = E.Engine(0, grep=grep)
    ts = []
    for i in range(12):
        r = eng.run_device(dev.data_ptr(), base, [n], since=(synth.T0 + 3301, 0), tail=100, stage_times=True)
        ts.append(r.timing()); r.free()
    ts = np.array(ts[2:])
    res[name] = {"scan_ms": float(np.median(ts[:, 0])), "total_ms": float(np.median(ts[:, 4])),
                 "k_scan_ms": float(np.median(ts[:, 6]))}
    eng.close()
print(json.dumps(res))
