"""Post-scan stage timings on the 4 GiB bench stream for several filters (run under
rocprofv3 --kernel-trace to split the stages into kernels)."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from klogs_amd import engine as E, synth
n = synth.size(synth.JSON, 42, 0, 4 << 30, permille=10)
host = np.empty(n + 1, np.uint8); synth.generate_into(host, synth.JSON, 42, 0, 4 << 30, permille=10)
base, total = E.layout([n])
dev = torch.empty(total, dtype=torch.uint8, device="cuda"); dev[:n].copy_(torch.from_numpy(host[:n])); torch.cuda.synchronize()
now = synth.T0 + synth.SPAN + 1
for name, grep, since, tail in [("grep_t100", [synth.NEEDLE], (now - 300, 0), 100),
                                ("grep_t10000", [synth.NEEDLE], (now - 300, 0), 10000),
                                ("nogrep_t100", [], (now - 300, 0), 100),
                                ("nogrep_all", [], None, -1)]:
    eng = E.Engine(0, grep=grep)
    ts = []
    for i in range(6):
        r = eng.run_device(dev.data_ptr(), base, [n], since=since, tail=tail)
        ts.append(r.timing()); tot = r.totals(); r.free()
    eng.close()
    print(json.dumps({"case": name, "stage_ms": [round(float(x), 4) for x in np.median(np.array(ts[2:]), axis=0)],
                      "selected": tot["selected"], "out_bytes": tot["out_bytes"]}), flush=True)
