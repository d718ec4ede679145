"""Scan-kernel time of libklf variants (KLF_LIB_DIR) on 4 GiB of C4 (1,024 literals) and
C5 (64 regexes) data; median of 8 runs.  Timing-only; ablated builds give wrong output."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from klogs_amd import engine as E, synth
res = {"lib": os.environ.get("KLF_LIB_DIR", "default")}
for name, kind, pats in (("c4", synth.MIXED, dict(grep=synth.c4_literals(1024))),
                         ("c5", synth.LONGJSON, dict(match=synth.c5_regexes()))):
    lens = [synth.size(kind, 42, i, 512 << 20, permille=5) for i in range(8)]
    base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    for i, n in enumerate(lens):
        h = np.empty(n + 1, np.uint8); synth.generate_into(h, kind, 42, i, 512 << 20, permille=5)
        dev[int(base[i]):int(base[i]) + n].copy_(torch.from_numpy(h[:n]))
    torch.cuda.synchronize()
    for tag, kw in (("plain", {}), ("gen", pats)):
        eng = E.Engine(0, **kw)
        ts = []
        for i in range(10):
            r = eng.run_device(dev.data_ptr(), base, lens, since=(synth.T0 + 3301, 0), tail=100, stage_times=True)
            ts.append(r.timing()); tot = r.totals(); r.free()
        ts = np.array(ts[2:])
        res[f"{name}_{tag}"] = {"scan_ms": round(float(np.median(ts[:, 6])), 3), "match_ms": round(float(np.median(ts[:, 1])), 3),
                                "total_ms": round(float(np.median(ts[:, 4])), 3), "matched": tot["matched"]}
        eng.close()
    del dev
    torch.cuda.empty_cache()
print(json.dumps(res))
