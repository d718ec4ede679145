"""Runs the diagnostic (KLF_TIMELINE) build on the bench stream and writes the per-tile
scan timeline to gpurun_out/timeline.bin (8 u64 per tile)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
os.environ["KLF_LIB_DIR"] = "klogs_amd/_lib_tl"
from klogs_amd import engine as E, synth
n = synth.size(synth.JSON, 42, 0, 4 << 30)
host = np.empty(n + 1, np.uint8); synth.generate_into(host, synth.JSON, 42, 0, 4 << 30)
base, total = E.layout([n])
dev = torch.empty(total, dtype=torch.uint8, device="cuda"); dev[:n].copy_(torch.from_numpy(host[:n])); torch.cuda.synchronize()
for name, grep in (("nogrep", []), ("lit", [synth.NEEDLE])):
    eng = E.Engine(0, grep=grep)
    for i in range(3):
        if i == 2:
            os.environ["KLF_TIMELINE_OUT"] = f"gpurun_out/timeline_{name}{i}.bin"
        else:
            os.environ.pop("KLF_TIMELINE_OUT", None)
        r = eng.run_device(dev.data_ptr(), base, [n], since=(synth.T0 + 3301, 0), tail=100)
        print(name, r.timing()); r.free()
    eng.close()
