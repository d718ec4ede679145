import sys, os, ctypes
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
mode = sys.argv[1]
if mode == "torch_first":
    import torch
    print("torch avail", torch.cuda.is_available())
from klogs_amd import engine as E
maps = open("/proc/self/maps").read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip" in l or "hsa-runtime" in l)))
try:
    e = E.Engine(0)
    print("engine ok")
    e.close()
except Exception as ex:
    print("engine fail", ex)
