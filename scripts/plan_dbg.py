import os, sys
sys.path.insert(0, '/root/repo')
import numpy as np


def run(plan, n, size):
    os.environ["KLF_PLAN_RUNS"] = plan
    import torch
    from klogs_amd import engine as E, synth
    lens = [synth.size(synth.TEXT, 42, i, size) for i in range(n)]
    base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    h = np.empty(max(lens) + 1, dtype=np.uint8)
    for i, m in enumerate(lens):
        synth.generate_into(h, synth.TEXT, 42, i, size)
        dev[int(base[i]):int(base[i]) + m].copy_(torch.from_numpy(h[:m]))
    torch.cuda.synchronize()
    with E.Engine(0) as eng:
        r = eng.run_device(dev.data_ptr(), base, lens)
        got = [(r.stream(i).out, dict(r.stream(i).counts)) for i in range(n)]
        r.free()
    del dev
    return got


if __name__ == "__main__":
    for n in (int(x) for x in sys.argv[1:]):
        a = run("1", n, 64 << 20)
        b = run("0", n, 64 << 20)
        bad = [i for i in range(n) if a[i] != b[i]]
        print(n, "streams: differing", len(bad), bad[:5], flush=True)
        for i in bad[:3]:
            print("  ", i, a[i][1], b[i][1], len(a[i][0]), len(b[i][0]), flush=True)
