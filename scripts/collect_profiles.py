#!/usr/bin/env python3
"""Copies one scripts/profile_round.sh result into profiles/<round> and derives what the
bench line cites from it:

    python3 scripts/collect_profiles.py gpurun_out/<tag> profiles/r02

  bench.json / bench_kernel_stats.csv    the driver's bench command and its kernel trace
  <cfg>_kernel_stats.csv                 per-config kernel traces (C3, C5)
  pmc_<cfg>.json                         per-kernel counter means (FETCH_SIZE x2, KiB -> B)
  traffic.json                           per-launch HBM bytes of C2's k_scan<1, ...> (bench.py
                                         reads it as roofline.traffic)
  summary.md                             per config: dominant kernel, trace average, the
                                         rocprof-derived roofline fraction beside the bench's
                                         HIP-event one, traffic / algorithmic bytes
"""
import csv
import json
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PEAK = 8000.0  # GB/s


def short(name):
    return re.sub(r"\(.*", "", name.replace("klf::(anonymous namespace)::", "").replace("void ", "")).strip()


def stats(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        rows[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                  "pct": float(r["Percentage"])}
    return rows


def steady_us(trace_csv, kernel):
    """Mean launch duration of `kernel` without its first launch (the warm-up the bench
    leaves out of its timed region too)."""
    if not Path(trace_csv).exists():
        return None
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(trace_csv))
         if short(r["Kernel_Name"]) == kernel]
    return sum(d[1:]) / len(d[1:]) if len(d) > 1 else None


def last_json(path):
    lines = [x for x in Path(path).read_text().splitlines() if x.startswith("{")]
    return json.loads(lines[-1])


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    shutil.copy(src / "bench.json", dst / "bench.json")
    shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / "bench_kernel_stats.csv")
    for c in ("c3", "c4", "c5"):
        f = src / f"trace_{c}" / "run_kernel_stats.csv"
        if f.exists():
            shutil.copy(f, dst / f"{c}_kernel_stats.csv")
    pmc = {}
    for c in ("c2", "c3", "c4", "c5"):
        d = src / f"pmc_{c}"
        if d.exists():
            subprocess.run([sys.executable, str(ROOT / "scripts/pmc_summary.py"), str(d), "--json",
                            str(dst / f"pmc_{c}.json")], check=True, stdout=subprocess.DEVNULL)
            pmc[c] = json.loads((dst / f"pmc_{c}.json").read_text())
    b = last_json(dst / "bench.json")
    tr = stats(dst / "bench_kernel_stats.csv")
    lines = ["# Profiles of this round", "",
             "Made by `scripts/profile_round.sh` on one MI355X (the driver's bench command under",
             "`rocprofv3 --kernel-trace --stats`, then counter passes per config) and",
             "`scripts/collect_profiles.py`.  frac = algorithmic bytes / average launch / 8 TB/s.", "",
             "| config | kernel | alg bytes / launch | config-run trace avg (µs) | frac (rocprof) | avg w/o 1st launch (µs; bench trace, C3: its config trace) | frac (rocprof, steady) | frac (bench HIP events) | HBM traffic / alg |",
             "|---|---|---|---|---|---|---|---|---|"]
    out = {}
    # C2: the headline line
    k2 = next(k for k in tr if k.startswith("k_scan<1"))
    alg2 = b["roofline"]["alg_bytes_per_launch"]
    fr2 = alg2 / (tr[k2]["avg_us"] * 1e-6) / 1e9 / PEAK
    t2 = None
    if "c2" in pmc and k2 in pmc["c2"]:
        p = pmc["c2"][k2]
        t2 = p.get("fetch_bytes_x2", 0) + p.get("write_bytes", 0)
        json.dump({"kernel": k2, "fetch_bytes": round(p.get("fetch_bytes_x2", 0)),
                   "write_bytes": round(p.get("write_bytes", 0)), "traffic_bytes": round(t2),
                   "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> B",
                   "sources": [str(src / "pmc_c2")]}, open(dst / "traffic.json", "w"), indent=1)
    st2 = steady_us(src / "trace" / "run_kernel_trace.csv", k2)
    fs2 = st2 and alg2 / (st2 * 1e-6) / 1e9 / PEAK
    out["c2"] = {"kernel": k2, "avg_us": tr[k2]["avg_us"], "frac_rocprof": round(fr2, 4),
                 "steady_us": st2 and round(st2, 1), "frac_rocprof_steady": fs2 and round(fs2, 4),
                 "frac_hip": b["roofline"]["frac"], "traffic_over_alg": t2 and round(t2 / alg2, 3)}
    lines.append(f"| C2 | `{k2}` | {alg2} | {tr[k2]['avg_us']:.1f} | {fr2:.4f} | "
                 f"{'%.1f' % st2 if st2 else '—'} | {'%.4f' % fs2 if fs2 else '—'} | {b['roofline']['frac']} | "
                 f"{'%.3f' % (t2 / alg2) if t2 else '—'} |")
    for c in ("c3", "c4", "c5"):
        f = dst / f"{c}_kernel_stats.csv"
        ex = b.get("extra", {}).get("configs", {}).get(c)
        if not f.exists() or not ex:
            continue
        ts = stats(f)
        ks = next(k for k in ts if k.startswith("k_scan<"))
        alg = ex["bytes"]
        fr = alg / (ts[ks]["avg_us"] * 1e-6) / 1e9 / PEAK
        tt = None
        if c in pmc and ks in pmc[c]:
            p = pmc[c][ks]
            tt = p.get("fetch_bytes_x2", 0) + p.get("write_bytes", 0)
        # steady state from the bench command's own trace (the line's numbers come from that
        # run), except C3: its scan instantiation also serves C1 there (k_scan<0,...>), so
        # C3's comes from its own config run
        tr_bench = src / "trace" / "run_kernel_trace.csv"
        tr_cfg = src / f"trace_{c}" / "run_kernel_trace.csv"
        st = (steady_us(tr_cfg, ks) or steady_us(tr_bench, ks)) if c == "c3" else \
            (steady_us(tr_bench, ks) or steady_us(tr_cfg, ks))
        fs = st and alg / (st * 1e-6) / 1e9 / PEAK
        out[c] = {"kernel": ks, "avg_us": ts[ks]["avg_us"], "frac_rocprof": round(fr, 4),
                  "steady_us": st and round(st, 1), "frac_rocprof_steady": fs and round(fs, 4),
                  "frac_hip": ex["roofline"]["frac"], "traffic_over_alg": tt and round(tt / alg, 3),
                  "kernels": {k: round(v["avg_us"], 1) for k, v in sorted(ts.items(), key=lambda kv: -kv[1]["pct"])[:8]}}
        lines.append(f"| {c.upper()} | `{ks}` | {alg} | {ts[ks]['avg_us']:.1f} | {fr:.4f} | "
                     f"{'%.1f' % st if st else '—'} | {'%.4f' % fs if fs else '—'} | {ex['roofline']['frac']} | "
                     f"{'%.3f' % (tt / alg) if tt else '—'} |")
    lines += ["", "Per-config kernel split (trace averages, µs):", ""]
    for c, v in out.items():
        if "kernels" in v:
            lines.append(f"* {c.upper()}: " + ", ".join(f"`{k}` {t}" for k, t in v["kernels"].items()))
    (dst / "summary.md").write_text("\n".join(lines) + "\n")
    json.dump(out, open(dst / "summary.json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
