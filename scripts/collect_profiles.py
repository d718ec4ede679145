#!/usr/bin/env python3
"""Copies one scripts/profile_round.sh result into profiles/<round> and derives what the
bench line cites from it:

    python3 scripts/collect_profiles.py gpurun_out/<tag> profiles/r05

  bench.json / bench_kernel_stats.csv    the driver's bench command and its kernel trace
  <cfg>_kernel_stats.csv                 per-config kernel traces (scripts/run_config.py)
  pmc_<cfg>.json                         per-kernel counter means (FETCH_SIZE x2, KiB -> B)
  traffic.json                           per config: per-launch HBM bytes of the roofline
                                         kernel (bench.py reads the headline's as
                                         roofline.traffic)
  summary.md / summary.json              per config: the roofline kernel (k_scan, C3:
                                         k_tcopy), its steady trace average, the rocprof
                                         roofline fraction beside the bench's HIP-event one,
                                         traffic / algorithmic bytes, the kernel split
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
CONFIGS = ("c5", "c2", "c3", "c4")


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


def bench_entry(b, c):
    """(roofline dict, bytes of the config) of config c in a bench line."""
    if c == "c5":
        return b["roofline"], b["extra"]["headline"]
    ex = b.get("extra", {}).get("configs", {}).get(c)
    return (ex["roofline"], ex) if ex and "roofline" in ex else (None, None)


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    shutil.copy(src / "bench.json", dst / "bench.json")
    shutil.copy(src / "trace" / "run_kernel_stats.csv", dst / "bench_kernel_stats.csv")
    for c in CONFIGS:
        f = src / f"trace_{c}" / "run_kernel_stats.csv"
        if f.exists():
            shutil.copy(f, dst / f"{c}_kernel_stats.csv")
    pmc = {}
    for c in CONFIGS:
        d = src / f"pmc_{c}"
        if d.exists():
            subprocess.run([sys.executable, str(ROOT / "scripts/pmc_summary.py"), str(d), "--json",
                            str(dst / f"pmc_{c}.json")], check=True, stdout=subprocess.DEVNULL)
            pmc[c] = json.loads((dst / f"pmc_{c}.json").read_text())
    b = last_json(dst / "bench.json")
    lines = ["# Profiles of this round", "",
             "Made by `scripts/profile_round.sh` on one MI355X (the driver's bench command under",
             "`rocprofv3 --kernel-trace --stats`, per-config traces of `scripts/run_config.py`, then counter",
             "passes per config) and `scripts/collect_profiles.py`.  frac = algorithmic bytes per launch /",
             "average launch / 8 TB/s; the steady average leaves the kernel's first launch out (C5, C2, C4: in the",
             "bench trace; C3: in its config run).", "",
             "| config | roofline kernel | alg bytes / launch | trace avg (µs) | steady avg (µs) | frac (rocprof, steady) "
             "| frac (bench HIP events) | HBM traffic / launch | traffic / alg |",
             "|---|---|---|---|---|---|---|---|---|"]
    out, traffic = {}, {}
    for c in CONFIGS:
        f = dst / f"{c}_kernel_stats.csv"
        roof, ex = bench_entry(b, c)
        if not f.exists() or roof is None:
            continue
        ts = stats(f)
        want = "k_tcopy" if roof["kernel"] == "k_tcopy" else "k_scan<"
        ks = next((k for k in ts if k.startswith(want)), None)
        if ks is None:
            continue
        alg = roof["alg_bytes_per_launch"]
        # steady state from the bench command's own trace (the line's numbers come from that
        # run) where the kernel is the config's alone there; C3's k_tcopy / plain scan also
        # run for other configs in that trace: its config run's
        st = steady_us(src / "trace" / "run_kernel_trace.csv", ks) if c != "c3" else None
        st = st or steady_us(src / f"trace_{c}" / "run_kernel_trace.csv", ks)
        fs = st and alg / (st * 1e-6) / 1e9 / PEAK
        tt = None
        if c in pmc and ks in pmc[c]:
            p = pmc[c][ks]
            tt = p.get("fetch_bytes_x2", 0) + p.get("write_bytes", 0)
            traffic[c] = {"kernel": ks, "fetch_bytes": round(p.get("fetch_bytes_x2", 0)),
                          "write_bytes": round(p.get("write_bytes", 0)), "traffic_bytes": round(tt),
                          "alg_bytes": alg,
                          "correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE x1; KiB -> B",
                          "source": str(src / f"pmc_{c}")}
        out[c] = {"kernel": ks, "alg_bytes": alg, "avg_us": round(ts[ks]["avg_us"], 1),
                  "steady_us": st and round(st, 1), "frac_rocprof_steady": fs and round(fs, 4),
                  "frac_hip": roof["frac"], "traffic_bytes": tt and round(tt),
                  "traffic_over_alg": tt and round(tt / alg, 3),
                  "kernels": {k: round(v["avg_us"], 1) for k, v in sorted(ts.items(), key=lambda kv: -kv[1]["pct"])[:10]}}
        lines.append(f"| {c.upper()} | `{ks}` | {alg} | {ts[ks]['avg_us']:.1f} | {'%.1f' % st if st else '—'} | "
                     f"{'%.4f' % fs if fs else '—'} | {roof['frac']} | {'%.4g' % tt if tt else '—'} | "
                     f"{'%.3f' % (tt / alg) if tt else '—'} |")
    if traffic:
        json.dump(traffic, open(dst / "traffic.json", "w"), indent=1)
    lines += ["", "Per-config kernel split (trace averages over the config run, µs):", ""]
    for c, v in out.items():
        lines.append(f"* {c.upper()}: " + ", ".join(f"`{k}` {t}" for k, t in v["kernels"].items()))
    # counters of the roofline kernels: VALU per 8 KiB tile, LDS bank conflicts / LDS-active
    lines += ["", "Counters of the scans (per launch; effective clock = GRBM_GUI_ACTIVE / 8 XCDs / the steady",
              "launch time, the DVFS clock the chip holds under the kernel, MI355X_MICROARCH.md):", "",
              "| config | kernel | SQ_INSTS_VALU / 8 KiB tile | SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS | effective clock (GHz) |",
              "|---|---|---|---|---|"]
    for c in CONFIGS:
        if c not in pmc or c not in out:
            continue
        ex = bench_entry(b, c)[1]
        tiles = ex["bytes"] / 8192 if ex else None
        for k, p in pmc[c].items():
            if not k.startswith("k_scan") or "SQ_INSTS_VALU" not in p:
                continue
            v = p["SQ_INSTS_VALU"] / tiles if tiles else None  # (summed over the dispatch's rows)
            bc = p.get("SQ_LDS_BANK_CONFLICT"), p.get("SQ_ACTIVE_INST_LDS")
            r = bc[0] / bc[1] if bc[0] is not None and bc[1] else None
            st = out[c].get("steady_us") if out[c]["kernel"] == k else None
            clk = p["GRBM_GUI_ACTIVE"] / 8 / (st * 1e-6) / 1e9 if st and p.get("GRBM_GUI_ACTIVE") else None
            if clk:
                out[c]["effective_clock_ghz"] = round(clk, 3)
            lines.append(f"| {c.upper()} | `{k}` | {'%.0f' % v if v else '—'} | {'%.2f' % r if r else '—'} | "
                         f"{'%.2f' % clk if clk else '—'} |")
    (dst / "summary.md").write_text("\n".join(lines) + "\n")
    json.dump(out, open(dst / "summary.json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
