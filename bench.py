#!/usr/bin/env python3
"""klogs filter-path benchmark (BASELINE.json configs[1], "C2"):

    one 4 GiB synthetic JSON log stream per GPU, --since 5m --tail 100 --grep <literal>

A step = one full klf_run_device pass (memsets, scan kernel, counts/tail, compaction)
over the device-resident batch plus the per-stream count gather across ranks.  Weak
scaling: every rank owns its own stream (streams shard across GPUs; no data-path
collective).  value = total input bytes of all ranks / max-over-ranks wall time.

At N = 1 the same line also carries BASELINE configs 4 and 5 under "extra.configs" (the
general matcher: the scan with the fused q-gram prefilter, then the per-candidate NFA):
  C4: 32 GiB of mixed-length lines (8 streams), 1,024 --grep literals, --since 5m --tail 100
  C5: 32 GiB of 1-32 KiB JSON lines, 8 pods with 1-2 init containers (-i stream table),
      64 --match regexes, --since 5m --tail 100
each measured the same way (device-resident, HIP events on the launch stream).

Launch: python bench.py [--gpus 1 --steps K --warmup W]; for N > 1 the driver runs
`python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...`.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

from klogs_amd import engine as E  # noqa: E402  (binds to torch's HIP runtime)
from klogs_amd import shard, synth  # noqa: E402

METRIC = "filtered log GB/s (whole node) at 1/2/4/8 MI355X; % of HBM peak"
HBM_PEAK_GBS = 8000.0  # MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md
STREAM_BYTES = 4 << 30
SINCE_S = 300  # --since 5m
TAIL = 100


def pmc_traffic():
    """Per-launch HBM bytes of k_scan<literal> from the newest committed rocprofv3 --pmc
    summary (profiles/<round>/traffic.json, written by scripts/collect_profiles.py from
    FETCH_SIZE / WRITE_SIZE passes over this same command), or None."""
    files = sorted(ROOT.glob("profiles/r*/traffic.json"))
    if not files:
        return None, None
    t = json.loads(files[-1].read_text())
    return int(t["traffic_bytes"]), str(files[-1].relative_to(ROOT))


def committed_trace_frac(cfg: str = "c2"):
    """The same roofline fraction from the newest committed kernel trace
    (profiles/<round>/summary.json, scripts/collect_profiles.py): bytes / rocprofv3's average
    launch / peak, measured on the profiling box -- reported beside the live HIP-event one."""
    files = sorted(ROOT.glob("profiles/r*/summary.json"))
    if not files:
        return None, None
    s = json.loads(files[-1].read_text()).get(cfg)
    return (s and s["frac_rocprof"]), str(files[-1].relative_to(ROOT))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--bytes", type=int, default=STREAM_BYTES, help="stream bytes per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-write", action="store_true", help="skip C3's file write path")
    ap.add_argument("--no-capture", action="store_true", help="skip the host-staged capture-path timing")
    ap.add_argument("--capture-piece", type=int, default=4 << 20, help="klf_stage piece size of the capture path")
    ap.add_argument("--extra-configs", default="c1,c3,c4,c5",
                    help="comma list of c1,c3,c4,c5 ('' = none); at N > 1: c3 and c5 run sharded")
    ap.add_argument("--extra-bytes", type=int, default=32 << 30, help="total bytes of each extra config")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knob for a one-GPU box: KLF_BENCH_BACKEND=gloo lets N ranks share cuda:0
    # (RCCL refuses two ranks on one device).  The driver's runs use RCCL, one GPU per rank.
    backend = os.environ.get("KLF_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    coll_dev = f"cuda:{local}" if backend == "nccl" else "cpu"
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    # ---- synthetic input: stream `rank` of the C2 family, generated on the host ----
    assert shard.local_streams([args.bytes] * world, world, rank) == [rank]  # LPT: equal streams 1:1
    t = time.time()
    n = synth.size(synth.JSON, 42, rank, args.bytes, permille=10)
    host = np.empty(n + 1, dtype=np.uint8)
    synth.generate_into(host, synth.JSON, 42, rank, args.bytes, permille=10)
    host = host[:n]
    seg_base, total = E.layout([n])
    dev = torch.empty(total, dtype=torch.uint8, device=f"cuda:{local}")
    torch.cuda.synchronize()
    t_h2d = time.time()
    dev[:n].copy_(torch.from_numpy(host), non_blocking=False)
    torch.cuda.synchronize()
    h2d_s = time.time() - t_h2d
    log(f"[rank {rank}] generated {n} B in {time.time() - t:.1f}s, H2D {n / h2d_s / 1e9:.1f} GB/s")

    now = synth.T0 + synth.SPAN + 1  # "now" = end of the stream + 1 s
    since = (now - SINCE_S, 0)
    stream = torch.cuda.current_stream()
    eng = E.Engine(local, grep=[synth.NEEDLE], hip_stream=stream.cuda_stream)
    ptr = dev.data_ptr()

    step_pending = []

    def step():
        # per-pattern counts ride along (one literal: no extra kernel work, SPEC.md S6)
        r = eng.run_device(ptr, seg_base, [n], since=since, tail=TAIL, pattern_counts=True)
        if world > 1:  # per-stream count records -> every rank (one all-gather, RCCL over xGMI),
            # left in flight while the next step filters; every gather is waited for before
            # the timed region closes (finish_gathers)
            rec = dict(r.totals(), patterns=r.pattern_counts(0))
            step_pending.append(shard.gather_counts_async({rank: rec}, [n] * world, world, device=coll_dev,
                                                          n_patterns=1))
            if len(step_pending) > 1:
                step_pending.pop(0).wait()
        return r

    def finish_gathers():
        while step_pending:
            step.table = step_pending.pop(0).wait()

    for _ in range(args.warmup):
        step().free()
    finish_gathers()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    scan_ms, total_ms = [], []
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        r = step()
        tm = r.timing()
        scan_ms.append(tm[6])  # the k_scan kernel alone
        total_ms.append(tm[4])
        if i + 1 < args.steps:
            r.free()
        else:
            last = r
    finish_gathers()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    tot = last.totals()
    lines = tot["lines"]
    out_bytes = tot["out_bytes"]
    # algorithmic bytes.  k_scan, the dominant kernel, reads every input
    # byte once; its staged per-line slots are intermediate (not counted).  The K1 stage
    # adds the u64 line-offset index (L + 1 per stream) and the match bitmap, written once.
    scan_alg = n
    k1_alg = n + 8 * (lines + 1) + 4 * (lines // 32 + 1)
    step_alg = k1_alg + out_bytes
    scan_avg_s = float(np.mean(scan_ms)) / 1e3

    dev_avg_s = float(np.mean(total_ms)) / 1e3
    achieved = scan_alg / scan_avg_s / 1e9

    log(f"[rank {rank}] timed {args.steps} steps: {dt / args.steps * 1e3:.3f} ms/step")
    cold = cold_run(local, dict(grep=[synth.NEEDLE]), ptr, seg_base, [n], since, TAIL) if world == 1 else None
    verified = None
    if not args.no_verify:  # every rank: its own stream in full against the C oracle
        sys.path.insert(0, str(ROOT / "oracle"))
        import c_oracle as co
        so = last.stream(0)
        t = time.perf_counter()
        ref_out, _, _, ref_c = co.filter_stream(host, since, TAIL, [synth.NEEDLE], want_lines=False,
                                                want_bits=False)
        cpu_s = time.perf_counter() - t
        verified = ref_out == so.out and ref_c["selected"] == tot["selected"] and ref_c["lines"] == lines
        lo = last.lines(0)
        verified = bool(verified and lo.shape[0] == lines + 1 and int(lo[-1]) == n)
        if world > 1:  # every rank's verdict (MIN)
            vt = torch.tensor([int(verified)], dtype=torch.int64, device=coll_dev)
            dist.all_reduce(vt, op=dist.ReduceOp.MIN)
            verified = bool(vt.item())
    records_ok = None
    if world > 1:  # the gathered table: every rank's row equals what that rank computed
        mine = step.table[rank].tolist()
        records_ok = mine == [tot[k] for k in shard.RECORD_FIELDS[1:]] + last.pattern_counts(0)
    cpu = None
    cpu_more = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(ROOT / "oracle"))
        import c_oracle as co
        # repeat whole passes over this run's stream until >= 10 s of CPU work
        passes, cpu_t = 0, 0.0
        while cpu_t < 10.0 and passes < 64:
            t = time.perf_counter()
            co.filter_stream(host, since, TAIL, [synth.NEEDLE], want_lines=False, want_bits=False)
            cpu_t += time.perf_counter() - t
            passes += 1
        cpu = {"value": round(n * passes / cpu_t / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
               "sample": f"{passes} full passes over this run's {n} B stream with oracle/klf_oracle_c.c "
                         f"(memchr line split, Go time.Parse restated, memmem grep, kubelet tail+since) "
                         f"on 1 host core, {cpu_t:.1f} s"}
        cpu_more = cpu_variants(host, since)

    # Capture path, N = 1 only: the product's host entry points on this
    # run's bytes -- klf_stage in 1 MiB pieces (io.Copy's role) into pinned chunks, then
    # klf_run (DMA H2D from the pinned chunks + the whole filter) and the output D2H.
    # Reported beside `value`, never as it (device-resident is the metric).
    capture = None
    log(f"[rank {rank}] verified={verified} cpu_baseline={cpu and cpu['value']}")
    if rank == 0 and world == 1 and not args.no_capture:
        ceng = E.Engine(local, grep=[synth.NEEDLE])
        want = last.stream(0).out
        piece = args.capture_piece
        runs = []
        for _ in range(2):  # the first pays the pinned-chunk allocation
            ceng.reset()
            ceng.set_streams(1)
            t0 = time.perf_counter()
            for off in range(0, n, piece):
                ceng.stage_array(0, host[off:off + piece])
            t1 = time.perf_counter()
            r = ceng.run(since=since, tail=TAIL, n_streams=1)
            got = r.stream(0).out
            t2 = time.perf_counter()
            r.free()
            runs.append((t1 - t0, t2 - t1, got == want))
        ceng.close()
        st_s, run_s, same = runs[-1]
        capture = {"stage_GBps": round(n / st_s / 1e9, 2), "h2d_filter_d2h_GBps": round(n / run_s / 1e9, 2),
                   "end_to_end_GBps": round(n / (st_s + run_s) / 1e9, 2), "piece_bytes": piece,
                   "staging": "pinned 64 MiB chunks (hipHostMalloc, reused across runs)",
                   "output_matches_device_run": bool(same and runs[0][2])}
        log(f"[rank 0] capture path: {capture}")

    # stage breakdown (after the checks: a later run invalidates `last`); outside the timed region (the stage events idle the GPU ~5 us each)
    k1_ms, staged = [], None
    for _ in range(3):
        if staged is not None:
            staged.free()
        staged = eng.run_device(ptr, seg_base, [n], since=since, tail=TAIL, stage_times=True)
        k1_ms.append(staged.timing()[0])  # K1 stage: k_scan + k_fixup + tile-base scan + scatter
    stage_last = staged.timing()
    staged.free()
    k1_avg_s = float(np.mean(k1_ms)) / 1e3
    traffic, traffic_src = pmc_traffic()
    trace_frac, trace_src = committed_trace_frac("c2")
    value = world * n * args.steps / dt / 1e9
    res = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded JSON kubelet log lines (200-599 B content, 31-B RFC3339Nano prefix, "
                "1% carry the grep literal), monotonic timestamps over 60 min",
        "config": {"workload": "C2: one 4 GiB JSON log stream per GPU, --since 5m --tail 100 --grep "
                               + synth.NEEDLE.decode(),
                   "stream_bytes": n, "lines_per_stream": lines, "global_bytes": world * n,
                   "parallelism": f"streams sharded, 1 stream per GPU x {world}"},
        "roofline": {"bound": "hbm", "kernel": "k_scan<literal>", "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "alg_bytes_per_launch": scan_alg,
                     "avg_launch_ms": round(scan_avg_s * 1e3, 4),
                     "frac_source": "HIP events carrying the k_scan dispatch's own start / end timestamps (hipExtLaunchKernel), this run",
                     "frac_rocprof_committed": trace_frac, "rocprof_source": trace_src},
        "cpu_baseline": cpu,
        "extra": {"device_ms_per_step": round(dev_avg_s * 1e3, 4),
                  "k1_stage": {"kernels": "k_scan+k_fixup+k_tsum+k_tbase+k_scatter", "alg_bytes": k1_alg,
                               "avg_ms": round(k1_avg_s * 1e3, 4),
                               "achieved_GBps": round(k1_alg / k1_avg_s / 1e9, 1)},
                  "step_alg_frac_of_peak": round(step_alg / dev_avg_s / 1e9 / HBM_PEAK_GBS, 4),
                  "stage_ms": [round(x, 4) for x in stage_last],
                  "selected_lines": tot["selected"], "matched_lines": tot["matched"], "out_bytes": out_bytes,
                  "h2d_inclusive_GBps": round(n / (h2d_s + dev_avg_s) / 1e9, 3),
                  "capture_path": capture,
                  "cold": cold,
                  "cpu_baseline_variants": cpu_more,
                  "gathered_records_consistent": records_ok,
                  "verified_vs_c_oracle": verified},
    }
    last.free()
    eng.close()
    del dev, host
    torch.cuda.empty_cache()
    if world == 1 and args.extra_configs:
        res["extra"]["configs"] = {}
        for name in [x for x in args.extra_configs.split(",") if x]:
            res["extra"]["configs"][name] = run_extra(name, args, local, now)
            torch.cuda.empty_cache()
    if world > 1:
        res["extra"]["configs"] = {}
        for name in [x for x in args.extra_configs.split(",") if x in ("c3", "c5")]:
            res["extra"]["configs"][name + "_sharded"] = run_sharded(name, args, world, rank, local, coll_dev, now)
            torch.cuda.empty_cache()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_variants(host: np.ndarray, since) -> dict:
    """More CPU reference points on the same stream, rank 0 at N = 1 (bounded, ~10 s):
    the C restatement on T host threads over line-aligned pieces (each piece with the run's
    --tail: the same per-line work; the split-tail exchange is O(1)), and the reference
    client's own ceiling -- klogs only io.Copy's each body into its file (cmd/root.go:359-374)
    -- as a host memcpy bound (1 and T threads) and a page-cache file write of the stream."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, str(ROOT / "oracle"))
    import c_oracle as co
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    n = len(host)
    cuts = [0]
    for k in range(1, threads):
        j = int(np.flatnonzero(host[k * n // threads:k * n // threads + (1 << 20)] == 10)[0]) + 1
        cuts.append(k * n // threads + j)
    cuts.append(n)
    pieces = [host[a:b] for a, b in zip(cuts, cuts[1:])]
    with ThreadPoolExecutor(threads) as ex:
        passes, t_mt = 0, 0.0
        while t_mt < 4.0 and passes < 64:
            t = time.perf_counter()
            list(ex.map(lambda p: co.filter_stream(p, since, TAIL, [synth.NEEDLE], want_lines=False,
                                                   want_bits=False), pieces))
            t_mt += time.perf_counter() - t
            passes += 1
        dst = np.empty_like(host)
        t = time.perf_counter()
        np.copyto(dst, host)
        t_cp1 = time.perf_counter() - t
        t = time.perf_counter()
        list(ex.map(lambda ab: np.copyto(dst[ab[0]:ab[1]], host[ab[0]:ab[1]]), zip(cuts, cuts[1:])))
        t_cpn = time.perf_counter() - t
    del dst
    wn = min(n, 1 << 30)
    with tempfile.NamedTemporaryFile(prefix="klf_cpy_") as f:
        t = time.perf_counter()
        mv = memoryview(host[:wn])
        off = 0
        while off < wn:
            off += os.write(f.fileno(), mv[off:off + (64 << 20)])
        t_w = time.perf_counter() - t
    return {
        "port_threads": {"value": round(n * passes / t_mt / 1e9, 3), "unit": "GB/s", "cores": threads,
                         "kind": "port", "sample": f"{passes} passes, {threads} line-aligned pieces of this run's "
                                                   f"stream, one host thread each, {t_mt:.1f} s"},
        "copy_bound_1t_GBps": round(n / t_cp1 / 1e9, 2),
        "copy_bound_threads_GBps": round(n / t_cpn / 1e9, 2),
        "file_write_GBps": round(wn / t_w / 1e9, 2),
        "copy_note": "the reference client's own work is io.Copy of each body into a file; host memcpy and "
                     "a page-cache write of the stream bound it from above",
    }


def sharded_table(name: str, world: int):
    """(stream sizes, kind, patterns, permille, since_tail, description) of config `name`
    at N ranks, weak scaling: each rank's share is the config's per-GPU workload.
      c3: 128 x 64 MiB TEXT streams per rank (256 pods x 4 containers over 8 GPUs), -l only;
      c5: 8 x N pods with 1-2 init containers + 2 containers (-i stream table, getPodLogs
          order), 32 GiB per rank of 1-32 KiB JSON lines, 64 --match regexes, since + tail."""
    if name == "c3":
        return [64 << 20] * (128 * world), synth.TEXT, {}, 10, "-l", \
            "C3 at N GPUs: 128 x 64 MiB TEXT streams per GPU, LPT-sharded, -l only (every line out)"
    from klogs_amd import host as H
    pods = [(f"synthetic-{p}", [f"init-{k}" for k in range(1 + p % 2)], ["app", "sidecar"]) for p in range(8 * world)]
    table = H.stream_table(pods, init=True)  # getPodLogs order with -i (cmd/root.go:240-262)
    w = [1 if is_init else 4 for _, _, is_init in table]
    per_rank = 32 << 30
    sizes = [per_rank * world * x // sum(w) for x in w]
    return sizes, synth.LONGJSON, dict(match=synth.c5_regexes()), 5, "since+tail", \
        (f"C5 at N GPUs: {len(table)} streams (8 pods per GPU, 1-2 init containers + 2 containers each, -i), "
         "32 GiB per GPU of 1-32 KiB JSON lines, 64 --match regexes, --since 5m --tail 100, LPT-sharded")


def run_sharded(name: str, args, world: int, rank: int, local: int, coll_dev, now: int) -> dict:
    """BASELINE config 3 or 5 across ranks: the stream table LPT-assigned
    (shard.assign), each rank one device batch of its own streams, then the one all-gather
    of per-stream count records (+ per-pattern counts for C5) per step over RCCL.  value =
    all ranks' bytes / max-over-ranks time.  After the timed region every rank checks its
    own rows of the gathered table and verifies its first and last stream in full against
    the C oracle (C5: the glibc-regex leg, ko_filter_rx); the flags are all-reduced (MIN)."""
    sizes, kind, pats, permille, mode, desc = sharded_table(name, world)
    since, tail = ((None, -1) if mode == "-l" else ((now - SINCE_S, 0), TAIL))
    lens_all = [synth.size(kind, 42, i, sz, permille=permille) for i, sz in enumerate(sizes)]
    mine = shard.local_streams(lens_all, world, rank)
    lens = [lens_all[i] for i in mine]
    seg_base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device=f"cuda:{local}")
    h = np.empty(max(lens) + 1, dtype=np.uint8)
    t = time.time()
    for j, i in enumerate(mine):
        synth.generate_into(h, kind, 42, i, sizes[i], permille=permille)
        dev[int(seg_base[j]):int(seg_base[j]) + lens[j]].copy_(torch.from_numpy(h[:lens[j]]))
    torch.cuda.synchronize()
    del h
    log(f"[rank {rank}] {name} share: {len(mine)} streams, {sum(lens)} B in {time.time() - t:.1f}s")
    eng = E.Engine(local, hip_stream=torch.cuda.current_stream().cuda_stream, **pats)
    ptr = dev.data_ptr()
    npat = len(pats.get("match", [])) + len(pats.get("grep", []))

    pending = []

    def records(r):
        recs = {}
        for j, sid in enumerate(mine):
            c = r.stream_counts(j)
            if npat:
                c = dict(c, patterns=r.pattern_counts(j))
            recs[sid] = c
        return recs

    def step():
        r = eng.run_device(ptr, seg_base, lens, since=since, tail=tail, pattern_counts=bool(npat))
        pending.append(shard.gather_counts_async(records(r), lens_all, world, device=coll_dev, n_patterns=npat))
        if len(pending) > 1:
            pending.pop(0).wait()
        return r

    def finish():
        while pending:
            step.table = pending.pop(0).wait()
    for _ in range(args.warmup):
        step().free()
    finish()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        r = step()
        if i + 1 < args.steps:
            r.free()
        else:
            last = r
    finish()
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    tt = torch.tensor([dt], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    # every rank's own rows of the gathered table equal its own counts; totals add up
    mine_rec = records(last)
    fields = shard.RECORD_FIELDS[1:]
    rec_ok = all(step.table[sid].tolist() == [mine_rec[sid][k] for k in fields] + list(mine_rec[sid].get("patterns", []))
                 for sid in mine)
    rec_ok = rec_ok and int(step.table[:, 0].sum()) > 0 and int(step.table[:, 5].sum()) > 0
    ver = None
    if not args.no_verify:  # the rank's first and last stream in full vs the C oracle
        sys.path.insert(0, str(ROOT / "oracle"))
        import c_oracle as co
        rs = co.RegexSet(pats["match"]) if "match" in pats else None
        sn = since if since is not None else co.GO_ZERO_TIME
        got = {j: (last.stream(j), last.match_bits(j) if npat else None) for j in sorted({0, len(mine) - 1})}
        del dev
        torch.cuda.empty_cache()
        dev = None

        def check(j):
            i = mine[j]
            hh = np.empty(lens[j] + 1, dtype=np.uint8)
            synth.generate_into(hh, kind, 42, i, sizes[i], permille=permille)
            if rs is not None:
                out, _, bits, c = co.filter_stream_rx(hh[:lens[j]], sn, tail, rs, want_lines=False)
            else:
                out, _, bits, c = co.filter_stream(hh[:lens[j]], sn, tail, [], want_lines=False, want_bits=False)
            so, gb = got[j]
            return so.out == out and all(so.counts[k] == c[k] for k in c) and (gb is None or gb == bits)
        from concurrent.futures import ThreadPoolExecutor
        tv = time.perf_counter()
        with ThreadPoolExecutor(len(got)) as ex:
            ver = all(ex.map(check, list(got)))
        log(f"[rank {rank}] {name} verified={ver} ({time.perf_counter() - tv:.1f}s)")
    flags = torch.tensor([int(rec_ok), -1 if ver is None else int(ver)], dtype=torch.int64, device=coll_dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    last.free()
    eng.close()
    del dev
    out = {"workload": desc, "streams": len(lens_all), "bytes": int(sum(lens_all)),
           "value_GBps": round(sum(lens_all) * args.steps / dt / 1e9, 1),
           "ms_per_step": round(dt / args.steps * 1e3, 3),
           "records_consistent": bool(flags[0].item()),
           "collective": f"one all-gather per step of {len(lens_all)} x {shard.NREC + npat} int64 records "
                         f"({'RCCL' if coll_dev != 'cpu' else 'gloo'})"}
    if ver is not None:
        out["verified_vs_oracle"] = bool(flags[1].item() == 1)
        out["verify_scope"] = ("on every rank: its first and last stream in full (output bytes, all counts"
                               + (", match bitmap" if npat else "") + ") against "
                               + ("the C oracle's glibc-regex leg (ko_filter_rx)" if npat else "the C oracle"))
    return out


def extra_streams(name: str, total: int):
    """(stream sizes, generator kind, patterns, permille, description) of BASELINE configs
    3 / 4 / 5."""
    if name == "c2":  # the headline workload, for scripts/run_config.py
        return [STREAM_BYTES], synth.JSON, dict(grep=[synth.NEEDLE]), 10, \
            "C2: one 4 GiB JSON log stream, --since 5m --tail 100 --grep " + synth.NEEDLE.decode()
    if name == "c1":  # the reference's own CPU-runnable case (BASELINE configs[0])
        return [64 << 20], synth.TEXT, {}, 10, \
            "C1: one 64 MiB stream (lognormal line lengths, median 96 B), --since 5m --tail 100"
    if name == "c3":  # one GPU's share of C3 at 8 GPUs (fixed size: --extra-bytes is for C4/C5)
        n = 128
        return [64 << 20] * n, synth.TEXT, {}, 10, \
            "C3 per-GPU share at 8 GPUs: 128 streams x 64 MiB (256 pods x 4 containers / 8), -l selection " \
            "only: no --since, no --tail, no grep (every line out, prefix stripped)"
    if name == "c4":
        n = 8
        return [total // n] * n, synth.MIXED, dict(grep=synth.c4_literals(1024)), 5, \
            "C4: 8 streams of mixed-length lines (16 B-8 KiB, lognormal), 1,024 --grep literals (6-24 B, " \
            "0.5% of lines hold one), --since 5m --tail 100"
    if name == "c5":
        from klogs_amd import host as H
        pods = [(f"synthetic-{p}", [f"init-{k}" for k in range(1 + p % 2)], ["app", "sidecar"]) for p in range(8)]
        table = H.stream_table(pods, init=True)  # getPodLogs order with -i (cmd/root.go:240-262)
        w = [1 if is_init else 4 for _, _, is_init in table]
        sizes = [total * x // sum(w) for x in w]
        return sizes, synth.LONGJSON, dict(match=synth.c5_regexes()), 5, \
            f"C5: {len(table)} streams (8 pods x 1-2 init containers + 2 containers, -i), 1-32 KiB JSON " \
            "lines, 64 --match regexes (0.5% of lines match one, 1% hold a factor but no match), " \
            "--since 5m --tail 100"
    raise ValueError(name)


def cpu_extra(name: str, kind: int, pats: dict, permille: int, since, tail: int) -> dict:
    """CPU reference points for configs 1 and 3-5 (rank 0, N = 1; bounded, a few seconds
    each) on samples of the same generator and shape: the C restatement on 1 and on T host
    threads (one stream per thread, as the reference runs one goroutine per stream).  Literal
    paths: oracle/klf_oracle_c.c ko_filter (memmem / Aho-Corasick).  The regex set (C5):
    ko_filter_rx, glibc POSIX ERE translated from the Go subset (oracle/posix_re.py) behind an
    Aho-Corasick pass over each pattern's required literal, first checked against the Python
    oracle on one sample stream; the Python oracle's own rate (one core, Python `re`) beside it.
    C1 is one 64 MiB stream: one core only."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, str(ROOT / "oracle"))
    import c_oracle as co
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    sample = {"c1": 64 << 20, "c3": 64 << 20, "c4": 2 << 20, "c5": 8 << 20}[name]
    nstreams = 1 if name == "c1" else threads
    streams = [synth.generate(kind, 7, i, sample, permille=permille) for i in range(nstreams)]
    grep = pats.get("grep", [])
    sn = since if since is not None else co.GO_ZERO_TIME

    if name == "c5":
        rs = co.RegexSet(pats["match"])

        def one(b):
            return co.filter_stream_rx(b, sn, tail, rs, want_lines=False, want_bits=False)
    else:
        def one(b):
            return co.filter_stream(b, sn, tail, grep, want_lines=False, want_bits=False)

    def timed(f, budget):
        n, t = 0, 0.0
        while t < budget and n < 64:
            t0 = time.perf_counter()
            f()
            t += time.perf_counter() - t0
            n += 1
        return n, t
    what = {"c5": "oracle/klf_oracle_c.c ko_filter_rx (glibc regexec behind the required-literal Aho-Corasick pass)"}
    impl = what.get(name, "oracle/klf_oracle_c.c")
    res = {}
    if name == "c5":  # the C leg decides every line as the Python oracle does (one sample stream)
        from oracle import klf_oracle as ko
        cp = ko.compile_patterns(match=pats["match"])
        probe = streams[0][:2 << 20]
        probe = probe[:probe.rfind(b"\n") + 1]
        ref = ko.filter_stream(probe, sn, tail, cp)
        got = co.filter_stream_rx(probe, sn, tail, rs, want_lines=False)
        res["c_leg_equals_python_oracle"] = bool(got[0] == ref.out and got[2] == ref.match_bits)
        n, t = timed(lambda: ko.filter_stream(probe, sn, tail, cp), 3.0)
        res["python_1_core"] = {"value": round(len(probe) * n / t / 1e9, 4), "unit": "GB/s", "cores": 1,
                                "kind": "port", "sample": f"{n} passes over {len(probe)} B of the C5 generator, "
                                                          f"oracle/klf_oracle.py (Python re), {t:.1f} s"}
    n, t = timed(lambda: one(streams[0]), 3.0)
    res["port_1_core"] = {"value": round(sample * n / t / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
                          "sample": f"{n} passes over one {sample >> 20} MiB stream of the {name.upper()} generator, "
                                    f"{impl}, {t:.1f} s"}
    if nstreams > 1:
        with ThreadPoolExecutor(threads) as ex:
            n, t = timed(lambda: list(ex.map(one, streams)), 3.0)
        res["port_threads"] = {"value": round(sample * threads * n / t / 1e9, 4), "unit": "GB/s",
                               "cores": threads, "kind": "port",
                               "sample": f"{n} passes over {threads} streams of {sample >> 20} MiB, one host thread "
                                         f"per stream, {impl}, {t:.1f} s"}
    return res


def cold_run(local: int, pats: dict, ptr: int, seg_base, lens, since, tail: int) -> dict:
    """One-shot cost, as one klogs invocation pays it (klf_run once per
    run): a fresh engine (klf_open: pattern compile + table uploads) and its first run on
    the device-resident batch (first-batch statistics + layout choice + uploads, the
    pipeline, the readback), host wall clock; beside it the steady step of the same
    engine's second run."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng = E.Engine(local, hip_stream=torch.cuda.current_stream().cuda_stream, **pats)
    t1 = time.perf_counter()
    r = eng.run_device(ptr, seg_base, lens, since=since, tail=tail)
    t2 = time.perf_counter()
    r.free()
    t3 = time.perf_counter()
    r = eng.run_device(ptr, seg_base, lens, since=since, tail=tail)
    t4 = time.perf_counter()
    r.free()
    eng.close()
    return {"open_ms": round((t1 - t0) * 1e3, 3), "first_run_ms": round((t2 - t1) * 1e3, 3),
            "cold_ms": round((t2 - t0) * 1e3, 3), "second_run_ms": round((t4 - t3) * 1e3, 3)}


def verify_large(name, sizes, lens, kind, permille, pats, since, tail, r) -> dict:
    """Checks the last timed run of C4 / C5 against the oracles (after the timed region),
    every stream in full, one host thread per stream: output bytes, all counts and the match
    bitmap.  C4: the C oracle (Aho-Corasick over the 1,024 literals).  C5: the C oracle's
    regex leg (ko_filter_rx: the 64 regexes as glibc POSIX ERE behind a required-literal
    pass, itself checked against the Python oracle in tests/test_oracle.py and, on a sample
    of this run's generator, in cpu_baseline.c_leg_equals_python_oracle)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, str(ROOT / "oracle"))
    import c_oracle as co
    t = time.perf_counter()
    got = [(r.stream(i), r.match_bits(i)) for i in range(len(lens))]
    sn = since if since is not None else co.GO_ZERO_TIME
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    rs = co.RegexSet(pats["match"]) if name == "c5" else None

    def check(i):
        h = np.empty(lens[i] + 1, dtype=np.uint8)
        synth.generate_into(h, kind, 42, i, sizes[i], permille=permille, threads=1)
        if rs is not None:
            out, _, bits, c = co.filter_stream_rx(h[:lens[i]], sn, tail, rs, want_lines=False)
        else:
            out, _, bits, c = co.filter_stream(h[:lens[i]], sn, tail, pats["grep"], want_lines=False)
        so, gbits = got[i]
        return so.out == out and gbits == bits and all(so.counts[k] == c[k] for k in c)
    with ThreadPoolExecutor(min(threads, len(lens))) as ex:
        ok = list(ex.map(check, range(len(lens))))
    bad = [i for i, x in enumerate(ok) if not x]
    scope = ("every stream in full: output bytes, all counts, match bitmap ("
             + ("C oracle regex leg: glibc POSIX ERE behind the required-literal pass" if rs is not None
                else "C oracle, Aho-Corasick") + ")")
    return {"ok": not bad, "streams": len(lens), "failed_streams": bad, "scope": scope,
            "s": round(time.perf_counter() - t, 1)}


def run_extra(name: str, args, local: int, now: int) -> dict:
    sizes, kind, pats, permille, desc = extra_streams(name, args.extra_bytes)
    t = time.time()
    lens = [synth.size(kind, 42, i, sz, permille=permille) for i, sz in enumerate(sizes)]
    seg_base, total = E.layout(lens)
    dev = torch.empty(total, dtype=torch.uint8, device=f"cuda:{local}")
    for i, (sz, n) in enumerate(zip(sizes, lens)):  # one stream at a time through host memory
        h = np.empty(n + 1, dtype=np.uint8)
        synth.generate_into(h, kind, 42, i, sz, permille=permille)
        dev[int(seg_base[i]):int(seg_base[i]) + n].copy_(torch.from_numpy(h[:n]))
        del h
    torch.cuda.synchronize()
    log(f"[{name}] generated + uploaded {sum(lens)} B in {time.time() - t:.1f}s")
    since, tail = ((None, -1) if name == "c3" else ((now - SINCE_S, 0), TAIL))
    stream = torch.cuda.current_stream()
    eng = E.Engine(local, hip_stream=stream.cuda_stream, **pats)
    ptr = dev.data_ptr()
    for _ in range(args.warmup):
        eng.run_device(ptr, seg_base, lens, since=since, tail=tail).free()
    torch.cuda.synchronize()
    scan_ms, total_ms = [], []
    t0 = time.perf_counter()
    last = None
    for i in range(args.steps):
        r = eng.run_device(ptr, seg_base, lens, since=since, tail=tail)
        tm = r.timing()
        scan_ms.append(tm[6])
        total_ms.append(tm[4])
        if i + 1 < args.steps:
            r.free()
        else:
            last = r
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    cold = cold_run(local, pats, ptr, seg_base, lens, since, tail)
    verified = None
    write = None
    wdir = None
    if name == "c3" and not args.no_write:  # §8f-3 output write path: every stream into its own file (klf_result_write)
        wdir = tempfile.TemporaryDirectory(prefix="klf_c3_")
        paths = [os.path.join(wdir.name, f"pod{i // 4}__c{i % 4}.log") for i in range(len(lens))]
        tw = time.perf_counter()
        try:
            wbytes = last.write_files(paths)
        except E.KlfError as ex:  # e.g. no room for 6.9 GB in the temp dir: reported, not fatal
            wbytes, write = None, {"error": str(ex), "dir": wdir.name}
        wdt = time.perf_counter() - tw
    if write is None and wdir is not None:
        write = {"GBps": round(wbytes / wdt / 1e9, 2), "bytes": wbytes, "files": len(paths), "s": round(wdt, 3),
                 "how": "klf_result_write: 64 MiB pinned D2H chunks, double-buffered, 8 writer threads each owning whole files (own HIP stream + 2x32 MiB pinned halves), "
                        "into page-cache files under " + os.path.dirname(wdir.name)}
    if name == "c3" and not args.no_verify and write is not None and wbytes is not None:  # first and last stream vs the C oracle
        sys.path.insert(0, str(ROOT / "oracle"))
        import c_oracle as co
        verified = True
        for i in (0, len(lens) - 1):
            h = np.empty(lens[i] + 1, dtype=np.uint8)
            synth.generate_into(h, kind, 42, i, sizes[i], permille=permille)
            want = co.filter_stream(h[:lens[i]], co.GO_ZERO_TIME, -1, [], want_lines=False, want_bits=False)[0]
            with open(paths[i], "rb") as f:  # the written file, i.e. the D2H + write path too
                verified = verified and f.read() == want
        write["verified_vs_c_oracle"] = bool(verified)
    if wdir is not None:
        wdir.cleanup()
    if name == "c1" and not args.no_verify:  # the whole stream vs the C oracle
        sys.path.insert(0, str(ROOT / "oracle"))
        import c_oracle as co
        h = np.empty(lens[0] + 1, dtype=np.uint8)
        synth.generate_into(h, kind, 42, 0, sizes[0], permille=permille)
        ref_out, ref_lo, _, ref_c = co.filter_stream(h[:lens[0]], since, tail, [], want_bits=False)
        so = last.stream(0)
        verified = bool(so.out == ref_out and all(so.counts[k] == ref_c[k] for k in ref_c)
                        and np.array_equal(last.lines(0), ref_lo))
    vlarge = None
    if name in ("c4", "c5") and not args.no_verify:
        del dev  # the checks regenerate the streams on the host
        torch.cuda.empty_cache()
        dev = None
        vlarge = verify_large(name, sizes, lens, kind, permille, pats, since, tail, last)
    tot = last.totals()
    if dev is not None:
        staged = eng.run_device(ptr, seg_base, lens, since=since, tail=tail, stage_times=True)
        stage = staged.timing()
        staged.free()
    else:  # the batch was dropped for the checks: the stage split of the timed runs' last
        stage = last.timing()
    n = sum(lens)
    scan_s = max(float(np.mean(scan_ms)) / 1e3, 1e-12)  # (0: a build without the scan's events)
    dev_s = float(np.mean(total_ms)) / 1e3
    step_alg = n + 8 * (tot["lines"] + len(lens)) + 4 * (tot["lines"] // 32 + 1) + tot["out_bytes"]
    out = {
        "workload": desc, "streams": len(lens), "bytes": n, "lines": tot["lines"],
        "value_GBps": round(n * args.steps / dt / 1e9, 1), "ms_per_step": round(dt / args.steps * 1e3, 3),
        "device_ms_per_step": round(dev_s * 1e3, 3),
        "roofline": {"bound": "hbm", "kernel": "k_scan<plain>" if not pats else "k_scan<general, q-gram prefilter>",
                     "achieved": round(n / scan_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(n / scan_s / 1e9 / HBM_PEAK_GBS, 4), "avg_launch_ms": round(scan_s * 1e3, 4)},
        "cold": cold,
        "matcher_ms": round(stage[1], 4),
        "step_alg_frac_of_peak": round(step_alg / dev_s / 1e9 / HBM_PEAK_GBS, 4),
        "matched_lines": tot["matched"], "selected_lines": tot["selected"], "out_bytes": tot["out_bytes"],
        "stage_ms": [round(x, 4) for x in stage],
    }
    if not getattr(args, "no_cpu_baseline", True):
        out["cpu_baseline"] = cpu_extra(name, kind, pats, permille, since, tail)
    if verified is not None:
        out["verified_vs_c_oracle"] = bool(verified)
    if vlarge is not None:
        out["verified_vs_oracle"] = vlarge.pop("ok")
        out["verify"] = vlarge
    if write is not None:
        out["write_path"] = write
    last.free()
    eng.close()
    del dev
    return out


if __name__ == "__main__":
    main()
