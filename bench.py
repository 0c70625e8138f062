#!/usr/bin/env python3
"""Benchmark: edges/sec into the streaming connected-components summary on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one synthetic stream already resident in HBM: reset the summary to its
initial value, then per merge window fold this rank's chunk of the window into the device forest and emit the
summary (canonicalising compress; with N > 1 the cross-GPU forest merge over RCCL/xGMI first).

Partitioning (the reference's: SummaryBulkAggregation.java:93-106 tags each edge with an arbitrary upstream
subtask, so a partition is any split of each window): every workload is ONE fixed stream, and rank r of N folds the
r-th contiguous 1/N of every window. Strong scaling: value = (edges of the whole stream) * K / max-over-ranks time.

N=1 default workload: C4, Kronecker scale 26 (64M vertices, 2^30 edges, 8 GiB of edges), one merge window — the
config the north-star target is quoted on; it fits one GPU. Extra legs on rank 0 at N=1 (outside the timed
region of the headline value): host-fed rate (pinned host memory + H2D), C2 R-MAT s20 rotating over 4 distinct
batches (537 MB: no batch is still in the 256 MiB Infinity Cache when it is folded again), CPU baseline (the C
restatement of the reference topology, oracle/cc_oracle.c) at T = 1, the box's CPU quota and nproc threads.
Parity: the final labels' digest vs tests/golden/stream_digests.json (oracle digests computed on the CPU).

Launch: python bench.py [--gpus N --steps K --warmup W]  (N>1 under torch.distributed.run, one rank per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, Chip-level parameters)
BYTES_PER_EDGE = 16  # algorithmic, whole fold: 8 B edge stream + 2 x 4 B parent reads
# per-kernel algorithmic bytes: (bytes, per "edge" of the launch | per "id" of the forest)
KERNEL_BYTES = {
    "fold_filtered_kernel": (8, "edge"),    # the edge stream (skipped edges need no parent access)
    "seed_bfs_kernel": (8, "edge"),         # the prefix edge stream (bitmap in LDS)
    "fold_kernel": (16, "edge"),            # edge + both parents
    "compress_bits_kernel": (8.125, "id"),  # parent read + label write + 1 bitmap bit
    "compress_inc_kernel": (8.125, "id"),   # the same, incremental (bloom of the window's mutations in LDS)
    "fold_pipe_kernel": (16, "edge"),       # fold_kernel's bytes (its touched-id marks are atomics on 2 bits per id)
    # the pipelined emission's scan: the label read + the new-id and tracked-component bits (it writes changed labels only)
    "compress_pipe_kernel": (4.25, "id"),
    "seed_pack_kernel": (5.125, "id"),      # flag byte read + parent write + 1 bitmap bit (the init variant)
    "seed_hub_kernel": (1.125, "id"),       # flag byte + bitmap bit cleared
    # the bucketed fold's P1 runs over every edge of the batch once: priced at SURVEY §8(d)'s 16 B per edge (its own
    # traffic is 8 B read + 6 B bucket entry written, round 3)
    "bucket_kernel": (16, "edge"),
    "slice_filter_kernel<true>": (9, "edge"),    # FINAL P2: read the 6-B bucket entry + write the 3-B v-list entry
    "slice_filter_kernel<false>": (9, "edge"),   # a seeding level's P2 over the bucket samples
    "slice_hook_kernel<true>": (3, "edge"),      # FINAL P3: read the 3-B v-list entries (units: the batch's edges)
    "slice_hook_kernel<false>": (3, "edge"),     # a seeding level's P3
    "bucket_init_kernel": (4.125, "id"),    # parent write + 1 bitmap bit
}
C2_BATCHES = 4  # rotating C2 batches (tests/golden/stream_digests.json c2_rmat20@k)
# DESIGN.md §6's predicted curve (round 6): per workload and N, the per-rank fold, the merge kernels, the message and the
# modelled all_gather (ms; bytes per rank), so that a multi-GPU line can be read against its prediction
PREDICTED = {
    "c4_kron26": {1: {"fold_ms": 9.04, "ms_per_step": 9.04},
                  2: {"fold_ms": 5.03, "merge_kernels_ms": 0.24, "message_bytes": 8.9e6, "all_gather_ms": 0.25, "ms_per_step": 5.52},
                  4: {"fold_ms": 2.86, "merge_kernels_ms": 0.28, "message_bytes": 9.3e6, "all_gather_ms": 0.26, "ms_per_step": 3.40},
                  8: {"fold_ms": 1.78, "merge_kernels_ms": 0.36, "message_bytes": 10.0e6, "all_gather_ms": 0.27, "ms_per_step": 2.41}},
    "c5_adversarial": {n: {"ms_per_window": 0.06, "message_bytes_per_window": 16 * (1 << 16) // n + 16, "ms_per_step": 15.0}
                       for n in (2, 4, 8)},
}
HOST_FED_MAX_EDGES = 1 << 28  # the host-fed leg's sample (2 GiB of pinned host edges)
CPU_SAMPLE_EDGES = 1 << 24    # the CPU baseline's sample (a prefix of the workload's stream)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4_kron26")
    ap.add_argument("--window-edges", type=int, default=0, help="edges per merge window (0 = config default)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target CPU-baseline work per thread count (0 = skip)")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the host-fed and rotating-C2 legs")
    ap.add_argument("--tune", default="", help="fold-pipeline knobs k=v,... (gcc_forest_tune; speed only)")
    ap.add_argument("--phase-timing", choices=["timed", "after", "off"], default="after",
                    help="per-kernel dispatch events in the timed steps, in extra steps after them, or not at all")
    ap.add_argument("--step-marker", action="store_true",
                    help="launch gcc_step_mark_kernel once per step (rocprofv3 runs count steps by it)")
    return ap.parse_args()


def golden_digests():
    p = os.path.join(ROOT, "tests", "golden", "stream_digests.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def label_digest(labels):
    """sum_v splitmix64((label[v] << 32) | v) mod 2^64 (the fixture's digest; same formula as the oracle's)."""
    import numpy as np

    lab = np.asarray(labels, dtype=np.uint64)
    x = (lab << np.uint64(32)) | np.arange(lab.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        return int(np.sum(x, dtype=np.uint64))


def window_starts(cfg, override):
    from gelly_stream import generators as G

    E, _ = cfg.info()
    if override:
        return list(range(0, E, override)) + [E]
    return [int(x) for x in G.window_starts(cfg)]


def rank_chunks(starts, rank, world):
    """Rank r's contiguous 1/world of every window: [(lo, hi)] per window."""
    out = []
    for b, e in zip(starts[:-1], starts[1:]):
        out.append((b + (e - b) * rank // world, b + (e - b) * (rank + 1) // world))
    return out


def pmc_kernel_match(label, kname):
    """Does a rocprof kernel name belong to bench's kernel label? 'slice_filter_kernel<true>' matches
    'void bk::slice_filter_kernel<true, false>(...)' (the label's template arguments are a prefix of the name's)."""
    base, _, targs = label.partition("<")
    at = kname.find(base + "<") if targs else kname.find(base + "(")
    if at < 0:
        at = kname.find(base)
        return at >= 0 and not targs
    if not targs:
        return True
    got = kname[at + len(base) + 1:].split(">")[0].replace(" ", "")
    return got.startswith(targs.rstrip(">").replace(" ", ""))


def record_order(fname):
    """Sort key of a profiles/ file by when it was recorded: the session tag r<round><letters><n> of its name (a..z,
    aa..az, ba.. within a round: longer tags are later, so 'r5ba' > 'r5k'), then the record's own
    'recorded' sequence number for records written since round 6."""
    m = re.match(r"r(\d+)([a-z]*)(\d*)", fname)
    if not m:
        return (-1, 0, "", 0)
    return (int(m.group(1)), len(m.group(2)), m.group(2), int(m.group(3) or 0))


def profile_record(workload, kernel=None, units=None):
    """The newest committed rocprofv3 PMC summary for this workload (profiles/*_pmc_<workload>*.json) whose kernel is
    `kernel` and whose units per launch match `units` (within 1 %), or None. Newest = the latest session tag
    (record_order), and within one tag the highest 'recorded' field (tools/pmc_summary.py writes it)."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    cands = []
    for f in os.listdir(pdir):
        if f"_pmc_{workload}" not in f or not f.endswith(".json"):
            continue
        try:
            rec = json.load(open(os.path.join(pdir, f)))
        except Exception:
            continue
        cands.append((record_order(f) + (float(rec.get("recorded", 0)),), f, rec))
    for _, f, rec in sorted(cands, key=lambda c: c[0], reverse=True):
        if kernel and not pmc_kernel_match(kernel, rec.get("kernel", "")):
            continue
        if units is not None and abs(rec.get("edges_per_launch", 0) - units) > 0.01 * max(1, units):
            continue
        rec["file"] = f"profiles/{f}"
        return rec
    return None


def cpu_quota():
    """CPUs this process may use: cgroup v2 cpu.max quota, else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(int(q) / int(p))))
    except Exception:
        pass
    return n


def cpu_baseline(cfg, target_s):
    """The CPU restatement of the reference (oracle/cc_oracle.c: HashMap union-by-rank DisjointSets, one per
    partition/thread, serial CombineCC merge into the running summary) timed on this host over a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # cpu_baseline leg only

    from gelly_stream import generators as G

    E, V = cfg.info()
    n = min(E, CPU_SAMPLE_EDGES)
    pairs = G.generate_host(cfg, 0, n)
    nproc = os.cpu_count() or 1
    res = {}
    for label, threads in (("t1", 1), ("tquota", cpu_quota()), ("tnproc", nproc)):
        if label == "tnproc" and threads == res.get("tquota", {}).get("cores"):
            res[label] = dict(res["tquota"])
            continue
        reps, total = 0, 0.0
        while True:
            out = orc.cc_stream(pairs, [0, n], V, partitions=threads, threads=threads, want_digest=False)
            total += out["fold_seconds"]
            reps += 1
            if total >= target_s or reps >= 20:
                break
        res[label] = {"value": n * reps / total, "cores": threads, "reps": reps, "seconds": round(total, 2)}
    # the headline is T = the CPUs this process may use (the cgroup quota); T = nproc beside it oversubscribes
    # them whenever nproc > quota (a GPU box's nproc counts the whole machine)
    main = res["tquota"]
    quota = cpu_quota()
    return {
        "value": main["value"], "unit": "edges/s", "cores": main["cores"], "kind": "port",
        "sample": f"first {n} edges of the {cfg.name} stream, 1 window; T partitions = T threads folding "
                  f"HashMap union-by-rank DisjointSets + serial CombineCC merge (oracle/cc_oracle.c); "
                  f"headline T = cpu quota = {quota}; nproc={nproc}"
                  + (" (tnproc oversubscribes the quota)" if nproc > quota else ""),
        "t1": res["t1"], "tquota": res["tquota"], "tnproc": res["tnproc"],
    }


def kernel_stats(log, V, inst_steps):
    """Per-kernel durations from the forest's dispatch-event log, grouped by kernel."""
    kernel_of = {"filtered": "fold_filtered_kernel", "sample": "fold_kernel", "plain": "fold_kernel",
                 "seed_hub": "seed_hub_kernel", "seed_bfs": "seed_bfs_kernel", "seed_pack": "seed_pack_kernel",
                 "seed_init": "seed_pack_kernel", "refresh": "compress_bits_kernel", "compress": "compress_bits_kernel",
                 "refresh_bits": "compress_bits_kernel", "compress_inc": "compress_inc_kernel",
                 "refresh_inc": "compress_inc_kernel", "vote": "giant_vote_kernel", "bucket": "bucket_kernel",
                 "bucket_hist": "bucket_hist_kernel", "slice_filter": "slice_filter_kernel<true>",
                 "seed_filter": "slice_filter_kernel<false>", "slice_hook": "slice_hook_kernel<true>",
                 "seed_hook": "slice_hook_kernel<false>", "bucket_hook": "bucket_hook_kernel",
                 "bucket_slow": "bucket_slow_kernel", "bucket_rest": "bucket_rest_kernel",
                 "bucket_layout": "bucket_layout_kernel", "bucket_hub": "bucket_hub_kernel", "bucket_init": "bucket_init_kernel", "overflow": "fold_filtered_kernel",
                 "slice_filter2": "slice_filter_kernel<true,true>", "slice_hook2": "slice_hook_kernel<true> (level 2)",
                 "bucket_hook2": "bucket_hook_kernel (level 2)", "plain_pipe": "fold_pipe_kernel",
                 "resolve": "pipe_resolve_kernel", "compress_pipe": "compress_pipe_kernel"}
    phases, kernels, spans = {}, {}, []
    for name, ms, n in log:
        if name in ("begin", "slow_edges"):
            continue
        if name == "fold_span":
            spans.append((ms, n))
            continue
        phases.setdefault(name, []).append(ms)
        kernels.setdefault(kernel_of.get(name, name), []).append((ms, n))

    def kernel_bytes(k, units):
        per = KERNEL_BYTES.get(k)
        if per is None:
            return None
        return per[0] * (units if per[1] == "edge" else V)

    kstats = {}
    for k, v in kernels.items():
        ms_avg = sum(ms for ms, _ in v) / len(v)
        units = sum(n for _, n in v) / len(v)
        by = kernel_bytes(k, units)
        kstats[k] = {"launches_per_step": len(v) / max(1, inst_steps), "ms_avg": ms_avg,
                     "ms_per_step": sum(ms for ms, _ in v) / max(1, inst_steps), "units_avg": units,
                     "achieved_gbs": (by / (ms_avg / 1e3) / 1e9) if by and ms_avg > 0 else None}
    return kstats, phases, spans


def make_roofline(kstats, phases, spans, inst_steps, workload, timing_note, host_fold_s):
    """The roofline of the fold: achieved = SURVEY §8(d)'s 16 B per edge x the edges of one fold /
    the fold's device span (first kernel start -> last kernel stop, every kernel of the fold incl. its closing compress,
    from dispatch events); traffic = the committed rocprofv3 PMC bytes of every kernel of one step (tools/pmc_summary.py)
    when that record was measured on a fold of the same size. The dominant kernel's own figure (priced at its own
    algorithmic bytes, KERNEL_BYTES) stays under roofline.dominant, every kernel under roofline.kernels."""
    dominant = max(kstats, key=lambda k: kstats[k]["ms_per_step"]) if kstats else None
    dom = kstats.get(dominant, {})
    prof = profile_record(workload, dominant, dom.get("units_avg", 0)) if dominant else None
    dom_traffic = prof["hbm_bytes_per_launch"] if prof else None
    # the committed PMC record is only this kernel's traffic if the kernel still runs as it did then: its duration in
    # the PMC run's trace pass must be within 15 % of the live one; otherwise traffic is withheld
    stale = None
    if prof is not None and dom.get("ms_avg"):
        at = prof.get("kernel_ms_at_pmc")
        if at is None:
            stale = "the PMC record has no kernel duration to check against"
        elif abs(at - dom["ms_avg"]) > 0.15 * at:
            stale = f"kernel {dom['ms_avg']:.3f} ms live vs {at:.3f} ms in the PMC run"
        if stale and at is not None:
            dom_traffic = None
    avg_fold_s = (sum(ms for ms, _ in spans) / len(spans) / 1e3) if spans else None
    avg_fold_edges = (sum(n for _, n in spans) / len(spans)) if spans else None
    pipeline_gbs = BYTES_PER_EDGE * avg_fold_edges / avg_fold_s / 1e9 if spans and avg_fold_s else None
    # the whole step's measured HBM bytes (every kernel's PMC bytes x launches, per step), only from a record whose
    # fold had this fold's edge count (at N > 1 a rank folds 1/N of the stream: VERDICT r4 weak 5)
    pipe_prof = profile_record(workload, None, avg_fold_edges) if avg_fold_edges else None
    pipe_traffic = pipe_prof.get("pipeline_traffic_per_step") if pipe_prof else None
    return {
        "bound": "hbm", "kernel": "fold (every kernel of one step's fold, closing compress included)",
        "achieved": pipeline_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": (pipeline_gbs / HBM_PEAK_GBS) if pipeline_gbs else None,
        "traffic": pipe_traffic, "traffic_unit": "bytes per step (fold)",
        "traffic_ratio": (pipe_traffic / (BYTES_PER_EDGE * avg_fold_edges)) if pipe_traffic and avg_fold_edges else None,
        "traffic_source": pipe_prof["file"] if pipe_traffic else None,
        "kernel_ms_avg": avg_fold_s * 1e3 if avg_fold_s else None, "edges_per_fold": int(avg_fold_edges or 0),
        "bytes_per_unit": [BYTES_PER_EDGE, "edge"], "timing": timing_note,
        "host_enqueue_ms_avg": (sum(host_fold_s) / len(host_fold_s) * 1e3) if host_fold_s else None,
        "dominant": {"kernel": dominant, "achieved": dom.get("achieved_gbs"),
                     "frac": (dom["achieved_gbs"] / HBM_PEAK_GBS) if dom.get("achieved_gbs") else None,
                     "ms_avg": dom.get("ms_avg"), "units_per_launch": int(dom.get("units_avg", 0)),
                     "bytes_per_unit": KERNEL_BYTES.get(dominant),
                     "traffic": dom_traffic, "traffic_unit": "bytes per launch",
                     "traffic_check": stale or ("duration matches the PMC run" if dom_traffic else None),
                     "traffic_source": (prof["source"] + (f"; L2 hit rate {prof['l2_hit_rate']:.2f}"
                                                          if "l2_hit_rate" in prof else "") + f"; {prof['file']}")
                     if dom_traffic else None},
        "kernels": kstats,
        "phases_ms_per_step": {k: sum(v) / max(1, inst_steps) for k, v in phases.items()},
    }


def host_fed_leg(cfg, V, local, steps, tune):
    """Edges in pinned host memory, folded through gcc_forest_fold_pinned (chunked H2D on a copy stream,
    overlapped with the folds): the PCIe-inclusive rate (never the headline value)."""
    import torch

    from gelly_stream import DisjointSet
    from gelly_stream import generators as G

    E, _ = cfg.info()
    n = min(E, HOST_FED_MAX_EDGES)
    d = torch.empty(2 * n, dtype=torch.int32, device=f"cuda:{local}")
    G.generate_device(cfg, 0, n, d.data_ptr(), torch.cuda.current_stream(local).cuda_stream)
    h = torch.empty(2 * n, dtype=torch.int32, pin_memory=True)
    h.copy_(d)
    torch.cuda.synchronize()
    del d
    ds = DisjointSet(V, local)
    if tune:
        ds.tune(**tune)
    ds.reset()
    ds.fold_pinned(h.data_ptr(), n)
    ds.sync()
    reps = max(1, min(steps, 5))
    t0 = time.perf_counter()
    for _ in range(reps):
        ds.reset()
        ds.fold_pinned(h.data_ptr(), n)
        ds.compress()
        ds.sync()
    el = (time.perf_counter() - t0) / reps
    lab = ds.labels()
    ds.close()
    return {"value": n / el, "unit": "edges/s", "ms_per_step": el * 1e3, "edges": n,
            "sample": f"first {n} edges of {cfg.name} in pinned host memory, one window per step",
            "pcie_gbs": 8 * n / el / 1e9}, lab


def c2_rotating_leg(local, steps, warmup, digests, tune):
    """C2 (R-MAT s20, 16M edges, one window per step) rotating over C2_BATCHES distinct batches."""
    import torch

    from gelly_stream import DisjointSet
    from gelly_stream import generators as G

    cfg = G.CONFIGS["c2_rmat20"]
    E, V = cfg.info()
    bufs = []
    for k in range(C2_BATCHES):
        t = torch.empty(2 * E, dtype=torch.int32, device=f"cuda:{local}")
        G.generate_device(cfg, k * E, E, t.data_ptr(), torch.cuda.current_stream(local).cuda_stream)
        bufs.append(t)
    torch.cuda.synchronize()
    ds = DisjointSet(V, local)
    if tune:
        ds.tune(**tune)
    ok = True

    def step(i):
        ds.reset()
        ds.fold_device(bufs[i % C2_BATCHES].data_ptr(), E)
        ds.compress()

    for i in range(warmup):
        step(i)
    ds.sync()
    steps = max(steps, 2 * C2_BATCHES)
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    ds.sync()
    el = time.perf_counter() - t0
    for k in range(C2_BATCHES):  # parity of every batch (after the timed region)
        step(k)
        key = "c2_rmat20" if k == 0 else f"c2_rmat20@{k}"
        if key in digests:
            ok &= label_digest(ds.labels()) == int(digests[key]["digest"])
    ds.enable_timing(1)
    ds.fold_profile()
    inst = 2 * C2_BATCHES
    for i in range(inst):
        step(i)
    kstats, phases, spans = kernel_stats(ds.fold_profile(), V, inst)
    ds.enable_timing(0)
    ds.close()
    roof = make_roofline(kstats, phases, spans, inst, "c2_rmat20", "dispatch events, after the timed steps", [])
    return {"value": E * steps / el, "unit": "edges/s", "ms_per_step": el / steps * 1e3, "steps": steps,
            "batches": C2_BATCHES, "batch_bytes": 8 * E, "parity": "bit-exact" if ok else "MISMATCH",
            "roofline": {k: roof[k] for k in ("kernel", "achieved", "frac", "kernel_ms_avg", "dominant")}}


def windows_leg(name, ds_factory, windows, steps, warmup, digest, V, workload_key, note):
    """One extra workload at N = 1, from edges already in HBM: per step reset + for every window (device pointer,
    edge count) a fold and an emission (compress). Timed bare, then instrumented steps for the per-kernel stats and
    the dominant kernel's roofline; parity of the final summary (and, when the fixture has them, of every window of
    one more step) against the oracle's digests."""
    import torch

    ds = ds_factory()
    E = sum(n for _, n in windows)

    def step(check=None):
        ds.reset()
        for w, (ptr, n) in enumerate(windows):
            ds.fold_device(ptr, n)
            ds.compress()  # the window's emission (lazy in the plain regime: tune emit_div)
            if check is not None:
                check(w)
        ds.labels_device()  # the stream's last summary materialised as canonical labels, inside the step

    for _ in range(warmup):
        step()
    ds.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ds.sync()
    el = (time.perf_counter() - t0) / steps
    parity = None
    if digest is not None:
        bad = []
        per_window = digest.get("windows")

        def check(w):
            if per_window is not None:
                got, seen, comps = ds.label_digest()
                want = per_window[w]
                if (str(got), seen, comps) != (want["digest"], want["seen"], want["components"]):
                    bad.append(w)

        step(check)
        got, seen, comps = ds.label_digest()
        final = digest if per_window is None else per_window[-1]
        ok = (str(got), seen, comps) == (final["digest"], final["seen"], final["components"]) and not bad
        parity = ("bit-exact" + (" (every window)" if per_window is not None else "")) if ok else f"MISMATCH {bad}"
    inst = max(1, min(steps, 3))
    ds.enable_timing(1)
    ds.fold_profile()
    for _ in range(inst):
        step()
    kstats, phases, spans = kernel_stats(ds.fold_profile(), V, inst)
    ds.enable_timing(0)
    ds.close()
    roof = make_roofline(kstats, phases, spans, inst, workload_key, "dispatch events, after the timed steps", [])
    return {"value": E / el, "unit": "edges/s", "ms_per_step": el * 1e3, "windows": len(windows),
            "ms_per_window": el * 1e3 / len(windows), "edges": E, "steps": steps, "parity": parity, "note": note,
            "roofline": {k: roof[k] for k in ("kernel", "achieved", "frac", "kernel_ms_avg", "traffic", "traffic_source",
                                              "dominant")},
            "kernels_ms_per_step": {k: round(v["ms_per_step"], 5) for k, v in kstats.items()}}


def bip_digests():
    p = os.path.join(ROOT, "tests", "golden", "digests_bip.json")
    return json.load(open(p)) if os.path.exists(p) else {}


def bip_leg(ptr, E, V, steps, warmup, want, note, tune=None):
    """BipartitenessCheck's summary (the signed forest, gcc_signed_*) at N = 1, edges already in HBM: per step reset +
    fold + the emission on the device (compress). Timed bare on torch's stream, then fold and compress apart with
    events; parity of the final words (digest, seen ids) and the success flag against tests/golden/digests_bip.json.
    Roofline: the fold, priced like the CC plain fold (16 B per edge: the edge + both ends' words)."""
    import torch

    from gelly_stream import Candidates

    c = Candidates(V).tune(**(tune or {}))
    c.set_stream(torch.cuda.current_stream().cuda_stream)

    def step():
        c.reset()
        c.fold_device(ptr, E)
        c.compress()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fold_ms, comp_ms = [], []
    for _ in range(max(1, min(steps, 3))):
        c.reset()
        ev[0].record()
        c.fold_device(ptr, E)
        ev[1].record()
        c.compress()
        ev[2].record()
        torch.cuda.synchronize()
        fold_ms.append(ev[0].elapsed_time(ev[1]))
        comp_ms.append(ev[1].elapsed_time(ev[2]))
    parity = None
    if want is not None:
        ok = c.getSuccess() == want["success"]
        if ok and want["success"]:
            w = c.words()
            ok = str(label_digest(w)) == want["digest"] and int((w != 0xFFFFFFFF).sum()) == want["seen"]
        parity = "bit-exact" if ok else "MISMATCH"
    c.close()
    fold_s = sorted(fold_ms)[len(fold_ms) // 2] / 1e3
    achieved = 16 * E / fold_s / 1e9
    return {"value": E / el, "unit": "edges/s", "ms_per_step": el * 1e3, "edges": E, "steps": steps, "parity": parity,
            "success": want["success"] if want else None, "note": note,
            "fold_ms": fold_s * 1e3, "compress_ms": sorted(comp_ms)[len(comp_ms) // 2],
            "roofline": {"kernel": "signed_fold_kernel", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "bytes_per_unit": [16, "edge"],
                         "timing": "torch events around the fold's launches on the forest's stream"}}


def bip_legs(local, steps, warmup, d_edges=None, tune=None):
    """BipartitenessCheck (VERDICT r3 missing 5): C3's and C4's per-rank share mapped bipartite
    (generators.to_bipartite: every edge joins an even id to an odd one), and C3 as it is (an odd cycle early: the
    fold stops once the summary has failed)."""
    import torch

    from gelly_stream import generators as G

    digs = bip_digests()
    out = {}
    E3, V3 = G.CONFIGS["c3_gnm24"].info()
    try:
        d = torch.empty(2 * E3, dtype=torch.int32, device=f"cuda:{local}")
        G.generate_device(G.CONFIGS["c3_gnm24"], 0, E3, d.data_ptr(), torch.cuda.current_stream(local).cuda_stream)
        out["c3_gnm24"] = bip_leg(d.data_ptr(), E3, V3, steps, warmup, digs.get("c3_gnm24"),
                                  "C3 as it is: not bipartite (an odd cycle once its giant forms)", tune)
        G.to_bipartite_device(d)
        out["bip_c3_gnm24"] = bip_leg(d.data_ptr(), E3, V3, steps, warmup, digs.get("bip_c3_gnm24"),
                                      "to_bipartite(C3): 9.2M edges over 2^24 ids, one window", tune)
        del d
    except Exception as e:
        out["bip_c3_gnm24"] = {"error": repr(e)}
    if d_edges is not None:
        try:
            E4, V4 = G.CONFIGS["c4_kron26"].info()
            share = 1 << 27
            d = d_edges[: 2 * share].clone()
            G.to_bipartite_device(d)
            out["bip_c4_share"] = bip_leg(d.data_ptr(), share, V4, steps, warmup, digs.get("bip_c4_share"),
                                          "to_bipartite(C4's first 2^27 edges): the kron hubs, one window", tune)
            del d
        except Exception as e:
            out["bip_c4_share"] = {"error": repr(e)}
    torch.cuda.empty_cache()
    return out


def config_legs(local, steps, warmup, digests, tune, d_edges=None):
    """Every other bench config of BASELINE.json at N = 1 beside the headline: C4's 1/8
    share (one rank's fold at N = 8), C4 in 8 windows (the windowed big-id-range path), C5 in 256 windows, C2 in 16
    windows, C3 in one window and in 1M-edge windows. d_edges: C4's whole stream, already in HBM."""
    import torch

    from gelly_stream import DisjointSet
    from gelly_stream import generators as G

    out = {}

    def factory(V):
        def make():
            ds = DisjointSet(V, local)
            if tune:
                ds.tune(**tune)
            return ds
        return make

    def wins(ptr, starts):
        return [(ptr + 8 * b, e - b) for b, e in zip(starts[:-1], starts[1:])]

    if d_edges is not None:
        E4, V4 = G.CONFIGS["c4_kron26"].info()
        base = d_edges.data_ptr()
        share = 1 << 27
        try:
            out["c4_share"] = windows_leg("c4_share", factory(V4), [(base, share)], steps, warmup,
                                          digests.get("c4_share"), V4, "c4_share",
                                          "C4's first 2^27 edges into a fresh summary: what each rank folds at N = 8")
        except Exception as e:
            out["c4_share"] = {"error": repr(e)}
        for key, n in (("c4_quarter", 1 << 28), ("c4_half", 1 << 29)):  # the per-rank folds at N = 4 and 2
            try:
                out[key] = windows_leg(key, factory(V4), [(base, n)], max(2, steps // 2), 1, digests.get(key), V4, key,
                                       f"C4's first 2^{n.bit_length() - 1} edges into a fresh summary: what each rank "
                                       f"folds at N = {E4 // n} (DESIGN.md §6's predicted curve)")
            except Exception as e:
                out[key] = {"error": repr(e)}
        try:
            w = 1 << 27
            out["c4_kron26/w8"] = windows_leg("c4_kron26/w8", factory(V4), wins(base, list(range(0, E4 + 1, w))),
                                              max(2, steps // 4), 1, digests.get("c4_kron26/w8"), V4, "c4_w8",
                                              "C4 in 8 windows of 2^27 edges, an emission (compress) per window")
        except Exception as e:
            out["c4_kron26/w8"] = {"error": repr(e)}
    for key, cfg_name, wedges in (("c5_adversarial/w64K", "c5_adversarial", 1 << 16),
                                  ("c2_rmat20/w1M", "c2_rmat20", 1 << 20),
                                  ("c3_gnm24", "c3_gnm24", 0),
                                  ("c3_gnm24/w1M", "c3_gnm24", 1 << 20)):
        try:
            cfg = G.CONFIGS[cfg_name]
            E, V = cfg.info()
            d = torch.empty(2 * E, dtype=torch.int32, device=f"cuda:{local}")
            G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream(local).cuda_stream)
            torch.cuda.synchronize()
            starts = list(range(0, E, wedges)) + [E] if wedges else [0, E]
            dig = digests.get(key)  # every window's digest (tests/golden/make_stream_digests.py WINDOWED)
            out[key] = windows_leg(key, factory(V), wins(d.data_ptr(), starts), steps, warmup, dig, V, cfg_name,
                                   f"{cfg_name} in {len(starts) - 1} window(s), an emission per window")
            del d
            torch.cuda.empty_cache()
        except Exception as e:
            out[key] = {"error": repr(e)}
    return out


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if os.environ.get("GELLY_SHARE_GPU"):  # rehearsal: every rank on cuda:0 (never for a measurement)
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        backend = os.environ.get("GELLY_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI; gloo: 1-GPU rehearsal
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)

    from gelly_stream import generators as G
    from gelly_stream.distributed import ForestGroup, TorchDisjointSet

    cfg = G.CONFIGS[args.workload]
    E, V = cfg.info()
    starts = window_starts(cfg, args.window_edges)
    n_windows = len(starts) - 1
    chunks = rank_chunks(starts, rank, world)
    my_edges = sum(hi - lo for lo, hi in chunks)
    tune = {k: float(v) for k, v in (kv.split("=") for kv in args.tune.split(","))} if args.tune else {}

    # this rank's chunks of every window, generated straight into HBM (outside any timed region)
    d_edges = torch.empty(2 * max(1, my_edges), dtype=torch.int32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream(local)
    offs, off = [], 0
    for lo, hi in chunks:
        G.generate_device(cfg, lo, hi - lo, d_edges.data_ptr() + 8 * off, stream.cuda_stream)
        offs.append((off, hi - lo))
        off += hi - lo
    forest = TorchDisjointSet(V, local)
    if tune:
        forest.ds.tune(**tune)
    group = ForestGroup() if world > 1 else None
    base_ptr = d_edges.data_ptr()

    host_fold_s = []
    merge_events = []  # (before merge, after merge) on the forest's stream, N > 1, instrumented steps only

    mark = None
    if args.step_marker:
        from gelly_stream.native import call as native_call

        def mark():
            native_call("gcc_step_mark", stream.cuda_stream)

    def step(instrument):
        if mark is not None:
            mark()
        forest.ds.reset()
        for w in range(n_windows):
            o, n = offs[w]
            th = time.perf_counter()
            forest.ds.fold_device(base_ptr + 8 * o, n)
            if instrument:
                host_fold_s.append(time.perf_counter() - th)
            if group is not None:
                if instrument:
                    ev1 = torch.cuda.Event(enable_timing=True)
                    ev1.record(stream)
                group.merge_forest(forest)
                if instrument:
                    ev2 = torch.cuda.Event(enable_timing=True)
                    ev2.record(stream)
                    merge_events.append((ev1, ev2))
            else:
                forest.compress()
        forest.ds.labels_device()  # the stream's last summary as canonical labels (a lazy emission's deferred compress)

    for _ in range(args.warmup):
        step(False)
    # "timed": every kernel of the timed steps carries its own dispatch start/stop events (hipExtLaunchKernel, no
    # extra packets); "after": the timed steps run bare and min(steps, 5) instrumented steps follow them
    timed_inst = args.phase_timing == "timed"
    forest.ds.enable_timing(1 if timed_inst else 0)
    forest.ds.fold_profile()  # drain the warmup log
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed_inst)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    inst_steps = args.steps if timed_inst else 0
    if args.phase_timing == "after":
        inst_steps = min(args.steps, 5)
        forest.ds.enable_timing(1)
        for _ in range(inst_steps):
            step(True)
        torch.cuda.synchronize()
    log = forest.ds.fold_profile()
    forest.ds.enable_timing(0)
    kstats, phases, spans = kernel_stats(log, V, inst_steps)
    timing_note = ("hipExtLaunchKernel dispatch events on the forest's stream, every timed step" if timed_inst
                   else f"hipExtLaunchKernel dispatch events, {inst_steps} steps after the timed region")
    roofline = make_roofline(kstats, phases, spans, inst_steps, args.workload, timing_note, host_fold_s)

    merge_ms = [a.elapsed_time(b) for a, b in merge_events]
    labels = forest.ds.labels()
    seen = int(np.count_nonzero(labels != 0xFFFFFFFF))
    comps = int(np.count_nonzero(labels == np.arange(V, dtype=np.uint32)))
    digests = golden_digests()
    parity = None
    if not args.no_parity and args.workload in digests:  # any window size: the final partition is the stream's
        parity = "bit-exact" if label_digest(labels) == int(digests[args.workload]["digest"]) else "MISMATCH"
    if dist:  # every rank holds the global partition after the merge: all must agree with the fixture
        ok = torch.tensor([0 if parity == "MISMATCH" else 1], dtype=torch.int32, device=f"cuda:{local}")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if parity is not None and int(ok.item()) == 0:
            parity = "MISMATCH"

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    result = {
        "metric": "edges/sec into CC summary",
        "value": E * args.steps / elapsed,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": f"{cfg.name}: " + {
                "c1_example": "ConnectedComponentsExample default data, 1000 ms event-time windows",
                "c2_rmat20": "R-MAT scale 20 (A,B,C,D=0.57,0.19,0.19,0.05), edge factor 16, seeded permutation",
                "c3_gnm24": "uniform G(n,m) n=2^24 m=9227469",
                "c4_kron26": "Kronecker scale 26, edge factor 16 (2^30 edges), seeded permutation",
                "c4_share": "Kronecker scale 26, the first 2^27 edges of C4's stream",
                "c5_adversarial": "shuffled 2^23-path + 1024 stars of 8192, windows of 2^16 edges",
            }.get(cfg.name, cfg.name),
            "stream_edges": E,
            "edges_per_gpu": my_edges,
            "vertices": V,
            "windows_per_step": n_windows,
            "parallelism": f"dp{world}",
            "partition": "rank r folds the r-th contiguous 1/N of every window (strong scaling of one stream)",
            "merge": ("gcc_forest_group_merge: delta all_gather over RCCL ((x, root) of the ids each rank's window changed) "
                      "when every rank is armed, else compact (giant bitmap + others list; label all_gather fallback)"
                      if world > 1 else "none"),
        },
        "roofline": roofline,
        "predicted": (dict(PREDICTED.get(args.workload, {}).get(world, {}),
                           source="DESIGN.md §6 (per-rank folds and merge kernels measured on one GPU; all_gather modelled)")
                      if PREDICTED.get(args.workload, {}).get(world) else None),
        "parity": parity,
        "summary": {"seen": seen, "components": comps},
        "merge": ({"ms_per_window": sum(merge_ms) / len(merge_ms), "windows_per_step": n_windows,
                   "ms_per_step": sum(merge_ms) / max(1, inst_steps),
                   "message_bytes": group.last.get("bytes"),
                   "gathered_bytes_per_window": (group.last.get("bytes") or 0) * world,
                   "all_gathers_last_window": group.last.get("rounds"), "label_exchange": group.last.get("labels"),
                   "kind_last_window": group.last.get("kind"),
                   "bytes_all_rounds_last_window": group.last.get("bytes_all_rounds"),
                   "full_label_bytes": 4 * V,
                   "timing": "torch events around gcc_forest_group_merge on the forest's stream, instrumented steps"}
                  if group is not None and merge_ms else None),
    }
    if world == 1 and not args.no_extras:
        forest.ds.close()
        try:
            result["configs"] = config_legs(local, args.steps, args.warmup, digests, tune,
                                            d_edges if args.workload == "c4_kron26" else None)
        except Exception as e:
            result["configs"] = {"error": repr(e)}
        try:
            result["bipartiteness"] = bip_legs(local, args.steps, args.warmup,
                                               d_edges if args.workload == "c4_kron26" else None)
        except Exception as e:
            result["bipartiteness"] = {"error": repr(e)}
        del d_edges
        torch.cuda.empty_cache()
        try:
            hf, hl = host_fed_leg(cfg, V, local, args.steps, tune)
            if hf["edges"] == E and digests.get(args.workload):
                hf["parity"] = "bit-exact" if label_digest(hl) == int(digests[args.workload]["digest"]) else "MISMATCH"
            result["host_fed"] = hf
        except Exception as e:  # a failed extra leg must not hide the headline measurement
            result["host_fed"] = {"error": repr(e)}
        torch.cuda.empty_cache()
        if args.workload != "c2_rmat20":
            try:
                result["c2_rotating"] = c2_rotating_leg(local, args.steps, args.warmup, digests, tune)
            except Exception as e:
                result["c2_rotating"] = {"error": repr(e)}
    if world == 1 and args.cpu_seconds > 0:
        result["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
    print(json.dumps(result))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
