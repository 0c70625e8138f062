#!/usr/bin/env python3
"""Benchmark: edges/sec into the streaming connected-components summary on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of synthetic input: reset the summary to its initial
value, fold this rank's edge chunk (already resident in HBM) window by window into the device forest,
and emit the summary after every window (canonicalising compress; with N>1 the butterfly forest merge
over RCCL/xGMI first). Weak scaling: every rank folds the same number of edges of one shared stream
(rank r owns chunk r), so value = N * edges_per_rank * K / max-over-ranks time.

N=1 default workload: configs[1] = R-MAT scale 20 (1M vertices, 16M edges), one merge window per step.
Launch: python bench.py [--gpus N --steps K --warmup W]  (N>1 under torch.distributed.run, one rank per GPU).
"""
from __future__ import annotations

import argparse
import json
import math
import os
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
    "seed_pack_kernel": (5.125, "id"),      # flag byte read + parent write + 1 bitmap bit (the init variant)
    "seed_hub_kernel": (1.125, "id"),       # flag byte + bitmap bit cleared
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2_rmat20")
    ap.add_argument("--window-edges", type=int, default=0, help="edges per merge window per rank (0 = config default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline work (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU-baseline threads (0 = min(16, cores))")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--tune", default="", help="fold-pipeline knobs k=v,... (gcc_forest_tune; speed only)")
    ap.add_argument("--phase-timing", choices=["timed", "after", "off"], default="after",
                    help="per-kernel dispatch events in the timed steps, in extra steps after them, or not at all")
    return ap.parse_args()


def rank_stream(cfg, world):
    """The shared stream all ranks draw from, and the per-rank edge count (weak scaling)."""
    from gelly_stream import generators as G

    E1, V = cfg.info()
    if world > 1 and cfg.kind in (2, 3):  # RMAT / GNM: a world-times longer stream over the same ids
        cfg = G.scaled(cfg, n_edges=cfg.n_edges * world)
    return cfg, E1, V


def profile_record(workload):
    """The newest committed rocprofv3 PMC summary for this workload (profiles/*_pmc_<workload>.json), or None."""
    pdir = os.path.join(ROOT, "profiles")
    best = None
    if os.path.isdir(pdir):
        for f in sorted(os.listdir(pdir)):
            if f.endswith(f"_pmc_{workload}.json"):
                try:
                    best = json.load(open(os.path.join(pdir, f)))
                except Exception:
                    continue
    return best


def cpu_baseline(cfg, E, V, target_s, threads):
    """The CPU oracle (restated reference topology) timed on this host: the same stream, one window."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc  # cpu_baseline leg only

    from gelly_stream import generators as G

    pairs = G.generate_host(cfg, 0, E)
    starts = [0, E]
    reps, total, digest = 0, 0.0, None
    while True:
        out = orc.cc_stream(pairs, starts, V, partitions=threads, threads=threads, want_digest=(reps == 0))
        if reps == 0:
            digest = int(out["digest"][0])
        total += out["fold_seconds"]
        reps += 1
        if total >= target_s or reps >= 50:
            break
    return {
        "value": E * reps / total,
        "unit": "edges/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full {cfg.name} stream ({E} edges, 1 window) x {reps} reps = {total:.1f} s; "
                  f"{threads} partitions/threads folding HashMap union-by-rank DisjointSets + serial CombineCC merge "
                  f"(oracle/cc_oracle.c); host cores visible: {os.cpu_count()}",
    }, digest


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

    base = G.CONFIGS[args.workload]
    cfg, E1, V = rank_stream(base, world)
    W = args.window_edges or base.window_edges or E1
    starts = list(range(0, E1, W)) + [E1]
    n_windows = len(starts) - 1

    # edges of this rank's chunk, generated straight into HBM (outside any timed region)
    d_edges = torch.empty(2 * E1, dtype=torch.int32, device=f"cuda:{local}")
    stream = torch.cuda.current_stream(local)
    G.generate_device(cfg, rank * E1, E1, d_edges.data_ptr(), stream.cuda_stream)
    forest = TorchDisjointSet(V, local)
    if args.tune:
        forest.ds.tune(**{k: float(v) for k, v in (kv.split("=") for kv in args.tune.split(","))})
    group = ForestGroup() if world > 1 else None
    base_ptr = d_edges.data_ptr()

    host_fold_s = []
    merge_events = []  # (before merge, after merge) on the forest's stream, N > 1, instrumented steps only

    def step(instrument):
        forest.ds.reset()
        for w in range(n_windows):
            b, e = starts[w], starts[w + 1]
            th = time.perf_counter()
            forest.ds.fold_device(base_ptr + 8 * b, e - b)
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

    for _ in range(args.warmup):
        step(False)
    # "timed": every kernel of the timed steps carries its own dispatch start/stop events (hipExtLaunchKernel, no
    # extra packets); "after": the timed steps run bare and min(steps, 10) instrumented steps follow them
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
        inst_steps = min(args.steps, 10)
        forest.ds.enable_timing(1)
        for _ in range(inst_steps):
            step(True)
        torch.cuda.synchronize()
    log = forest.ds.fold_profile()
    forest.ds.enable_timing(0)

    # per-kernel durations (each kernel's own dispatch events) and per-fold device spans, grouped by kernel
    kernel_of = {"filtered": "fold_filtered_kernel", "sample": "fold_kernel", "plain": "fold_kernel",
                 "seed_hub": "seed_hub_kernel", "seed_bfs": "seed_bfs_kernel", "seed_pack": "seed_pack_kernel",
                 "seed_init": "seed_pack_kernel", "refresh": "compress_bits_kernel", "compress": "compress_bits_kernel", "refresh_bits": "compress_bits_kernel",
                 "compress_inc": "compress_inc_kernel", "refresh_inc": "compress_inc_kernel",
                 "vote": "giant_vote_kernel"}
    phases, kernels, spans = {}, {}, []
    for name, ms, n in log:
        if name == "begin" or name == "slow_edges":
            continue
        if name == "fold_span":
            spans.append((ms, n))
            continue
        phases.setdefault(name, []).append(ms)
        kernels.setdefault(kernel_of.get(name, name), []).append((ms, n))
    avg_fold_s = (sum(ms for ms, _ in spans) / len(spans) / 1e3) if spans else float("nan")
    avg_fold_edges = (sum(n for _, n in spans) / len(spans)) if spans else E1 / n_windows
    pipeline_gbs = BYTES_PER_EDGE * avg_fold_edges / avg_fold_s / 1e9 if spans else None

    def kernel_bytes(k, units):
        """Algorithmic bytes of one launch: per edge for the edge kernels, per id otherwise."""
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
                     "ms_per_step": sum(ms for ms, _ in v) / max(1, inst_steps),
                     "achieved_gbs": (by / (ms_avg / 1e3) / 1e9) if by and ms_avg > 0 else None}
    prof = profile_record(args.workload)
    # the dominant kernel: the largest device time per step
    dominant = max(kstats, key=lambda k: kstats[k]["ms_per_step"]) if kstats else None
    dom_ms = kstats[dominant]["ms_avg"] if dominant else float("nan")
    dom_units = (sum(n for _, n in kernels[dominant]) / len(kernels[dominant])) if dominant else 0
    achieved = kstats[dominant]["achieved_gbs"] if dominant else None
    traffic = None
    if prof and dominant and dominant in prof.get("kernel", "") and \
            abs(prof.get("edges_per_launch", 0) - dom_units) <= 0.01 * max(1, dom_units):
        traffic = prof["hbm_bytes_per_launch"]

    merge_ms = [a.elapsed_time(b) for a, b in merge_events]
    labels = forest.ds.labels()
    seen = int(np.count_nonzero(labels != 0xFFFFFFFF))
    comps = int(np.count_nonzero(labels == np.arange(V, dtype=np.uint32)))

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    total_edges = world * E1 * args.steps
    result = {
        "metric": "edges/sec into CC summary",
        "value": total_edges / elapsed,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": {
            "workload": f"{base.name}: " + {
                "c2_rmat20": "R-MAT scale 20 (A,B,C,D=0.57,0.19,0.19,0.05), edge factor 16, seeded permutation",
                "c3_gnm24": "uniform G(n,m) n=2^24 m=9227469",
                "c4_kron26": "Kronecker scale 26, edge factor 16",
                "c4_share": "Kronecker scale 26, 2^27 edges per GPU of C4's stream (x8 GPUs = C4's 2^30 edges)",
                "c5_adversarial": "shuffled 2^23-path + 1024 stars of 8192",
            }.get(base.name, base.name),
            "edges_per_gpu": E1,
            "vertices": V,
            "windows_per_step": n_windows,
            "window_edges": W,
            "parallelism": f"dp{world}",
            "merge": ("compact all_gather over RCCL (giant bitmap + others list; label butterfly fallback)"
                      if world > 1 else "none"),
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dominant,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": traffic,
            "traffic_unit": "bytes per launch",
            "traffic_source": (prof["source"] + f"; L2 hit rate {prof['l2_hit_rate']:.2f}") if traffic else None,
            "kernel_ms_avg": dom_ms,
            "kernel_units_per_launch": int(dom_units),
            "bytes_per_unit": KERNEL_BYTES.get(dominant),
            "timing": ("hipExtLaunchKernel dispatch events on the forest's stream, every timed step"
                       if timed_inst else f"hipExtLaunchKernel dispatch events, {inst_steps} steps after the timed region"),
            "kernels": kstats,
            "phases_ms_per_step": {k: sum(v) / max(1, inst_steps) for k, v in phases.items()},
            "pipeline": {"fold_ms_avg": avg_fold_s * 1e3, "edges_per_fold": int(avg_fold_edges),
                         "bytes_per_edge": BYTES_PER_EDGE, "achieved": pipeline_gbs,
                         "frac": (pipeline_gbs / HBM_PEAK_GBS) if pipeline_gbs else None,
                         "host_enqueue_ms_avg": (sum(host_fold_s) / len(host_fold_s) * 1e3) if host_fold_s else None},
        },
        "summary": {"seen": seen, "components": comps},
        "merge": ({"ms_avg": sum(merge_ms) / len(merge_ms), "last": group.last} if group is not None and merge_ms
                  else None),
    }
    if world == 1 and args.cpu_seconds > 0:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        cb, digest = cpu_baseline(cfg, E1, V, args.cpu_seconds, threads)
        result["cpu_baseline"] = cb
        if not args.no_parity:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as orc

            result["parity"] = "bit-exact" if orc.label_digest(labels) == digest else "MISMATCH"
    print(json.dumps(result))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
