"""Why is the filtered pass of a fresh (seeded) fold slower than a refold? Times the filtered kernel (dispatch
events) in: fresh fold; refold right after it (bitmap = the seeded C); refold after a compress (bitmap = the
final giant); and a fresh fold whose batch was just streamed by another kernel (warm MALL). Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def filt(ds):
    return [round(ms * 1e3, 1) for k, ms, _ in ds.fold_profile() if k == "filtered"]


def main():
    cfg = G.CONFIGS["c2_rmat20"]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    junk = torch.empty(64 << 20, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    ds = DisjointSet(V)
    ds.set_stream(torch.cuda.current_stream().cuda_stream)
    ds.enable_timing(1)
    for rep in range(4):
        ds.reset()
        ds.fold_device(d.data_ptr(), E)
        a = filt(ds)
        ds.fold_device(d.data_ptr(), E)       # refold, no compress in between (bitmap = seeded C)
        b = filt(ds)
        ds.compress()
        ds.fold_device(d.data_ptr(), E)       # refold after compress (bitmap = final giant)
        c = filt(ds)
        junk.add_(1)                           # 256 MiB of other traffic: evict the edges from the MALL
        ds.fold_device(d.data_ptr(), E)       # refold from cold caches
        e = filt(ds)
        ds.reset()
        s = d.sum()                            # stream the batch right before a fresh fold (warm MALL)
        ds.fold_device(d.data_ptr(), E)
        f = filt(ds)
        torch.cuda.synchronize()
        print(f"rep {rep}: fresh {a} | refold(seed C) {b} | refold(final) {c} | refold cold {e} | fresh warm {f} us",
              flush=True)


if __name__ == "__main__":
    main()
