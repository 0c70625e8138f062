"""Host-side cost of one bench step on one GPU: async steps (host runs ahead), steps with a host sync after each
(what a per-window merge that reads gathered headers forces at N > 1), and the host enqueue time per step.
Usage: python tools/probe_host.py [workload] [steps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gelly-streaming_amd"))
import torch  # noqa: E402

from gelly_stream import generators as G  # noqa: E402
from gelly_stream.distributed import TorchDisjointSet  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2_rmat20"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    cfg = G.CONFIGS[wl]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), torch.cuda.current_stream().cuda_stream)
    f = TorchDisjointSet(V, 0)
    tune = {}
    for kv in sys.argv[3:]:
        k, v = kv.split("=")
        tune[k] = float(v)
    if tune:
        f.ds.tune(**tune)

    def step():
        f.ds.reset()
        f.ds.fold_device(d.data_ptr(), E)
        f.ds.compress()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    for mode in ("async", "sync", "async", "sync"):
        enq = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            a = time.perf_counter()
            step()
            enq.append(time.perf_counter() - a)
            if mode == "sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        print(f"{wl} {mode:5s} {ms * 1e3:8.1f} us/step  enqueue median {statistics.median(enq) * 1e6:7.1f} us "
              f"min {min(enq) * 1e6:7.1f} us  {E / ms / 1e6:.1f} Gedge/s", flush=True)


if __name__ == "__main__":
    main()
