"""Serialized timing of one rank's merge at C4's strong split (what bench.py runs at N > 1 per window, minus the
RCCL transfer): P forests fold the r-th 1/P of the C4 stream on one GPU; then, one step at a time with a sync
after each, every forest's encode (of its uncompressed forest, as gcc_forest_group_merge does) into one all_gather-shaped buffer, and forest 0's
absorb of the P-1 peer messages + its final compress. Kernels never overlap, so a rocprofv3 kernel trace of this
script gives clean per-kernel durations. Usage: python tools/merge_probe.py [P]"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402
from gelly_stream.native import call, msg_bytes  # noqa: E402


def ms(t0):
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cfg = G.CONFIGS["c4_kron26"]
    E, V = cfg.info()
    d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E, d.data_ptr(), 0)
    torch.cuda.synchronize()
    forests = [DisjointSet(V) for _ in range(P)]

    def fold(r):
        lo, hi = E * r // P, E * (r + 1) // P
        forests[r].reset()
        forests[r].fold_device(d.data_ptr() + 8 * lo, hi - lo)
        forests[r].sync()

    for r in range(P):
        fold(r)
    cap = max(1024, V // 256)  # about what gcc_forest_group_merge settles on at C4 (1.5x the longest list)
    stride = (msg_bytes(V, cap) + 15) // 16 * 16
    buf = torch.empty(P * stride, dtype=torch.uint8, device="cuda:0")
    for rep in range(3):
        fold(0)
        t = {}
        enc = []
        for r in range(P):  # one at a time (each forest has its own stream)
            t0 = time.perf_counter()
            call("gcc_forest_encode", forests[r].handle, ctypes.c_void_p(buf.data_ptr() + r * stride), cap)
            enc.append(ms(t0))
        t["encode_max"] = max(enc)
        hdr = buf.view(P, stride)[:, :16].cpu().view(torch.int32)
        t0 = time.perf_counter()
        call("gcc_forest_absorb_many", forests[0].handle, ctypes.c_void_p(buf.data_ptr()), stride, P, 0, cap)
        forests[0].sync()
        t["absorb"] = ms(t0)
        t0 = time.perf_counter()
        forests[0].compress()
        forests[0].sync()
        t["compress_post"] = ms(t0)
        print(f"P={P} rep {rep}: " + ", ".join(f"{k} {v:.3f} ms" for k, v in t.items()) +
              f"; list entries per peer max {int(hdr[:, 1].max())}", flush=True)
    for f in forests:
        f.close()


if __name__ == "__main__":
    main()
