"""inc_div by speed: per-window fold + compress kernel time on C3 (G(n, m), 2^24 ids) and C5
(path + stars, 2^24 ids) for window sizes from 1/256 to 1/4 of the id range, with the incremental compress
allowed up to 1/inc_div of the ids. Prints, per (config, window, inc_div), the summed kernel ms per window of the
fold and of the emission (compress_inc or the full compress), from the forest's dispatch events.
Usage: python tools/sweep_inc_div.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def main():
    for cfg_name in ("c3_gnm24", "c5_adversarial"):
        cfg = G.CONFIGS[cfg_name]
        E, V = cfg.info()
        d = torch.empty(2 * E, dtype=torch.int32, device="cuda:0")
        G.generate_device(cfg, 0, E, d.data_ptr(), 0)
        torch.cuda.synchronize()
        for wl in (16, 18, 20, 21, 22):
            W = 1 << wl
            for inc_div in (4, 8, 16, 32, 64, 1 << 30):
                with DisjointSet(V) as ds:
                    ds.tune(incremental=1, inc_div=inc_div)
                    n_w = min(E // W, 24)
                    for rep in range(2):  # rep 0 warms up (allocations); rep 1 is timed
                        ds.reset()
                        if rep == 1:
                            ds.enable_timing(1)
                            ds.fold_profile()
                        for w in range(n_w):
                            ds.fold_device(d.data_ptr() + 8 * w * W, W)
                            ds.compress()
                        ds.sync()
                    prof = ds.fold_profile()
                    ds.enable_timing(0)
                # skip the first window (a fresh forest's start) in the averages
                fold = comp = 0.0
                inc = full = 0
                k = -1
                for name, ms, n in prof:
                    if name == "begin":
                        k += 1
                        continue
                    if k < 1 or name in ("fold_span", "slow_edges"):
                        continue
                    if name in ("compress", "compress_inc"):
                        comp += ms
                        inc += name == "compress_inc"
                        full += name == "compress"
                    else:
                        fold += ms
                nw = max(1, n_w - 1)
                print(f"{cfg_name} W=2^{wl} inc_div={inc_div}: fold {1e3 * fold / nw:8.1f} us  emission "
                      f"{1e3 * comp / nw:8.1f} us per window ({inc} incremental, {full} full)", flush=True)
        del d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
