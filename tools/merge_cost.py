"""One-GPU estimate of the device side of ForestGroup's compact merge at the bench's weak-scaling shape:
P forests on cuda:0 each fold 16M edges of one shared R-MAT s20 stream (rank r = chunk r), then the merge's
device work is timed with HIP events — encode, the P-1 absorbs of one rank, its final compress — and compared
with the label-butterfly's absorb+compress per round. The RCCL transfer itself (one all_gather of the
messages) needs P GPUs and is not in these numbers. Usage: python tools/merge_cost.py [P]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gelly-streaming_amd")]
import torch  # noqa: E402

from gelly_stream import DisjointSet, native  # noqa: E402
from gelly_stream import generators as G  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    base = G.CONFIGS["c2_rmat20"]
    E1, V = base.info()
    cfg = G.scaled(base, n_edges=E1 * P)
    d = torch.empty(2 * E1 * P, dtype=torch.int32, device="cuda:0")
    G.generate_device(cfg, 0, E1 * P, d.data_ptr(), 0)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream().cuda_stream
    ranks = [DisjointSet(V) for _ in range(P)]
    for r, ds in enumerate(ranks):
        ds.set_stream(s)
    cap = V // 16
    stride = (native.msg_bytes(V, cap) + 15) // 16 * 16
    packed = torch.empty(P * stride, dtype=torch.uint8, device="cuda:0")
    msgs = [packed[r * stride:(r + 1) * stride] for r in range(P)]
    for rep in range(4):
        for r, ds in enumerate(ranks):
            ds.reset()
            ds.fold_device(d.data_ptr() + 8 * E1 * r, E1)
            ds.compress()
        torch.cuda.synchronize()
        t = [ev() for _ in range(4)]
        t[0].record()
        for r, ds in enumerate(ranks):
            ds.encode_message(msgs[r].data_ptr(), cap)
        t[1].record()
        hdr = [m[:16].cpu().numpy().view("<u4") for m in msgs]
        nmax = max(int(h[1]) for h in hdr)
        t2 = ev()
        t2.record()
        ranks[0].absorb_messages(packed.data_ptr(), stride, P, 0, cap)  # rank 0 absorbs everyone else
        t[2].record()
        ranks[0].compress()
        t[3].record()
        torch.cuda.synchronize()
        enc = t[0].elapsed_time(t[1]) / P
        print(f"P={P} rep={rep}: encode {enc * 1e3:.1f} us/rank, absorb {P - 1} msgs (1 launch) {t2.elapsed_time(t[2]) * 1e3:.1f} us, "
              f"compress {t[2].elapsed_time(t[3]) * 1e3:.1f} us; n_others max {nmax}, message "
              f"{native.msg_bytes(V, nmax) / 1024:.0f} KiB vs labels {4 * V / 1024:.0f} KiB", flush=True)
    # label butterfly, device side of one round: absorb a partner's label array + compress
    for rep in range(3):
        lab = torch.empty(V, dtype=torch.int32, device="cuda:0")
        ranks[1].compress()
        torch.cuda.synchronize()
        lab.copy_(torch.from_numpy(ranks[1].labels().view("int32")).cuda())
        t = [ev() for _ in range(3)]
        t[0].record()
        ranks[0].merge_labels_device(lab.data_ptr(), V)
        t[1].record()
        ranks[0].compress()
        t[2].record()
        torch.cuda.synchronize()
        print(f"butterfly round (device side): absorb labels {t[0].elapsed_time(t[1]) * 1e3:.1f} us, "
              f"compress {t[1].elapsed_time(t[2]) * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
