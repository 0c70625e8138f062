"""Cross-GPU combine of the per-rank CC forests (replaces the reference's all-to-one window gather).

Reference: SummaryBulkAggregation.run (…/SummaryBulkAggregation.java:81-83) gathers every partition's
partial DisjointSet, Kryo-serialised, to ONE task: ``timeWindowAll(t).reduce(CombineCC)`` then the
parallelism-1 ``Merger`` (…/SummaryAggregation.java:107-119). SummaryTreeReduce (…/SummaryTreeReduce.java:95-123)
pairs partitions up in a log2 tree instead.

MI355X form: every rank (one process per GPU) keeps a full-range forest, and the whole merge runs inside
libgelly_cc (csrc/gelly_group.cpp, ``gcc_forest_group_merge``) over its own RCCL communicator: each rank compresses
and encodes its forest as a compact message (include/gelly_cc.h: header, bitmap of the largest component, (v, label)
list of the other seen ids), ONE ncclAllGather over xGMI moves every message to every rank, and each rank absorbs
the P-1 others on its device. The list capacity is speculative (the last window's need x1.5; the gathered headers
say whether a repeat round is needed); when the compact form stops paying, the label arrays are all-gathered. Every
rank ends with the global partition — the forest the reference's reduce + Merger emit — with no serial bottleneck.
torch.distributed only carries the communicator's unique id (bootstrap bytes); it is never on the data path, and
this module has no second (Python) implementation of the protocol: with several ranks on ONE device (tests, the
one-GPU rehearsal) GELLY_RCCL_LIB points the same C++ loop at the shared-memory stand-in tests/cpp/shm_rccl.cpp.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence


class TorchDisjointSet:
    """A DisjointSet whose two id-range buffers are torch tensors on this rank's GPU and whose HIP stream is
    torch's current stream, so that torch work (events, the bench's barriers) orders with the forest's kernels."""

    def __init__(self, id_capacity: int, device: int = 0):
        import torch

        from .summaries import DisjointSet

        self.id_capacity = int(id_capacity)
        self.device = int(device)
        self.bufs = [torch.empty(self.id_capacity, dtype=torch.int32, device=f"cuda:{self.device}") for _ in range(2)]
        self.ds = DisjointSet(self.id_capacity, self.device, d_buffers=(self.bufs[0].data_ptr(), self.bufs[1].data_ptr()))
        self.ds.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def __getattr__(self, name):  # delegate the DisjointSet surface (find, getMatches, fold_device, compress, ...)
        return getattr(self.ds, name)


class RcclComm:
    """One rank's RCCL communicator behind the C ABI (gcc_comm_*, csrc/gelly_group.cpp): the merge of
    timeWindowAll(t).reduce(CombineCC) + Merger (SummaryBulkAggregation.java:81-83) as ONE all_gather of compact
    forest messages over xGMI, run entirely by libgelly_cc (no torch collective on the data path)."""

    ID_BYTES = 128  # GCC_COMM_ID_BYTES

    def __init__(self, device: int, nranks: int, rank: int, uid: bytes, _handle=None):
        from .native import call

        self.device, self.nranks, self.rank = int(device), int(nranks), int(rank)
        if _handle is not None:
            self._h = _handle
            return
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), self.ID_BYTES)
        call("gcc_comm_init", self.device, self.nranks, self.rank, buf, ctypes.byref(h))
        self._h = h

    @classmethod
    def unique_id(cls) -> bytes:
        from .native import call

        buf = ctypes.create_string_buffer(cls.ID_BYTES)
        call("gcc_comm_unique_id", buf)
        return buf.raw

    @classmethod
    def init_all(cls, devices: Sequence[int]) -> list["RcclComm"]:
        """One process driving several GPUs: rank i on devices[i] (ncclCommInitAll)."""
        from .native import call

        n = len(devices)
        devs = (ctypes.c_int * n)(*devices)
        hs = (ctypes.c_void_p * n)()
        call("gcc_comm_init_all", n, devs, hs)
        return [cls(d, n, i, b"", _handle=ctypes.c_void_p(hs[i])) for i, d in enumerate(devices)]

    def merge(self, ds) -> None:
        """Collective: ds (a DisjointSet on this rank's device) := the union of every rank's forest."""
        from .native import call

        call("gcc_forest_group_merge", ds.handle, self._h)
        if hasattr(ds, "_dirty"):  # the forest changed under the Python view: drop its cached labels
            ds._dirty()

    def last_bytes(self) -> int:
        from .native import call

        b = ctypes.c_uint64()
        call("gcc_comm_info", self._h, None, None, ctypes.byref(b))
        return b.value

    def last_merge(self) -> dict:
        """The last merge: all_gathers it took (compact rounds + the label exchange), whether it ended with the
        label exchange, the bytes each rank contributed to its last all_gather, the next merge's list capacity."""
        from .native import call

        rounds, labels, cap = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint64()
        call("gcc_comm_last_merge", self._h, ctypes.byref(rounds), ctypes.byref(labels), ctypes.byref(cap))
        kind, total, dcap = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        call("gcc_comm_last_merge_kind", self._h, ctypes.byref(kind), ctypes.byref(total), ctypes.byref(dcap))
        return {"rounds": rounds.value, "labels": bool(labels.value), "bytes": self.last_bytes(),
                "cap_others": cap.value, "kind": ("compact", "labels", "delta")[kind.value],
                "bytes_all_rounds": total.value, "cap_delta": dcap.value}

    def close(self) -> None:
        from .native import call

        if getattr(self, "_h", None):
            call("gcc_comm_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def group_merge(forests: Sequence, comms: Optional[Sequence[RcclComm]] = None) -> None:
    """Single process: every forest := the union of all of them (gcc_group_merge). Forests on one device need no
    comms; forests on several devices need RcclComm.init_all over their devices (comms[i] for forests[i])."""
    from .native import call

    n = len(forests)
    hs = (ctypes.c_void_p * n)(*[f.handle.value for f in forests])
    cs = None if comms is None else (ctypes.c_void_p * n)(*[c._h.value for c in comms])
    call("gcc_group_merge", hs, n, cs)
    for f in forests:
        f._dirty()


class ForestGroup:
    """Cross-rank merge of one forest per rank: SummaryBulkAggregation's timeWindowAll(t).reduce(CombineCC) + Merger
    (…/SummaryBulkAggregation.java:81-83) over every rank of a torch.distributed group. Rank 0 creates the RCCL unique
    id, torch.distributed broadcasts its bytes (any backend: nccl, or gloo for rehearsals), and every merge is
    gcc_forest_group_merge on this rank's communicator."""

    def __init__(self, group=None, device: Optional[int] = None):
        import torch
        import torch.distributed as dist

        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        dev = torch.cuda.current_device() if device is None else int(device)
        uid = [RcclComm.unique_id() if self.rank == 0 else None]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        dist.broadcast_object_list(uid, src=src, group=group)  # bootstrap bytes only
        self.comm = RcclComm(dev, self.world, self.rank, uid[0])
        self.last = {}  # what the last merge did (measurement / tests): RcclComm.last_merge()

    def merge_forest(self, forest) -> None:
        """forest := union of every rank's forest (collective: every rank must call it)."""
        self.comm.merge(forest.ds if hasattr(forest, "ds") else forest)
        self.last = self.comm.last_merge()

    def reduce(self, summary, combineFun=None):
        """SummaryBulkAggregation's timeWindowAll(...).reduce(combineFun) across ranks, for a forest summary."""
        self.merge_forest(summary)
        return summary

    def close(self) -> None:
        self.comm.close()
