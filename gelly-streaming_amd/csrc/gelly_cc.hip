// gelly_cc.hip — gfx950 implementation of the C ABI in include/gelly_cc.h.
//
// What it replaces (reference = gelly-streaming, `…/` = src/main/java/org/apache/flink/graph/streaming/):
//   DisjointSet<Long>            …/summaries/DisjointSet.java:30-154  HashMap<K,K> matches + HashMap<K,Integer> ranks
//   UpdateCC.foldEdges           …/library/ConnectedComponents.java:83-86  ds.union(src, trg) per edge
//   CombineCC.reduce / merge     …/library/ConnectedComponents.java:116-125, DisjointSet.java:132-136
//
// Device representation: one u32 parent[id_capacity] per forest, resident in HBM.
//   parent[v] == GCC_UNSEEN  -> v is not in the key set (matches.containsKey(v) == false)
//   parent[v] == v           -> v is a root
//   parent[v] <  v           -> v hangs under parent[v]           (invariant: parent[v] <= v once seen)
// Hooking is min-id: a root is only ever hooked under a SMALLER root, with atomicCAS(parent[hi], hi, lo),
// so every root is the minimum id of its tree and a full compress leaves parent[] == canonical labels.
// Union-by-rank (DisjointSet.java:113-122) only decides which root survives; it never changes the
// partition, which is all the parity contract (min-id labels after every window) observes.
//
// Memory model (gfx950: per-CU L1 and per-XCD L2 are not coherent). Plain loads of parent[] may return
// stale — but always historically valid — values: a vertex's parent only ever moves to an ancestor in the
// same tree, and a root only leaves root state through a device-scope CAS that executes at the memory side.
// A stale read therefore costs at most a failed CAS, whose return value is fresh and strictly smaller, so
// every loop terminates. Path-splitting stores are plain stores to NON-root slots only (a slot once
// non-root never becomes root again: all values written are < v), so they never race with a hook.

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "abi_common.h"
#include "edge_gen.h"
#include "gelly_cc.h"
#include "uf_device.h"

typedef uint32_t u32;
typedef uint64_t u64;

#define UNSEEN GCC_UNSEEN

// ------------------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

int gcc_set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define set_err gcc_set_err  // HIP_TRY / CHECK_ARG / DeviceGuard: abi_common.h

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
using gcc::Count;
using gcc::NoCount;
using gcc::UF;
using gcc::UFRead;
using gcc::unite_entry;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
typedef uint8_t u8;

constexpr int kBlock = 256;
constexpr int kFilterBlockLds = 1024;       // one workgroup per CU holding the whole giant bitmap in LDS
constexpr u32 kLdsBitmapMaxWords = 18176;   // 142 KiB of the CU's 160 KiB LDS (+16 KiB of rings) -> ids < 1,163,264
constexpr unsigned kMaxGrid = 2048;         // 256 CUs x 8 resident 256-thread blocks

// Fold a batch of edges (interleaved u32 pairs) into the forest: one edge per lane per iteration, 8 B/lane
// coalesced non-temporal stream (read once; it must not evict parent[] lines from L2).
// REC: every id that leaves UNSEEN or root state is marked in bloom (uf_device.h BloomRec), so the next
// compress can be incremental (compress_inc_kernel).
// Device-side id validation (gcc_forest_fold_device takes raw device pairs): an edge with an id >= cap is
// skipped — never dereferenced — and *err is set; the host reports it at the next synchronising call
// (stream_sync_checked). The ids of a bad edge are replaced by 0 so that later bitmap lookups stay in range.
__device__ __forceinline__ bool edge_ok(u32& a, u32& b, u32 cap, u32* err) {
    const bool ok = a < cap && b < cap;
    if (!ok) {
        *err = 1u;
        a = 0;
        b = 0;
    }
    return ok;
}

// Kernel-start trace (diagnostics, GELLY_TRACE=1): block 0's thread 0 of each traced kernel stores the kernel's id
// into one pinned host word (system scope, a vector store). A stream's kernels start in order and a fault stops its
// queue, so after an asynchronous fault the word names the kernel that faulted (or one of another stream).
__device__ u32* gcc_trace_slot = nullptr;
enum : u32 {
    kTrFold = 1, kTrFiltered, kTrCompressBits, kTrCompressInc, kTrSeedBfs, kTrSeedPack, kTrMergeLabels,
    kTrBkLayout, kTrBkP1, kTrBkHub, kTrBkP2Seed, kTrBkP3Seed, kTrBkInit, kTrBkP2, kTrBkP3, kTrBkHook, kTrBkSlow, kTrBkRest,
    kTrFoldPipe, kTrResolve, kTrCompressPipe,
    kTrCount
};
static const char* const kTraceNames[kTrCount] = {
    "none", "fold_kernel", "fold_filtered_kernel", "compress_bits_kernel", "compress_inc_kernel", "seed_bfs_kernel",
    "seed_pack_kernel", "merge_labels_kernel", "bucket_layout_kernel", "bucket_kernel (P1)", "bucket_hub_kernel",
    "slice_filter_kernel<false> (P2 seed)", "slice_hook_kernel<false> (P3 seed)", "bucket_init_kernel",
    "slice_filter_kernel<true> (P2)", "slice_hook_kernel<true> (P3)", "bucket_hook_kernel", "bucket_slow_kernel",
    "bucket_rest_kernel", "fold_pipe_kernel", "pipe_resolve_kernel", "compress_pipe_kernel"};
__device__ __forceinline__ void trace_start(u32 id) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        u32* t = gcc_trace_slot;
        if (t) __hip_atomic_store(t, id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The delta merge's lists (round 6; gcc_forest_encode_delta): kDeltaStripes stripes of `subcap` ids
// each; cnt[s] = the ids stripe s has taken (it may run past subcap: then the delta is unusable and the merge takes the
// compact message), cnt[kDeltaStripes] = some lane had more events than its slots. A wave appends its lanes' events to
// stripe (its global wave index mod kDeltaStripes) with ONE atomicAdd: a per-event atomic on one counter would
// serialise at the memory side (round 1's encode: 16K same-address atomics took 476 us).
constexpr u32 kDeltaStripes = 64;
struct DeltaLists {
    u32* ids;
    u32* cnt;
    u32 subcap;
};

__device__ __forceinline__ void delta_append(const DeltaLists& d, const gcc::LaneEvents& ev) {
    const u32 lane = threadIdx.x & 63;
    const u32 k = min(ev.n, gcc::kLaneEvents);
    if (ev.n > gcc::kLaneEvents) atomicOr(&d.cnt[kDeltaStripes], 1u);
    u32 incl = k;
    for (int off = 1; off < 64; off <<= 1) {
        const u32 y = __shfl_up(incl, off, 64);
        if (lane >= (u32)off) incl += y;
    }
    const u32 total = __shfl(incl, 63, 64);
    if (total == 0) return;
    const u32 stripe = (blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) & (kDeltaStripes - 1);
    u32 base = 0;
    if (lane == 63) base = atomicAdd(&d.cnt[stripe], total);
    base = __shfl(base, 63, 64);
    u32* out = d.ids + (size_t)stripe * d.subcap;
    u32 pos = base + incl - k;
    for (u32 j = 0; j < k; ++j, ++pos)
        if (pos < d.subcap) out[pos] = ev.x[j];
}

// SPLIT: path splitting in the finds (plain stores). END: 0 nothing; 1 every block ends with an agent-scope release
// (its XCD's dirty L2 lines written back before the kernel ends); 2 every wave ends with s_waitcnt vmcnt(0) (its
// stores and atomics acknowledged before it ends). A/B knobs of the recording fold (tune inc_split / fold_release).
// DELTA: every hooked root and new id also goes into the delta lists (the delta merge; the loop's trip count is then
// wave-uniform, so the wave can aggregate its events).
template <bool REC, bool SPLIT = true, int END = 0, bool DELTA = false>
__global__ __launch_bounds__(kBlock) void fold_kernel(u32* __restrict__ parent, const u64* __restrict__ edges,
                                                      u64 n_edges, u32* __restrict__ bloom, u32 cap,
                                                      u32* __restrict__ err, DeltaLists dl) {
    trace_start(kTrFold);
    NoCount c;
    typedef gcc::UnionFind<gcc::LoadPlain, SPLIT> U;
    const u64 stride = (u64)gridDim.x * kBlock;
    if constexpr (DELTA) {
        for (u64 b0 = (u64)blockIdx.x * kBlock; b0 < n_edges; b0 += stride) {
            const u64 i = b0 + threadIdx.x;
            gcc::LaneEvents ev;
            if (i < n_edges) {
                const u64 e = __builtin_nontemporal_load(edges + i);
                u32 a = (u32)e, b = (u32)(e >> 32);
                if (edge_ok(a, b, cap, err)) {
                    if constexpr (REC) U::unite(parent, a, b, c, gcc::BloomDeltaRec{bloom, &ev});
                    else U::unite(parent, a, b, c, gcc::DeltaRec{&ev});
                }
            }
            delta_append(dl, ev);
        }
    } else {
        for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n_edges; i += stride) {
            const u64 e = __builtin_nontemporal_load(edges + i);
            u32 a = (u32)e, b = (u32)(e >> 32);
            if (!edge_ok(a, b, cap, err)) continue;
            if constexpr (REC) U::unite(parent, a, b, c, gcc::BloomRec{bloom});
            else U::unite(parent, a, b, c);
        }
    }
    if constexpr (END == 1) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    } else if constexpr (END == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// Global -> LDS copy of n 16-B words by a whole block: U loads in flight per thread before any store. A plain
// `dst[w] = src[w]` loop waits for each load before it issues the next (measured: 6.7 us for a 128 KiB bitmap).
template <int BLOCK>
__device__ __forceinline__ void lds_fill(u32x4* dst, const u32x4* __restrict__ src, u32 n) {
    constexpr int U = 8;
    for (u32 base = 0; base < n; base += U * BLOCK) {
        u32x4 r[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {  // unconditional (clamped) loads: the compiler can count them
            const u32 w = base + k * BLOCK + threadIdx.x;
            r[k] = src[w < n ? w : n - 1];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const u32 w = base + k * BLOCK + threadIdx.x;
            if (w < n) dst[w] = r[k];
        }
    }
}

// Giant-filtered fold (Afforest-style skip): bits[] is a bitmap of one component C of the forest at some
// earlier time (normally the largest). Components only grow, so an edge with both endpoints in C is already
// folded in: it is skipped without touching parent[]. Every other edge is appended to the slow queue (or,
// past its capacity, united inline). Edges stream as 16 B per lane (two edges), four loads in flight.
// LDS = true: the bitmap lives in LDS (id range <= kLdsBitmapMaxWords * 64), one 1024-thread block per CU.
template <bool LDS>
__device__ __forceinline__ u32 in_c(const u32* bm, u32 v) {
    return (bm[v >> 5] >> (v & 31)) & 1u;
}

// Per-wave slow-edge ring in LDS: a wave appends its slow edges (ballot + popcount, wave-uniform cursor, no
// atomics at all) and, whenever 64 are pending, unites them one per lane right away. The slow edges' CAS /
// find latency then overlaps the other waves' streaming instead of forming a tail after it (measured: a
// per-block queue drained at the end left ~25 us of tail on C2; one global queue counter capped appends at
// ~88/us).
constexpr u32 kRing = 128;  // u64 entries per wave (1 KiB): pending stays < 64 + 64

// One drain round: the wave unites up to 64 ring entries, one per lane. Out of line: it runs rarely, and
// inlined at each of the hot loop's 8 push sites it multiplied the loop body ~8x (I-cache, registers).
// The union of one ring entry (uf_device.h unite_entry): an entry (g, x) with x > g (an edge from the tracked
// component to an id outside it) takes the hook of filter_round: ONE atomicMin(parent[x], g); only if x already hung
// under some other id p (old not in {UNSEEN, x, g}) is the link to p restored by union(g, p). Else the full union.

__device__ __attribute__((noinline)) void ring_drain(const u64* ring, u32 wd, u32 pending, u32* parent, u32 g) {
    const u32 lane = threadIdx.x & 63;
    if (lane < pending) {
        const u64 e = ring[(wd + lane) & (kRing - 1)];
        unite_entry(parent, (u32)e, (u32)(e >> 32), g);
    }
}

__device__ __forceinline__ void ring_push(bool slow, u32 a, u32 b, u64* ring, u32& wq, u32& wd, u32* parent,
                                          u32 drain_at, u32 g) {
    const unsigned long long m = __ballot(slow);
    if (m == 0) return;
    const u32 lane = threadIdx.x & 63;
    if (slow) ring[(wq + (u32)__popcll(m & ((1ull << lane) - 1ull))) & (kRing - 1)] = ((u64)b << 32) | a;
    wq += (u32)__popcll(m);
    const u32 pending = wq - wd;
    if (pending >= drain_at) {  // wave-uniform: drain one round (up to 64 edges), one edge per lane
        ring_drain(ring, wd, pending, parent, g);
        wd += pending < 64 ? pending : 64;
    }
}

// One edge of the filtered stream. Both ends in C: already folded, skip. One end in C: it is connected to g
// (C's root when the bitmap was built), so union(u, v) == union(g, other end) — pushed in that form, which
// saves the slow path a dependent find through the C-side endpoint. Otherwise pushed as is.
template <bool LDS>
__device__ __forceinline__ void filter_edge(bool valid, u32 a, u32 b, const u32* bm, u32 g, u64* ring, u32& wq,
                                            u32& wd, u32* parent, u32 drain_at) {
    const u32 ia = in_c<LDS>(bm, a), ib = in_c<LDS>(bm, b);
    // (g, other end) when exactly one end is in C: the drain's hook form (unite_entry)
    ring_push(valid && !(ia & ib), ia ? g : (ib ? g : a), ia ? b : (ib ? a : b), ring, wq, wd, parent, drain_at, g);
}

// A round of N edges of the filtered stream with the direct hook (HOOK): an edge with exactly one end in C and
// the other end b > g is folded by ONE atomicMin(parent[b], g), issued for the whole round before any result
// is looked at. old = UNSEEN (b was new: the common case), b (b was a root) or g: b now hangs under g, done.
// Otherwise b left the tree of old, or already hung under something smaller: (g, old) goes to the ring, whose
// union restores the connection. Every write still lowers a parent, so the forest stays a forest and roots stay
// minimal (b's descendants are all > b > g). Other non-skipped edges take the ring as in filter_edge.
// The hooks' results are checked one round later (HookCarry): the atomics' latency overlaps the next round's
// loads and filtering instead of stalling the wave.
template <int N>
struct HookCarry {
    u32 other[N], old[N];
    bool hook[N];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int k = 0; k < N; ++k) hook[k] = false;
    }
    __device__ __forceinline__ void settle(u32 g, u64* ring, u32& wq, u32& wd, u32* parent, u32 drain_at) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const bool again = hook[k] && gcc::hook_needs_union(old[k], other[k], g);
            ring_push(again, g, again ? old[k] : 0u, ring, wq, wd, parent, drain_at, g);
        }
    }
};

template <bool LDS, int N>
__device__ __forceinline__ void filter_round(const bool* valid, const u32* a, const u32* b, const u32* bm, u32 g,
                                             u64* ring, u32& wq, u32& wd, u32* parent, u32 drain_at,
                                             HookCarry<N>& carry) {
    HookCarry<N> cur;
    bool slow[N];
    u32 pa[N], pb[N], wa[N], wb[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {  // every bitmap lookup of the round first: one LDS wait, not one per edge
        wa[k] = bm[a[k] >> 5];
        wb[k] = bm[b[k] >> 5];
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const u32 ia = (wa[k] >> (a[k] & 31)) & 1u, ib = (wb[k] >> (b[k] & 31)) & 1u;
        cur.other[k] = ia ? b[k] : a[k];
        cur.hook[k] = valid[k] && (ia ^ ib) && cur.other[k] > g;
        slow[k] = valid[k] && !(ia & ib) && !cur.hook[k];
        pa[k] = ia ? g : a[k];
        pb[k] = ib ? g : b[k];
        if (cur.hook[k]) cur.old[k] = gcc::hook_min(parent, cur.other[k], g);
    }
    carry.settle(g, ring, wq, wd, parent, drain_at);  // the previous round's hooks (their atomics have returned)
#pragma unroll
    for (int k = 0; k < N; ++k) ring_push(slow[k], pa[k], pb[k], ring, wq, wd, parent, drain_at, g);
    carry = cur;
}

// Dynamic LDS: [bitmap (LDS variant), 16-B aligned][BLOCK/64 rings of kRing u64]. slow_count[blockIdx.x] =
// the block's slow edges (measurement).
template <bool LDS, int BLOCK, int DEPTH, bool PIPE, bool HOOK>
__global__ __launch_bounds__(BLOCK) void fold_filtered_kernel(u32* __restrict__ parent, const u64* __restrict__ edges,
                                                              u64 n_edges, const u32* __restrict__ bits, u32 nwords,
                                                              const u32* __restrict__ giant,
                                                              u32* __restrict__ slow_count, u32 drain_at, u32 cap,
                                                              u32* __restrict__ err) {
    trace_start(kTrFiltered);
    extern __shared__ __attribute__((aligned(16))) u32 s_dyn[];
    __shared__ u32 s_slow;
    const u32 bitmap_u32 = LDS ? nwords * 2 : 0;  // nwords = u64 words, even
    u64* ring = reinterpret_cast<u64*>(s_dyn + bitmap_u32) + (threadIdx.x >> 6) * kRing;
    // split the batch into an aligned body of 16-B pairs of edges and a scalar head/tail
    const u64 head = ((reinterpret_cast<uintptr_t>(edges) & 15) && n_edges) ? 1 : 0;
    const u64 n2 = (n_edges - head) / 2;
    const u32x4* body = reinterpret_cast<const u32x4*>(edges + head);
    const u64 stride = (u64)gridDim.x * BLOCK;
    const u32 lane = threadIdx.x & 63;
    // Whole waves run both loops with the same trip count (the ring cursors wq/wd must stay wave-uniform):
    // the loops are driven by the wave's first pair index, lanes past the end are predicated off.
    u64 base = (u64)blockIdx.x * BLOCK + (threadIdx.x - lane);
    u32x4 q[DEPTH];
    const bool first_round = PIPE && base + 63 + (DEPTH - 1) * stride < n2;
    if (first_round) {  // in flight while the bitmap is copied into LDS
#pragma unroll
        for (int k = 0; k < DEPTH; ++k) q[k] = __builtin_nontemporal_load(body + base + lane + k * stride);
    }
    const u32* bm = bits;
    if (threadIdx.x == 0) s_slow = 0;
    if constexpr (LDS) {
        const u32x4* src = reinterpret_cast<const u32x4*>(bits);
        u32x4* dst = reinterpret_cast<u32x4*>(s_dyn);
        if (nwords) lds_fill<BLOCK>(dst, src, nwords / 2);
        bm = s_dyn;
    }
    __syncthreads();
    const u32 g = *giant;
    u32 wq = 0, wd = 0;  // this wave's ring: pushed / drained (wave-uniform)
    HookCarry<2 * DEPTH> carry;  // HOOK: the last round's atomicMin results, settled one round later
    HookCarry<2> carry2;
    carry.clear();
    carry2.clear();
    if constexpr (PIPE) {
        // software-pipelined: the next DEPTH loads are in flight while this round is filtered (and while a
        // ring drain waits on its union chains)
        if (first_round) {
            while (true) {
                const u64 nb = base + DEPTH * stride;
                const bool more = nb + 63 + (DEPTH - 1) * stride < n2;  // wave-uniform
                // issued unconditionally (clamped in range; the last, unused round re-reads a valid pair): a load
                // under a branch leaves the compiler unable to count it, and its s_waitcnt then drains the whole
                // queue, prefetch included, before the current round is filtered
                u32x4 nq[DEPTH];
#pragma unroll
                for (int k = 0; k < DEPTH; ++k) {
                    const u64 j = nb + lane + k * stride;
                    nq[k] = __builtin_nontemporal_load(body + (j < n2 ? j : n2 - 1));
                }
                if constexpr (HOOK) {
                    bool vv[2 * DEPTH];
                    u32 ea[2 * DEPTH], eb[2 * DEPTH];
#pragma unroll
                    for (int k = 0; k < DEPTH; ++k) {
                        ea[2 * k] = q[k].x;
                        eb[2 * k] = q[k].y;
                        ea[2 * k + 1] = q[k].z;
                        eb[2 * k + 1] = q[k].w;
                        vv[2 * k] = edge_ok(ea[2 * k], eb[2 * k], cap, err);
                        vv[2 * k + 1] = edge_ok(ea[2 * k + 1], eb[2 * k + 1], cap, err);
                    }
                    filter_round<LDS, 2 * DEPTH>(vv, ea, eb, bm, g, ring, wq, wd, parent, drain_at, carry);
                } else {
#pragma unroll
                    for (int k = 0; k < DEPTH; ++k) {
                        u32 a0 = q[k].x, b0 = q[k].y, a1 = q[k].z, b1 = q[k].w;
                        const bool v0 = edge_ok(a0, b0, cap, err), v1 = edge_ok(a1, b1, cap, err);
                        filter_edge<LDS>(v0, a0, b0, bm, g, ring, wq, wd, parent, drain_at);
                        filter_edge<LDS>(v1, a1, b1, bm, g, ring, wq, wd, parent, drain_at);
                    }
                }
                base = nb;
                if (!more) break;
#pragma unroll
                for (int k = 0; k < DEPTH; ++k) q[k] = nq[k];
            }
        }
    } else {
        for (; base + 63 + (DEPTH - 1) * stride < n2; base += DEPTH * stride) {
            const u64 i = base + lane;
            u32x4 q[DEPTH];
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) q[k] = __builtin_nontemporal_load(body + i + k * stride);
#pragma unroll
            for (int k = 0; k < DEPTH; ++k) {
                u32 a0 = q[k].x, b0 = q[k].y, a1 = q[k].z, b1 = q[k].w;
                const bool v0 = edge_ok(a0, b0, cap, err), v1 = edge_ok(a1, b1, cap, err);
                filter_edge<LDS>(v0, a0, b0, bm, g, ring, wq, wd, parent, drain_at);
                filter_edge<LDS>(v1, a1, b1, bm, g, ring, wq, wd, parent, drain_at);
            }
        }
    }
    for (; base < n2; base += stride) {
        const u64 i = base + lane;
        const bool valid = i < n2;
        u32x4 q = {0, 0, 0, 0};
        if (valid) q = __builtin_nontemporal_load(body + i);
        u32 ea[2] = {q.x, q.z}, eb[2] = {q.y, q.w};
        const bool v0 = edge_ok(ea[0], eb[0], cap, err) && valid, v1 = edge_ok(ea[1], eb[1], cap, err) && valid;
        if constexpr (HOOK) {
            const bool vv[2] = {v0, v1};
            filter_round<LDS, 2>(vv, ea, eb, bm, g, ring, wq, wd, parent, drain_at, carry2);
        } else {
            filter_edge<LDS>(v0, ea[0], eb[0], bm, g, ring, wq, wd, parent, drain_at);
            filter_edge<LDS>(v1, ea[1], eb[1], bm, g, ring, wq, wd, parent, drain_at);
        }
    }
    if constexpr (HOOK) {  // the last rounds' hooks
        carry.settle(g, ring, wq, wd, parent, drain_at);
        carry2.settle(g, ring, wq, wd, parent, drain_at);
    }
    NoCount c;
    // the rest of this wave's ring (< 64 + 64 entries)
    for (; wd < wq; wd += 64) {
        if (lane < wq - wd) {
            const u64 e = ring[(wd + lane) & (kRing - 1)];
            unite_entry(parent, (u32)e, (u32)(e >> 32), g);
        }
    }
    if (lane == 0 && wq) atomicAdd(&s_slow, wq);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // scalar head / tail edges
        if (head) {
            u32 a = (u32)edges[0], b = (u32)(edges[0] >> 32);
            if (edge_ok(a, b, cap, err)) UF::unite(parent, a, b, c);
        }
        if (head + 2 * n2 < n_edges) {
            const u64 e = edges[n_edges - 1];
            u32 a = (u32)e, b = (u32)(e >> 32);
            if (edge_ok(a, b, cap, err)) UF::unite(parent, a, b, c);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) slow_count[blockIdx.x] = s_slow;  // measurement (profile mode reads it)
}

// Merge: into ∪ {(v, labels[v])}. labels may be any parent array of a forest over the same id range
// (compressed or not) — its (key, parent) pairs generate its partition (DisjointSet.merge :132-136).
// A label array comes from outside (another forest, rank or device: gcc_forest_merge_labels_device), so a label
// is validated like a device batch's ids: one >= cap is skipped (never dereferenced) and *err is set.
__global__ __launch_bounds__(kBlock) void merge_labels_kernel(u32* __restrict__ parent, const u32* __restrict__ labels,
                                                              u32 n, u32 cap, u32* __restrict__ err) {
    trace_start(kTrMergeLabels);
    NoCount c;
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 vv = (u64)blockIdx.x * kBlock + threadIdx.x; vv < n; vv += stride) {
        const u32 v = (u32)vv;
        const u32 l = labels[v];
        if (l == UNSEEN) continue;
        if (l >= cap) {
            *err = 1u;
            continue;
        }
        UF::unite(parent, v, l, c);
    }
}

// Canonicalise (compress_bits_kernel below): labels[v] := root(v) = min id of v's component, UNSEEN stays UNSEEN
// (multi-level pointer jumping). Out of place on purpose: the path-splitting stores that let all threads collapse a
// deep chain together (O(log d) instead of O(d) per thread) write intermediate ancestors into parent[], and such a
// store can land after another thread's final root store — in place that would leave a vertex pointing at a
// non-root (the race, replayed in tests/cpp/test_uf_replay.cpp). labels[] is written exactly once per
// slot, by its own lane, so it is race-free; parent[] only needs to stay a valid forest (every store is an
// ancestor, roots never move: no hook is in flight). Algorithmic traffic: 4 B read + 4 B write per id.

// Majority vote (Boyer-Moore in its associative pair form) over the labels of 4096 pseudo-random seen ids:
// the winner is the giant component's label whenever one component holds most of the seen ids. Any
// component is a correct filter; the vote only decides how useful it is.
__device__ __forceinline__ void bm_merge(u32& c1, u32& n1, u32 c2, u32 n2) {
    if (c1 == c2) n1 += n2;
    else if (n1 >= n2) n1 -= n2;
    else {
        c1 = c2;
        n1 = n2 - n1;
    }
}

// share[0] = how many seen samples the winner holds, share[1] = how many samples were seen (exact counts: the
// host turns the filter off for a forest whose largest component is no giant).
__global__ __launch_bounds__(1024) void giant_vote_kernel(u32* __restrict__ parent, u32 n, u32* __restrict__ giant,
                                                          u32* __restrict__ share) {
    __shared__ u32 sc[16], sn[16], s_win, s_hit[16], s_seen[16];
    u32 l[4];
    NoCount c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32 v = (u32)(gcc_splitmix64(threadIdx.x * 4u + k) % n);
        l[k] = parent[v];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // roots of the sampled ids (UNSEEN stays UNSEEN)
        const u32 v = (u32)(gcc_splitmix64(threadIdx.x * 4u + k) % n);
        if (l[k] != UNSEEN) l[k] = UF::find_from(parent, v, l[k], c);
    }
    u32 cand = UNSEEN, cnt = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (l[k] != UNSEEN) bm_merge(cand, cnt, l[k], 1);
    for (int off = 32; off > 0; off >>= 1) {
        const u32 c2 = __shfl_down(cand, off, 64), n2 = __shfl_down(cnt, off, 64);
        bm_merge(cand, cnt, c2, n2);
    }
    if ((threadIdx.x & 63) == 0) {
        sc[threadIdx.x >> 6] = cand;
        sn[threadIdx.x >> 6] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) bm_merge(sc[0], sn[0], sc[w], sn[w]);
        s_win = sn[0] ? sc[0] : UNSEEN;
        *giant = s_win;
    }
    __syncthreads();
    u32 hit = 0, seen = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        seen += l[k] != UNSEEN;
        hit += l[k] != UNSEEN && l[k] == s_win;
    }
    for (int off = 32; off > 0; off >>= 1) {
        hit += __shfl_down(hit, off, 64);
        seen += __shfl_down(seen, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        s_hit[threadIdx.x >> 6] = hit;
        s_seen[threadIdx.x >> 6] = seen;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) {
            s_hit[0] += s_hit[w];
            s_seen[0] += s_seen[w];
        }
        share[0] = s_hit[0];
        share[1] = s_seen[0];
    }
}

// Compress fused with the giant bitmap: labels[v] = root(v) as compress_kernel, and bits[w] bit b =
// (labels[64w + b] == g) where g = the current root of the tracked component (the root of giant_prev: roots
// only move to smaller ids, so following the old root finds the same, grown, component). giant_next receives g.
// A wave labels 256-id chunks, 4 ids per lane (16-B loads and stores), kBitsU chunks in flight per wave before any
// is labelled (one id per lane and one load at a time kept too little in flight: C4's 64M ids at ~1.9 TB/s); the
// lanes' 4-bit nibbles are OR-ed into the chunk's 4 bitmap words. labels == nullptr: a mid-fold refresh of the
// bitmap alone (refresh_now); bits == nullptr (the filter off): the labels alone. Prefetched parent values are historically valid (splitting stores only write
// ancestors), so a find from one is exact.
constexpr int kBitsU = 1;  // chunks per wave per batch (A/B: 1 beat 2, 4, 8 on C2 x 16)
__device__ __forceinline__ void chunk_bits(u64* bits, u64 nwords, u64 ch, u32 lane, u32 g, const u32 (&lab)[4]) {
    u64 w = 0;
    if (g != UNSEEN)
        w = (u64)((lab[0] == g) | ((lab[1] == g) << 1) | ((lab[2] == g) << 2) | ((lab[3] == g) << 3)) << (4 * (lane & 15));
    w |= __shfl_xor(w, 1, 64);
    w |= __shfl_xor(w, 2, 64);
    w |= __shfl_xor(w, 4, 64);
    w |= __shfl_xor(w, 8, 64);
    const u64 wi = ch * 4 + (lane >> 4);
    if ((lane & 15) == 0 && wi < nwords) bits[wi] = w;
}

// The same packing for the merge message's "others" mask: seen ids outside g's component (all seen ids if no g).
__device__ __forceinline__ void chunk_oth(u64* oth, u64 nwords, u64 ch, u32 lane, u32 g, const u32 (&lab)[4]) {
    auto o = [&](u32 l) { return (u32)(l != UNSEEN && l != g); };
    u64 w = (u64)(o(lab[0]) | (o(lab[1]) << 1) | (o(lab[2]) << 2) | (o(lab[3]) << 3)) << (4 * (lane & 15));
    w |= __shfl_xor(w, 1, 64);
    w |= __shfl_xor(w, 2, 64);
    w |= __shfl_xor(w, 4, 64);
    w |= __shfl_xor(w, 8, 64);
    const u64 wi = ch * 4 + (lane >> 4);
    if ((lane & 15) == 0 && wi < nwords) oth[wi] = w;
}

static inline unsigned chunk_grid(u64 n, int per_wave, int block, unsigned max_blocks) {  // waves for 256-id chunks
    const u64 waves = ((n + 255) / 256 + per_wave - 1) / per_wave;
    const u64 b = (waves * 64 + block - 1) / block;
    return (unsigned)(b < 1 ? 1 : (b > max_blocks ? max_blocks : b));
}

// SPLIT: the finds split paths in `parent` (plain stores). Only the mid-fold refresh (labels == nullptr) does: it
// shortens the chains the rest of the fold walks. A compress that writes labels uses read-only finds (round 5): its
// split stores went into the buffer that becomes the spare after the swap, i.e. the OUTPUT of the compress two kernels
// later, and a plain store landing that late would overwrite a label (the host replay's late-store model,
// tests/cpp/test_uf_replay.cpp). tune key compress_split = 1 restores them (A/B only).
template <bool SPLIT>
__global__ __launch_bounds__(kBlock) void compress_bits_kernel(u32* __restrict__ parent, u32* __restrict__ labels, u32 n,
                                                               const u32* __restrict__ giant_prev,
                                                               u32* __restrict__ giant_next, u64* __restrict__ bits,
                                                               u32* __restrict__ bloom_clear, u64* __restrict__ oth,
                                                               const u64* __restrict__ newbits) {
    trace_start(kTrCompressBits);
    typedef gcc::UnionFind<gcc::LoadPlain, SPLIT> CF;
    __shared__ u32 s_g, s_g0;
    NoCount c;
    const u32 lane = threadIdx.x & 63;
    const u64 nwords = ((u64)n + 63) / 64;
    const u64 nfull = (u64)n / 256;
    const u64 nwaves = (u64)gridDim.x * (kBlock / 64);
    const u64 wave = (u64)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    u32x4 pv[kBitsU];
    auto load_batch = [&](u64 base) {
#pragma unroll
        for (int k = 0; k < kBitsU; ++k) {  // clamped, unconditional: countable loads
            const u64 ch = base + (u64)k * nwaves;
            pv[k] = *reinterpret_cast<const u32x4*>(parent + (ch < nfull ? ch : nfull - 1) * 256 + 4 * lane);
        }
    };
    if (wave < nfull) load_batch(wave);
    if (bloom_clear)  // the bloom buffer the next fold records into (compress_inc_kernel): memory-side atomics
        for (u32 w = blockIdx.x * kBlock + threadIdx.x; w < gcc::kBloomBits / 32; w += gridDim.x * kBlock)
            atomicAnd(&bloom_clear[w], 0u);
    if (threadIdx.x == 0) {
        const u32 g0 = giant_prev ? *giant_prev : UNSEEN;
        s_g = (g0 == UNSEEN) ? UNSEEN : CF::find_from(parent, g0, parent[g0], c);
        s_g0 = g0;
        if (blockIdx.x == 0 && giant_next) *giant_next = s_g;
    }
    __syncthreads();
    const u32 g = s_g;
    // the tracked component's previous root g0 (now under g, or g itself): the bucketed fold and the seeding hang
    // most of a giant's ids straight under it, so its children are labelled g without a walk
    const u32 g0 = s_g0;
    for (u64 base = wave; base < nfull; base += (u64)kBitsU * nwaves) {
        u32x4 cur[kBitsU];
#pragma unroll
        for (int k = 0; k < kBitsU; ++k) cur[k] = pv[k];
        const u64 nb = base + (u64)kBitsU * nwaves;
        if (nb < nfull) load_batch(nb);  // wave-uniform
#pragma unroll
        for (int k = 0; k < kBitsU; ++k) {
            const u64 ch = base + (u64)k * nwaves;
            if (ch >= nfull) break;  // wave-uniform
            const u32 v0 = (u32)(ch * 256 + 4 * lane);
            const u32x4 p = cur[k];
            u32 lab[4];
            // a child of the tracked root g (a root during the compress) needs no find: most ids of a giant
            lab[0] = (p.x >= v0 || p.x == g) ? p.x : (p.x == g0 ? g : CF::find_from(parent, v0, p.x, c));
            lab[1] = (p.y >= v0 + 1 || p.y == g) ? p.y : (p.y == g0 ? g : CF::find_from(parent, v0 + 1, p.y, c));
            lab[2] = (p.z >= v0 + 2 || p.z == g) ? p.z : (p.z == g0 ? g : CF::find_from(parent, v0 + 2, p.z, c));
            lab[3] = (p.w >= v0 + 3 || p.w == g) ? p.w : (p.w == g0 ? g : CF::find_from(parent, v0 + 3, p.w, c));
            if (newbits) {  // an absorb's deferred new ids (msg_absorb_bits_kernel): still UNSEEN, in g's component
                const u32 nb = (u32)(newbits[v0 >> 6] >> (v0 & 63)) & 15u;
                if (nb) {
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (((nb >> k) & 1u) && lab[k] == UNSEEN) lab[k] = g;
                }
            }
            if (labels) {
                const u32x4 o = {lab[0], lab[1], lab[2], lab[3]};
                *reinterpret_cast<u32x4*>(labels + v0) = o;
            }
            if (bits) chunk_bits(bits, nwords, ch, lane, g, lab);
            if (oth) chunk_oth(oth, nwords, ch, lane, g, lab);
        }
    }
    if (nfull * 256 < n && wave == nfull % nwaves) {  // the partial last chunk: id by id
        const u64 v0 = nfull * 256 + 4 * lane;
        u32 lab[4] = {UNSEEN, UNSEEN, UNSEEN, UNSEEN};
        for (u32 k = 0; k < 4; ++k)
            if (v0 + k < n) {
                const u32 pk = parent[v0 + k];
                lab[k] = pk >= (u32)(v0 + k) ? pk : CF::find_from(parent, (u32)(v0 + k), pk, c);
                if (newbits && lab[k] == UNSEEN && ((newbits[(v0 + k) >> 6] >> ((v0 + k) & 63)) & 1ull)) lab[k] = g;
                if (labels) labels[v0 + k] = lab[k];
            }
        if (bits) chunk_bits(bits, nwords, nfull, lane, g, lab);
        if (oth) chunk_oth(oth, nwords, nfull, lane, g, lab);
    }
}

// Incremental compress: parent[] was compressed at the last compress and every mutation since was recorded in
// `bloom` (fold_kernel<true>; uf_device.h explains why an unmarked parent is still a root). labels[v] = p =
// parent[v] unless p is marked, and only then a (read-only) find. So the pass is a coalesced stream of parent[]
// and labels[] instead of a random read of parent[p] per seen non-root. One 1024-thread block per CU holds the
// bloom in LDS; a wave covers 256 ids = 4 bitmap words of the tracked component per chunk, lane l the ids 64 j + l.
// The block also clears its share of the other bloom buffer.
constexpr int kIncBlock = 1024;
#ifndef GCC_INC_U  // A/B builds only (tools/gpu_c5.sh)
#define GCC_INC_U 2
#endif
constexpr int kIncU = GCC_INC_U;  // 256-id chunks per wave per batch (A/B: 2 beat 1, 4 and 8 on C5; profiles/r2_ab_chunk_batches.log)
constexpr int kIncQ = 128;  // queued finds per wave (two per lane per flush): 16 KiB of LDS beside the 128 KiB bloom
using gcc::inc_label;  // uf_device.h: shared with the host replay

// INPLACE: labels == parent. parent[] is already canonical except where a marked parent needs the find, so only
// those slots are written (with the root; each slot by its own lane only). That is race-free: the finds are
// read-only, no root moves during a compress, and a lane that reads a slot before or after its owner rewrites it
// gets an ancestor either way (the old parent or the root). The pass then reads parent[] and writes only the
// changed slots instead of streaming a second 4 B per id into the spare buffer.
// CHECK (diagnostics, tune key inc_check): after the LDS fill every block also reads each bloom word with a
// memory-side atomic (fresh by construction) and counts the words whose LDS copy differs: dbg[0] = words where the
// memory holds a mark the LDS copy lacks (a lost mark: a wrong label can follow), dbg[1] = the reverse.
template <bool INPLACE, bool CHECK>
__global__ __launch_bounds__(kIncBlock) void compress_inc_kernel(const u32* parent, u32* labels,
                                                                 u32 n, const u32* __restrict__ bloom,
                                                                 u32* __restrict__ bloom_clear,
                                                                 const u32* __restrict__ giant_prev,
                                                                 u32* __restrict__ giant_next, u64* __restrict__ bits,
                                                                 u32* __restrict__ dbg) {
    trace_start(kTrCompressInc);
    extern __shared__ __attribute__((aligned(16))) u32 s_bloom[];
    __shared__ u32 s_g;
    __shared__ u32 s_qv[kIncBlock / 64][kIncQ], s_qp[kIncBlock / 64][kIncQ];  // queued finds per wave: id, parent
    constexpr u32 kW4 = gcc::kBloomBits / 128;  // bloom size in 16-B words
    const u32 lane = threadIdx.x & 63;
    const u64 nwords = ((u64)n + 63) / 64;
    const u64 nfull = (u64)n / 256;  // whole 256-id chunks (one 16-B load per lane); the partial tail: below
    const u64 nwaves = (u64)gridDim.x * (kIncBlock / 64);
    const u64 wave = (u64)blockIdx.x * (kIncBlock / 64) + (threadIdx.x >> 6);
    // the first batch of parent[] loads is issued before the bloom's LDS fill and lands behind it. Lane l of a wave
    // takes ids 64 j + l (j < 4) of each 256-id chunk: four coalesced 256-B loads per chunk, and a ballot over the
    // wave of one predicate per j is then the chunk's bitmap word j itself (no cross-lane shuffles)
    u32 pv[kIncU][4];
    auto load_batch = [&](u64 base) {
#pragma unroll
        for (int k = 0; k < kIncU; ++k) {  // clamped, unconditional: the compiler can count them
            const u64 ch = base + (u64)k * nwaves;
            const u32* src = parent + (ch < nfull ? ch : nfull - 1) * 256 + lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) pv[k][j] = src[64 * j];
        }
    };
    if (wave < nfull) load_batch(wave);
    {
        const u32x4* src = reinterpret_cast<const u32x4*>(bloom);
        u32x4* dst = reinterpret_cast<u32x4*>(s_bloom);
        lds_fill<kIncBlock>(dst, src, kW4);
        // the other bloom is cleared with memory-side atomics, never with plain stores: the next fold's marks are
        // memory-side atomics, and a plain store of this kernel can still land after the next kernel's atomics
        const u32 per = (kW4 + gridDim.x - 1) / gridDim.x, a = blockIdx.x * per, b = min(kW4, a + per);
        for (u32 w = 4 * a + threadIdx.x; w < 4 * b; w += kIncBlock) atomicAnd(&bloom_clear[w], 0u);
    }
    if (threadIdx.x == 0) {
        NoCount c;
        const u32 g0 = *giant_prev;
        s_g = (g0 == UNSEEN) ? UNSEEN : UFRead::find_from(const_cast<u32*>(parent), g0, parent[g0], c);
        if (blockIdx.x == 0) *giant_next = s_g;
    }
    __syncthreads();
    if constexpr (CHECK) {
        for (u32 w = threadIdx.x; w < gcc::kBloomBits / 32; w += kIncBlock) {
            const u32 mem = __hip_atomic_fetch_or(const_cast<u32*>(bloom) + w, 0u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
            const u32 lds = s_bloom[w];
            if (mem & ~lds) {
                const u32 k = atomicAdd(&dbg[0], 1u);
                if (k < 4) {
                    dbg[16 + 4 * k] = blockIdx.x;
                    dbg[17 + 4 * k] = w;
                    dbg[18 + 4 * k] = lds;
                    dbg[19 + 4 * k] = mem;
                }
            }
            if (lds & ~mem) atomicAdd(&dbg[1], 1u);
        }
    }
    const u32 g = s_g;
    // The ids whose parent is marked need a find: a chain of dependent loads. Walked inline (inc_label), each hop
    // waited for every load in flight (vmcnt is in order), the next batch's prefetch included, and with 512 ids
    // per wave per batch almost every batch of C5 had a marked parent somewhere. So the stream only labels the
    // unmarked ids (their label is the parent: nothing to store in place), writes the bitmap words from them, and
    // queues the marked ones per wave in LDS; a flush walks up to kIncQ queued finds at once (two chains per lane
    // in lock step), stores their roots and ORs their bits into the words already written. The flush's fences
    // order those stores after the stream's stores to the same words / slots (other lanes of the same wave).
    const u32 wv = threadIdx.x >> 6;
    u32 qn = 0;  // queued finds of this wave (wave-uniform)
    auto order = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    // in place, a label is stored write-through (gcc::st_through): the next in-place compress may rewrite the same
    // slot two kernels later, and a plain store still on its way could land over that
    auto settle = [&](u32 v, u32 p, u32 r) {  // a resolved find: the label and the tracked component's bit
        if constexpr (INPLACE) {
            if (r != p) gcc::st_through(labels + v, r);
        } else {
            labels[v] = r;
        }
        if (r == g) __hip_atomic_fetch_or(bits + (v >> 6), 1ull << (v & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto flush = [&]() {
        order();
        const bool ha = lane < qn, hb = lane + 64 < qn;
        const u32 va = ha ? s_qv[wv][lane] : 0, pa = ha ? s_qp[wv][lane] : 0;
        const u32 vb = hb ? s_qv[wv][lane + 64] : 0, pb = hb ? s_qp[wv][lane + 64] : 0;
        u32 ra = pa, rb = pb;  // an idle chain starts at 0: parent[0] is 0 or UNSEEN, never below it
        for (;;) {
            const u32 na = parent[ra], nb = parent[rb];
            const bool ma = na < ra, mb = nb < rb;
            if (!ma && !mb) break;
            if (ma) ra = na;
            if (mb) rb = nb;
        }
        if (ha) settle(va, pa, ra);
        if (hb) settle(vb, pb, rb);
        qn = 0;
    };
    const u64 lt = (1ull << lane) - 1;
    const bool track = g != UNSEEN;  // no tracked component: no bit is set
    // kIncU chunks per wave in flight before any is labelled: a wave that waited for each chunk in turn kept ~4 MB
    // in flight device-wide and streamed C5's 64 MB parent[] at ~2.2 TB/s
    for (u64 base = wave; base < nfull; base += (u64)kIncU * nwaves) {
        u32 cur[kIncU][4];
#pragma unroll
        for (int k = 0; k < kIncU; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[k][j] = pv[k][j];
        const u64 nb = base + (u64)kIncU * nwaves;
        if (nb < nfull) load_batch(nb);  // wave-uniform: the next batch streams in while this one is labelled
#pragma unroll
        for (int k = 0; k < kIncU; ++k) {
            const u64 ch = base + (u64)k * nwaves;
            if (ch >= nfull) break;  // wave-uniform
            const u32 v0 = (u32)(ch * 256) + lane;  // this lane's ids: v0 + 64 j
            // branch-free: every id reads its bloom word (roots and UNSEEN too), the four LDS reads in flight
            // together (a short-circuit test compiled to a branch and a wait per id)
            u32 bw[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bw[j] = s_bloom[gcc::bloom_word(cur[k][j])];
            u32 dm = 0;
            u64 wd[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32 p = cur[k][j];
                const u32 m = gcc::bloom_mask(p);
                const bool d = (p < v0 + 64 * j) & ((bw[j] & m) == m);
                dm |= (u32)d << j;
                wd[j] = __ballot(!d && p == g && track);
                if constexpr (!INPLACE) labels[v0 + 64 * j] = p;  // marked slots: rewritten by the flush
            }
            if (lane < 4) bits[ch * 4 + lane] = lane == 0 ? wd[0] : lane == 1 ? wd[1] : lane == 2 ? wd[2] : wd[3];
            if (__ballot(dm != 0) == 0) continue;  // wave-uniform: the common chunk
            const u32 cnt = __popc(dm);
            const u64 b1 = __ballot(cnt & 1), b2 = __ballot(cnt & 2), b4 = __ballot(cnt & 4);
            const u32 tot = __popcll(b1) + 2 * __popcll(b2) + 4 * __popcll(b4);
            if (qn + tot > (u32)kIncQ) flush();
            if (tot > (u32)kIncQ) {  // a dense chunk: its finds inline
                order();
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((dm >> j) & 1u) {
                        NoCount c;
                        const u32 v = v0 + 64 * j;
                        settle(v, cur[k][j], UFRead::find_from(const_cast<u32*>(parent), v, cur[k][j], c));
                    }
                continue;
            }
            u32 pos = qn + __popcll(b1 & lt) + 2 * __popcll(b2 & lt) + 4 * __popcll(b4 & lt);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((dm >> j) & 1u) {
                    s_qv[wv][pos] = v0 + 64 * j;
                    s_qp[wv][pos] = cur[k][j];
                    ++pos;
                }
            qn += tot;
        }
    }
    if (qn) flush();
    if (nfull * 256 < n && wave == nfull % nwaves) {  // the partial last chunk: id by id
        const u64 v0 = nfull * 256 + 4 * lane;
        u32 lab[4] = {UNSEEN, UNSEEN, UNSEEN, UNSEEN};
        for (u32 k = 0; k < 4; ++k)
            if (v0 + k < n) {
                const u32 pk = parent[v0 + k];
                lab[k] = inc_label(parent, s_bloom, (u32)(v0 + k), pk);
                if (!INPLACE) labels[v0 + k] = lab[k];
                else if (lab[k] != pk) gcc::st_through(labels + v0 + k, lab[k]);
            }
        chunk_bits(bits, nwords, nfull, lane, g, lab);
    }
}

// ---- The pipelined emission (round 5; tune key inc_pipe) ----------------------------------------------------------
// Short windows over a big forest (C5: 2^16 edges per window over 2^24 ids): the emission of window w — the
// incremental compress, a scan of the whole label array — no longer has to finish before window w+1's fold starts.
// The labels live in their own array L (d_spare), and the scan of window w reads only L and a snapshot taken right
// after the fold, never parent[]: so it runs on a second stream, beside the next window's fold.
//   fold w (fold_pipe_kernel, handle stream): the recording fold, which also marks every touched id exactly
//     (uf_device.h PipeRec: hooked roots and new ids, 2 bits per id in `touched`);
//   resolve w (pipe_resolve_kernel, handle stream, before fold w+1): for each touched id x, roots[x] = root(x) now,
//     the new ids' bits copied out (`born`), `touched` cleared; the tracked root followed;
//   scan w (compress_pipe_kernel, pipe stream, after resolve w): L[v] = roots[v] for a new v; else, when L[v]'s
//     root l is marked in the window's bloom, L[v] = roots[l] (one load: no find); the tracked component's bitmap.
// Why roots[l] is right: L[v] = l was a root at the end of window w-1. If l was hooked in w, roots[l] is its root at
// the end of w. If the bloom only says "maybe" (a false positive), l was not touched in w, and roots[l] is UNSEEN or
// was written in an earlier window of the same parity: when l was new then — and l, a root now, was one since (a
// root is never made a root again until a reset), so roots[l] = l. The roots arrays are filled with UNSEEN when the
// mode starts after a reset. Buffers alternate: roots and born by window parity, blooms in a ring of 3 (the scan of
// window w clears the one fold w+2 records into); fold w+2 waits for scan w (its bloom, roots, born buffers).
__global__ __launch_bounds__(kBlock) void fold_pipe_kernel(u32* __restrict__ parent, const u64* __restrict__ edges,
                                                           u64 n_edges, u32* __restrict__ bloom,
                                                           u32* __restrict__ touched, u32 cap, u32* __restrict__ err) {
    trace_start(kTrFoldPipe);
    NoCount c;
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n_edges; i += stride) {
        const u64 e = __builtin_nontemporal_load(edges + i);
        u32 a = (u32)e, b = (u32)(e >> 32);
        if (!edge_ok(a, b, cap, err)) continue;
        gcc::UFRec::unite(parent, a, b, c, gcc::PipeRec{bloom, touched});  // memory-side atomics only (UFRec)
    }
}

// One thread per 32 ids (a u64 of `touched`: hooked bits | new bits << 32). The forest is quiescent here (after
// the window's folds, before the next window's, on one stream): read-only finds. The touched words are cleared with
// memory-side atomics (the next fold ORs into them with atomics); roots and born are written through
// (gcc::st_through: the scan reads them from another stream, and both are rewritten two windows later).
__global__ __launch_bounds__(kBlock) void pipe_resolve_kernel(const u32* __restrict__ parent, u64* __restrict__ touched,
                                                              u32 nw, u32* __restrict__ roots, u32* __restrict__ born,
                                                              const u32* __restrict__ giant_prev,
                                                              u32* __restrict__ giant_next) {
    trace_start(kTrResolve);
    NoCount c;
    u32* par = const_cast<u32*>(parent);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const u32 g0 = *giant_prev;
        *giant_next = (g0 == UNSEEN) ? UNSEEN : UFRead::find_from(par, g0, parent[g0], c);
    }
    for (u32 w = blockIdx.x * kBlock + threadIdx.x; w < nw; w += gridDim.x * kBlock) {
        const u64 t = touched[w];
        if (!t) continue;
        atomicExch(reinterpret_cast<unsigned long long*>(touched + w), 0ull);
        const u32 nb = (u32)(t >> 32);
        if (nb) gcc::st_through(born + w, nb);
        for (u32 m = (u32)t | nb; m; m &= m - 1) {
            const u32 x = w * 32 + (u32)__builtin_ctz(m);
            gcc::st_through(roots + x, gcc::pipe_root(par, x));
        }
    }
}

// The scan of window w (one 1024-thread block per CU, the window's bloom in LDS, compress_inc_kernel's chunk layout:
// lane l takes ids 64 j + l of each 256-id chunk, so a ballot per j is the chunk's bitmap word j). Reads L and the
// chunk's 8 new-id words; the hits (new ids and marked labels) need a load of the roots snapshot, a load that depends
// on the stream's: done inline, every hit would wait for the next batch's prefetch too (vmcnt is in order; the lesson
// of compress_inc_kernel), so they are queued per wave in LDS and a flush resolves up to kIncQ at once, stores the
// changed labels (write-through) and ORs their tracked-component bits into the words the stream already wrote.
// Clears its new-id words and its share of `bloom_clear`.
__global__ __launch_bounds__(kIncBlock) void compress_pipe_kernel(u32* __restrict__ labels, u32* parent, u32 n,
                                                                  const u32* __restrict__ bloom,
                                                                  u32* __restrict__ bloom_clear, u32* __restrict__ born,
                                                                  const u32* __restrict__ roots,
                                                                  const u32* __restrict__ giant, u64* __restrict__ bits) {
    trace_start(kTrCompressPipe);
    extern __shared__ __attribute__((aligned(16))) u32 s_bloom[];
    __shared__ u32 s_g;
    __shared__ u32 s_qv[kIncBlock / 64][kIncQ], s_ql[kIncBlock / 64][kIncQ];  // queued hits per wave: id, label
    constexpr u32 kW4 = gcc::kBloomBits / 128;
    const u32 lane = threadIdx.x & 63;
    const u64 nwords = ((u64)n + 63) / 64;
    const u64 nfull = (u64)n / 256;
    const u64 nwaves = (u64)gridDim.x * (kIncBlock / 64);
    const u64 wave = (u64)blockIdx.x * (kIncBlock / 64) + (threadIdx.x >> 6);
    u32 pv[kIncU][4], pb[kIncU][4];
    auto load_batch = [&](u64 base) {
#pragma unroll
        for (int k = 0; k < kIncU; ++k) {  // clamped, unconditional
            const u64 ch = base + (u64)k * nwaves;
            const u64 cc = ch < nfull ? ch : nfull - 1;
            const u32* src = labels + cc * 256 + lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pv[k][j] = src[64 * j];
                pb[k][j] = born[cc * 8 + 2 * j + (lane >> 5)];
            }
        }
    };
    if (wave < nfull) load_batch(wave);
    {
        lds_fill<kIncBlock>(reinterpret_cast<u32x4*>(s_bloom), reinterpret_cast<const u32x4*>(bloom), kW4);
        const u32 per = (kW4 + gridDim.x - 1) / gridDim.x, a = blockIdx.x * per, b = min(kW4, a + per);
        for (u32 w = 4 * a + threadIdx.x; w < 4 * b; w += kIncBlock) atomicAnd(&bloom_clear[w], 0u);
    }
    if (threadIdx.x == 0) s_g = *giant;
    __syncthreads();
    const u32 g = s_g;
    const bool track = g != UNSEEN;
    const u32 wv = threadIdx.x >> 6;
    u32 qn = 0;  // queued hits of this wave (wave-uniform)
    auto order = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    auto settle = [&](u32 v, u32 l, u32 r) {
        if (r != l) {
            gcc::st_through(labels + v, r);
            // the forest follows (a memory-side atomicMin: the next window's fold may run; r is v's root at the end
            // of this window, the smallest id on its path now and later), so that parent[] stays as flat as the
            // labels, as the in-place incremental compress keeps it
            atomicMin(parent + v, r);
        }
        if (track && r == g)
            __hip_atomic_fetch_or(bits + (v >> 6), 1ull << (v & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    auto flush = [&]() {
        order();
        const bool ha = lane < qn, hb = lane + 64 < qn;
        const u32 va = ha ? s_qv[wv][lane] : 0, la = ha ? s_ql[wv][lane] : 0;
        const u32 vb = hb ? s_qv[wv][lane + 64] : 0, lb = hb ? s_ql[wv][lane + 64] : 0;
        const u32 qa = roots[gcc::pipe_key(va, la)], qb = roots[gcc::pipe_key(vb, lb)];  // both in flight
        if (ha) settle(va, la, gcc::pipe_settle(la, qa));
        if (hb) settle(vb, lb, gcc::pipe_settle(lb, qb));
        qn = 0;
    };
    const u64 lt = (1ull << lane) - 1;
    for (u64 base = wave; base < nfull; base += (u64)kIncU * nwaves) {
        u32 cur[kIncU][4], cb[kIncU][4];
#pragma unroll
        for (int k = 0; k < kIncU; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) cur[k][j] = pv[k][j], cb[k][j] = pb[k][j];
        const u64 nb = base + (u64)kIncU * nwaves;
        if (nb < nfull) load_batch(nb);  // wave-uniform
#pragma unroll
        for (int k = 0; k < kIncU; ++k) {
            const u64 ch = base + (u64)k * nwaves;
            if (ch >= nfull) break;  // wave-uniform
            const u32 v0 = (u32)(ch * 256) + lane;
            u32 dm = 0;
            u64 wd[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const u32 l = cur[k][j];
                const bool d = gcc::pipe_hit(s_bloom, l, (cb[k][j] >> (lane & 31)) & 1u);
                dm |= (u32)d << j;
                wd[j] = __ballot(!d && track && l == g);
                if ((lane & 31) == 0 && cb[k][j]) gcc::st_through(born + ch * 8 + 2 * j + (lane >> 5), 0u);
            }
            if (lane < 4) bits[ch * 4 + lane] = lane == 0 ? wd[0] : lane == 1 ? wd[1] : lane == 2 ? wd[2] : wd[3];
            if (__ballot(dm != 0) == 0) continue;  // wave-uniform: the common chunk
            const u32 cnt = __popc(dm);
            const u64 b1 = __ballot(cnt & 1), b2 = __ballot(cnt & 2), b4 = __ballot(cnt & 4);
            const u32 tot = __popcll(b1) + 2 * __popcll(b2) + 4 * __popcll(b4);
            if (qn + tot > (u32)kIncQ) flush();
            if (tot > (u32)kIncQ) {  // a dense chunk (more hits than the queue holds): its lookups inline
                order();
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((dm >> j) & 1u) {
                        const u32 v = v0 + 64 * j, l = cur[k][j];
                        settle(v, l, gcc::pipe_settle(l, roots[gcc::pipe_key(v, l)]));
                    }
                continue;
            }
            u32 pos = qn + __popcll(b1 & lt) + 2 * __popcll(b2 & lt) + 4 * __popcll(b4 & lt);
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((dm >> j) & 1u) {
                    s_qv[wv][pos] = v0 + 64 * j;
                    s_ql[wv][pos] = cur[k][j];
                    ++pos;
                }
            qn += tot;
        }
    }
    if (qn) flush();
    if (nfull * 256 < n && wave == nfull % nwaves) {  // the partial last chunk: 4 consecutive ids per lane
        const u64 v0 = nfull * 256 + 4 * lane;
        u32 lab[4] = {UNSEEN, UNSEEN, UNSEEN, UNSEEN};
        for (u32 k = 0; k < 4; ++k)
            if (v0 + k < n) {
                const u32 v = (u32)(v0 + k), l = labels[v];
                lab[k] = gcc::pipe_label(s_bloom, roots, v, l, (born[v >> 5] >> (v & 31)) & 1u);
                if (lab[k] != l) {
                    gcc::st_through(labels + v, lab[k]);
                    atomicMin(parent + v, lab[k]);
                }
            }
        chunk_bits(bits, nwords, nfull, lane, g, lab);
        // the tail's new-id words (ids nfull * 256 .. n): cleared after every lane of the wave has read them
        __builtin_amdgcn_wave_barrier();
        if (lane < 8 && nfull * 8 + lane < ((u64)n + 31) / 32) gcc::st_through(born + nfull * 8 + lane, 0u);
    }
}

// Diagnostics (tune key inc_check): the incremental compress's labels vs the roots of the forest it started from
// (`pre`, a copy taken just before it; quiescent here, so a plain walk is exact). dbg[2] counts wrong labels and
// keeps the first four as (v, pre[v], label, root, is pre[v] marked in the bloom (memory-side reads), pre[pre[v]]);
// dbg[3] = the bloom's set bits (its fill).
__global__ __launch_bounds__(kBlock) void inc_verify_kernel(const u32* __restrict__ pre, const u32* __restrict__ labels,
                                                            u32 n, const u32* __restrict__ bloom, u32* __restrict__ dbg) {
    const u32 stride = gridDim.x * kBlock;
    for (u32 w = blockIdx.x * kBlock + threadIdx.x; w < gcc::kBloomBits / 32; w += stride)
        atomicAdd(&dbg[3], (u32)__builtin_popcount(bloom[w]));
    for (u32 v = blockIdx.x * kBlock + threadIdx.x; v < n; v += stride) {
        const u32 p = pre[v];
        u32 r = p;
        if (p != UNSEEN) {
            r = v;
            while (pre[r] < r) r = pre[r];
        }
        const u32 got = labels[v];
        if (got == r) continue;
        const u32 k = atomicAdd(&dbg[2], 1u);
        if (k < 4) {
            const u32 msk = gcc::bloom_mask(p);
            const u32 word = __hip_atomic_fetch_or(const_cast<u32*>(bloom) + gcc::bloom_word(p), 0u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            const u32 marked = (word & msk) == msk;
            u32* o = dbg + 32 + 6 * k;
            o[0] = v;
            o[1] = p;
            o[2] = got;
            o[3] = r;
            o[4] = marked;
            o[5] = p < n ? pre[p] : UNSEEN;
        }
    }
}

// Diagnostics (tune key post_check, round 4): a check that runs AFTER an incremental compress and changes nothing
// before or inside it (no copy of the forest, no host sync, no memory-side reads around the compress). For every
// seen v it tests the compress's output invariant labels[labels[v]] == labels[v]; the first kPostRecs offenders are
// recorded with what tells the candidate mechanisms apart: whether labels[v] is marked in the bloom the compress used
// (memory-side read; that bloom stays intact until the next compress clears it), the true root (a walk: the array is
// quiescent here), and, with post_check 2, the labels after the previous compress (prev: whether labels[v] was
// already a non-root when the window started, so that no fold of this window could have hooked it).
// d[0] = offenders (all checks), d[1] = checks run; records at d[16 + 8 k]: check#, v, l, labels[l], root, marked,
// prev[v], prev[l].
constexpr u32 kPostRecs = 6;
__global__ __launch_bounds__(kBlock) void inc_post_check_kernel(const u32* __restrict__ labels, u32 n,
                                                                const u32* __restrict__ bloom,
                                                                const u32* __restrict__ prev, u32 check_no,
                                                                u32* __restrict__ d) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&d[1], 1u);
    const u32 stride = gridDim.x * kBlock;
    for (u32 v = blockIdx.x * kBlock + threadIdx.x; v < n; v += stride) {
        const u32 l = labels[v];
        if (l == UNSEEN || l >= n) continue;
        const u32 ll = labels[l];
        if (ll == l) continue;
        const u32 k = atomicAdd(&d[0], 1u);
        if (k < kPostRecs) {
            u32 r = l;
            for (u32 hop = 0; hop < 64 && labels[r] < r; ++hop) r = labels[r];
            const u32 word = __hip_atomic_fetch_or(const_cast<u32*>(bloom) + gcc::bloom_word(l), 0u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
            u32* o = d + 16 + 8 * k;
            o[0] = check_no;
            o[1] = v;
            o[2] = l;
            o[3] = ll;
            o[4] = r;
            o[5] = (word & gcc::bloom_mask(l)) == gcc::bloom_mask(l);
            o[6] = prev ? prev[v] : UNSEEN;
            o[7] = prev ? prev[l] : UNSEEN;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Seeding a FRESH forest without parent[] atomics (DESIGN.md §4 "seeded fold").
// A from-scratch fold of a skewed stream spends its time in CAS storms on the hubs' roots. Instead:
//  (1) seed_hub_kernel: the most frequent endpoint h of the batch's first edges (LDS hash count) —
//      on a skewed stream a hub, in the eventual giant component. Also clears the flag bytes;
//  (2) seed_bfs_kernel (a few passes over a prefix of the batch): C := C ∪ {x} for every edge (y, x) with
//      y ∈ C — a BFS from h over the prefix edges, on one flag byte per id. Setting a flag is an idempotent
//      plain byte store (no atomics: a stale read only delays a flag to the next pass). Every id in C is
//      connected to h by edges of this batch, so C lies inside one component of the folded forest;
//      gmin = min C: each block stores its minimum discovery in a slot of its own, the last pack reduces them;
//  (3) seed_init_kernel: parent[v] = (v ∈ C) ? gmin : UNSEEN and the bitmap of C — the reset and all of C's
//      union work in one pass. The filtered kernel then folds the WHOLE batch against C: edges inside C are
//      skipped, every other edge (prefix included) takes the union path, so the result is exact.
// ------------------------------------------------------------------------------------------------
constexpr int kHubBlock = 1024;
constexpr u32 kHubSlots = 16384;  // LDS open-addressing table (key, count): 128 KiB, load factor <= 1/8
constexpr u32 kHubProbe = 64;
constexpr u64 kHubSample = 1024;  // edges sampled for the hub vote (1 per thread)

// Count one occurrence of x; returns x's count including this one (0 if the probe limit was hit). The thread
// that makes the last increment of a key holds its final count, so the argmax needs no scan of the table.
__device__ __forceinline__ u32 hub_count(u32 x, u32* s_key, u32* s_cnt) {
    u32 s = (x * 0x9E3779B1u) >> (32 - 14);
    static_assert(kHubSlots == (1u << 14), "hash width");
#pragma unroll 1
    for (u32 p = 0; p < kHubProbe; ++p, s = (s + 1) & (kHubSlots - 1)) {
        const u32 k = atomicCAS(&s_key[s], UNSEEN, x);
        if (k == UNSEEN || k == x) return atomicAdd(&s_cnt[s], 1u) + 1;
    }
    return 0;
}

__device__ __forceinline__ bool hub_better(u32 c, u32 k, u32 bc, u32 bk) { return c > bc || (c == bc && c && k < bk); }

// The hub election of one 1024-thread block: h = the most frequent endpoint of the first n_sample (<= 2048)
// edges, ties to the smaller id — deterministic, so every block that runs it elects the same h. s_tab: 2 x
// kHubSlots u32 of LDS (free again on return). Every thread returns h.
constexpr int kHubPer = (int)(kHubSample / kHubBlock);  // sample edges per thread

// This thread's share of the election sample (hub_elect's input). A caller that also streams edges issues
// these loads first: a wave's loads return in order, so a sample load queued behind the stream's first round
// would hold the election until that whole round had arrived.
__device__ __forceinline__ void hub_sample(const u64* __restrict__ edges, u64 n_sample, u64 (&e)[kHubPer]) {
#pragma unroll
    for (int k = 0; k < kHubPer; ++k) {  // all sample loads in flight at once
        const u64 i = threadIdx.x + (u64)k * kHubBlock;
        e[k] = i < n_sample ? edges[i] : ~0ull;
    }
}

__device__ __forceinline__ u32 hub_elect(const u64 (&e)[kHubPer], u32* s_tab, u32 cap) {
    u32* s_key = s_tab;
    u32* s_cnt = s_tab + kHubSlots;
    __shared__ u32 s_bc[kHubBlock / 64], s_bk[kHubBlock / 64];
    constexpr int kPer = kHubPer;
    {
        const u32x4 kz = {UNSEEN, UNSEEN, UNSEEN, UNSEEN}, cz = {0, 0, 0, 0};
#pragma unroll
        for (u32 s = threadIdx.x; s < kHubSlots / 4; s += kHubBlock) {
            reinterpret_cast<u32x4*>(s_key)[s] = kz;
            reinterpret_cast<u32x4*>(s_cnt)[s] = cz;
        }
    }
    __syncthreads();
    // each thread keeps the best (count, key) among its own increments; argmax: count desc, id asc
    u32 bc = 0, bk = UNSEEN;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (e[k] == ~0ull) continue;
        const u32 a = (u32)e[k], b = (u32)(e[k] >> 32);
        if (a >= cap || b >= cap) continue;  // a bad edge is flagged by the pass that folds it
        const u32 ca = hub_count(a, s_key, s_cnt);
        if (hub_better(ca, a, bc, bk)) {
            bc = ca;
            bk = a;
        }
        const u32 cb = hub_count(b, s_key, s_cnt);
        if (hub_better(cb, b, bc, bk)) {
            bc = cb;
            bk = b;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const u32 c2 = __shfl_down(bc, off, 64), k2 = __shfl_down(bk, off, 64);
        if (hub_better(c2, k2, bc, bk)) {
            bc = c2;
            bk = k2;
        }
    }
    if ((threadIdx.x & 63) == 0) {
        s_bc[threadIdx.x >> 6] = bc;
        s_bk[threadIdx.x >> 6] = bk;
    }
    __syncthreads();
    // every wave reduces the kHubBlock / 64 wave winners itself (no serial loop, no further barrier)
    const u32 lane = threadIdx.x & 63;
    bc = lane < kHubBlock / 64 ? s_bc[lane] : 0;
    bk = lane < kHubBlock / 64 ? s_bk[lane] : UNSEEN;
    for (int off = 8; off > 0; off >>= 1) {
        static_assert(kHubBlock / 64 == 16, "wave winners fit 16 lanes");
        const u32 c2 = __shfl_xor(bc, off, 64), k2 = __shfl_xor(bk, off, 64);
        if (hub_better(c2, k2, bc, bk)) {
            bc = c2;
            bk = k2;
        }
    }
    // UNSEEN when no sampled edge was valid: the seeding then starts from C = {} (every edge takes the union path)
    return __shfl(bk, 0, 64);
}

// Elects h and initialises C = {h}: flags (zeroed up to a whole bitmap word) and the bitmap. Every block of
// the grid elects the same h (deterministic argmax) and clears its own share of both arrays.
__global__ __launch_bounds__(kHubBlock) void seed_hub_kernel(const u64* __restrict__ edges, u64 n_sample,
                                                             u8* __restrict__ flags, u32* __restrict__ bits32, u32 n,
                                                             u32* __restrict__ gmin) {
    extern __shared__ __attribute__((aligned(16))) u32 s_dyn[];
    u64 e[kHubPer];
    hub_sample(edges, n_sample, e);
    const u32 h = hub_elect(e, s_dyn, n);
    // this block's share: 32 ids per unit = 32 flag bytes (two 16-B stores) + one bitmap word
    const u64 nu = ((u64)n + 31) / 32;
    const u64 per = (nu + gridDim.x - 1) / gridDim.x;
    const u64 u0 = blockIdx.x * per, u1 = min(nu, u0 + per);
    u32x4* f4 = reinterpret_cast<u32x4*>(flags);
    for (u64 u = u0 + threadIdx.x; u < u1; u += kHubBlock) {
        u32x4 z0 = {0, 0, 0, 0}, z1 = {0, 0, 0, 0};
        u32 w = 0;
        if (u == h / 32) {
            const u32 o = h & 31;
            if (o < 16) z0[o >> 2] = 1u << (8 * (o & 3));
            else z1[(o - 16) >> 2] = 1u << (8 * (o & 3));
            w = 1u << o;
        }
        f4[2 * u] = z0;
        f4[2 * u + 1] = z1;
        bits32[u] = w;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *gmin = h;  // the hub's own slot of the seeding's minimum
}

// One BFS pass over the prefix. LDS = true: every block (one per CU) holds the bitmap of C as of the last
// pack in LDS; a discovered id is set there too (LDS atomicOr: propagation inside the block, and each id is
// flagged once per block), then flagged in HBM. LDS = false: lookups go to the global bitmap.
// HUB (first pass of the fused seeding, LDS only): there is no C yet — the block elects h itself (hub_elect,
// the same h in every block), starts from the LDS bitmap {h} instead of copying one in, and block 0 flags h.
// Flags hold the seeding's epoch (1..255) instead of 1, so no pass ever has to clear them.
template <bool LDS, int BLOCK, bool NT, bool HUB>
__global__ __launch_bounds__(BLOCK) void seed_bfs_kernel(const u64* __restrict__ edges, u64 n,
                                                         const u32* __restrict__ bits32, u32 nwords32,
                                                         u8* __restrict__ flags, u32* __restrict__ bmin, u8 epoch,
                                                         u32 cap, u32* __restrict__ err) {
    trace_start(kTrSeedBfs);
    static_assert(!HUB || (LDS && BLOCK == kHubBlock), "the fused hub election needs the LDS variant");
    extern __shared__ __attribute__((aligned(16))) u32 s_dyn[];
    __shared__ u32 s_min;
    constexpr int D = 8;  // 16-B edge pairs in flight per lane
    auto ld = [](const u32x4* p) -> u32x4 {
        if constexpr (NT) return __builtin_nontemporal_load(p);
        else return *p;
    };
    // aligned body of 16-B edge pairs + scalar head/tail edges; this lane's pairs are i, i + stride, ...
    const u64 head = ((reinterpret_cast<uintptr_t>(edges) & 15) && n) ? 1 : 0;
    const u64 n2 = (n - head) / 2;
    const u32x4* body = reinterpret_cast<const u32x4*>(edges + head);
    const u64 stride = (u64)gridDim.x * BLOCK;
    const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
    const u64 cnt = i < n2 ? (n2 - 1 - i) / stride + 1 : 0;
    u64 e[kHubPer];
    if constexpr (HUB) hub_sample(edges, n < kHubSample ? n : kHubSample, e);  // ahead of the stream (hub_sample)
    u32x4 q[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {  // the first round is in flight while the bitmap is copied into LDS
        // unconditional (clamped in range; launch_seed guarantees n2 >= 1): the compiler can then count them
        // and wait for the sample alone before the election
        const u64 j = i + k * stride;
        q[k] = ld(body + (j < n2 ? j : n2 - 1));
    }
    u32* bm = const_cast<u32*>(bits32);
    if (threadIdx.x == 0) s_min = UNSEEN;
    u32 lmin = UNSEEN;
    if constexpr (HUB) {
        const u32 h = hub_elect(e, s_dyn, cap);  // ends with a barrier
        const u32x4 z = {0, 0, 0, 0};
        for (u32 w = threadIdx.x; w < nwords32 / 4; w += BLOCK) reinterpret_cast<u32x4*>(s_dyn)[w] = z;
        __syncthreads();
        if (threadIdx.x == 0 && h != UNSEEN) {
            s_dyn[h >> 5] = 1u << (h & 31);
            if (blockIdx.x == 0) {
                flags[h] = epoch;
                lmin = h;
            }
        }
        bm = s_dyn;
    } else if constexpr (LDS) {
        const u32x4* src = reinterpret_cast<const u32x4*>(bits32);
        u32x4* dst = reinterpret_cast<u32x4*>(s_dyn);
        if (nwords32) lds_fill<BLOCK>(dst, src, nwords32 / 4);
        bm = s_dyn;
    }
    __syncthreads();
    auto visit = [&](u32 a, u32 b) {
        if (!edge_ok(a, b, cap, err)) return;
        const u32 ia = (bm[a >> 5] >> (a & 31)) & 1u, ib = (bm[b >> 5] >> (b & 31)) & 1u;
        if (ia != ib) {
            const u32 x = ia ? b : a, m = 1u << (x & 31);
            bool fresh = true;
            if constexpr (LDS) fresh = !(atomicOr(&bm[x >> 5], m) & m);
            if (fresh) {
                flags[x] = epoch;
                lmin = min(lmin, x);
            }
        }
    };
    for (u64 r = 0; r < cnt; r += D) {  // software-pipelined: round r + D is loading while round r is visited
        u32x4 nq[D];
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (r + D + k < cnt) nq[k] = ld(body + i + (r + D + k) * stride);
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (r + k < cnt) {
                visit(q[k].x, q[k].y);
                visit(q[k].z, q[k].w);
            }
#pragma unroll
        for (int k = 0; k < D; ++k) q[k] = nq[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (head) visit((u32)edges[0], (u32)(edges[0] >> 32));
        if (head + 2 * n2 < n) visit((u32)edges[n - 1], (u32)(edges[n - 1] >> 32));
    }
    for (int off = 32; off > 0; off >>= 1) lmin = min(lmin, (u32)__shfl_down(lmin, off, 64));
    if ((threadIdx.x & 63) == 0 && lmin != UNSEEN) atomicMin(&s_min, lmin);
    __syncthreads();
    // the block's minimum discovery, in its own slot (seed_pack_kernel<true> reduces the slots): no global atomic
    if (threadIdx.x == 0) bmin[blockIdx.x] = s_min;
}

// Pack the flag bytes into the bitmap of C (8 lanes = one u32 word, 4 ids per lane). PARENT = true (the
// last step of the seeding): also parent[v] = (v in C) ? gmin : UNSEEN with 16-B stores, and publish gmin as
// the tracked component.
// A flag byte marks C iff it equals the seeding's epoch.
template <bool PARENT>
__global__ __launch_bounds__(kBlock) void seed_pack_kernel(u32* __restrict__ parent, u32 n, const u8* __restrict__ flags,
                                                           u32* __restrict__ bits32, const u32* __restrict__ bmin,
                                                           u32 n_bmin, u32* __restrict__ giant, u8 epoch) {
    trace_start(kTrSeedPack);
    u32 g = 0;
    if constexpr (PARENT) {  // g = min C = the minimum of the BFS blocks' (and the hub's) slots
        __shared__ u32 s_g[kBlock / 64];
        u32 m = UNSEEN;
        for (u32 j = threadIdx.x; j < n_bmin; j += kBlock) m = min(m, bmin[j]);
        for (int off = 32; off > 0; off >>= 1) m = min(m, (u32)__shfl_down(m, off, 64));
        if ((threadIdx.x & 63) == 0) s_g[threadIdx.x >> 6] = m;
        __syncthreads();
        g = s_g[0];
#pragma unroll
        for (int w = 1; w < kBlock / 64; ++w) g = min(g, s_g[w]);
        if (blockIdx.x == 0 && threadIdx.x == 0) *giant = g;
    }
    const u32 ep4 = 0x01010101u * epoch;
    const u64 stride = (u64)gridDim.x * kBlock;
    const u64 nq = ((u64)n + 31) / 32 * 8;  // whole bitmap words
    const u32* f32 = reinterpret_cast<const u32*>(flags);
    u32x4* p4 = reinterpret_cast<u32x4*>(parent);
    const u32 lane = threadIdx.x & 63;
    for (u64 q0 = (u64)blockIdx.x * kBlock + (threadIdx.x - lane); q0 < nq; q0 += stride) {  // whole waves
        const u64 q = q0 + lane;
        u32 nib = 0;
        if (q < nq) {
            const u32 f = f32[q] ^ ep4;  // flag bytes of ids 4q..4q+3: 0 iff in C
            nib = ((f & 0xFFu) == 0) | (((f & 0xFF00u) == 0) << 1) | (((f & 0xFF0000u) == 0) << 2) |
                  (((f & 0xFF000000u) == 0) << 3);
            if constexpr (PARENT) {
                const u64 v = 4 * q;
                if (v + 3 < n) {
                    u32x4 o;
                    o.x = (nib & 1u) ? g : UNSEEN;
                    o.y = (nib & 2u) ? g : UNSEEN;
                    o.z = (nib & 4u) ? g : UNSEEN;
                    o.w = (nib & 8u) ? g : UNSEEN;
                    p4[q] = o;
                } else {
                    for (u32 k = 0; k < 4; ++k)
                        if (v + k < n) parent[v + k] = ((nib >> k) & 1u) ? g : UNSEEN;
                }
            }
        }
        u32 w = nib << ((lane & 7) * 4);
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        if ((lane & 7) == 0 && q < nq) bits32[q >> 3] = w;
    }
}

// ------------------------------------------------------------------------------------------------
// Cross-GPU merge message (include/gelly_cc.h: header, giant bitmap, (v, label) list of the other seen ids).
// ------------------------------------------------------------------------------------------------
constexpr unsigned kMsgWordsPerBlock = 256;  // 16K ids per count block: 16 waves x 16 words
constexpr int kMsgBlock = 1024;

// The label of v from a forest that may not be compressed: FIND follows parent pointers with read-only loads
// (no path splitting: a find of the encode and the same id's find in msg_write_kernel must agree, and nothing
// mutates parent[] between them), otherwise parent[] already holds the canonical labels. g is the tracked
// component's current root and g0 its root at the last refresh (now under g, or g itself): their children are
// labelled without a walk.
template <bool FIND>
__device__ __forceinline__ u32 msg_label(const u32* __restrict__ parent, u32 v, u32 p, u32 g, u32 g0) {
    if (!FIND || p >= v || p == g) return p;  // a label, a root or UNSEEN
    if (p == g0) return g;
    NoCount c;
    return UFRead::find_from(const_cast<u32*>(parent), v, p, c);
}

// Encode, pass 1 of 3: each block owns kMsgWordsPerBlock consecutive 64-id words (16 per wave). It writes the
// giant bitmap words (into the message and, with `mine`, into the forest's own tracked-component bitmap), the
// mask of every word's "other" seen ids (scratch, 8 B per word) and its count of others. No atomics: round 1's
// single kernel reserved list space with one atomicAdd per 4096-id block on one header word, and 16K
// same-address atomics serialised at the memory side (476 us of a 64M-id encode, tools/merge_probe.py).
template <bool FIND>
__global__ __launch_bounds__(kMsgBlock) void msg_count_kernel(const u32* __restrict__ parent, u32 n,
                                                              const u32* __restrict__ hdr, const u32* __restrict__ giant_prev,
                                                              u64* __restrict__ bits, u64* __restrict__ mine,
                                                              u64* __restrict__ oth, u32* __restrict__ cnt) {
    __shared__ u32 s_cnt[kMsgBlock / 64];
    constexpr int kW = kMsgWordsPerBlock / (kMsgBlock / 64);  // words per wave
    const u32 g = hdr[0];
    const u32 g0 = giant_prev ? *giant_prev : UNSEEN;
    const u64 nw = ((u64)n + 63) / 64;
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 w0 = (u64)blockIdx.x * kMsgWordsPerBlock + (u64)wave * kW;
    u32 l[kW];
#pragma unroll
    for (int k = 0; k < kW; ++k) {  // all loads of the wave in flight before any find
        const u64 v = (w0 + k) * 64 + lane;
        l[k] = (w0 + k < nw && v < n) ? parent[v] : UNSEEN;
    }
    u32 total = 0;
#pragma unroll
    for (int k = 0; k < kW; ++k) {
        const u64 w = w0 + k;
        const u32 lab = msg_label<FIND>(parent, (u32)(w * 64 + lane), l[k], g, g0);
        const unsigned long long in_g = __ballot(lab != UNSEEN && lab == g);
        const unsigned long long o = __ballot(lab != UNSEEN && lab != g);
        if (lane == 0 && w < nw) {
            bits[w] = in_g;
            if (mine) mine[w] = in_g;
            oth[w] = o;
        }
        total += (u32)__popcll(o);
    }
    if (lane == 0) s_cnt[wave] = total;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 t = 0;
        for (int k = 0; k < kMsgBlock / 64; ++k) t += s_cnt[k];
        cnt[blockIdx.x] = t;
    }
}

// Encode, pass 1 after a compress that wrote the masks (compress_bits_kernel's chunk_oth): per count block the
// number of other seen ids, read from the 8-B masks instead of the 4-B labels, and the forest's giant bitmap
// copied into the message. One word per thread.
__global__ __launch_bounds__(kBlock) void msg_cnt_kernel(const u64* __restrict__ oth, const u64* __restrict__ mine,
                                                         u64* __restrict__ bits, u64 nw, u32* __restrict__ cnt) {
    static_assert(kMsgWordsPerBlock == kBlock, "one word per thread");
    __shared__ u32 s_tot[kBlock / 64];
    const u64 w = (u64)blockIdx.x * kMsgWordsPerBlock + threadIdx.x;
    u32 c = 0;
    if (w < nw) {
        c = (u32)__popcll(oth[w]);
        bits[w] = mine[w];
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) s_tot[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 t = 0;
        for (int k = 0; k < kBlock / 64; ++k) t += s_tot[k];
        cnt[blockIdx.x] = t;
    }
}

// Encode, pass 2: one block, the exclusive prefix of the count blocks' totals -> base[]; hdr[1] = the list's
// true length (a receiver compares it with the capacity: a longer list means a repair round).
constexpr int kScanBlock = 1024;
constexpr int kScanPer = 4;  // items per thread and round: 4096 count blocks (C4's 64M ids) in one round
__global__ __launch_bounds__(kScanBlock) void msg_scan_kernel(const u32* __restrict__ cnt, u32 nb, u32* __restrict__ base,
                                                              u32* __restrict__ hdr) {
    __shared__ u64 s_wave[kScanBlock / 64];
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 carry = 0;
    for (u32 r0 = 0; r0 < nb; r0 += kScanBlock * kScanPer) {
        const u32 b0 = r0 + threadIdx.x * kScanPer;
        u32 x[kScanPer];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) x[k] = (b0 + k < nb) ? cnt[b0 + k] : 0;  // all in flight
        u64 t = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) t += x[k];
        u64 incl = t;  // wave inclusive scan of the threads' sums
        for (int off = 1; off < 64; off <<= 1) {
            const u64 y = __shfl_up(incl, off, 64);
            if (lane >= (u32)off) incl += y;
        }
        if (lane == 63) s_wave[wave] = incl;
        __syncthreads();
        u64 before = carry, total = carry;
        for (u32 k = 0; k < kScanBlock / 64; ++k) {
            if (k < wave) before += s_wave[k];
            total += s_wave[k];
        }
        u64 run = before + incl - t;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            if (b0 + k < nb) base[b0 + k] = (u32)min<u64>(run, 0xFFFFFFFFull);
            run += x[k];
        }
        carry = total;
        __syncthreads();  // s_wave is rewritten by the next round
    }
    if (threadIdx.x == 0) hdr[1] = (u32)min<u64>(carry, 0xFFFFFFFFull);
}

// Encode, pass 3: one 256-thread block per count block, one word per lane. The masks locate the other seen ids
// (sparse: 0.2 % of C4's ids at an 8-way split), wave and block prefixes of their counts place them, and only
// those ids are read again. Pairs come out in id order, so a message (and a serialized summary) is deterministic.
template <bool FIND>
__global__ __launch_bounds__(kBlock) void msg_write_kernel(const u32* __restrict__ parent, u32 n, const u64* __restrict__ oth,
                                                           const u32* __restrict__ base, const u32* __restrict__ hdr,
                                                           const u32* __restrict__ giant_prev, u32* __restrict__ others,
                                                           u64 cap) {
    static_assert(kMsgWordsPerBlock == kBlock, "one word per lane");
    __shared__ u32 s_tot[kBlock / 64];
    const u32 lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 nw = ((u64)n + 63) / 64;
    const u64 w = (u64)blockIdx.x * kMsgWordsPerBlock + threadIdx.x;
    u64 m = w < nw ? oth[w] : 0;
    const u32 c = (u32)__popcll(m);
    u32 incl = c;
    for (int off = 1; off < 64; off <<= 1) {
        const u32 x = __shfl_up(incl, off, 64);
        if (lane >= (u32)off) incl += x;
    }
    if (lane == 63) s_tot[wave] = incl;
    __syncthreads();
    u64 pos = (u64)base[blockIdx.x] + (incl - c);
    for (u32 k = 0; k < wave; ++k) pos += s_tot[k];
    if (!m) return;
    const u32 g = hdr[0];
    const u32 g0 = giant_prev ? *giant_prev : UNSEEN;
    while (m) {
        const u32 v = (u32)(w * 64 + (u64)__builtin_ctzll(m));
        m &= m - 1;
        if (pos < cap) {
            others[2 * pos] = v;
            others[2 * pos + 1] = msg_label<FIND>(parent, v, parent[v], g, g0);
        }
        ++pos;
    }
}

// One wave: the header, and the witness slots of the absorb that follows a merge's all_gather re-armed to UNSEEN
// (saves that absorb a memset launch). With `parent` (an uncompressed forest) the tracked root is followed to the
// component's current root, which is also stored in giant_next (the forest's next tracked-root slot).
__global__ void msg_header_kernel(u32* __restrict__ hdr, const u32* __restrict__ giant_root, u32 has_giant, u32 n,
                                  u32* __restrict__ witness, const u32* __restrict__ parent, u32* __restrict__ giant_next) {
    if (threadIdx.x == 0) {
        u32 g = has_giant ? *giant_root : UNSEEN;
        if (parent && g < n) {
            NoCount c;
            g = UFRead::find_from(const_cast<u32*>(parent), g, parent[g], c);
        }
        hdr[0] = g;
        hdr[1] = 0;
        hdr[2] = n;
        hdr[3] = 0;
        if (giant_next) *giant_next = g;
    }
    if (witness) witness[threadIdx.x] = UNSEEN;
}

// Absorbing the P-1 peer messages of an all_gather (gcc_forest_absorb_many), three launches:
//  msg_overlap_kernel: for each peer p, does its giant G_p share an id with this forest's tracked component T
//    (bitmap `mine`, root R; valid forever since components only grow)? If so, witness[p] = one shared id.
//  msg_absorb_bits_kernel: an overlapping peer's giant G_p is connected to T (root R) through the witness, so
//    the union U of their bitmaps only needs its ids OUTSIDE T joined to R, each ONCE however many peers hold it
//    (one 64-id word per wave, one id per lane); a new id above R by one CAS (or deferred to the compress);
//  msg_absorb_kernel: the giants without overlap (or all of them when there is no T: id by id against their
//    own root), then the (v, label) lists.
constexpr u32 kMaxPeers = 64;

// The ids < n of bitmap word w: a peer's or a deserialized message's last word may carry bits past the id range
// (a well-formed encode never sets them; gcc_forest_deserialize's bytes are untrusted), which must not index parent[].
__device__ __forceinline__ u64 id_range_mask(u64 w, u32 n) {
    const u64 lo = w * 64;
    return lo + 64 <= n ? ~0ull : (lo >= n ? 0ull : (1ull << (n - lo)) - 1);
}

__global__ __launch_bounds__(kBlock) void msg_overlap_kernel(const char* __restrict__ msgs, u64 stride, u32 count,
                                                             u32 skip, u32 n, const u64* __restrict__ mine,
                                                             u32* __restrict__ witness) {
    const u64 nw = ((u64)n + 63) / 64;
    const u64 chunks = (nw + 63) / 64;  // one word per lane
    const u32 lane = threadIdx.x & 63;
    const u64 wave = (u64)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const u64 waves = (u64)gridDim.x * (kBlock / 64);
    for (u64 t = wave; t < (u64)count * chunks; t += waves) {
        const u32 p = (u32)(t / chunks);
        if (p == skip) continue;
        const u32* hdr = reinterpret_cast<const u32*>(msgs + p * stride);
        if (hdr[2] != n || hdr[0] >= n) continue;
        if (__hip_atomic_load(&witness[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != UNSEEN) continue;
        const u64 w = (t - (u64)p * chunks) * 64 + lane;
        u64 both = 0;
        if (w < nw)
            both = reinterpret_cast<const u64*>(msgs + p * stride + GCC_MSG_HEADER_BYTES)[w] & mine[w] & id_range_mask(w, n);
        const unsigned long long wb = __ballot(both != 0);
        if (wb && lane == (u32)__builtin_ctzll(wb)) witness[p] = (u32)(w * 64 + __builtin_ctzll(both));  // any one
    }
}

// Peer p's giant root g_p and its witness (an id shared with T), or UNSEEN; the same in every block.
__device__ __forceinline__ void msg_peers(const char* __restrict__ msgs, u64 stride, u32 count, u32 skip, u32 n,
                                          bool tracked, const u32* __restrict__ witness, u32* s_g, u32* s_w) {
    if (threadIdx.x < kMaxPeers) {
        u32 g = UNSEEN, wv = UNSEEN;
        if (threadIdx.x < count && threadIdx.x != skip) {
            const u32* hdr = reinterpret_cast<const u32*>(msgs + threadIdx.x * stride);
            if (hdr[2] == n && hdr[0] < n) {
                g = hdr[0];
                wv = tracked ? witness[threadIdx.x] : UNSEEN;
            }
        }
        s_g[threadIdx.x] = g;
        s_w[threadIdx.x] = wv;
    }
    __syncthreads();
}

// Absorb, phase 1 (after msg_overlap_kernel): the union U of the giants that meet T, minus T, one 64-id word per
// wave, each id once however many peers hold it. Every id of such a giant is connected to T (through the
// witness), so x in U \ T joins T's root R. A new id above R — the common case — is hung under R by ONE CAS
// (UNSEEN -> R). Round 1-3 used a plain store (in this kernel x has no other writer), but phase 2's list unions may
// CAS the same slot in the next kernel, and on gfx950 a plain store can land after the next kernel's memory-side
// atomics. The default absorb defers the new ids to its compress (newbits) and stores nothing here.
// Anything else takes the full union.
__global__ __launch_bounds__(kBlock) void msg_absorb_bits_kernel(u32* __restrict__ parent, const char* __restrict__ msgs,
                                                                 u64 stride, u32 count, u32 skip, u32 n,
                                                                 const u64* __restrict__ mine,
                                                                 const u32* __restrict__ tracked,
                                                                 const u32* __restrict__ witness,
                                                                 const u64* __restrict__ seen_oth,
                                                                 u64* __restrict__ newbits) {
    __shared__ u32 s_g[kMaxPeers];
    __shared__ u32 s_w[kMaxPeers];
    msg_peers(msgs, stride, count, skip, n, true, witness, s_g, s_w);
    const u32 lane = threadIdx.x & 63;
    const u32 R = *tracked;
    const u64 nw = ((u64)n + 63) / 64;
    const u64 wave = (u64)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const u64 waves = (u64)gridDim.x * (kBlock / 64);
    // 64 words per wave and round, one per lane: the overlapping peers' words and T's word of every lane in flight
    // at once (coalesced: consecutive words across the lanes), then the new ids word by word, one id per lane, four
    // words' parent loads in flight before their stores. (Round 1 took one word per wave and round: its peer
    // loads, OR-shuffles, T load and stores were one dependent chain per 64 ids, 284 us on C4's 64M ids.)
    for (u64 w0 = wave * 64; w0 < nw; w0 += waves * 64) {
        const u64 w = w0 + lane;
        u64 m = 0, so = ~0ull;
        if (w < nw) {
            for (u32 p = 0; p < count; ++p)
                if (s_g[p] != UNSEEN && s_w[p] != UNSEEN)
                    m |= reinterpret_cast<const u64*>(msgs + p * stride + GCC_MSG_HEADER_BYTES)[w];
            if (m) m &= ~mine[w] & id_range_mask(w, n);
            if (m && seen_oth) so = seen_oth[w];
        }
        if (newbits) {  // deferred: the new ids above R only go into newbits, the compress right after labels them
            u64 nb = 0, seen_todo = 0;
            if (w < nw) {
                const u64 above = (R >= w * 64 + 63) ? 0ull
                                : (R < w * 64 ? ~0ull : (~0ull << (R - w * 64)) << 1);  // ids > R of this word
                nb = m & ~so & above;
                seen_todo = m & ~nb;  // seen outside T (or a new id below R): the union
                newbits[w] = nb;      // overwrites this word's mask (read above, same lane)
            }
            unsigned long long sw = __ballot(seen_todo != 0);
            while (sw) {
                const int j = __builtin_ctzll(sw);
                sw &= sw - 1;
                const u64 t = __shfl(seen_todo, j, 64);
                const u32 v = (u32)((w0 + (u64)j) * 64 + lane);
                if ((t >> lane) & 1ull) {
                    NoCount c;
                    UF::unite(parent, v, R, c);
                }
            }
            continue;
        }
        unsigned long long todo_words = __ballot(m != 0);
        if (seen_oth) {  // the encode's masks say which ids outside T are seen: the others are new, no load needed
            while (todo_words) {
                const int j = __builtin_ctzll(todo_words);
                todo_words &= todo_words - 1;
                const u64 t = __shfl(m, j, 64);
                const u64 sj = __shfl(so, j, 64);
                const u32 v = (u32)((w0 + (u64)j) * 64 + lane);
                if (((t >> lane) & 1ull) && v != R) {
                    // a new id: one CAS (a plain store could land after msg_absorb_kernel's CASes: DESIGN §3)
                    if (!(v > R && !((sj >> lane) & 1ull) && gcc::cas(&parent[v], UNSEEN, R) == UNSEEN))
                        gcc::absorb_join(parent, v, R);
                }
            }
            continue;
        }
        while (todo_words) {
            constexpr int kU = 4;
            u32 v[kU];
            bool on[kU];
            u32 pv[kU];
#pragma unroll
            for (int k = 0; k < kU; ++k) {
                on[k] = false;
                v[k] = 0;
                if (todo_words) {
                    const int j = __builtin_ctzll(todo_words);
                    todo_words &= todo_words - 1;
                    const u64 t = __shfl(m, j, 64);
                    v[k] = (u32)((w0 + (u64)j) * 64 + lane);
                    on[k] = ((t >> lane) & 1ull) && v[k] != R;
                }
                pv[k] = on[k] ? gcc::ld(&parent[v[k]]) : 0;
            }
#pragma unroll
            for (int k = 0; k < kU; ++k)
                if (on[k]) {
                    if (!(v[k] > R && pv[k] == UNSEEN && gcc::cas(&parent[v[k]], UNSEEN, R) == UNSEEN))  // a new id: one CAS
                        gcc::absorb_join(parent, v[k], R);
                }
        }
    }
}

// Absorb, phase 2 (or the whole absorb when this forest tracks no component): the giants that do not meet T
// (each id against its own root g_p) and every peer's (v, label) list.
__global__ __launch_bounds__(kBlock) void msg_absorb_kernel(u32* __restrict__ parent, const char* __restrict__ msgs,
                                                            u64 stride, u32 count, u32 skip, u64 cap, u32 n,
                                                            bool tracked, const u32* __restrict__ witness,
                                                            const u64* __restrict__ newbits,
                                                            const u32* __restrict__ tracked_root) {
    __shared__ u32 s_g[kMaxPeers];
    __shared__ u32 s_w[kMaxPeers];
    msg_peers(msgs, stride, count, skip, n, tracked, witness, s_g, s_w);
    NoCount c;
    // (an overlapping peer's giant needs no union of its own: phase 1 joined every id of it outside T to R)
    const u32 lane = threadIdx.x & 63;
    const u64 nw = ((u64)n + 63) / 64;
    const u64 wave = (u64)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const u64 waves = (u64)gridDim.x * (kBlock / 64);
    bool any_lone = false;
    for (u32 p = 0; p < count; ++p) any_lone |= s_g[p] != UNSEEN && s_w[p] == UNSEEN;
    if (any_lone) {  // rare: peers whose giant does not touch T (or no T)
        for (u64 w = wave; w < nw; w += waves) {
            u64 lone = 0;
            if (lane < count && s_g[lane] != UNSEEN && s_w[lane] == UNSEEN)
                lone = reinterpret_cast<const u64*>(msgs + lane * stride + GCC_MSG_HEADER_BYTES)[w] & id_range_mask(w, n);
            const u64 v = w * 64 + lane;
            unsigned long long lb = __ballot(lone != 0);
            bool in_lone = false;
            while (lb) {
                const u32 p = (u32)__builtin_ctzll(lb);
                lb &= lb - 1;
                const u64 mp = __shfl(lone, (int)p, 64);
                if ((mp >> lane) & 1ull) {
                    in_lone = true;
                    if ((u32)v != s_g[p]) UF::unite(parent, (u32)v, s_g[p], c);
                }
            }
            // a deferred new id (absorb_bits' newbits) in a lone giant: that union made it seen, so it joins R here
            if (in_lone && newbits && v < n && ((newbits[w] >> lane) & 1ull)) UF::unite(parent, (u32)v, *tracked_root, c);
        }
    }
    // the lists as one flat index over (peer, entry): one header load per entry, every union in flight at once
    const u64 stride_t = (u64)gridDim.x * kBlock;
    for (u64 t = (u64)blockIdx.x * kBlock + threadIdx.x; t < (u64)count * cap; t += stride_t) {
        const u32 p = (u32)(t / cap);
        const u64 k = t - (u64)p * cap;
        if (p == skip) continue;
        const u32* hdr = reinterpret_cast<const u32*>(msgs + p * stride);
        if (hdr[2] != n || k >= min((u64)hdr[1], cap)) continue;
        const u32* others = reinterpret_cast<const u32*>(msgs + p * stride + GCC_MSG_HEADER_BYTES + nw * sizeof(u64));
        const u32 v = others[2 * k], l = others[2 * k + 1];
        if (v < n && l < n) {
            UF::unite(parent, v, l, c);
            // a deferred new id (absorb_bits' newbits) is in R's component too: this union made it seen, so the
            // compress would no longer label it through newbits
            if (newbits && (((newbits[v >> 6] >> (v & 63)) | (newbits[l >> 6] >> (l & 63))) & 1ull))
                UF::unite(parent, v, *tracked_root, c);
        }
    }
}

// ---- the delta merge's message (round 6; include/gelly_cc.h "delta message") ----------------------
// u32 header[4] = {edges the sender folded since it armed, n_pairs (true count), id_capacity, status}, then n_pairs
// (x, root(x)) pairs: one per id of the sender's delta lists, its root found in the sender's forest (read-only finds).
// Every block loads the stripes' counts and their prefix (wave 0), then the flat index over the pairs maps to a stripe
// by binary search: one kernel, no global atomics.
__global__ __launch_bounds__(kBlock) void delta_encode_kernel(const u32* __restrict__ parent, const u32* __restrict__ ids,
                                                              const u32* __restrict__ cnt, u32 subcap,
                                                              u32* __restrict__ msg, u64 cap, u32 n, u32 edges,
                                                              u32 armed) {
    __shared__ u32 s_pre[kDeltaStripes + 1];
    __shared__ u32 s_bad;
    if (threadIdx.x < 64) {
        const u32 lane = threadIdx.x;
        u32 k = armed ? cnt[lane] : 0;
        const bool over = k > subcap;
        k = min(k, subcap);
        u32 incl = k;
        for (int off = 1; off < 64; off <<= 1) {
            const u32 y = __shfl_up(incl, off, 64);
            if (lane >= (u32)off) incl += y;
        }
        s_pre[lane + 1] = incl;
        const unsigned long long ob = __ballot(over);
        if (lane == 0) {
            s_pre[0] = 0;
            s_bad = (ob != 0 || (armed && cnt[kDeltaStripes] != 0)) ? 1u : 0u;
        }
    }
    __syncthreads();
    const u32 total = s_pre[kDeltaStripes];
    const u32 status = !armed ? GCC_DELTA_STATUS_UNARMED : (s_bad ? GCC_DELTA_STATUS_OVERFLOW : 0u);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        msg[0] = edges;
        msg[1] = total;
        msg[2] = n;
        msg[3] = status;
    }
    if (status) return;
    u32* pairs = msg + GCC_MSG_HEADER_BYTES / sizeof(u32);
    const u64 end = min((u64)total, cap);
    for (u64 t = (u64)blockIdx.x * kBlock + threadIdx.x; t < end; t += (u64)gridDim.x * kBlock) {
        u32 lo = 0, hi = kDeltaStripes;  // the last stripe s with s_pre[s] <= t (a non-empty one)
        while (hi - lo > 1) {
            const u32 mid = (lo + hi) >> 1;
            if (s_pre[mid] <= (u32)t) lo = mid;
            else hi = mid;
        }
        const u32 x = ids[(size_t)lo * subcap + ((u32)t - s_pre[lo])];
        NoCount c;
        const u32 p = parent[x];
        pairs[2 * t] = x;
        pairs[2 * t + 1] = (p >= x) ? x : UFRead::find_from(const_cast<u32*>(parent), x, p, c);
    }
}

// Absorb the peers' delta messages: unite(x, r) for every pair, one pair per lane over a flat (peer, pair) index. The
// unions write parent[] with memory-side atomics only (UFRec) and, when every mutation since the last compress was
// recorded (bloom != null), mark their hooks in the incremental compress's bloom, so that compress stays incremental.
// Block 0 also zeroes this forest's own stripe counters (the encode read them one kernel before): the delta is armed
// again from here (the merge is complete once this kernel has run).
template <bool BLOOM>
__global__ __launch_bounds__(kBlock) void delta_absorb_kernel(u32* __restrict__ parent, const char* __restrict__ msgs,
                                                              u64 stride, u32 count, u32 skip, u64 cap, u32 n,
                                                              u32* __restrict__ bloom, u32* __restrict__ own_cnt,
                                                              u32* __restrict__ err) {
    if (blockIdx.x == 0 && own_cnt && threadIdx.x <= kDeltaStripes) atomicExch(&own_cnt[threadIdx.x], 0u);
    NoCount c;
    const u64 stride_t = (u64)gridDim.x * kBlock;
    for (u64 t = (u64)blockIdx.x * kBlock + threadIdx.x; t < (u64)count * cap; t += stride_t) {
        const u32 p = (u32)(t / cap);
        const u64 k = t - (u64)p * cap;
        if (p == skip) continue;
        const u32* hdr = reinterpret_cast<const u32*>(msgs + p * stride);
        if (hdr[2] != n || hdr[3] != 0 || k >= min((u64)hdr[1], cap)) continue;
        const u32* pairs = hdr + GCC_MSG_HEADER_BYTES / sizeof(u32);
        const u32 x = pairs[2 * k], r = pairs[2 * k + 1];
        if (x >= n || r >= n) {
            *err = 1u;
            continue;
        }
        if constexpr (BLOOM) gcc::UFRec::unite(parent, x, r, c, gcc::BloomRec{bloom});
        else gcc::UFRec::unite(parent, x, r, c);
    }
}

#include "bucket_fold.h"
#include "signed_bucket.h"  // the signed forest's bucketed fold (gelly_bip.hip), reusing bucket_fold.h's P1
#include "signed_bucket_api.h"

static constexpr size_t slice_filter_lds(int per = 8, int vw = 4) {  // bucket_fold.h slice_filter_kernel's dynamic LDS
    return (bk::kSliceWords + bk::p2_tile(per, vw) + 10 * bk::kMaxVLists) * sizeof(u32) + bk::kMaxVLists * sizeof(u64) +
           (bk::kP2Block / 64) * kRing * sizeof(u64);
}

// counts[0] += #seen, counts[1] += #roots (= #components)
__global__ __launch_bounds__(kBlock) void count_kernel(const u32* __restrict__ parent, u32 n,
                                                       unsigned long long* __restrict__ counts) {
    __shared__ unsigned long long s_seen[kBlock / 64], s_root[kBlock / 64];
    const u64 stride = (u64)gridDim.x * kBlock;
    unsigned long long seen = 0, roots = 0;
    for (u64 v = (u64)blockIdx.x * kBlock + threadIdx.x; v < n; v += stride) {
        const u32 p = parent[v];
        seen += (p != UNSEEN);
        roots += (p == v);
    }
    for (int off = 32; off > 0; off >>= 1) {
        seen += __shfl_down(seen, off, 64);
        roots += __shfl_down(roots, off, 64);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        s_seen[wave] = seen;
        s_root[wave] = roots;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0, b = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            a += s_seen[w];
            b += s_root[w];
        }
        if (a) atomicAdd(&counts[0], a);
        if (b) atomicAdd(&counts[1], b);
    }
}

// The parity digest of a compressed forest (= its canonical labels), as tests/golden/stream_digests.json and
// oracle.label_digest compute it: out[2] += sum_v splitmix64((label[v] << 32) | v) mod 2^64, over every id (UNSEEN
// labels included); out[0] += #seen, out[1] += #roots. Lets a test check every window of a long stream without
// copying 4 B per id to the host.
__device__ __forceinline__ u64 splitmix_fin(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ __launch_bounds__(kBlock) void digest_kernel(const u32* __restrict__ labels, u32 n,
                                                        unsigned long long* __restrict__ out) {
    __shared__ unsigned long long s_acc[3][kBlock / 64];
    const u64 stride = (u64)gridDim.x * kBlock;
    unsigned long long seen = 0, roots = 0, dig = 0;
    for (u64 v = (u64)blockIdx.x * kBlock + threadIdx.x; v < n; v += stride) {
        const u32 l = labels[v];
        seen += (l != UNSEEN);
        roots += (l == v);
        dig += splitmix_fin(((u64)l << 32) | v);
    }
    for (int off = 32; off > 0; off >>= 1) {
        seen += __shfl_down(seen, off, 64);
        roots += __shfl_down(roots, off, 64);
        dig += __shfl_down(dig, off, 64);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        s_acc[0][wave] = seen;
        s_acc[1][wave] = roots;
        s_acc[2][wave] = dig;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long a = 0;
        for (int w = 0; w < kBlock / 64; ++w) a += s_acc[threadIdx.x][w];
        atomicAdd(&out[threadIdx.x], a);  // mod 2^64, like the digest
    }
}

__global__ __launch_bounds__(kBlock) void gen_kernel(gcc_gen_params prm, u64 first, u64 count, uint2* __restrict__ out) {
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
        u32 u, v;
        gcc_gen_edge(&prm, first + i, &u, &v);
        out[i] = make_uint2(u, v);
    }
}

// gcc_step_mark: an empty kernel that profilers count as the bench's once-per-step marker
__global__ void gcc_step_mark_kernel() {}

static inline unsigned grid_for(u64 n, unsigned max_blocks) {
    u64 b = (n + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (unsigned)b;
}

// ------------------------------------------------------------------------------------------------
// host-side forest handle
// ------------------------------------------------------------------------------------------------
// fold pipeline tuning (defaults measured on C2, tools/sweep_fold.py; gcc_forest_tune overrides)
struct FoldTune {
    u64 filter_min_batch = 1ull << 16;  // below this a fresh forest's batch is folded by fold_kernel alone
    // first sampling launch; each next one is sample_growth x larger (round 6: 2^14, one launch fewer than 2^12: C3
    // 1.040 -> 1.028 ms, C5 and C3 in 1M-edge windows unchanged within noise, profiles/r6z_sweep_sampled_start.txt)
    u64 sample_first = 1ull << 14;
    u64 sample_growth = 4;
    u64 sample_div = 128;               // the sampling prefix is 1/sample_div of a fresh forest's first batch
    u64 sample_min = 9ull << 15;        // ... and at least this many edges (C3: a shorter prefix left more CAS work)
    u64 refresh_min_batch = 1ull << 22; // batches above this refresh the giant bitmap at the refresh points
    // refresh points (fractions of the batch), increasing, 0 = unused. C4's per-GPU share: 5.37 -> 4.49 ms with
    // a 1/128 sample and three early refreshes instead of 1/32 and one at 1/4 (profiles/r1_sweep_c4_refresh.log)
    double refresh[3] = {0.04, 0.12, 0.30};
    bool filter = true;
    double filter_min_share = 0.5;  // the voted component must hold this share of the seen samples (0: no check)
    // the share is read back asynchronously (1): the sampled start does not wait for the device; the batch's rest
    // folds plain (correct either way) and the first fold that finds the share landed turns the filter on if it
    // holds. 0: the host waits for the vote mid-batch (rounds 1-5)
    int share_async = 1;
    int depth = 4;  // 16-B edge-pair loads in flight per lane in the filtered kernel (4 or 8)
    // seeded fold of a fresh forest (seed_* kernels): BFS from a hub over the first 1/seed_div of the batch
    bool seed = true;
    int seed_passes = 2;
    u64 seed_div = 3;
    u64 seed_div1 = 3;  // the first BFS pass covers 1/seed_div1 of the batch (>= 1/seed_div)
    double seed_refresh = 0;  // refresh point of a seeded batch (fraction; 0 = none)
    bool hook = true;  // direct atomicMin hook of (T, new id) edges in the filtered stream (filter_round)
    // the filtered fold copies the bitmap into every CU's LDS only when the batch has at least lds_edges_per_word
    // edges per bitmap word (u64); a shorter batch looks its endpoints up in the global (L2-resident) bitmap
    double lds_edges_per_word = 0.0;
    u32 drain_at = 64;  // a wave drains its slow-edge ring once this many edges are pending (1..64)
    bool seed_nt = true;  // non-temporal loads in the BFS passes (false: the prefix may stay in the MALL)
    bool seed_global = false;  // also seed when the bitmap does not fit LDS (global-bitmap BFS lookups)
    bool seed_fuse = true;  // the first BFS pass elects the hub itself (no seed_hub launch, no flag clearing)
    // incremental compress (compress_inc_kernel): plain folds record their mutations in a bloom filter when the
    // forest spans >= inc_min_ids ids and a batch is at most 1/inc_div of them (a short window of a big forest)
    bool refresh_labels = false;  // mid-fold refreshes: bitmap only (false) or a full compress (true)
    // On again since round 4. Rounds 2-3's stale label (a label left at a root hooked in the window, counts intact;
    // profiles/r3ai_gpu_tests_c3_w1M_stale_label.log) was a PLAIN store of the recording fold's path splitting that
    // reached memory after the in-place compress had rewritten the same slot (tools/stress_inc.py: 747 of 7854 C3/w1M
    // streams at round 3's defaults; tools/probe_late_store.hip). The recording fold now writes parent[]
    // with memory-side atomics only (inc_split = 0) and the blooms are cleared with atomics: 0 in the same stress
    bool incremental = true;
    bool inc_inplace = true;  // the incremental compress rewrites only changed parent[] slots (no spare buffer)
    u64 inc_min_ids = 1ull << 22;
    // chosen by speed (round 3, tools/sweep_inc_div.py, profiles/r3c_sweep_inc_div.log): on C3 and C5 the recording
    // fold + incremental compress beat the plain fold + full compress at every window size up to 1/4 of the ids
    // (C3 at 1/4: 555 vs 574 us per window; at 1/16: 170 vs 214). Round 2 had raised it to 64 after a stale label
    // it could not explain; round 3's hardware probe and in-library checks did not reproduce it.
    u64 inc_div = 4;
    // diagnostics: every incremental compress is checked against the roots of the forest it started from and its
    // bloom LDS copies against memory-side reads; failures go to stderr and to gcc_forest_inc_check_stats
    bool inc_check = false;
    // diagnostics that leave the compress itself alone: a check kernel after every incremental compress (1), and the
    // previous labels kept for its records (2); gcc_forest_post_check_stats
    int post_check = 0;
    // the recording fold (fold_kernel<true>): path splitting (plain stores) on / off (OFF: the stale label above; no
    // splitting is also faster on C3 / C5 windows: chains stay short between compresses), and fold_release: an agent
    // release at the end of every block (1) or an s_waitcnt vmcnt(0) at the end of every wave (2) — A/B knobs of the
    // mechanism (1 repairs the split fold, 2 does not: profiles/r4b_*)
    bool inc_split = false;
    int fold_release = 0;
    bool experimental = false;  // unlocks settings known to produce wrong results (inc_split = 1), for reproductions
    // bucketed fold of a fresh forest (bucket_fold.h): batches of >= bucket_min_batch edges over >= bucket_min_ids
    // ids (default: exactly the forests whose giant bitmap does not fit LDS); seeding = bucket_levels P2 + P3 levels
    // over the first bucket_sample of every bucket
    bool bucket = true;
    u64 bucket_min_batch = 1ull << 25;
    u64 bucket_min_ids = (u64)kLdsBitmapMaxWords * 64 + 1;
    // since the first level streams only the hub's slice, the whole of it (C1 = every neighbour of h in the batch)
    // + one level over a quarter of every bucket beat three levels over 15 % (profiles/r2c_sweep_seeding.log:
    // C4 11.0 -> 10.8 ms, the share equal; round 2's first sweep, r2_sweep_c4_p1.log, predates the hub level).
    // Round 3 (6-B entries, faster P2): 15 % of every bucket for the second level, C4 10.22 -> 10.04 ms (0.15 / 0.2 /
    // 0.25 / 0.3: 10.04 / 10.06 / 10.22 / 10.33 ms, profiles/r3h_sweep_seed_sample.log)
    int bucket_levels = 2;
    double bucket_sample = 0.15;
    // ... and for a SPARSE batch (fewer than 4 edges per id of the range: C4's 1/8 share has 2), where 36.5 % of the
    // edges still had a source outside C after seeding at 0.15 and went through the second level: 0.3 (round 5, one box,
    // interleaved: the share 1.875 -> 1.851 ms; 0.5: 1.936; a third level at 0.15: 1.849-1.853; profiles/r5n_*)
    double bucket_sample_sparse = 0.3;
    double bucket_hub_sample = 1.0;  // the first level's share of the hub's bucket (C = {h}: one slice)
    u64 pin_chunk = 1ull << 25;  // gcc_forest_fold_pinned: edges per H2D chunk (256 MiB)
    int bucket_defer = 1;        // N labelled by the fold's closing compress instead of a store per id (bucket_join_kernel)
    // a fresh forest's C deferred like N, the reset done by P1 (round 5) instead of bucket_init_kernel's 4 B per id
    // measured (profiles/r5c_ab_defer_c.txt, one box, interleaved): the reset's stores slow P1 by more than the launch
    // they save (C4's share P1 0.485 -> 0.564 ms for bucket_init's 0.07), so off
    // 2 (round 5): C deferred the same way, the reset a memset of parent[] on a second stream beside P1 and the seeding
    // (neither touches parent[]), joined before the first kernel that does
    int bucket_defer_c = 0;
    int bucket_slow2 = 1;        // second filter level over the slow edges with C | N (C4's 1/8 share: 19 % slow edges)
    int bucket_p1 = 1;           // P1 geometry (bucket_fold.h): 0 = 512 x 16, 1 = 1024 x 16 (C4: 4.43 -> 4.25 ms), 2 = 1024 x 12,
                                 // 3 = 1024 x 16 with 8-entry write-out lanes (16-B hi stores)
    // FINAL P2 entries per thread per round: 8 or 12 (fewer barriers per entry; C4: P2 3.73 -> 3.23 ms,
    // profiles/r3c_ab_p2_per.log)
    int bucket_p2_per = 12;
    int bucket_p2_vw = 4;      // FINAL P2's write-out: v-list entries per lane (4: 8-B + 4-B stores; 8: 16-B + 8-B)
    int bucket_chunk = 0;      // entries per chunk reservation in the bucketed fold's lists (0: by batch size)
    // diagnostics (tools/placement_probe.py): the next bucketed fold takes freshly allocated scratch (1: every list;
    // 2: the bucket storage only; 3: the v-lists only), the old buffers held a while so the new ones land elsewhere
    int scratch_realloc = 0;
    // the bucketed fold also for a later window of a forest tracking a giant (C4 in 8 windows: every window after the
    // first took the filtered fold over an 8 MiB global bitmap, 2.2 ms per 2^27 edges; round 4)
    int bucket_windows = 1;
    int bucket_items = 4;  // P2 work items per CU (each loads its slice's bitmap into LDS)
    int bucket_items_p3 = 2;  // FINAL / second-level P3 work items per CU
    // tests only: the fail_absorb-th next gcc_forest_absorb_many call fails with GCC_E_INTERNAL before it launches
    // anything (0: never) — a rank's absorb failing inside the cross-GPU group merge (tests/test_gpu_group.py)
    int fail_absorb = 0;
    // the full compress's finds: read-only (0, round 5) or splitting paths in the old buffer (1, rounds 1-4; A/B only —
    // compress_bits_kernel says why not)
    int compress_split = 0;
    int fold_split = 1;  // the plain (non-recording) fold's finds split paths (1) or are read-only (0)
    // the pipelined emission (round 5, compress_pipe_kernel): the incremental regime's scan of window w runs on a second
    // stream beside window w+1's fold (2: that stream at the device's highest priority, set when it is created).
    // Measured slower, so off (profiles/r5j_ab_inc_pipe.txt, interleaved on one box: C5 8.02 -> 12.5 ms, C3/w1M 1.59 ->
    // 2.7 ms): the recording fold with the touched marks, the resolve and the scan sharing the CUs with the next fold
    // cost more than the overlap returns
    int inc_pipe = 0;
    // Lazy emission (round 6, VERDICT r5 next-4: short windows). gcc_forest_compress is the per-window emission
    // (Merger.flatMap emits the running summary, …/SummaryAggregation.java:107-111). The emitted summary is the forest
    // itself, as in the reference (DisjointSet.getMatches exposes the parent map and find compresses lazily,
    // …/summaries/DisjointSet.java:49-51, :71-85): every root is its component's minimum id, so find(v) is exact on it.
    // In the plain regime (no tracked giant: C3, C5) the emission compresses only once the edges folded since the last
    // compress reach id_capacity / emit_div (and whenever a read needs the labels: labels, find, size, digest,
    // serialize, a merge message), so a window pays its fold plus an amortised O(1) per edge for the O(id_capacity)
    // compress, not an O(id_capacity) scan per window. 0 = every emission compresses (rounds 1-5).
    // Measured on C5 (256 windows of 2^16 edges; profiles/r6c_*, every window's emitted forest bit-exact): a compress
    // every 4 / 8 / 16 / 32 windows: 3.70 / 4.22 / 4.55 / 4.78 G edges/s (recording folds + incremental compress), 4.55 /
    // 5.25 G at 16 / 32 with splitting folds + full compress, against 2.08 eager. The giant-filtered regime (C2) keeps
    // the eager emission: its compress refreshes the filter's bitmap (lazy there measured slower: C2 x 16 at 4 / 8
    // windows 0.296 / 0.417 ms against 0.259).
    int emit_div = 1;
    // the plain folds between lazy emissions: record their mutations for an incremental compress (1) or split paths
    // and leave the compress that follows full (0: measured faster at C5's 32 windows per compress)
    int emit_rec = 0;
    // the giant-filtered regime's lazy emission (A/B, round 6): the emission refreshes only the tracked component's
    // bitmap (compress_bits_kernel without labels: 4 B per id read instead of 4 read + 4 written), and the labels
    // wait for a read (1); or it compresses (0)
    int emit_filtered = 0;
};
constexpr u32 kFilterMinIds = 1u << 16;  // forests over fewer ids never use the filter

struct gcc_forest {
    int device = 0;
    u32 cap = 0;
    // two id-range buffers: d_parent (the working forest) and d_spare; compress writes the canonical labels
    // into d_spare and the two swap roles, so after a compress d_parent IS the label array
    u32* d_parent = nullptr;
    u32* d_spare = nullptr;
    bool own_bufs = true;
    bool compressed = false;  // d_parent holds canonical labels (no mutation since the last compress)
    // reset() is lazy: the next fold of a fresh forest writes parent[] itself (seed_init_kernel); any other
    // use materialises the all-UNSEEN forest first (materialize_reset)
    bool pending_reset = false;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    int n_cu = 256;

    // giant-component filter: bitmap of one component (valid forever: components only grow)
    u64* d_bits = nullptr;
    u32* d_giant = nullptr;  // [0], [1]: tracked-component root slots; [4], [5]: the vote's share (giant_vote_kernel)
    bool filter_off = false;  // the vote found no giant: this forest folds without the filter until reset
    bool has_giant = false;
    // a compress (not a fold's sample) elected the tracked component: its share was not checked yet (round 6: a short
    // first window, e.g. C5's 2^15-edge chunks at N = 2, went straight to the filtered regime over a component of a few
    // ids, and the filtered fold keeps no delta lists). launch_fold reads the share once and decides filter_off
    bool share_unchecked = false;
    // the sampled start's vote-share check read back without a host sync (FoldTune::share_async): the share lands in
    // h_share behind share_ev, the batch's rest and later batches fold plain until a fold finds the event complete
    bool share_pending = false;
    hipEvent_t share_ev = nullptr;
    u32* h_share = nullptr;
    int giant_slot = 0;  // d_giant[giant_slot] = root of the tracked component as of the last refresh
    u32* d_qcount = nullptr;  // per-block slow-edge counts of the last filtered launch (measurement)
    // fused seeding: dedicated flag bytes (one per id, rounded up to a bitmap word), marked with an epoch
    // 1..255 so they need clearing once per 255 seedings
    u8* d_flags = nullptr;
    u32 flag_epoch = 0;  // the last epoch written into d_flags (0: needs clearing)
    u32* d_bmin = nullptr;  // seeding: per-block minima of the BFS passes (seed_pack_kernel<true> reduces them)
    // incremental compress: two bloom buffers of gcc::kBloomBits bits. The folds record into d_bloom[bloom_cur];
    // every compress clears the other one and flips. rec_all: every mutation since the last compress was recorded
    u32* d_bloom = nullptr;
    int bloom_cur = 0;
    bool rec_all = false;
    u32* bloom(int i) const { return d_bloom + (size_t)i * (gcc::kBloomBits / 32); }
    u32* d_dbg = nullptr;  // tune inc_check: 64 words (compress_inc_kernel<.., true>, inc_verify_kernel)
    u32* h_dbg = nullptr;
    u64 inc_checks = 0, inc_bad_labels = 0, inc_lost_marks = 0;
    u32* d_post = nullptr;  // tune post_check: inc_post_check_kernel's counters and records (64 words)
    u32* d_prev = nullptr;  // post_check 2: the labels after the previous checked compress
    u32 post_checks = 0;

    // pinned double-buffered staging for host-fed edges (per-edge foldEdges appends here)
    static constexpr u64 kStageEdges = 1ull << 20;  // 8 MiB per slot
    u32* h_stage[2] = {nullptr, nullptr};
    u32* d_stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int slot = 0;
    u64 staged = 0;

    // scratch for cross-device merges
    u32* d_scratch = nullptr;
    u32* d_witness = nullptr;  // absorb_many: per-peer id shared with the tracked component
    u64* d_msg_oth = nullptr;  // encode scratch (gcc_forest_encode): per word, the seen ids outside the tracked component
    u64 version = 0;      // bumped by every mutation of parent[] (with host_valid = false)
    u64 enc_version = ~0ull;  // `version` when d_msg_oth was written: equal = the masks still describe parent[]
    u64 mask_version = ~0ull;  // `version` when a compress last wrote the others' masks into d_msg_oth
    bool deferred_n = false;   // the bucketed fold left N in d_nbits for its closing compress
    bool witness_armed = false;  // the last encode already reset d_witness (stream-ordered before the next absorb)

    unsigned long long* d_counts = nullptr;

    // the pipelined emission (compress_pipe_kernel's comment). While `pipe` is on, d_spare holds the labels of the last
    // compressed window (L) and d_parent the live forest; fold + resolve run on `stream`, the scans on pipe_stream.
    bool pipe = false;
    bool pipe_dirty = false;         // folds since the last pipelined compress
    bool pipe_roots_stale = true;    // d_proots may hold roots from before the last reset
    u64 pipe_w = 0;                  // windows compressed since the mode started
    hipStream_t pipe_stream = nullptr;
    hipEvent_t pipe_ev_fold = nullptr, pipe_ev_scan[2] = {nullptr, nullptr};
    u32* d_pbloom = nullptr;   // 3 bloom buffers (a ring)
    u64* d_touched = nullptr;  // per 32 ids: hooked bits | new bits << 32 (zero outside a window)
    u32* d_pborn = nullptr;    // 2 parities x nw32 words: the window's new ids (zeroed by its scan)
    u32* d_proots = nullptr;   // 2 parities x cap: roots of the window's touched ids
    u32 nw32() const { return (u32)(((u64)cap + 31) / 32); }
    u32* pbloom(u64 i) const { return d_pbloom + (size_t)(i % 3) * (gcc::kBloomBits / 32); }

    // device-side id validation of raw device batches (edge_ok): set by a kernel, reported and cleared by the next
    // synchronising call (stream_sync_checked)
    u32* d_err = nullptr;
    u32* h_err = nullptr;  // pinned copy

    // gcc_forest_fold_pinned: chunks of a pinned host batch go H2D on copy_stream into two device slots while
    // the previous chunk folds on `stream`
    hipStream_t copy_stream = nullptr;
    hipStream_t aux_stream = nullptr;  // tune bucket_defer_c = 2: the fresh forest's reset beside P1
    hipEvent_t aux_ev[2] = {nullptr, nullptr};
    u32* d_pin[2] = {nullptr, nullptr};
    u64 pin_cap = 0;  // edges per slot
    hipEvent_t pin_copied[2] = {nullptr, nullptr}, pin_folded[2] = {nullptr, nullptr};

    // bucketed fold (bucket_fold.h): metadata, bucket storage, overflow list, v-lists (grown on demand)
    bk::Meta* d_meta = nullptr;
    std::vector<void*> held_scratch;  // FoldTune::scratch_realloc: earlier scratch buffers, freed two generations on
    uint8_t* d_bk = nullptr;  // bucket storage: bk::bk_bytes(S) bytes = S 6-B entries (lo array, then hi array)
    u64 bk_cap_bytes = 0;
    u64* d_ovf = nullptr;
    u64 ovf_cap = 0;
    uint8_t* d_vl = nullptr;  // v-lists: bk::vl_bytes(S) bytes = S 3-B entries (lo array, then hi array)
    u64 vl_cap = 0;           // bytes
    u64* d_slow = nullptr;  // FINAL P2's slow edges, one region per block
    u64 slow_cap_total = 0;
    u32* d_nbits = nullptr;  // N: ids reached from C by the FINAL pass (kept all-zero between batches)
    bk::SlowSeg* d_seg = nullptr;  // FINAL P2's slow-list runs (the second filter level's items)
    u64 seg_cap = 0;

    // lazy host view of the labels (getMatches()/find() consumers)
    std::vector<u32> host_labels;
    bool host_valid = false;

    int timing = 0;  // 1: every pipeline kernel timed by its own dispatch (start/stop events); 2: + slow-edge counts
    // timing mode: per-kernel log (name, event pair index or -1 for a fold's "begin" marker, edges processed)
    struct KLog {
        const char* name;
        int ev;
        u64 edges;
    };
    std::vector<std::pair<hipEvent_t, hipEvent_t>> kev;  // event-pair pool, reused after each drain
    size_t kev_used = 0;
    std::vector<KLog> klog;
    int last_fold_first = -1, last_fold_last = -1;  // event pairs spanning the last timed fold
    u32* h_segcount = nullptr;  // pinned copies of the slow-queue segment counts, one row per filtered round
    std::vector<u32> slow_rounds;

    // the delta merge (round 6): while armed (gcc_forest_delta_arm, after a group merge), every plain fold
    // also lists the ids it changes (fold_kernel<.., DELTA>) in kDeltaStripes stripes of delta_subcap ids; any other
    // mutation disarms it. delta_need: the per-stripe worst case of the folds since arming (the lists are grown before a
    // fold that could overflow them); delta_edges: the edges folded since arming (the message header's)
    bool delta_armed = false;
    bool delta_cnt_zero = false;  // the stripe counters are known to be zero (memset, or zeroed by the delta absorb)
    u32* d_delta = nullptr;
    u32* d_delta_cnt = nullptr;  // kDeltaStripes counters + the lane-overflow flag
    u32 delta_subcap = 0;
    u64 delta_need = 0;
    u64 delta_edges = 0;

    FoldTune tune;
    u64 edges_since_compress = 0;  // lazy emission (FoldTune::emit_div)

    u32 nwords() const { return (u32)(((u64)cap + 63) / 64); }
    bool filter_enabled() const { return tune.filter && cap >= kFilterMinIds; }
};

int gcc_check_device(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return set_err(GCC_E_NODEV, "no HIP device visible (%s)", hipGetErrorString(e));
    if (device < 0 || device >= n) return set_err(GCC_E_INVALID, "device %d out of range (have %d)", device, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(GCC_E_NODEV, "device %d is %s, this library is built for gfx950 only", device, prop.gcnArchName);
    return GCC_OK;
}

// recorded: the mutation was recorded in the bloom (or cleared rec_all itself); anything else rules out an
// incremental compress until the next full one
static void mark_mutated(gcc_forest* h, bool recorded = false) {
    h->host_valid = false;
    ++h->version;
    h->compressed = false;
    if (!recorded) {
        h->delta_armed = false;  // a mutation the delta lists did not see
        h->rec_all = false;
        h->pipe_roots_stale = true;  // conservatively: the pipelined emission's roots arrays start from UNSEEN again
    }
}

// Every kernel of the fold pipeline goes through launch_k. Timing mode launches it with hipExtLaunchKernelGGL's
// start/stop events, which the runtime records from the dispatch itself: the logged duration is the kernel's
// own execution, and no extra packets (hipEventRecord markers cost ~4 us each between dependent kernels) are
// put between the pipeline's launches.
// GELLY_BUCKET_STATS=1 (diagnostics): after each bucketed fold, print its lists' fill to stderr (synchronises).
static bool bucket_stats() {
    static const bool on = [] {
        const char* e = std::getenv("GELLY_BUCKET_STATS");
        return e && *e && *e != '0';
    }();
    return on;
}

// GELLY_BUCKET_ADDR=1 (diagnostics): every bucketed fold prints its buffers' device addresses (no synchronisation):
// P1's time varies by up to 25 % between forests of one process (profiles/r4o_*), i.e. with where its buffers lie.
static bool bucket_addr() {
    static const bool on = [] {
        const char* e = std::getenv("GELLY_BUCKET_ADDR");
        return e && *e && *e != '0';
    }();
    return on;
}

// GELLY_SYNC_EACH=1 (diagnostics): synchronise after every launch, so that an asynchronous fault names its kernel.
static bool sync_each_launch() {
    static const bool on = [] {
        const char* e = std::getenv("GELLY_SYNC_EACH");
        return e && *e && *e != '0';
    }();
    return on;
}

// GELLY_SYNC_EACH for the merge-message kernels (launched directly, not through launch_k)
static int msg_launched(gcc_forest* h, const char* name) {
    HIP_TRY(hipGetLastError());
    if (sync_each_launch()) {
        const hipError_t e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return set_err(GCC_E_HIP, "kernel %s: %s", name, hipGetErrorString(e));
    }
    return GCC_OK;
}

template <typename F, typename... Args>
static int launch_ks(gcc_forest* h, hipStream_t st, const char* name, u64 edges, F kernel, dim3 grid, dim3 block,
                     size_t shmem, Args... args) {
    if (!h->timing) {
        hipLaunchKernelGGL(kernel, grid, block, (unsigned)shmem, st, args...);
    } else {
        if (h->klog.size() > 16384) {  // nobody drains the log: keep it bounded
            h->klog.clear();
            h->kev_used = 0;
            h->last_fold_first = h->last_fold_last = -1;
        }
        if (h->kev_used == h->kev.size()) {
            hipEvent_t a, b;
            HIP_TRY(hipEventCreate(&a));
            HIP_TRY(hipEventCreate(&b));
            h->kev.push_back({a, b});
        }
        const int ev = (int)h->kev_used++;
        hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)shmem, st, h->kev[ev].first, h->kev[ev].second, 0,
                              args...);
        h->klog.push_back({name, ev, edges});
    }
    HIP_TRY(hipGetLastError());
    if (sync_each_launch()) {  // diagnostics: a fault is reported by the launch that caused it
        const hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) return set_err(GCC_E_HIP, "kernel %s: %s", name, hipGetErrorString(e));
    }
    return GCC_OK;
}

template <typename F, typename... Args>
static int launch_k(gcc_forest* h, const char* name, u64 edges, F kernel, dim3 grid, dim3 block, size_t shmem,
                    Args... args) {
    return launch_ks(h, h->stream, name, edges, kernel, grid, block, shmem, args...);
}

// Synchronise the handle's stream and report an id-range error that a kernel recorded since the last check
// (edge_ok: those edges were skipped, the batch's other edges folded). Every synchronising entry point uses it.
static int stream_sync_checked(gcc_forest* h) {
    HIP_TRY(hipMemcpyAsync(h->h_err, h->d_err, sizeof(u32), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (*h->h_err) {
        const u32 e = *h->h_err;
        *h->h_err = 0;
        HIP_TRY(hipMemsetAsync(h->d_err, 0, sizeof(u32), h->stream));
        if (e & ~1u)  // bucket_fold.h's internal checks (kErr*): an entry of an internal list was out of range
            return set_err(GCC_E_INTERNAL, "bucketed fold consistency check failed (flags 0x%x: %s%s%s%s)", e,
                           (e & bk::kErrP2) ? "P2 bucket entry " : "", "",
                           (e & bk::kErrSlow) ? "slow-list entry " : "", (e & bk::kErrOvf) ? "overflow entry" : "");
        return set_err(GCC_E_INVALID, "a device batch or label array held an id >= id_capacity %u (those entries were skipped)",
                       h->cap);
    }
    return GCC_OK;
}

static int materialize_reset(gcc_forest* h) {
    if (!h->pending_reset) return GCC_OK;
    h->rec_all = false;
    h->delta_armed = false;
    HIP_TRY(hipMemsetAsync(h->d_parent, 0xFF, (size_t)h->cap * sizeof(u32), h->stream));
    h->pending_reset = false;
    return GCC_OK;
}

static int alloc_filter(gcc_forest* h) {
    if (h->d_bits) return GCC_OK;
    HIP_TRY(hipMalloc((void**)&h->d_bits, (size_t)h->nwords() * sizeof(u64) + 16));
    HIP_TRY(hipMalloc((void**)&h->d_giant, 6 * sizeof(u32)));
    return GCC_OK;
}

// incremental compresses are only worth their recording for big forests (the full compress of a few MiB is a
// launch floor anyway); they also need 16-B aligned id-range buffers (the inc kernel's vector loads)
static bool inc_forest(const gcc_forest* h) {
    return h->tune.incremental && h->filter_enabled() && (u64)h->cap >= h->tune.inc_min_ids &&
           ((reinterpret_cast<uintptr_t>(h->d_parent) | reinterpret_cast<uintptr_t>(h->d_spare)) & 15) == 0;
}

// tune inc_check (diagnostics): zero the debug words and, for the in-place compress, keep a copy of the forest it
// starts from in d_spare (free: an in-place compress does not swap)
static int inc_check_begin(gcc_forest* h, bool inplace) {
    if (!h->d_dbg) {
        HIP_TRY(hipMalloc((void**)&h->d_dbg, 64 * sizeof(u32)));
        HIP_TRY(hipHostMalloc((void**)&h->h_dbg, 64 * sizeof(u32), hipHostMallocDefault));
    }
    HIP_TRY(hipMemsetAsync(h->d_dbg, 0, 64 * sizeof(u32), h->stream));
    if (inplace) HIP_TRY(hipMemcpyAsync(h->d_spare, h->d_parent, (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToDevice,
                                        h->stream));
    return GCC_OK;
}

static int inc_check_end(gcc_forest* h, const u32* pre, const u32* labels, const u32* bloom) {
    hipLaunchKernelGGL(inc_verify_kernel, dim3(kMaxGrid), dim3(kBlock), 0, h->stream, pre, labels, h->cap, bloom, h->d_dbg);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h->h_dbg, h->d_dbg, 64 * sizeof(u32), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const u32* d = h->h_dbg;
    ++h->inc_checks;
    h->inc_lost_marks += d[0];
    h->inc_bad_labels += d[2];
    if (d[0] || d[2]) {
        fprintf(stderr, "[inc_check] compress %llu: bloom fill %u bits; LDS words missing marks %u (extra %u); wrong labels %u\n",
                (unsigned long long)h->inc_checks, d[3], d[0], d[1], d[2]);
        for (u32 k = 0; k < std::min<u32>(d[0], 4); ++k)
            fprintf(stderr, "[inc_check]   block %u word %u: lds %08x memory %08x\n", d[16 + 4 * k], d[17 + 4 * k],
                    d[18 + 4 * k], d[19 + 4 * k]);
        for (u32 k = 0; k < std::min<u32>(d[2], 4); ++k) {
            const u32* o = d + 32 + 6 * k;
            fprintf(stderr, "[inc_check]   v %u: pre parent %u (marked in memory %u, its parent %u) label %u root %u\n", o[0],
                    o[1], o[4], o[5], o[2], o[3]);
        }
    }
    return GCC_OK;
}

// tune post_check (diagnostics): inc_post_check_kernel after the incremental compress, stream-ordered, no sync; with
// post_check 2 the labels are also copied into d_prev after the check (for the next check's records)
static int post_check_launch(gcc_forest* h, const u32* labels, const u32* bloom) {
    if (!h->d_post) {
        HIP_TRY(hipMalloc((void**)&h->d_post, 64 * sizeof(u32)));
        HIP_TRY(hipMemsetAsync(h->d_post, 0, 64 * sizeof(u32), h->stream));
    }
    const bool keep = h->tune.post_check >= 2;
    if (keep && !h->d_prev) {
        HIP_TRY(hipMalloc((void**)&h->d_prev, (size_t)h->cap * sizeof(u32)));
        HIP_TRY(hipMemsetAsync(h->d_prev, 0xFF, (size_t)h->cap * sizeof(u32), h->stream));
    }
    hipLaunchKernelGGL(inc_post_check_kernel, dim3(kMaxGrid), dim3(kBlock), 0, h->stream, labels, h->cap, bloom,
                       (const u32*)(keep ? h->d_prev : nullptr), h->post_checks++, h->d_post);
    HIP_TRY(hipGetLastError());
    if (keep)
        HIP_TRY(hipMemcpyAsync(h->d_prev, labels, (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToDevice, h->stream));
    return GCC_OK;
}

// compress into the spare buffer and swap; with the filter on, refresh the giant bitmap from the new labels.
// Incremental (compress_inc_kernel) when every mutation since the last compress was recorded.
// oth (the merge encode): a full compress also writes the others mask of every 64-id word (chunk_oth); returns
// whether it did (only the full compress of a filtered forest can).
// newbits (gcc_forest_absorb_many): ids still UNSEEN that belong to the tracked component (a full compress of a
// filtered forest; the caller checks).
// ---- the pipelined emission's host side (compress_pipe_kernel's comment) ------------------------------------------
// Entered by a recording fold of a compressed forest (pipe_fold); every entry point that reads the labels waits for
// the last scan (pipe_labels_ready) and reads d_spare (labels_ptr); every other entry point leaves the mode first
// (pipe_exit, from flush()).
static u32* labels_ptr(const gcc_forest* h) { return h->pipe ? h->d_spare : h->d_parent; }

static int pipe_labels_ready(gcc_forest* h) {  // the handle's stream waits for the last scan
    if (h->pipe && h->pipe_w > 0) HIP_TRY(hipStreamWaitEvent(h->stream, h->pipe_ev_scan[(h->pipe_w - 1) & 1], 0));
    return GCC_OK;
}

// Leave the mode: the handle's stream waits for the last scan. With no fold since it, L is canonical and becomes
// d_parent (compressed, the normal bloom untouched and clear since the mode started: rec_all stays). With folds since
// it, d_parent (the live forest) stays, its pending window's touched marks are dropped, and the next compress is full.
static int pipe_exit(gcc_forest* h) {
    if (!h->pipe) return GCC_OK;
    int rc = pipe_labels_ready(h);
    if (rc) return rc;
    if (h->pipe_dirty) {
        HIP_TRY(hipMemsetAsync(h->d_touched, 0, (size_t)h->nw32() * sizeof(u64), h->stream));
        h->compressed = false;
        h->rec_all = false;
    } else {
        std::swap(h->d_parent, h->d_spare);
        h->compressed = true;
    }
    h->pipe = false;
    h->pipe_dirty = false;
    h->host_valid = false;
    return GCC_OK;
}

static int pipe_enter(gcc_forest* h) {
    const size_t bl = gcc::kBloomBits / 8;
    if (!h->pipe_stream) {
        int lo = 0, hi = 0;  // the scan first: the window's fold waits for it two windows later anyway
        HIP_TRY(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIP_TRY(hipStreamCreateWithPriority(&h->pipe_stream, hipStreamNonBlocking, h->tune.inc_pipe >= 2 ? hi : lo));
        HIP_TRY(hipEventCreateWithFlags(&h->pipe_ev_fold, hipEventDisableTiming));
        for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&h->pipe_ev_scan[i], hipEventDisableTiming));
        HIP_TRY(hipMalloc((void**)&h->d_pbloom, 3 * bl));
        HIP_TRY(hipMalloc((void**)&h->d_touched, (size_t)h->nw32() * sizeof(u64)));
        HIP_TRY(hipMalloc((void**)&h->d_pborn, 2 * (size_t)h->nw32() * sizeof(u32)));
        HIP_TRY(hipMalloc((void**)&h->d_proots, 2 * (size_t)h->cap * sizeof(u32)));
        HIP_TRY(hipMemsetAsync(h->d_touched, 0, (size_t)h->nw32() * sizeof(u64), h->stream));
        HIP_TRY(hipMemsetAsync(h->d_pborn, 0, 2 * (size_t)h->nw32() * sizeof(u32), h->stream));
        h->pipe_roots_stale = true;
    }
    // the labels stay where the last compress wrote them (d_parent) and become L; the forest goes on in a copy in the
    // other buffer. Not the other way round: the other buffer held the forest two kernels ago, and a plain (path
    // splitting) store of that fold landing late would overwrite a label (the late-store model); over the
    // forest's copy it only writes an ancestor (tests/cpp/test_uf_replay.cpp, pipeline "pipe")
    HIP_TRY(hipMemcpyAsync(h->d_spare, h->d_parent, (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToDevice, h->stream));
    std::swap(h->d_parent, h->d_spare);
    if (h->pipe_roots_stale) {
        HIP_TRY(hipMemsetAsync(h->d_proots, 0xFF, 2 * (size_t)h->cap * sizeof(u32), h->stream));
        h->pipe_roots_stale = false;
    }
    HIP_TRY(hipMemsetAsync(h->d_pbloom, 0, 3 * bl, h->stream));
    h->pipe = true;
    h->pipe_w = 0;
    h->pipe_dirty = false;
    return GCC_OK;
}

// The eligibility of a recording fold for the mode: entered only from a compressed forest (d_parent = the labels)
static bool pipe_applies(const gcc_forest* h) {
    return h->tune.inc_pipe && !h->tune.inc_check && !h->tune.post_check && h->has_giant && h->d_bits &&
           (h->pipe || h->compressed);
}

static int pipe_fold(gcc_forest* h, const u64* edges, u64 n) {
    int rc = GCC_OK;
    if (!h->pipe) rc = pipe_enter(h);
    if (rc) return rc;
    // the window's first fold: scan w-2 must be done (this fold's bloom, and resolve's roots / born buffers)
    if (!h->pipe_dirty && h->pipe_w >= 2) HIP_TRY(hipStreamWaitEvent(h->stream, h->pipe_ev_scan[h->pipe_w & 1], 0));
    rc = launch_k(h, "plain_pipe", n, fold_pipe_kernel, dim3(grid_for(n, kMaxGrid)), dim3(kBlock), 0, h->d_parent, edges, n,
                  h->pbloom(h->pipe_w), reinterpret_cast<u32*>(h->d_touched), h->cap, h->d_err);
    if (rc) return rc;
    h->pipe_dirty = true;
    return GCC_OK;
}

static int pipe_compress(gcc_forest* h) {
    if (!h->pipe_dirty) return GCC_OK;
    const u64 w = h->pipe_w;
    const int par = (int)(w & 1);
    u32* roots = h->d_proots + (size_t)par * h->cap;
    u32* born = h->d_pborn + (size_t)par * h->nw32();
    const u32* gp = h->d_giant + h->giant_slot;
    u32* gn = h->d_giant + (h->giant_slot ^ 1);
    int rc = launch_k(h, "resolve", 0, pipe_resolve_kernel, dim3(grid_for(h->nw32(), kMaxGrid)), dim3(kBlock), 0,
                      (const u32*)h->d_parent, h->d_touched, h->nw32(), roots, born, gp, gn);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(h->pipe_ev_fold, h->stream));
    HIP_TRY(hipStreamWaitEvent(h->pipe_stream, h->pipe_ev_fold, 0));
    rc = launch_ks(h, h->pipe_stream, "compress_pipe", 0, compress_pipe_kernel, dim3(h->n_cu), dim3(kIncBlock),
                   gcc::kBloomBits / 8, h->d_spare, h->d_parent, h->cap, (const u32*)h->pbloom(w), h->pbloom(w + 2), born,
                   (const u32*)roots, (const u32*)gn, h->d_bits);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(h->pipe_ev_scan[par], h->pipe_stream));
    h->giant_slot ^= 1;
    h->pipe_w = w + 1;
    h->pipe_dirty = false;
    h->host_valid = false;
    return GCC_OK;
}

static int compress_now(gcc_forest* h, const char* name = "compress", u64* oth = nullptr, bool* oth_done = nullptr,
                        const u64* newbits = nullptr) {
    int rc = pipe_exit(h);
    if (rc) return rc;
    bool inplace = false;  // the compress rewrote d_parent itself (no swap)
    const bool inc_here = inc_forest(h) && !oth && !newbits;  // masks in or out: a full compress
    if (!h->filter_enabled()) {
        rc = h->tune.compress_split
                 ? launch_k(h, name, 0, compress_bits_kernel<true>, dim3(chunk_grid(h->cap, kBitsU, kBlock, kMaxGrid)),
                            dim3(kBlock), 0, h->d_parent, h->d_spare, h->cap, (const u32*)nullptr, (u32*)nullptr,
                            (u64*)nullptr, (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr)
                 : launch_k(h, name, 0, compress_bits_kernel<false>, dim3(chunk_grid(h->cap, kBitsU, kBlock, kMaxGrid)),
                            dim3(kBlock), 0, h->d_parent, h->d_spare, h->cap, (const u32*)nullptr, (u32*)nullptr,
                            (u64*)nullptr, (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr);
    } else {
        rc = alloc_filter(h);
        if (rc) return rc;
        if (inc_here && !h->d_bloom) {
            HIP_TRY(hipMalloc((void**)&h->d_bloom, 2 * (size_t)(gcc::kBloomBits / 8)));
            HIP_TRY(hipMemsetAsync(h->d_bloom, 0, 2 * (size_t)(gcc::kBloomBits / 8), h->stream));
            h->rec_all = false;
        }
        if (!h->has_giant) {  // first refresh of this forest: elect the component to track
            rc = launch_k(h, "vote", 0, giant_vote_kernel, dim3(1), dim3(1024), 0, h->d_parent, h->cap,
                          h->d_giant + h->giant_slot, h->d_giant + 4);
            h->share_unchecked = true;  // the next fold checks the vote's share (launch_fold)
        }
        u32* clear = h->d_bloom ? h->bloom(h->bloom_cur ^ 1) : nullptr;
        if (!rc && inc_here && h->rec_all) {
            const char* kname = std::strcmp(name, "refresh") ? "compress_inc" : "refresh_inc";
            inplace = h->tune.inc_inplace;
            const bool check = h->tune.inc_check;
            if (check) rc = inc_check_begin(h, inplace);
            const u32* bl = h->bloom(h->bloom_cur);
            const u32* gp = h->d_giant + h->giant_slot;
            u32* gn = h->d_giant + (h->giant_slot ^ 1);
            u32* out = inplace ? h->d_parent : h->d_spare;
            if (!rc) {
                if (inplace && check)
                    rc = launch_k(h, kname, 0, compress_inc_kernel<true, true>, dim3(h->n_cu), dim3(kIncBlock),
                                  gcc::kBloomBits / 8, (const u32*)h->d_parent, out, h->cap, bl, clear, gp, gn, h->d_bits,
                                  h->d_dbg);
                else if (inplace)
                    rc = launch_k(h, kname, 0, compress_inc_kernel<true, false>, dim3(h->n_cu), dim3(kIncBlock),
                                  gcc::kBloomBits / 8, (const u32*)h->d_parent, out, h->cap, bl, clear, gp, gn, h->d_bits,
                                  (u32*)nullptr);
                else if (check)
                    rc = launch_k(h, kname, 0, compress_inc_kernel<false, true>, dim3(h->n_cu), dim3(kIncBlock),
                                  gcc::kBloomBits / 8, (const u32*)h->d_parent, out, h->cap, bl, clear, gp, gn, h->d_bits,
                                  h->d_dbg);
                else
                    rc = launch_k(h, kname, 0, compress_inc_kernel<false, false>, dim3(h->n_cu), dim3(kIncBlock),
                                  gcc::kBloomBits / 8, (const u32*)h->d_parent, out, h->cap, bl, clear, gp, gn, h->d_bits,
                                  (u32*)nullptr);
            }
            // the forest the compress started from: the copy in d_spare (in place), or d_parent itself
            if (!rc && check) rc = inc_check_end(h, inplace ? h->d_spare : h->d_parent, out, bl);
            if (!rc && h->tune.post_check) rc = post_check_launch(h, out, bl);
        } else if (!rc) {
            rc = h->tune.compress_split
                     ? launch_k(h, name, 0, compress_bits_kernel<true>, dim3(chunk_grid(h->cap, kBitsU, kBlock, kMaxGrid)),
                                dim3(kBlock), 0, h->d_parent, h->d_spare, h->cap, (const u32*)(h->d_giant + h->giant_slot),
                                h->d_giant + (h->giant_slot ^ 1), h->d_bits, clear, oth, newbits)
                     : launch_k(h, name, 0, compress_bits_kernel<false>, dim3(chunk_grid(h->cap, kBitsU, kBlock, kMaxGrid)),
                                dim3(kBlock), 0, h->d_parent, h->d_spare, h->cap, (const u32*)(h->d_giant + h->giant_slot),
                                h->d_giant + (h->giant_slot ^ 1), h->d_bits, clear, oth, newbits);
            if (oth_done) *oth_done = oth != nullptr;
        }
        h->giant_slot ^= 1;
        h->has_giant = true;
        h->bloom_cur ^= 1;
    }
    if (rc) return rc;
    if (!inplace) std::swap(h->d_parent, h->d_spare);
    h->compressed = true;
    h->rec_all = inc_here && h->d_bloom;  // parent[] is compressed and the next fold's bloom is clear
    h->edges_since_compress = 0;
    return GCC_OK;
}

// Mid-fold refresh of the tracked component's bitmap (and its root) without a compress: the filter only needs
// the bitmap, and writing 4 B of labels per id (then swapping buffers) doubles the pass's traffic. Path
// splitting in the finds still shortens the forest. tune.refresh_labels = 1: a full compress instead.
static int refresh_now(gcc_forest* h) {
    if (h->tune.refresh_labels || !h->filter_enabled()) return compress_now(h, "refresh");
    int rc = pipe_exit(h);
    if (!rc) rc = alloc_filter(h);
    if (rc) return rc;
    if (!h->has_giant) {
        rc = launch_k(h, "vote", 0, giant_vote_kernel, dim3(1), dim3(1024), 0, h->d_parent, h->cap,
                      h->d_giant + h->giant_slot, h->d_giant + 4);
        h->share_unchecked = true;
    }
    if (!rc)
        rc = launch_k(h, "refresh_bits", 0, compress_bits_kernel<true>, dim3(chunk_grid(h->cap, kBitsU, kBlock, kMaxGrid)),
                      dim3(kBlock), 0, h->d_parent, (u32*)nullptr, h->cap, (const u32*)(h->d_giant + h->giant_slot),
                      h->d_giant + (h->giant_slot ^ 1), h->d_bits, (u32*)nullptr, (u64*)nullptr, (const u64*)nullptr);
    if (rc) return rc;
    h->giant_slot ^= 1;
    h->has_giant = true;
    return GCC_OK;
}

// The delta lists must hold the worst case of this fold on top of what they hold (a wave appends at most
// kLaneEvents ids per lane per iteration into its stripe): grown here, before the launch, if they could overflow.
static int delta_reserve(gcc_forest* h, u64 n, u32 grid) {
    const u64 waves = (u64)grid * (kBlock / 64);
    const u64 iters = (n + (u64)grid * kBlock - 1) / ((u64)grid * kBlock);
    const u64 need = h->delta_need + (waves + kDeltaStripes - 1) / kDeltaStripes * iters * 64 * gcc::kLaneEvents;
    if (need > (1ull << 26)) {  // past 4G ids of lists: this window takes the compact message
        h->delta_armed = false;
        return GCC_OK;
    }
    if (need > h->delta_subcap) {
        const u64 nc = std::max<u64>({need, 2ull * h->delta_subcap, 1024});
        u32* nb = nullptr;
        HIP_TRY(hipMalloc((void**)&nb, (size_t)kDeltaStripes * nc * sizeof(u32)));
        if (h->d_delta) {
            if (h->delta_need)
                HIP_TRY(hipMemcpy2DAsync(nb, nc * sizeof(u32), h->d_delta, (size_t)h->delta_subcap * sizeof(u32),
                                         (size_t)h->delta_subcap * sizeof(u32), kDeltaStripes, hipMemcpyDeviceToDevice,
                                         h->stream));
            HIP_TRY(hipStreamSynchronize(h->stream));  // (growth only: the old lists may still be read)
            HIP_TRY(hipFree(h->d_delta));
        }
        h->d_delta = nb;
        h->delta_subcap = (u32)nc;
    }
    h->delta_need = need;
    h->delta_edges += n;
    h->delta_cnt_zero = false;
    return GCC_OK;
}

static int launch_plain(gcc_forest* h, const u32* d_pairs, u64 n, const char* name) {
    if (n == 0) return GCC_OK;
    const u64* edges = reinterpret_cast<const u64*>(d_pairs);
    // the recording fold: every mutation since the last compress recorded, a short window of a big forest, and (lazy
    // emission with emit_rec = 0: the folds between compresses split paths instead) recording wanted
    const bool rec = h->rec_all && n * std::max<u64>(1, h->tune.inc_div) <= (u64)h->cap &&
                     (h->tune.emit_div <= 0 || h->tune.emit_rec);
    if (rec && pipe_applies(h)) {
        h->delta_armed = false;  // the pipelined fold keeps no delta lists
        return pipe_fold(h, edges, n);
    }
    int rc = pipe_exit(h);
    if (rc) return rc;
    const dim3 g(grid_for(n, kMaxGrid));
    if (h->delta_armed && (rc = delta_reserve(h, n, g.x))) return rc;
    const bool delta = h->delta_armed;
    const DeltaLists dl{h->d_delta, h->d_delta_cnt, h->delta_subcap};
    if (rec) {
        u32* bl = h->bloom(h->bloom_cur);
        const int v = (h->tune.inc_split ? 0 : 1) + 2 * std::max(0, std::min(2, h->tune.fold_release));
        if (delta && v == 1)
            return launch_k(h, name, n, fold_kernel<true, false, 0, true>, g, dim3(kBlock), 0, h->d_parent, edges, n, bl,
                            h->cap, h->d_err, dl);
        h->delta_armed = false;  // the A/B variants below keep no delta lists
#define GCC_REC(S, E) launch_k(h, name, n, fold_kernel<true, S, E>, g, dim3(kBlock), 0, h->d_parent, edges, n, bl, h->cap, h->d_err, DeltaLists{})
        switch (v) {
        case 0: return GCC_REC(true, 0);
        case 1: return GCC_REC(false, 0);
        case 2: return GCC_REC(true, 1);
        case 3: return GCC_REC(false, 1);
        case 4: return GCC_REC(true, 2);
        default: return GCC_REC(false, 2);
        }
#undef GCC_REC
    }
    h->rec_all = false;
    if (!h->tune.fold_split)  // read-only finds in the plain fold too (A/B, round 5: the compress measured faster so)
        return delta ? launch_k(h, name, n, fold_kernel<false, false, 0, true>, g, dim3(kBlock), 0, h->d_parent, edges, n,
                                (u32*)nullptr, h->cap, h->d_err, dl)
                     : launch_k(h, name, n, fold_kernel<false, false>, g, dim3(kBlock), 0, h->d_parent, edges, n,
                                (u32*)nullptr, h->cap, h->d_err, DeltaLists{});
    return delta ? launch_k(h, name, n, fold_kernel<false, true, 0, true>, g, dim3(kBlock), 0, h->d_parent, edges, n,
                            (u32*)nullptr, h->cap, h->d_err, dl)
                 : launch_k(h, name, n, fold_kernel<false>, g, dim3(kBlock), 0, h->d_parent, edges, n, (u32*)nullptr,
                            h->cap, h->d_err, DeltaLists{});
}

static int launch_filtered(gcc_forest* h, const u32* d_pairs, u64 n) {
    if (n == 0) return GCC_OK;
    if (int rc = pipe_exit(h)) return rc;
    h->rec_all = false;  // the filtered fold does not record its mutations
    h->delta_armed = false;  // nor list them for the delta merge
    const u32 nw = h->nwords() + (h->nwords() & 1);  // u64 bitmap words, rounded to 16 B
    const bool lds = nw <= kLdsBitmapMaxWords && (double)n >= h->tune.lds_edges_per_word * (double)nw;
    const u32 nblocks = lds ? (u32)h->n_cu : kMaxGrid;
    if (!h->d_qcount) HIP_TRY(hipMalloc((void**)&h->d_qcount, kMaxGrid * sizeof(u32)));
    const u64* edges = reinterpret_cast<const u64*>(d_pairs);
    const u32* bits = reinterpret_cast<const u32*>(h->d_bits);
    const u32* giant = h->d_giant + h->giant_slot;
    // instantiated variants: depth 4 with / without the direct hook, depth 8 without; software-pipelined stream
    // depth 8 with the hook carry exceeds 128 VGPRs (1024-thread blocks) and spills: it runs without the hook
    const int variant = h->tune.depth == 8 ? 1 : (h->tune.hook ? 2 : 0);
    int rc = GCC_OK;
    if (lds) {
        const size_t lds_bytes = (size_t)nw * sizeof(u64) + (kFilterBlockLds / 64) * kRing * sizeof(u64);
#define GCC_FILTERED(D, H)                                                                                     \
    launch_k(h, "filtered", n, fold_filtered_kernel<true, kFilterBlockLds, D, true, H>, dim3(nblocks),         \
             dim3(kFilterBlockLds), lds_bytes, h->d_parent, edges, n, bits, nw, giant, h->d_qcount, h->tune.drain_at,   \
             h->cap, h->d_err)
        switch (variant) {
        case 0: rc = GCC_FILTERED(4, false); break;
        case 1: rc = GCC_FILTERED(8, false); break;
        case 2: rc = GCC_FILTERED(4, true); break;
        default: rc = GCC_FILTERED(8, true); break;
        }
#undef GCC_FILTERED
    } else {
        const size_t lds_bytes = (kBlock / 64) * kRing * sizeof(u64);
#define GCC_FILTERED(D, H)                                                                                  \
    launch_k(h, "filtered", n, fold_filtered_kernel<false, kBlock, D, true, H>, dim3(nblocks), dim3(kBlock), \
             lds_bytes, h->d_parent, edges, n, bits, nw, giant, h->d_qcount, h->tune.drain_at, h->cap, h->d_err)
        switch (variant) {
        case 0: rc = GCC_FILTERED(4, false); break;
        case 1: rc = GCC_FILTERED(8, false); break;
        case 2: rc = GCC_FILTERED(4, true); break;
        default: rc = GCC_FILTERED(8, true); break;
        }
#undef GCC_FILTERED
    }
    if (rc) return rc;
    if (h->timing > 1) {  // measurement only (profile mode): how many edges took the slow path
        if (!h->h_segcount) HIP_TRY(hipHostMalloc((void**)&h->h_segcount, 8 * kMaxGrid * sizeof(u32), hipHostMallocDefault));
        if (h->slow_rounds.size() < 8) {
            const size_t row = h->slow_rounds.size();
            HIP_TRY(hipMemcpyAsync(h->h_segcount + row * kMaxGrid, h->d_qcount, nblocks * sizeof(u32),
                                   hipMemcpyDeviceToHost, h->stream));
            h->slow_rounds.push_back(nblocks);
        }
    }
    return GCC_OK;
}

// Seeded start of a fresh forest's first batch (seed_* kernels above): hub vote, BFS passes over the
// prefix, parent[] := C ? gmin : UNSEEN. Replaces the reset memset; leaves has_giant set, bitmap = C.
static int launch_seed(gcc_forest* h, const u32* d_pairs, u64 n) {
    if (int rc = pipe_exit(h)) return rc;
    const FoldTune& t = h->tune;
    h->rec_all = false;
    h->delta_armed = false;
    int rc = alloc_filter(h);
    if (rc) return rc;
    const u64* edges = reinterpret_cast<const u64*>(d_pairs);
    u32* bits = reinterpret_cast<u32*>(h->d_bits);
    const u32 nw32 = 2 * (h->nwords() + (h->nwords() & 1));  // u32 bitmap words, rounded to 16 B
    const bool lds = nw32 / 2 <= kLdsBitmapMaxWords;
    const bool fuse = t.seed_fuse && lds && t.seed_passes > 0;
    // per-block minimum slots: [0] the hub (seed_hub_kernel; unused when fused), then one per BFS block and pass
    if (!h->d_bmin) HIP_TRY(hipMalloc((void**)&h->d_bmin, (1 + 16 * (size_t)kMaxGrid) * sizeof(u32)));
    u32* gmin = h->d_bmin;
    u32 n_bmin = 1;
    u8* flags;
    u8 epoch = 1;
    if (fuse) {  // dedicated epoch-marked flags: nothing to clear
        const size_t flag_bytes = (size_t)nw32 * 32;  // one byte per id of every bitmap word
        if (!h->d_flags) {
            HIP_TRY(hipMalloc((void**)&h->d_flags, flag_bytes));
            h->flag_epoch = 0;
        }
        if (h->flag_epoch == 0 || h->flag_epoch == 255) {
            HIP_TRY(hipMemsetAsync(h->d_flags, 0, flag_bytes, h->stream));
            h->flag_epoch = 0;
        }
        epoch = (u8)++h->flag_epoch;
        flags = h->d_flags;
    } else {
        flags = reinterpret_cast<u8*>(h->d_spare);  // free until the next compress: one flag byte per id
        const unsigned hub_grid = (unsigned)std::max<u64>(1, std::min<u64>((u64)h->n_cu, (u64)h->cap >> 16));
        rc = launch_k(h, "seed_hub", 0, seed_hub_kernel, dim3(hub_grid), dim3(kHubBlock), 2 * kHubSlots * sizeof(u32),
                      edges, std::min(n, kHubSample), flags, bits, h->cap, gmin);
        if (rc) return rc;
    }
    // BFS prefixes hold at least 64 edges (the kernel's clamped loads need a non-empty body; n >= 64 here)
    const u64 pref = std::min(n, std::max<u64>({64, t.filter_min_batch, n / std::max<u64>(1, t.seed_div)}));
    // the first pass only has to reach the hubs next to h: a shorter prefix
    const u64 pref1 = std::min(pref, std::max<u64>({64, t.filter_min_batch, n / std::max<u64>(1, t.seed_div1)}));
    const unsigned pack_grid = grid_for(((u64)h->cap + 3) / 4, kMaxGrid);
    for (int p = 0; p < t.seed_passes; ++p) {
        const u64 np = p == 0 ? pref1 : pref;
        if (lds) {
            const bool hub = fuse && p == 0;
            // the fused first pass also holds the election's hash table (2 x kHubSlots u32) in the same LDS
            const size_t sh = std::max<size_t>((size_t)nw32 * sizeof(u32), hub ? 2 * kHubSlots * sizeof(u32) : 0);
#define GCC_BFS(NT, HUB)                                                                                       \
    launch_k(h, "seed_bfs", np, seed_bfs_kernel<true, kFilterBlockLds, NT, HUB>, dim3(h->n_cu), dim3(kFilterBlockLds), \
             sh, edges, np, (const u32*)bits, nw32, flags, h->d_bmin + n_bmin, epoch, h->cap, h->d_err)
            rc = t.seed_nt ? (hub ? GCC_BFS(true, true) : GCC_BFS(true, false))
                           : (hub ? GCC_BFS(false, true) : GCC_BFS(false, false));
#undef GCC_BFS
        } else {
            const unsigned grid = grid_for((np + 1) / 2, kMaxGrid);
            rc = t.seed_nt ? launch_k(h, "seed_bfs", np, seed_bfs_kernel<false, kBlock, true, false>, dim3(grid),
                                      dim3(kBlock), 0, edges, np, (const u32*)bits, nw32, flags, h->d_bmin + n_bmin, epoch,
                                      h->cap, h->d_err)
                           : launch_k(h, "seed_bfs", np, seed_bfs_kernel<false, kBlock, false, false>, dim3(grid),
                                      dim3(kBlock), 0, edges, np, (const u32*)bits, nw32, flags, h->d_bmin + n_bmin, epoch,
                                      h->cap, h->d_err);
            n_bmin += grid;
        }
        if (rc) return rc;
        if (lds) n_bmin += (u32)h->n_cu;
        if (p + 1 < t.seed_passes) {
            rc = launch_k(h, "seed_pack", 0, seed_pack_kernel<false>, dim3(pack_grid), dim3(kBlock), 0, h->d_parent, h->cap,
                          (const u8*)flags, bits, (const u32*)nullptr, 0u, h->d_giant + h->giant_slot, epoch);
            if (rc) return rc;
        }
    }
    // fused: slot 0 (the hub's) is not written; h is in block 0's slot of the first pass
    rc = launch_k(h, "seed_init", 0, seed_pack_kernel<true>, dim3(pack_grid), dim3(kBlock), 0, h->d_parent, h->cap,
                  (const u8*)flags, bits, (const u32*)(fuse ? h->d_bmin + 1 : h->d_bmin), fuse ? n_bmin - 1 : n_bmin,
                  h->d_giant + h->giant_slot, epoch);
    if (rc) return rc;
    h->pending_reset = false;
    h->has_giant = true;
    return GCC_OK;
}

// The bucketed fold of a fresh forest (bucket_fold.h): when it applies, and the pipeline.
static u32 bucket_slices(const gcc_forest* h) { return (u32)(((u64)h->cap + bk::kSliceIds - 1) / bk::kSliceIds); }

// A fresh forest (seeded from a hub), or (round 4, tune bucket_windows) a later window of a forest that tracks a giant:
// then C is the tracked component's bitmap from the last compress, and the seeding and the reset are skipped.
static bool bucket_applies(const gcc_forest* h, const u32* d_pairs, u64 n) {
    const FoldTune& t = h->tune;
    const bool later = !h->pending_reset && t.bucket_windows && h->has_giant && !h->filter_off && h->compressed;
    return t.bucket && (h->pending_reset || later) && h->filter_enabled() && (u64)h->cap >= t.bucket_min_ids &&
           n >= std::max<u64>(t.bucket_min_batch, 2 * bk::kP1Tile) && n < (1ull << 31) &&
           bucket_slices(h) <= bk::kMaxBuckets &&
           ((reinterpret_cast<uintptr_t>(d_pairs) | reinterpret_cast<uintptr_t>(h->d_parent) |
             reinterpret_cast<uintptr_t>(h->d_spare)) & 15) == 0;
}

// GELLY_POISON=1 (diagnostics): the bucketed fold's scratch buffers start as 0xA5 bytes instead of whatever the
// allocator hands back, so that a read of an entry no kernel wrote trips the kErr* checks deterministically.
static bool poison_scratch() {
    static const bool on = [] {
        const char* e = std::getenv("GELLY_POISON");
        return e && *e && *e != '0';
    }();
    return on;
}

template <typename T>
static int grow(T*& p, u64& cap, u64 need, hipStream_t st) {
    if (cap >= need) return GCC_OK;
    if (p) {
        HIP_TRY(hipStreamSynchronize(st));  // the stream's earlier launches may still read the old buffer
        HIP_TRY(hipFree(p));
    }
    p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc((void**)&p, (size_t)need * sizeof(T)));
    if (poison_scratch()) HIP_TRY(hipMemsetAsync(p, 0xA5, (size_t)need * sizeof(T), st));  // stream-ordered
    cap = need;
    return GCC_OK;
}

// encode scratch (msg kernels): per 64-id word the others' mask, then per count block its count and list base
static u32 msg_blocks(const gcc_forest* h) { return (u32)((((u64)h->cap + 63) / 64 + kMsgWordsPerBlock - 1) / kMsgWordsPerBlock); }
static int ensure_msg_scratch(gcc_forest* h) {
    if (h->d_msg_oth) return GCC_OK;
    const u64 nw = ((u64)h->cap + 63) / 64;
    HIP_TRY(hipMalloc((void**)&h->d_msg_oth, nw * sizeof(u64) + 2 * (size_t)msg_blocks(h) * sizeof(u32)));
    return GCC_OK;
}

static int launch_bucket(gcc_forest* h, const u32* d_pairs, u64 n) {
    if (int rc = pipe_exit(h)) return rc;
    const FoldTune& t = h->tune;
    const bool fresh = h->pending_reset;  // else: a later window, C = the tracked component (bucket_applies)
    h->rec_all = false;
    int rc = alloc_filter(h);
    if (rc) return rc;
    const u32 ns = bucket_slices(h);
    if (!h->d_meta) {
        HIP_TRY(hipMalloc((void**)&h->d_meta, sizeof(bk::Meta)));
        if (poison_scratch()) HIP_TRY(hipMemsetAsync(h->d_meta, 0xA5, sizeof(bk::Meta), h->stream));
    }
    const u32 p1_blocks = 2 * (u32)h->n_cu;  // (bucket_p1 = 1 runs n_cu blocks: fewer writers, same slack bound)
    const u32 p2_blocks = std::min<u32>((u32)h->n_cu, bk::kMaxP2Blocks);
    const u32 chunk = bk::chunk_entries(n, (u32)t.bucket_chunk);
    if (h->tune.scratch_realloc) {  // diagnostics: fresh scratch for this fold
        const int mode = h->tune.scratch_realloc;
        h->tune.scratch_realloc = 0;
        HIP_TRY(hipStreamSynchronize(h->stream));
        while (h->held_scratch.size() > 8) {
            (void)hipFree(h->held_scratch.front());
            h->held_scratch.erase(h->held_scratch.begin());
        }
        if ((mode == 1 || mode == 2) && h->d_bk) {
            h->held_scratch.push_back(h->d_bk);
            h->d_bk = nullptr;
            h->bk_cap_bytes = 0;
        }
        if ((mode == 1 || mode == 3) && h->d_vl) {
            h->held_scratch.push_back(h->d_vl);
            h->d_vl = nullptr;
            h->vl_cap = 0;
        }
        if (mode == 1) {
            if (h->d_slow) h->held_scratch.push_back(h->d_slow);
            if (h->d_ovf) h->held_scratch.push_back(h->d_ovf);
            h->d_slow = nullptr;
            h->slow_cap_total = 0;
            h->d_ovf = nullptr;
            h->ovf_cap = 0;
        }
    }
    const u64 bk_S = bk::bk_entries(bk::storage_edges(n, ns, p1_blocks, bk::bk_aligned(n), chunk));  // entries (a multiple of 2^19)
    if ((rc = grow(h->d_bk, h->bk_cap_bytes, bk::bk_bytes(bk_S), h->stream))) return rc;
    u32* bk_lo = reinterpret_cast<u32*>(h->d_bk);
    if (bucket_addr())
        std::fprintf(stderr, "[bucket-addr] edges %p bk %p (%llu entries) vl %p parent %p bits %p\n", (const void*)d_pairs,
                     (const void*)h->d_bk, (unsigned long long)bk_S, (const void*)h->d_vl, (const void*)h->d_parent,
                     (const void*)h->d_bits);
    bk::u16* bk_hi = reinterpret_cast<bk::u16*>(h->d_bk + 4 * bk_S);
    if ((rc = grow(h->d_ovf, h->ovf_cap, n / 8 + 65536, h->stream))) return rc;
    const u64 vl_S = bk::vl_entries(bk::storage_edges(n, bk::vslices(h->cap), p2_blocks, false, chunk));
    if ((rc = grow(h->d_vl, h->vl_cap, bk::vl_bytes(vl_S), h->stream))) return rc;
    const bk::VList vl{reinterpret_cast<bk::u16*>(h->d_vl), h->d_vl + 2 * vl_S};
    // room for half the batch in the slow lists (C4: 3.9 % slow; C4's 1/8 share: more than the 12.5 % an n/8
    // capacity held, and the rest took P2's inline ring unions: 1.03 ms instead of ~0.5)
    const u32 slow_cap = (u32)std::min<u64>(0x7FFFFFFEull, std::max<u64>(4096, n / p2_blocks / 2)) & ~1u;  // even: runs pair-aligned
    if ((rc = grow(h->d_slow, h->slow_cap_total, (u64)p2_blocks * slow_cap, h->stream))) return rc;
    const u64* edges = reinterpret_cast<const u64*>(d_pairs);
    u32* bits = reinterpret_cast<u32*>(h->d_bits);
    const u32 nw32 = 2 * (h->nwords() + (h->nwords() & 1));
    u32* giant = h->d_giant + h->giant_slot;
    if (!h->d_nbits) {
        HIP_TRY(hipMalloc((void**)&h->d_nbits, (size_t)nw32 * sizeof(u32)));
        HIP_TRY(hipMemsetAsync(h->d_nbits, 0, (size_t)nw32 * sizeof(u32), h->stream));
    }
    const u32 ovf_cap = (u32)std::min<u64>(h->ovf_cap, 0xFFFFFFF0ull);
    const u32 items = (u32)std::max(1, t.bucket_items) * (u32)h->n_cu;  // dequeue items per P2 / P3 launch (parts of the slices)
    const u32 cps = std::max<u32>(1, (items + ns - 1) / ns);
    // A block loads a part's 64 KiB bitmap slice into LDS per item: a pass over few edges (the seeding levels of a
    // small batch) takes fewer, longer parts, about 64K edges per part at least
    const bool slow2 = t.bucket_slow2 != 0;
    if (slow2 && (rc = grow(h->d_seg, h->seg_cap, (u64)ns * cps + 64, h->stream))) return rc;
    const double sample = n < 4 * (u64)h->cap ? t.bucket_sample_sparse : t.bucket_sample;
    const u32 cps_seed = (u32)std::max<u64>(1, std::min<u64>(cps, (u64)((double)n * sample) / ((u64)ns << 16)));
    // the first level streams only the hub's slice: one slice's sample, about 16K edges per part (one part per
    // P2 block at most)
    const u32 cps_hub = (u32)std::max<u64>(1, std::min<u64>(p2_blocks, (u64)((double)n * t.bucket_hub_sample) / ns / 16384));
    const u32 frac_hub = (u32)std::max(0.0, std::min(65536.0, t.bucket_hub_sample * 65536.0));
    const size_t f_lds = slice_filter_lds(), h_lds = bk::kVSliceWords * sizeof(u32);
    // P3's items: parts of the v-lists (target slices of 2^kVSliceBits ids, fewer than the buckets). Each item loads
    // its list's bitmap slice into LDS: as many parts per list as the buckets have per slice would load twice the
    // bytes of slices, so a v-list has (slice size ratio) times fewer parts
    const u32 nvs = bk::vslices(h->cap);
    const u32 vratio = 1u << (bk::kVSliceBits - bk::kSliceBits);
    // (round 5: P3's own count, bucket_items_p3 = 2 per CU: half P2's — fewer 128 KiB slice loads; C4 9.17 -> 9.1 ms,
    // the share 1.82 -> 1.78 with both at 2, P2 itself slower at 2: profiles/r5aq_sweep_cc_items.txt)
    const u32 cps3 = std::max<u32>(1, ((u32)std::max(1, t.bucket_items_p3) * (u32)h->n_cu + ns - 1) / ns);
    const u32 cps_v = std::max<u32>(1, cps3 * ns / nvs / vratio);
    const u32 cps_seed_v = std::max<u32>(1, cps_seed * ns / nvs / vratio);
    u32 slot = 0;
    // a fresh forest with the deferred N: C is deferred too (round 5), and P1 performs the lazy reset itself
    const bool defer = t.bucket_defer != 0;
    const bool defer_c = fresh && defer && t.bucket_defer_c;
    u32* p1_reset = defer_c && t.bucket_defer_c == 1 ? h->d_parent : nullptr;
    if (defer_c && t.bucket_defer_c == 2) {  // the reset beside P1, ordered after everything queued before this fold
        if (!h->aux_stream) {
            HIP_TRY(hipStreamCreateWithFlags(&h->aux_stream, hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&h->aux_ev[0], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&h->aux_ev[1], hipEventDisableTiming));
        }
        HIP_TRY(hipEventRecord(h->aux_ev[0], h->stream));
        HIP_TRY(hipStreamWaitEvent(h->aux_stream, h->aux_ev[0], 0));
        HIP_TRY(hipMemsetAsync(h->d_parent, 0xFF, (size_t)h->cap * sizeof(u32), h->aux_stream));
        HIP_TRY(hipEventRecord(h->aux_ev[1], h->aux_stream));
    }
    rc = launch_k(h, "bucket_layout", 0, bk::bucket_layout_kernel, dim3(1), dim3(1024), 0, edges, n, ns, h->cap, h->d_meta,
                  p1_blocks, p2_blocks, chunk, (const u32*)nullptr, (const u32*)nullptr);
    if (!rc)
        rc = ns > 256  // beyond 2^27 ids: 512 buckets' state and the 16K-edge tile exceed the LDS; 12K-edge tiles
                 ? launch_k(h, "bucket", n, bk::bucket_kernel<1024, 12, 512>, dim3(h->n_cu), dim3(1024),
                            bk::p1_lds(1024, 12, 512), edges, n, ns, h->cap, h->d_meta, bk_lo, bk_hi, h->d_ovf, ovf_cap,
                            h->d_err, p1_reset)
             : t.bucket_p1 == 1
                 ? launch_k(h, "bucket", n, bk::bucket_kernel<1024, 16>, dim3(h->n_cu), dim3(1024), bk::p1_lds(1024, 16),
                            edges, n, ns, h->cap, h->d_meta, bk_lo, bk_hi, h->d_ovf, ovf_cap, h->d_err, p1_reset)
             : t.bucket_p1 == 3
                 ? launch_k(h, "bucket", n, bk::bucket_kernel<1024, 16, 256, 8>, dim3(h->n_cu), dim3(1024),
                            bk::p1_lds(1024, 16, 256, 8), edges, n, ns, h->cap, h->d_meta, bk_lo, bk_hi, h->d_ovf, ovf_cap,
                            h->d_err, p1_reset)
             : t.bucket_p1 == 2
                 ? launch_k(h, "bucket", n, bk::bucket_kernel<1024, 12>, dim3(h->n_cu), dim3(1024), bk::p1_lds(1024, 12),
                            edges, n, ns, h->cap, h->d_meta, bk_lo, bk_hi, h->d_ovf, ovf_cap, h->d_err, p1_reset)
                 : launch_k(h, "bucket", n, bk::bucket_kernel<512, 16>, dim3(p1_blocks), dim3(512), bk::p1_lds(512, 16),
                            edges, n, ns, h->cap, h->d_meta, bk_lo, bk_hi, h->d_ovf, ovf_cap, h->d_err, p1_reset);
    if (rc) return rc;
    if (fresh) {
        HIP_TRY(hipMemsetAsync(bits, 0, (size_t)nw32 * sizeof(u32), h->stream));
        rc = launch_k(h, "bucket_hub", 0, bk::bucket_hub_kernel, dim3(1), dim3(kHubBlock), 2 * kHubSlots * sizeof(u32),
                      edges, n, h->cap, bits, h->d_meta);
    }
    // seeding (a fresh forest): C := {hub}, then levels over the sample. A later window keeps C = the tracked
    // component's bitmap and its root (the last compress wrote both), and parent[] as it is.
    const u32 frac = (u32)std::max(0.0, std::min(65536.0, sample * 65536.0));
    const u64 sample_edges = (u64)((double)n * frac / 65536.0);
    const int levels = fresh ? std::max(0, std::min(6, t.bucket_levels)) : 0;
    for (int l = 0; l < levels && !rc; ++l) {
        rc = launch_k(h, "seed_filter", sample_edges, bk::slice_filter_kernel<false>, dim3(p2_blocks), dim3(bk::kP2Block),
                      f_lds, h->d_parent, (const u32*)bk_lo, (const bk::u16*)bk_hi, (const u64*)nullptr,
                      (const u32*)bits, nw32, ns, h->d_meta, vl, l == 0 ? cps_hub : cps_seed, l == 0 ? frac_hub : frac, slot++, h->tune.drain_at, (u32)(l == 0),
                      (const u32*)giant, h->d_slow, slow_cap, h->cap, h->d_err,
                      (bk::SlowSeg*)nullptr, (u32)l);
        if (!rc)
            rc = launch_k(h, "seed_hook", 0, bk::slice_hook_kernel<false>, dim3(h->n_cu), dim3(bk::kP3Block), h_lds, bits,
                          bits, nw32, nvs, h->d_meta, vl, cps_seed_v, slot++, h->cap, h->d_err, (u32)l);
    }
    // parent[] := C ? g : UNSEEN (the reset), then every bucketed edge, the overflow list, a spill. With C deferred,
    // P1 did the reset and only g is published here
    if (!rc && defer_c && t.bucket_defer_c == 2) HIP_TRY(hipStreamWaitEvent(h->stream, h->aux_ev[1], 0));  // the reset
    if (!rc && fresh)
        rc = defer_c ? launch_k(h, "bucket_init", 0, bk::bucket_root_kernel, dim3(1), dim3(1), 0,
                                (const bk::Meta*)h->d_meta, giant)
                     : launch_k(h, "bucket_init", 0, bk::bucket_init_kernel, dim3(grid_for(((u64)h->cap + 3) / 4, kMaxGrid)),
                                dim3(kBlock), 0, h->d_parent, h->cap, (const u32*)bits, (const bk::Meta*)h->d_meta, giant);
    if (rc) return rc;
#define GCC_P2_FINAL(PER, VW)                                                                                      \
    launch_k(h, "slice_filter", n, bk::slice_filter_kernel<true, false, PER, VW>, dim3(p2_blocks), dim3(bk::kP2Block), \
             slice_filter_lds(PER, VW), h->d_parent, (const u32*)bk_lo, (const bk::u16*)bk_hi, (const u64*)nullptr,   \
             (const u32*)bits, nw32, ns, h->d_meta, vl, cps, 65536u, slot++, h->tune.drain_at, 0u, (const u32*)giant, \
             h->d_slow, slow_cap, h->cap, h->d_err, slow2 ? h->d_seg : nullptr, bk::kVlFinal)
    rc = t.bucket_p2_per == 12 ? (t.bucket_p2_vw == 8 ? GCC_P2_FINAL(12, 8) : GCC_P2_FINAL(12, 4)) : GCC_P2_FINAL(8, 4);
#undef GCC_P2_FINAL
    if (!rc && bucket_stats()) {  // diagnostics: FINAL P2's output (synchronises)
        bk::Meta hm;
        HIP_TRY(hipMemcpyAsync(&hm, h->d_meta, sizeof(hm), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        u64 vl_used = 0, slow = 0;
        for (u32 s = 0; s < nvs; ++s) vl_used += std::min(hm.vl_cur[bk::kVlFinal][s], hm.vl_cap[s]);
        for (u32 b = 0; b < p2_blocks; ++b) slow += hm.slow_cnt[b];
        std::fprintf(stderr, "[bucket] FINAL P2: v-list entries %llu, slow %llu (%.1f %%), slow runs %u\n",
                     (unsigned long long)vl_used, (unsigned long long)slow, 100.0 * slow / n, hm.nseg);
    }
    if (!rc)
        rc = launch_k(h, "slice_hook", 0, bk::slice_hook_kernel<true>, dim3(h->n_cu), dim3(bk::kP3Block), h_lds, bits,
                      h->d_nbits, nw32, nvs, h->d_meta, vl, cps_v, slot++, h->cap, h->d_err, bk::kVlFinal);
    if (!rc)
        rc = defer ? launch_k(h, "bucket_join", 0, bk::bucket_join_kernel, dim3(grid_for(nw32, kMaxGrid)), dim3(kBlock), 0,
                              h->d_parent, bits, h->d_nbits, nw32, (const u32*)giant, (const bk::Meta*)h->d_meta,
                              (u32)!fresh, (u32)defer_c)
                   : launch_k(h, "bucket_hook", 0, bk::bucket_hook_kernel, dim3(grid_for(nw32, kMaxGrid)), dim3(kBlock), 0,
                              h->d_parent, bits, h->d_nbits, nw32, (const u32*)giant);
    // Second level over the slow edges, now against C | N: a slow edge whose source joined N is a hook of its
    // target (its v-list again), one whose target is in C | N (the global bitmap) a hook of its source (round 4),
    // only the rest stays slow. Its input is FINAL P2's slow runs (one source slice
    // each); its slow edges go to the bucket storage, which P2 has consumed.
    const u64* slow_list = h->d_slow;
    u32 slow_list_cap = slow_cap;
    if (slow2 && !rc) {
        // the bucket storage (consumed by FINAL P2) as u64 slow entries
        const u32 slow_cap2 = (u32)std::min<u64>(0x7FFFFFFEull, h->bk_cap_bytes / 8 / p2_blocks) & ~1u;
        rc = launch_k(h, "slice_filter2", 0, bk::slice_filter_kernel<true, true>, dim3(p2_blocks), dim3(bk::kP2Block),
                      f_lds, h->d_parent, (const u32*)nullptr, (const bk::u16*)nullptr, (const u64*)h->d_slow,
                      (const u32*)bits, nw32, ns, h->d_meta, vl, 1u, 65536u, slot++, h->tune.drain_at, 0u,
                      (const u32*)giant, reinterpret_cast<u64*>(h->d_bk), slow_cap2, h->cap, h->d_err, h->d_seg,
                      bk::kVlLevel2);
        if (!rc)
            rc = launch_k(h, "slice_hook2", 0, bk::slice_hook_kernel<true>, dim3(h->n_cu), dim3(bk::kP3Block), h_lds, bits,
                          h->d_nbits, nw32, nvs, h->d_meta, vl, cps_v, slot++, h->cap, h->d_err, bk::kVlLevel2);
        if (!rc)
            rc = defer ? launch_k(h, "bucket_join2", 0, bk::bucket_join_kernel, dim3(grid_for(nw32, kMaxGrid)), dim3(kBlock),
                                  0, h->d_parent, bits, h->d_nbits, nw32, (const u32*)giant,
                                  (const bk::Meta*)h->d_meta, (u32)!fresh, (u32)defer_c)
                       : launch_k(h, "bucket_hook2", 0, bk::bucket_hook_kernel, dim3(grid_for(nw32, kMaxGrid)), dim3(kBlock),
                                  0, h->d_parent, bits, h->d_nbits, nw32, (const u32*)giant);
        slow_list = reinterpret_cast<const u64*>(h->d_bk);
        slow_list_cap = slow_cap2;
    }
    if (!rc)
        rc = launch_k(h, "bucket_slow", 0, bk::bucket_slow_kernel, dim3(p2_blocks * bk::kSlowSplit), dim3(kBlock), 0,
                      h->d_parent, slow_list, slow_list_cap, (const bk::Meta*)h->d_meta, p2_blocks, (const u32*)bits,
                      (const u32*)giant, h->cap, h->d_err);
    if (!rc)
        rc = launch_k(h, "bucket_rest", 0, bk::bucket_rest_kernel, dim3(grid_for(n / 64 + 1, kMaxGrid)), dim3(kBlock), 0,
                      h->d_parent, (const u64*)h->d_ovf, ovf_cap, (const bk::Meta*)h->d_meta, (const u32*)bits, edges, n,
                      h->cap, h->d_err, (const u32*)giant);
    if (rc) return rc;
    h->deferred_n = defer;
    h->pending_reset = false;
    h->has_giant = true;
    if (bucket_stats()) {  // diagnostics: the lists' fill (synchronises)
        bk::Meta hm;
        HIP_TRY(hipMemcpyAsync(&hm, h->d_meta, sizeof(hm), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        u64 bk_used = 0, vl_used = 0, slow = 0;
        for (u32 s = 0; s < ns; ++s) {
            bk_used += std::min(hm.bk_cur[s], hm.bk_cap[s]);
            vl_used += std::min(hm.vl_cur[bk::kVlFinal][s], hm.vl_cap[s]);
        }
        for (u32 b = 0; b < p2_blocks; ++b) slow += hm.slow_cnt[b];
        std::fprintf(stderr, "[bucket] n=%llu ns=%u bucket entries %llu, v-list entries %llu (%.1f %%), slow %llu "
                     "(%.1f %%), overflow %u, spill %u, g=%u\n", (unsigned long long)n, ns,
                     (unsigned long long)bk_used, (unsigned long long)vl_used, 100.0 * vl_used / n,
                     (unsigned long long)slow, 100.0 * slow / n, hm.ovf_cur, hm.spill, hm.gmin);
        // the slow kernel's input by kind, against the final C | N: both ends in it (nothing to do), one end (a hook
        // of the other), neither (a union)
        std::vector<u32> hb(nw32);
        HIP_TRY(hipMemcpy(hb.data(), bits, (size_t)nw32 * sizeof(u32), hipMemcpyDeviceToHost));
        u64 kinds[3] = {0, 0, 0};
        std::vector<u64> seg;
        for (u32 b = 0; b < p2_blocks; ++b) {
            const u32 c = std::min(hm.slow_cnt[b], slow_list_cap);
            seg.resize(c);
            if (c) HIP_TRY(hipMemcpy(seg.data(), slow_list + (u64)b * slow_list_cap, (size_t)c * sizeof(u64), hipMemcpyDeviceToHost));
            for (u64 e : seg) {
                if (e == ~0ull) continue;
                const u32 a = (u32)e, bb = (u32)(e >> 32);
                const int ia = (hb[a >> 5] >> (a & 31)) & 1, ib = (hb[bb >> 5] >> (bb & 31)) & 1;
                ++kinds[ia + ib == 2 ? 0 : ia + ib == 1 ? 1 : 2];
            }
        }
        std::fprintf(stderr, "[bucket] slow kernel input vs C|N: both ends %llu, one end %llu, neither %llu\n",
                     (unsigned long long)kinds[0], (unsigned long long)kinds[1], (unsigned long long)kinds[2]);
#ifdef GCC_PHASES
        unsigned long long ph[2][16];
        HIP_TRY(hipMemcpyFromSymbol(ph, HIP_SYMBOL(bk::gcc_phase_acc), sizeof(ph)));
        static const char* const names[2][8] = {
            {"loads", "count", "barrier1", "scan", "barrier2", "reserve+scatter", "barrier3", "write-out"},
            {"loads+decode", "lookup+count", "slow stores", "barrier1", "scan+barrier2", "reserve+scatter", "barrier3",
             "write-out/item"}};
        for (int k = 0; k < 2; ++k)
            for (int grp = 0; grp < 2; ++grp) {
                unsigned long long tot = 0;
                for (int j = 0; j < 8; ++j) tot += ph[k][8 * grp + j];
                std::fprintf(stderr, "[phases] %s %s:", k ? "P2" : "P1", grp ? "other waves" : "waves 0-1");
                for (int j = 0; j < 8; ++j)
                    std::fprintf(stderr, " %s %.1f%%", names[k][j], 100.0 * ph[k][8 * grp + j] / (tot ? tot : 1));
                std::fprintf(stderr, " (total %.3g clk)\n", (double)tot);
            }
        unsigned long long zero[2][16] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(bk::gcc_phase_acc), zero, sizeof(zero)));
        // every block's working time against the kernel's span (load balance of the persistent / work-queue kernels)
        std::vector<unsigned long long> bt((size_t)bk::kBtKinds * bk::kBtBlocks * 2);
        HIP_TRY(hipMemcpyFromSymbol(bt.data(), HIP_SYMBOL(bk::gcc_blk_time), bt.size() * sizeof(unsigned long long)));
        static const char* const bt_names[bk::kBtKinds] = {"P1", "FINAL P2", "level-2 P2", "FINAL P3", "level-2 P3",
                                                        "seed P2", "seed P3", "slow"};
        for (int k = 0; k < bk::kBtKinds; ++k) {
            unsigned long long lo = ~0ull, hi = 0, busy = 0, mx = 0;
            u32 nb = 0;
            std::vector<unsigned long long> d;
            for (int b = 0; b < bk::kBtBlocks; ++b) {
                const unsigned long long t0 = bt[((size_t)k * bk::kBtBlocks + b) * 2], t1 = bt[((size_t)k * bk::kBtBlocks + b) * 2 + 1];
                if (!t0 || t1 < t0) continue;
                lo = std::min(lo, t0);
                hi = std::max(hi, t1);
                busy += t1 - t0;
                mx = std::max(mx, t1 - t0);
                d.push_back(t1 - t0);
                ++nb;
            }
            if (!nb) continue;
            std::sort(d.begin(), d.end());
            std::fprintf(stderr, "[blocks] %s: %u blocks, span %.1f us, block time median %.1f / max %.1f us, "
                         "utilisation %.2f\n", bt_names[k], nb, (hi - lo) / 100.0, d[d.size() / 2] / 100.0, mx / 100.0,
                         (double)busy / ((double)nb * (double)(hi - lo ? hi - lo : 1)));
        }
        std::fill(bt.begin(), bt.end(), 0ull);
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(bk::gcc_blk_time), bt.data(), bt.size() * sizeof(unsigned long long)));
#endif
    }
    return GCC_OK;
}

// The sampled start's share, read back without a host sync (FoldTune::share_async): not landed yet -> nothing (this
// batch folds plain, as every batch since the vote did); landed -> the filter turns on if the voted component holds
// filter_min_share of the samples, after a refresh of its bitmap (the empty set until then).
static int share_poll(gcc_forest* h) {
    const hipError_t q = hipEventQuery(h->share_ev);
    if (q == hipErrorNotReady) return GCC_OK;
    HIP_TRY(q);
    h->share_pending = false;
    const u32 hit = __atomic_load_n(&h->h_share[0], __ATOMIC_ACQUIRE), seen = __atomic_load_n(&h->h_share[1], __ATOMIC_ACQUIRE);
    if (!h->has_giant || hit < h->tune.filter_min_share * seen) return GCC_OK;
    h->filter_off = false;
    return refresh_now(h);
}

// The fold pipeline for one batch (UpdateCC.foldEdges over the batch, DisjointSet.union per edge):
//  0. a FRESH forest (reset, nothing folded since) is seeded: launch_seed builds the component of a hub
//     over a prefix on a bitmap and writes parent[] from it; the filtered kernel then folds the whole batch;
//  1. otherwise a forest without a tracked component first folds a sampling prefix in geometrically growing
//     launches (4K, 16K, ... edges): few threads contend while the hubs are still unhooked, which avoids the
//     CAS storm a single full-width launch causes on the hubs of a skewed stream;
//  2. compress + vote + bitmap of the giant component;
//  3. the rest streams through the giant-filtered kernel; large batches refresh the bitmap at the refresh points.
static int launch_fold(gcc_forest* h, const u32* d_pairs, u64 n) {
    if (n == 0) return GCC_OK;
    const FoldTune& t = h->tune;
    h->edges_since_compress += n;
    const int ev_first = (int)h->kev_used;
    if (h->timing) h->klog.push_back({"begin", -1, 0});
    int rc = GCC_OK;
    u64 b = 0;
    // seeding pays when the BFS lookups are LDS-resident; beyond that (C4: 8 MiB bitmap) the sampled start
    // measured faster (profiles/r1_sweep_c4_seed.log)
    const bool seed_fits = (u64)h->nwords() + (h->nwords() & 1) <= kLdsBitmapMaxWords || t.seed_global;
    const bool seeded = h->pending_reset && h->filter_enabled() && t.seed && seed_fits && n >= t.filter_min_batch &&
                        n >= 64 &&
                        ((reinterpret_cast<uintptr_t>(h->d_parent) | reinterpret_cast<uintptr_t>(h->d_spare)) & 15) == 0;
    double refresh[3] = {t.refresh[0], t.refresh[1], t.refresh[2]};
    if (bucket_applies(h, d_pairs, n)) {  // a fresh forest over a big id range: the bucketed fold
        rc = launch_bucket(h, d_pairs, n);
        if (rc) return rc;
        if (h->timing && (int)h->kev_used > ev_first) {
            h->last_fold_first = ev_first;
            h->last_fold_last = (int)h->kev_used - 1;
        }
        mark_mutated(h);
        if (h->deferred_n) {  // the closing compress labels N (and writes the others' masks for a merge's encode)
            h->deferred_n = false;
            rc = ensure_msg_scratch(h);
            bool masks = false;
            if (!rc) rc = compress_now(h, "compress", h->d_msg_oth, &masks, reinterpret_cast<const u64*>(h->d_nbits));
            if (rc) return rc;
            HIP_TRY(hipMemsetAsync(h->d_nbits, 0, (size_t)2 * (h->nwords() + (h->nwords() & 1)) * sizeof(u32), h->stream));
            if (masks) h->mask_version = h->version;
        }
        return GCC_OK;
    }
    if (h->share_pending && !h->pending_reset && (rc = share_poll(h))) return rc;
    if (h->share_unchecked && !h->pending_reset) {
        h->share_unchecked = false;
        if (h->has_giant && !h->filter_off && h->filter_enabled() && t.filter_min_share > 0 && h->d_giant) {
            u32 share[2] = {0, 0};  // once per forest
            HIP_TRY(hipMemcpyAsync(share, h->d_giant + 4, sizeof(share), hipMemcpyDeviceToHost, h->stream));
            HIP_TRY(hipStreamSynchronize(h->stream));
            h->filter_off = share[0] < t.filter_min_share * share[1];
        }
    }
    if (seeded) {
        rc = launch_seed(h, d_pairs, n);
        refresh[0] = t.seed_refresh;
        refresh[1] = refresh[2] = 0;
    } else {
        rc = materialize_reset(h);
    }
    if (rc) return rc;
    if (!h->filter_enabled() || (!h->has_giant && n < t.filter_min_batch)) {
        rc = launch_plain(h, d_pairs, n, "plain");
        b = n;
    } else if (!h->has_giant) {
        // 1/sample_div of the batch, but at least min(sample_min, 1/32 of it): a short batch (a C5 window) keeps
        // a sample well below its length, so the vote-share check below still runs
        const u64 s_end = std::min(n, std::max<u64>({t.filter_min_batch / 4, n / std::max<u64>(1, t.sample_div),
                                                     std::min<u64>(t.sample_min, n / 32)}));
        for (u64 c = std::max<u64>(1, t.sample_first); b < s_end && !rc; c *= std::max<u64>(2, t.sample_growth)) {
            const u64 e = std::min(s_end, b + c);
            rc = launch_plain(h, d_pairs + 2 * b, e - b, "sample");
            b = e;
        }
        if (!rc && b < n && t.filter_min_share > 0) {
            // once per forest: is the voted component a giant among the seen samples? If not, the filter would
            // send almost every edge down its slow path, and the plain fold is faster (C3, C5). The vote alone
            // answers that; the bitmap refresh only runs when the filter stays on (C3: 1.135 -> 1.107 ms).
            rc = alloc_filter(h);
            if (!rc && !h->has_giant)
                rc = launch_k(h, "vote", 0, giant_vote_kernel, dim3(1), dim3(1024), 0, h->d_parent, h->cap,
                              h->d_giant + h->giant_slot, h->d_giant + 4);
            if (rc) return rc;
            h->has_giant = true;
            if (t.share_async) {
                // the batch's rest folds plain while the share travels; a later fold decides (share_poll)
                if (!h->h_share) HIP_TRY(hipHostMalloc((void**)&h->h_share, 2 * sizeof(u32), hipHostMallocDefault));
                if (!h->share_ev) HIP_TRY(hipEventCreateWithFlags(&h->share_ev, hipEventDisableTiming));
                HIP_TRY(hipMemcpyAsync(h->h_share, h->d_giant + 4, 2 * sizeof(u32), hipMemcpyDeviceToHost, h->stream));
                HIP_TRY(hipEventRecord(h->share_ev, h->stream));
                h->share_pending = true;
                h->filter_off = true;
            } else {
                u32 share[2] = {0, 0};
                HIP_TRY(hipMemcpyAsync(share, h->d_giant + 4, sizeof(share), hipMemcpyDeviceToHost, h->stream));
                HIP_TRY(hipStreamSynchronize(h->stream));
                h->filter_off = share[0] < t.filter_min_share * share[1];
            }
            if (!h->filter_off) rc = refresh_now(h);
            else  // no refresh: the tracked-component bitmap is the empty set (valid: components only grow)
                HIP_TRY(hipMemsetAsync(h->d_bits, 0, (size_t)h->nwords() * sizeof(u64), h->stream));
        } else if (!rc && b < n) {
            rc = refresh_now(h);
        }
        if (!rc && b < n && h->filter_off) {
            rc = launch_plain(h, d_pairs + 2 * b, n - b, "plain");
            b = n;
        }
    } else if (h->filter_off) {
        rc = launch_plain(h, d_pairs, n, "plain");
        b = n;
    }
    int next_refresh = 0;
    while (!rc && b < n) {
        u64 e = n;
        if (n > t.refresh_min_batch) {
            while (next_refresh < 3 && refresh[next_refresh] > 0 && (u64)(n * refresh[next_refresh]) <= b) ++next_refresh;
            if (next_refresh < 3 && refresh[next_refresh] > 0) e = std::max<u64>(b + 1, (u64)(n * refresh[next_refresh]));
        }
        rc = launch_filtered(h, d_pairs + 2 * b, e - b);
        b = e;
        if (!rc && b < n) {
            rc = refresh_now(h);
            ++next_refresh;
        }
    }
    if (rc) return rc;
    if (h->timing && (int)h->kev_used > ev_first) {
        h->last_fold_first = ev_first;
        h->last_fold_last = (int)h->kev_used - 1;
    }
    mark_mutated(h, true);  // the launches above cleared rec_all unless they recorded
    return GCC_OK;
}

// H2D the first n edges of the current staging slot and fold them; then switch slots.
static int submit_slot(gcc_forest* h, u64 n) {
    if (n == 0) return GCC_OK;
    const int s = h->slot;
    HIP_TRY(hipMemcpyAsync(h->d_stage[s], h->h_stage[s], n * 2 * sizeof(u32), hipMemcpyHostToDevice, h->stream));
    int rc = launch_fold(h, h->d_stage[s], n);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(h->stage_ev[s], h->stream));
    h->slot = s ^ 1;
    h->staged = 0;
    // the next slot may still be in flight from two submits ago
    HIP_TRY(hipEventSynchronize(h->stage_ev[h->slot]));
    return GCC_OK;
}

static int alloc_staging(gcc_forest* h) {
    if (h->h_stage[0]) return GCC_OK;
    for (int s = 0; s < 2; ++s) {
        HIP_TRY(hipHostMalloc((void**)&h->h_stage[s], gcc_forest::kStageEdges * 2 * sizeof(u32), hipHostMallocDefault));
        HIP_TRY(hipMalloc((void**)&h->d_stage[s], gcc_forest::kStageEdges * 2 * sizeof(u32)));
        HIP_TRY(hipEventCreateWithFlags(&h->stage_ev[s], hipEventDisableTiming));
        HIP_TRY(hipEventRecord(h->stage_ev[s], h->stream));
    }
    return GCC_OK;
}

// submit the staged host edges (a fold handles a pending reset itself)
static int flush_staged(gcc_forest* h) {
    if (h->staged == 0) return GCC_OK;
    return submit_slot(h, h->staged);
}

// everything queued and parent[] materialised, the pipelined emission still on (folds, compresses and label reads)
static int flush_fold(gcc_forest* h) {
    int rc = flush_staged(h);
    if (rc) return rc;
    return materialize_reset(h);
}

// everything queued, parent[] materialised, and the pipelined emission left: the state every other entry point
// works on
static int flush(gcc_forest* h) {
    int rc = flush_fold(h);
    if (rc) return rc;
    return pipe_exit(h);
}

// the labels of everything folded so far, in labels_ptr(h), stream-ordered on the handle's stream — except for the
// emission call itself in the pipelined regime (ready = false: gcc_forest_compress), whose scan the handle's stream
// does not wait for, so that the next window's fold runs beside it; every label read waits (ready = true)
static int compress_async(gcc_forest* h, bool ready = true) {
    int rc = flush_fold(h);
    if (rc) return rc;
    if (h->pipe) {
        rc = pipe_compress(h);
        return rc || !ready ? rc : pipe_labels_ready(h);
    }
    if (h->compressed) return GCC_OK;
    return compress_now(h);
}

static int refresh_host(gcc_forest* h) {
    if (h->host_valid) return GCC_OK;
    int rc = compress_async(h);
    if (rc) return rc;
    h->host_labels.resize(h->cap);
    HIP_TRY(hipMemcpyAsync(h->host_labels.data(), labels_ptr(h), (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToHost,
                           h->stream));
    rc = stream_sync_checked(h);
    if (rc) return rc;
    h->host_valid = true;
    return GCC_OK;
}

static int counts(gcc_forest* h, unsigned long long out[2]) {
    int rc = h->pipe ? compress_async(h) : flush(h);  // a forest's seen ids and roots, or the labels' (the same counts)
    if (rc) return rc;
    if (!h->d_counts) HIP_TRY(hipMalloc((void**)&h->d_counts, 3 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(h->d_counts, 0, 2 * sizeof(unsigned long long), h->stream));
    hipLaunchKernelGGL(count_kernel, dim3(grid_for(h->cap, kMaxGrid)), dim3(kBlock), 0, h->stream, labels_ptr(h), h->cap,
                       h->d_counts);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, h->d_counts, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    return stream_sync_checked(h);
}
// P1 of the bucketed fold alone (layout + bucket_kernel), into f's bucket storage: n u64 pairs split by the FIRST id's
// 2^19-id slice. For the signed forest's bucketed fold (signed_bucket.h), which treats P1 as a plain partition. n_dev:
// the list's length on the device (n: its bound), exact: its per-slice counts (no sampled layout).
static int bucketize(gcc_forest* f, const u64* edges, u64 n, u32** lo_out, bk::u16** hi_out, const u32* n_dev = nullptr,
                     const u32* exact = nullptr, bool key_only = false) {
    const u32 ns = bucket_slices(f);
    if (!f->d_meta) HIP_TRY(hipMalloc((void**)&f->d_meta, sizeof(bk::Meta)));
    const u32 p1_blocks = 2 * (u32)f->n_cu;
    const u32 p2_blocks = std::min<u32>((u32)f->n_cu, bk::kMaxP2Blocks);
    const u32 chunk = bk::chunk_entries(n, 0);
    const u64 bk_S = bk::bk_entries(bk::storage_edges(n, ns, p1_blocks, bk::bk_aligned(n), chunk));
    int rc = grow(f->d_bk, f->bk_cap_bytes, bk::bk_bytes(bk_S), f->stream);
    if (!rc) rc = grow(f->d_ovf, f->ovf_cap, n / 8 + 65536, f->stream);
    if (rc) return rc;
    u32* bk_lo = reinterpret_cast<u32*>(f->d_bk);
    bk::u16* bk_hi = reinterpret_cast<bk::u16*>(f->d_bk + 4 * bk_S);
    const u32 ovf_cap = (u32)std::min<u64>(f->ovf_cap, 0xFFFFFFF0ull);
    rc = launch_k(f, "sb_layout", 0, bk::bucket_layout_kernel, dim3(1), dim3(1024), 0, edges, n, ns, f->cap, f->d_meta,
                  p1_blocks, p2_blocks, chunk, n_dev, exact);
    const u64 nk = n_dev ? ~0ull : n;  // bucket_kernel: from the layout
    if (!rc && key_only && ns <= 256)  // 4-B entries (the emit lists: the second id is a parity bit)
        rc = launch_k(f, "sb_bucket", n, bk::bucket_kernel<1024, 16, 256, 4, true>, dim3(f->n_cu), dim3(1024),
                      bk::p1_lds(1024, 16), edges, nk, ns, f->cap, f->d_meta, bk_lo, bk_hi, f->d_ovf, ovf_cap, f->d_err,
                      (u32*)nullptr);
    else if (!rc)
        rc = ns > 256 ? launch_k(f, "sb_bucket", n, bk::bucket_kernel<1024, 12, 512>, dim3(f->n_cu), dim3(1024),
                                 bk::p1_lds(1024, 12, 512), edges, nk, ns, f->cap, f->d_meta, bk_lo, bk_hi, f->d_ovf,
                                 ovf_cap, f->d_err, (u32*)nullptr)
                      : launch_k(f, "sb_bucket", n, bk::bucket_kernel<1024, 16>, dim3(f->n_cu), dim3(1024),
                                 bk::p1_lds(1024, 16), edges, nk, ns, f->cap, f->d_meta, bk_lo, bk_hi, f->d_ovf, ovf_cap,
                                 f->d_err, (u32*)nullptr);
    *lo_out = bk_lo;
    *hi_out = bk_hi;
    return rc;
}

// The bucketed signed fold (signed_bucket.h's header comment): `levels` rounds of P1 + filter + P1 + check + join, the
// rest, the closing compress into a->out. No host synchronisation: the lists' lengths and per-slice counts stay on
// the device (ctr[1], ctr[2]; a->hist), and their P1 layouts take them from there (round 5: one sync per list and a
// sampled layout each cost 0.3 ms of the share's 4.65).
int gcc_internal_take_err(gcc_forest* f, hipStream_t stream) {
    if (!f) return GCC_OK;
    DeviceGuard g(f->device);
    const hipStream_t own = f->stream;
    f->stream = stream;
    const int rc = stream_sync_checked(f);
    f->stream = own;
    return rc;
}

int gcc_internal_signed_bucket(gcc_forest* f, GccSignedBucketArgs* a) {
    DeviceGuard g(f->device);
    // the scratch runs on the signed handle's stream for this fold only: its own stream is restored on every return
    // (gcc_forest_destroy synchronises f->stream, which must not be a stream the signed handle may have destroyed since)
    struct StreamRestore {
        gcc_forest* f;
        hipStream_t own;
        ~StreamRestore() { f->stream = own; }
    } restore{f, f->stream};
    f->stream = a->stream;
    const u32 ns = bucket_slices(f);
    const u32 nw16 = (u32)(((u64)a->cap + 15) / 16);
    const u32 items = (u32)std::max(1, a->items_per_cu) * (u32)f->n_cu;
    const u32 cps = std::max<u32>(1, (items + ns - 1) / ns);
    const size_t lds = sb::kSliceW * sizeof(u32);
    auto ovf_cap = [&]() -> u32 { return (u32)std::min<u64>(f->ovf_cap, 0xFFFFFFF0ull); };  // grows with the lists
    const int levels = std::max(1, std::min(3, a->levels));
    int rc = GCC_OK;
    u64* slow_out = a->slow0;
    HIP_TRY(hipMemsetAsync(a->ctr, 0, 8 * sizeof(u32), f->stream));
    HIP_TRY(hipMemsetAsync(a->hist, 0, 2 * levels * bk::kMaxBuckets * sizeof(u32), f->stream));
    const u64* src = a->edges;
    u32* lo;
    bk::u16* hi;
    for (int lv = 0; lv < levels && !rc; ++lv) {
        u32* he = a->hist + 2 * lv * bk::kMaxBuckets;
        u32* hs = he + bk::kMaxBuckets;
        // level 1: the batch (sampled layout); level 2: the previous level's slow list (its length ctr[2], its counts)
        rc = lv == 0 ? bucketize(f, src, a->n, &lo, &hi)
                     : bucketize(f, src, a->n, &lo, &hi, a->ctr + 2, he - bk::kMaxBuckets);
        if (!rc) HIP_TRY(hipMemsetAsync(a->ctr, 0, 3 * sizeof(u32), f->stream));
        if (!rc)
            rc = launch_k(f, "sb_filter", lv == 0 ? a->n : 0, sb::sb_filter_kernel, dim3(f->n_cu), dim3(sb::kBlock), lds,
                          (const u32*)lo, (const bk::u16*)hi, (const bk::Meta*)f->d_meta, ns, cps, a->ctr,
                          (const u32*)a->gbits, nw16, a->emit, slow_out, a->cap, he, hs, f->d_err);
        // the bucketing's overflow list (edges): the rest's rule now (exact at any time: deferred members are never
        // united directly); a spill sets ctr[3] for the whole batch at the end
        if (!rc)
            rc = launch_k(f, "sb_rest", 0, sb::sb_rest_kernel, dim3(grid_for(std::max<u64>(1, ovf_cap()), 1024)), dim3(256), 0,
                          a->word, (const u64*)f->d_ovf, (u64)ovf_cap(), (const u32*)&f->d_meta->ovf_cur, 0u,
                          (const bk::Meta*)f->d_meta, a->gbits, a->vote, a->cap, a->fail, a->ctr);
        // the emitted pairs by v's slice (their length ctr[1]), then checked / added with v's slice in LDS
        const bool key_only = ns <= 256;
        if (!rc) rc = bucketize(f, a->emit, a->n, &lo, &hi, a->ctr + 1, he, key_only);
        if (!rc) HIP_TRY(hipMemsetAsync(a->ctr, 0, sizeof(u32), f->stream));
        if (!rc)
            rc = launch_k(f, "sb_check", 0, key_only ? sb::sb_check_kernel<true> : sb::sb_check_kernel<false>, dim3(f->n_cu),
                          dim3(sb::kBlock), lds, (const u32*)lo,
                          (const bk::u16*)hi, (const bk::Meta*)f->d_meta, ns, cps, a->ctr, (const u32*)a->gbits, nw16,
                          a->n2, a->cap, a->fail, f->d_err);
        if (!rc)
            rc = launch_k(f, "sb_check_ovf", 0, sb::sb_check_list_kernel, dim3(grid_for(std::max<u64>(1, ovf_cap()), 1024)),
                          dim3(256), 0, (const u64*)f->d_ovf, ovf_cap(), (const bk::Meta*)f->d_meta,
                          (const u32*)a->gbits, a->n2, a->cap, a->fail, a->ctr);
        if (!rc)
            rc = launch_k(f, "sb_join_low", 0, sb::sb_join_low_kernel, dim3(64), dim3(256), 0, a->word, (const u32*)a->n2,
                          a->vote, a->fail);
        if (!rc)
            rc = launch_k(f, "sb_join", 0, sb::sb_join_kernel, dim3(grid_for(nw16, kMaxGrid)), dim3(256), 0, a->word,
                          a->gbits, a->n2, nw16, a->vote, a->fail);
        src = slow_out;
        slow_out = slow_out == a->slow0 ? a->slow1 : a->slow0;
    }
    // the last level's slow edges (ctr[2] of them), then (only after a spill: ctr[3]) the whole batch again
    if (!rc)
        rc = launch_k(f, "sb_rest", 0, sb::sb_rest_kernel, dim3(grid_for(a->n, kMaxGrid)), dim3(256), 0, a->word, src, a->n,
                      (const u32*)(a->ctr + 2), 0u, (const bk::Meta*)nullptr, a->gbits, a->vote, a->cap, a->fail, a->ctr);
    if (!rc)
        rc = launch_k(f, "sb_rest", 0, sb::sb_rest_kernel, dim3(grid_for(a->n, kMaxGrid)), dim3(256), 0, a->word,
                      a->edges, a->n, (const u32*)nullptr, 1u, (const bk::Meta*)nullptr, a->gbits, a->vote, a->cap,
                      a->fail, a->ctr);
    if (!rc)
        rc = launch_k(f, "sb_compress", 0, sb::sb_compress_kernel, dim3(grid_for(a->cap, kMaxGrid)), dim3(256), 0, a->word,
                      a->out, a->cap, (const u32*)a->gbits, a->vote);
    if (!rc && a->want_counts) {  // diagnostics: the lists' lengths from the per-slice counts
        std::vector<u32> h(2 * levels * bk::kMaxBuckets);
        HIP_TRY(hipMemcpyAsync(h.data(), a->hist, h.size() * sizeof(u32), hipMemcpyDeviceToHost, f->stream));
        rc = stream_sync_checked(f);
        for (int i = 0; i < 6; ++i) a->counts[i] = 0;
        for (size_t i = 0; i < h.size(); ++i) a->counts[i / bk::kMaxBuckets] += h[i];
    }
    return rc;
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

int gcc_forest_label_digest(gcc_forest* h, uint64_t* digest, uint64_t* n_seen, uint64_t* n_components) {
    CHECK_ARG(h && digest, "null argument");
    DeviceGuard g(h->device);
    int rc = compress_async(h);
    if (rc) return rc;
    if (!h->d_counts) HIP_TRY(hipMalloc((void**)&h->d_counts, 3 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(h->d_counts, 0, 3 * sizeof(unsigned long long), h->stream));
    hipLaunchKernelGGL(digest_kernel, dim3(grid_for(h->cap, kMaxGrid)), dim3(kBlock), 0, h->stream, labels_ptr(h), h->cap,
                       h->d_counts);
    HIP_TRY(hipGetLastError());
    unsigned long long c[3];
    HIP_TRY(hipMemcpyAsync(c, h->d_counts, sizeof(c), hipMemcpyDeviceToHost, h->stream));
    rc = stream_sync_checked(h);
    if (rc) return rc;
    *digest = c[2];
    if (n_seen) *n_seen = c[0];
    if (n_components) *n_components = c[1];
    return GCC_OK;
}

const char* gcc_last_error(void) { return g_last_error.c_str(); }

int gcc_version(void) { return 1; }

int gcc_device_count(int* n) {
    CHECK_ARG(n, "n is null");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return GCC_OK;
}

int gcc_init(int device) {
    int rc = gcc_check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    HIP_TRY(hipFree(nullptr));
    return GCC_OK;
}

int gcc_gen_info(const gcc_gen_params* p, uint64_t* n_edges, uint64_t* n_vertices) {
    CHECK_ARG(p, "params is null");
    CHECK_ARG(p->kind >= GCC_GEN_EXAMPLE && p->kind <= GCC_GEN_ADVERSARIAL, "unknown generator kind");
    if (p->kind == GCC_GEN_RMAT) CHECK_ARG(p->scale >= 1 && p->scale <= 31, "rmat scale must be in [1,31]");
    if (p->kind == GCC_GEN_GNM) CHECK_ARG(p->n_vertices >= 1 && p->n_vertices < UNSEEN, "gnm n out of range");
    if (p->kind == GCC_GEN_ADVERSARIAL) {
        CHECK_ARG(p->scale >= 1 && p->scale <= 30, "adversarial path bits must be in [1,30]");
        CHECK_ARG(p->star_size >= 2, "adversarial star_size must be >= 2");
        CHECK_ARG(gcc_gen_num_vertices(p) < UNSEEN, "adversarial id range too large");
    }
    if (n_edges) *n_edges = gcc_gen_num_edges(p);
    if (n_vertices) *n_vertices = gcc_gen_num_vertices(p);
    return GCC_OK;
}

int gcc_gen_host(const gcc_gen_params* p, uint64_t first, uint64_t count, uint32_t* out_pairs) {
    int rc = gcc_gen_info(p, nullptr, nullptr);
    if (rc) return rc;
    CHECK_ARG(out_pairs || count == 0, "out_pairs is null");
    for (u64 i = 0; i < count; ++i) gcc_gen_edge(p, first + i, &out_pairs[2 * i], &out_pairs[2 * i + 1]);
    return GCC_OK;
}

int gcc_gen_device(const gcc_gen_params* p, uint64_t first, uint64_t count, uint32_t* d_out_pairs, void* hip_stream) {
    int rc = gcc_gen_info(p, nullptr, nullptr);
    if (rc) return rc;
    CHECK_ARG(d_out_pairs || count == 0, "d_out_pairs is null");
    if (count == 0) return GCC_OK;
    hipLaunchKernelGGL(gen_kernel, dim3(grid_for(count, 8192)), dim3(kBlock), 0, (hipStream_t)hip_stream, *p, first,
                       count, reinterpret_cast<uint2*>(d_out_pairs));
    HIP_TRY(hipGetLastError());
    return GCC_OK;
}

// Kernels with > 64 KiB of dynamic LDS must be allowed it explicitly, and the attribute belongs to the function's
// code object on ONE device: it is set once per device (std::call_once per device index: thread-safe for task
// threads creating forests on several GPUs at once), before the device's first forest exists.
constexpr int kMaxDevices = 64;
static std::once_flag g_attr_once[kMaxDevices];
static int g_attr_rc[kMaxDevices];
static std::string g_attr_msg[kMaxDevices];

// The kernel-start trace word (trace_start): one pinned, device-mapped host word for the process, its address set
// into gcc_trace_slot once per device (with the LDS attributes).
static u32* g_trace_host = nullptr;
static std::once_flag g_trace_once;

extern "C++" const char* gcc_fault_note(hipError_t e) {  // abi_common.h (C++ linkage, inside this extern "C" block)
    static thread_local char buf[96];
    if (e != hipErrorIllegalAddress && e != hipErrorLaunchFailure) return "";
    const u32 id = g_trace_host ? __atomic_load_n(g_trace_host, __ATOMIC_RELAXED) : 0u;
    snprintf(buf, sizeof(buf), " [last kernel started: %s]", id < kTrCount ? kTraceNames[id] : "?");
    return buf;
}

static int set_trace_slot() {  // the current device
    std::call_once(g_trace_once, [] {
        // opt-in (GELLY_TRACE=1): the system-scope store costs the shortest launches (C2 x 16: 0.259 vs 0.267 ms per
        // step, profiles/r6u_ab_kernel_start_trace.txt)
        const char* e = std::getenv("GELLY_TRACE");
        if (!e || !*e || e[0] == '0') return;
        if (hipHostMalloc((void**)&g_trace_host, 64, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
            g_trace_host = nullptr;
        else
            *g_trace_host = 0;
    });
    if (!g_trace_host) return GCC_OK;  // diagnostics only
    u32* dev = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&dev, g_trace_host, 0));
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(gcc_trace_slot), &dev, sizeof(dev)));
    return GCC_OK;
}

static int set_lds_attrs_impl() {
    const int filtered = (int)(kLdsBitmapMaxWords * sizeof(u64) + (kFilterBlockLds / 64) * kRing * sizeof(u64));
    const int bitmap = (int)(kLdsBitmapMaxWords * sizeof(u64));
    const struct {
        const void* f;
        int bytes;
    } tab[] = {
        {(const void*)compress_inc_kernel<false, false>, (int)(gcc::kBloomBits / 8)},
        {(const void*)compress_inc_kernel<true, false>, (int)(gcc::kBloomBits / 8)},
        {(const void*)compress_inc_kernel<false, true>, (int)(gcc::kBloomBits / 8)},
        {(const void*)compress_inc_kernel<true, true>, (int)(gcc::kBloomBits / 8)},
        {(const void*)compress_pipe_kernel, (int)(gcc::kBloomBits / 8)},
        {(const void*)sb::sb_filter_kernel, (int)(sb::kSliceW * sizeof(u32))},
        {(const void*)sb::sb_check_kernel<true>, (int)(sb::kSliceW * sizeof(u32))},
        {(const void*)sb::sb_check_kernel<false>, (int)(sb::kSliceW * sizeof(u32))},
        {(const void*)fold_filtered_kernel<true, kFilterBlockLds, 4, true, false>, filtered},
        {(const void*)fold_filtered_kernel<true, kFilterBlockLds, 8, true, false>, filtered},
        {(const void*)fold_filtered_kernel<true, kFilterBlockLds, 4, true, true>, filtered},
        {(const void*)fold_filtered_kernel<true, kFilterBlockLds, 8, true, true>, filtered},
        {(const void*)seed_hub_kernel, (int)(2 * kHubSlots * sizeof(u32))},
        {(const void*)seed_bfs_kernel<true, kFilterBlockLds, true, false>, bitmap},
        {(const void*)seed_bfs_kernel<true, kFilterBlockLds, false, false>, bitmap},
        {(const void*)seed_bfs_kernel<true, kFilterBlockLds, true, true>, bitmap},
        {(const void*)seed_bfs_kernel<true, kFilterBlockLds, false, true>, bitmap},
        {(const void*)bk::slice_filter_kernel<false>, (int)slice_filter_lds()},
        {(const void*)bk::slice_filter_kernel<true>, (int)slice_filter_lds()},
        {(const void*)bk::slice_filter_kernel<true, true>, (int)slice_filter_lds()},
        {(const void*)bk::slice_filter_kernel<true, false, 12>, (int)slice_filter_lds(12)},
        {(const void*)bk::slice_filter_kernel<true, false, 12, 8>, (int)slice_filter_lds(12, 8)},
        {(const void*)bk::slice_hook_kernel<false>, (int)(bk::kVSliceWords * sizeof(u32))},
        {(const void*)bk::slice_hook_kernel<true>, (int)(bk::kVSliceWords * sizeof(u32))},
        {(const void*)bk::bucket_hub_kernel, (int)(2 * kHubSlots * sizeof(u32))},
        {(const void*)bk::bucket_kernel<512, 16>, (int)bk::p1_lds(512, 16)},
        {(const void*)bk::bucket_kernel<1024, 16>, (int)bk::p1_lds(1024, 16)},
        {(const void*)bk::bucket_kernel<1024, 16, 256, 4, true>, (int)bk::p1_lds(1024, 16)},
        {(const void*)bk::bucket_kernel<1024, 12>, (int)bk::p1_lds(1024, 12)},
        {(const void*)bk::bucket_kernel<1024, 12, 512>, (int)bk::p1_lds(1024, 12, 512)},
        {(const void*)bk::bucket_kernel<1024, 16, 256, 8>, (int)bk::p1_lds(1024, 16, 256, 8)},
    };
    for (const auto& t : tab) HIP_TRY(hipFuncSetAttribute(t.f, hipFuncAttributeMaxDynamicSharedMemorySize, t.bytes));
    return set_trace_slot();
}

static int ensure_lds_attrs(int device) {  // `device` is current
    if (device < 0 || device >= kMaxDevices) return set_err(GCC_E_INVALID, "device %d beyond %d", device, kMaxDevices);
    std::call_once(g_attr_once[device], [device] {
        g_attr_rc[device] = set_lds_attrs_impl();
        if (g_attr_rc[device]) g_attr_msg[device] = g_last_error;
    });
    if (g_attr_rc[device]) return set_err(g_attr_rc[device], "%s", g_attr_msg[device].c_str());
    return GCC_OK;
}

static int forest_create_impl(int device, uint32_t id_capacity, uint32_t* d_buf0, uint32_t* d_buf1,
                              gcc_forest** out) {
    CHECK_ARG(out, "out is null");
    *out = nullptr;
    CHECK_ARG(id_capacity >= 1 && id_capacity <= UNSEEN, "id_capacity must be in [1, 0xFFFFFFFF]");
    int rc = gcc_check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    rc = ensure_lds_attrs(device);
    if (rc) return rc;
    gcc_forest* h = new gcc_forest();
    h->device = device;
    h->cap = id_capacity;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            h->n_cu = prop.multiProcessorCount;
    }
    auto fail = [&](int code) {
        gcc_forest_destroy(h);
        return code;
    };
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return fail(set_err(GCC_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e)));
    h->stream = h->own_stream;
    e = hipMalloc((void**)&h->d_err, sizeof(u32));
    if (e == hipSuccess) e = hipMemsetAsync(h->d_err, 0, sizeof(u32), h->stream);  // ordered before its kernels
    if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_err, sizeof(u32), hipHostMallocDefault);
    if (e != hipSuccess) return fail(set_err(GCC_E_HIP, "error word: %s", hipGetErrorString(e)));
    *h->h_err = 0;
    if (d_buf0) {
        h->d_parent = d_buf0;
        h->d_spare = d_buf1;
        h->own_bufs = false;
    } else {
        e = hipMalloc((void**)&h->d_parent, (size_t)id_capacity * sizeof(u32));
        if (e == hipSuccess) e = hipMalloc((void**)&h->d_spare, (size_t)id_capacity * sizeof(u32));
        if (e != hipSuccess) return fail(set_err(GCC_E_OOM, "hipMalloc 2 x u32[%u]: %s", id_capacity, hipGetErrorString(e)));
    }
    rc = gcc_forest_reset(h);
    if (rc) return fail(rc);
    *out = h;
    return GCC_OK;
}

int gcc_forest_create(int device, uint32_t id_capacity, gcc_forest** out) {
    return forest_create_impl(device, id_capacity, nullptr, nullptr, out);
}

int gcc_forest_create_ext(int device, uint32_t id_capacity, uint32_t* d_buf0, uint32_t* d_buf1, gcc_forest** out) {
    CHECK_ARG(d_buf0 && d_buf1 && d_buf0 != d_buf1, "need two distinct device buffers");
    CHECK_ARG(((reinterpret_cast<uintptr_t>(d_buf0) | reinterpret_cast<uintptr_t>(d_buf1)) & 15) == 0,
              "the id-range buffers must be 16-byte aligned (the compress moves 4 ids per 16-B access)");
    return forest_create_impl(device, id_capacity, d_buf0, d_buf1, out);
}

int gcc_forest_destroy(gcc_forest* h) {
    if (!h) return GCC_OK;
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->pipe_stream) {
        (void)hipStreamSynchronize(h->pipe_stream);
        (void)hipStreamDestroy(h->pipe_stream);
    }
    if (h->pipe_ev_fold) (void)hipEventDestroy(h->pipe_ev_fold);
    if (h->share_ev) (void)hipEventDestroy(h->share_ev);
    if (h->h_share) (void)hipHostFree(h->h_share);
    if (h->aux_stream) {
        (void)hipStreamSynchronize(h->aux_stream);
        (void)hipStreamDestroy(h->aux_stream);
    }
    for (int s = 0; s < 2; ++s)
        if (h->aux_ev[s]) (void)hipEventDestroy(h->aux_ev[s]);
    for (int s = 0; s < 2; ++s)
        if (h->pipe_ev_scan[s]) (void)hipEventDestroy(h->pipe_ev_scan[s]);
    if (h->d_pbloom) (void)hipFree(h->d_pbloom);
    if (h->d_touched) (void)hipFree(h->d_touched);
    if (h->d_pborn) (void)hipFree(h->d_pborn);
    if (h->d_proots) (void)hipFree(h->d_proots);
    for (int s = 0; s < 2; ++s) {
        if (h->h_stage[s]) (void)hipHostFree(h->h_stage[s]);
        if (h->d_stage[s]) (void)hipFree(h->d_stage[s]);
        if (h->stage_ev[s]) (void)hipEventDestroy(h->stage_ev[s]);
    }
    if (h->own_bufs) {
        if (h->d_parent) (void)hipFree(h->d_parent);
        if (h->d_spare) (void)hipFree(h->d_spare);
    }
    if (h->d_scratch) (void)hipFree(h->d_scratch);
    if (h->d_witness) (void)hipFree(h->d_witness);
    if (h->d_seg) (void)hipFree(h->d_seg);
    if (h->d_delta) (void)hipFree(h->d_delta);
    if (h->d_delta_cnt) (void)hipFree(h->d_delta_cnt);
    if (h->d_msg_oth) (void)hipFree(h->d_msg_oth);
    if (h->d_bits) (void)hipFree(h->d_bits);
    if (h->d_bloom) (void)hipFree(h->d_bloom);
    if (h->d_dbg) (void)hipFree(h->d_dbg);
    if (h->d_post) (void)hipFree(h->d_post);
    if (h->d_prev) (void)hipFree(h->d_prev);
    if (h->h_dbg) (void)hipHostFree(h->h_dbg);
    if (h->d_giant) (void)hipFree(h->d_giant);
    if (h->d_flags) (void)hipFree(h->d_flags);
    if (h->d_bmin) (void)hipFree(h->d_bmin);
    if (h->d_qcount) (void)hipFree(h->d_qcount);
    if (h->d_counts) (void)hipFree(h->d_counts);
    if (h->d_err) (void)hipFree(h->d_err);
    if (h->d_meta) (void)hipFree(h->d_meta);
    for (void* p : h->held_scratch) (void)hipFree(p);
    if (h->d_bk) (void)hipFree(h->d_bk);
    if (h->d_ovf) (void)hipFree(h->d_ovf);
    if (h->d_vl) (void)hipFree(h->d_vl);
    if (h->d_slow) (void)hipFree(h->d_slow);
    if (h->d_nbits) (void)hipFree(h->d_nbits);
    if (h->h_err) (void)hipHostFree(h->h_err);
    for (int s = 0; s < 2; ++s) {
        if (h->d_pin[s]) (void)hipFree(h->d_pin[s]);
        if (h->pin_copied[s]) (void)hipEventDestroy(h->pin_copied[s]);
        if (h->pin_folded[s]) (void)hipEventDestroy(h->pin_folded[s]);
    }
    if (h->copy_stream) {
        (void)hipStreamSynchronize(h->copy_stream);
        (void)hipStreamDestroy(h->copy_stream);
    }
    for (auto& pe : h->kev) {
        (void)hipEventDestroy(pe.first);
        (void)hipEventDestroy(pe.second);
    }
    if (h->h_segcount) (void)hipHostFree(h->h_segcount);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return GCC_OK;
}

int gcc_forest_set_stream(gcc_forest* h, void* hip_stream, int use_own) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    hipStream_t next = use_own ? h->own_stream : (hipStream_t)hip_stream;  // NULL = the device's null stream
    if (next != h->stream) {
        // order: everything already queued on the old stream happens before work on the new one
        hipEvent_t ev;
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev, h->stream));
        HIP_TRY(hipStreamWaitEvent(next, ev, 0));
        HIP_TRY(hipEventDestroy(ev));
        h->stream = next;
    }
    return GCC_OK;
}

int gcc_forest_get_stream(gcc_forest* h, void** hip_stream) {
    CHECK_ARG(h && hip_stream, "null argument");
    *hip_stream = (void*)h->stream;
    return GCC_OK;
}

int gcc_forest_capacity(gcc_forest* h, uint32_t* id_capacity) {
    CHECK_ARG(h && id_capacity, "null argument");
    *id_capacity = h->cap;
    return GCC_OK;
}

int gcc_forest_device(gcc_forest* h, int* device) {
    CHECK_ARG(h && device, "null argument");
    *device = h->device;
    return GCC_OK;
}

int gcc_forest_device_ptr(gcc_forest* h, uint32_t** d_parent) {
    CHECK_ARG(h && d_parent, "null argument");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    // the caller may write through the pointer: nothing cached about parent[] holds any more (no incremental
    // compress until a full one; the next read compresses and re-reads)
    mark_mutated(h);
    *d_parent = h->d_parent;
    return GCC_OK;
}

int gcc_forest_labels_device(gcc_forest* h, const uint32_t** d_labels) {
    CHECK_ARG(h && d_labels, "null argument");
    DeviceGuard g(h->device);
    int rc = compress_async(h);  // read-only view: the forest's caches (rec_all, compressed) stay valid
    if (rc) return rc;
    *d_labels = labels_ptr(h);
    return GCC_OK;
}

int gcc_forest_reset(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = pipe_exit(h);
    if (rc) return rc;
    h->pipe_roots_stale = true;  // a root of the new forest may have been touched in the old one
    h->staged = 0;
    h->pending_reset = true;  // materialised lazily (see gcc_forest::pending_reset)
    h->rec_all = false;
    h->host_valid = false;
    ++h->version;
    h->compressed = true;  // all UNSEEN is canonical
    h->has_giant = false;  // the giant bitmap described the old forest
    h->filter_off = false;
    h->share_unchecked = false;
    h->share_pending = false;
    h->edges_since_compress = 0;
    h->delta_armed = false;
    return GCC_OK;
}

int gcc_forest_staging(gcc_forest* h, uint32_t** pairs, uint64_t* cap_edges) {
    CHECK_ARG(h && pairs && cap_edges, "null argument");
    DeviceGuard g(h->device);
    int rc = alloc_staging(h);
    if (rc) return rc;
    *pairs = h->h_stage[h->slot];
    *cap_edges = gcc_forest::kStageEdges;
    return GCC_OK;
}

int gcc_forest_submit(gcc_forest* h, uint64_t n_edges) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(n_edges <= gcc_forest::kStageEdges, "n_edges exceeds the staging capacity");
    DeviceGuard g(h->device);
    int rc = alloc_staging(h);
    if (rc) return rc;
    // validate ids on the host: a bad id would be an out-of-bounds device access
    const u32* p = h->h_stage[h->slot];
    for (u64 i = 0; i < 2 * n_edges; ++i)
        if (p[i] >= h->cap) return set_err(GCC_E_INVALID, "vertex id %u >= id_capacity %u", p[i], h->cap);
    h->staged = 0;
    return submit_slot(h, n_edges);
}

int gcc_forest_union(gcc_forest* h, uint32_t u, uint32_t v) {
    CHECK_ARG(h, "null forest");
    if (u >= h->cap || v >= h->cap) return set_err(GCC_E_INVALID, "vertex id >= id_capacity %u", h->cap);
    DeviceGuard g(h->device);
    int rc = alloc_staging(h);
    if (rc) return rc;
    u32* s = h->h_stage[h->slot];
    s[2 * h->staged] = u;
    s[2 * h->staged + 1] = v;
    h->staged++;
    h->host_valid = false;
    ++h->version;
    if (h->staged == gcc_forest::kStageEdges) return submit_slot(h, h->staged);
    return GCC_OK;
}

int gcc_forest_make_set(gcc_forest* h, uint32_t v) { return gcc_forest_union(h, v, v); }

int gcc_forest_fold_host(gcc_forest* h, const uint32_t* pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(pairs || n_edges == 0, "pairs is null");
    DeviceGuard g(h->device);
    int rc = alloc_staging(h);
    if (rc) return rc;
    u64 done = 0;
    while (done < n_edges) {
        const u64 room = gcc_forest::kStageEdges - h->staged;
        const u64 take = std::min(room, n_edges - done);
        u32* dst = h->h_stage[h->slot] + 2 * h->staged;
        const u32* src = pairs + 2 * done;
        for (u64 i = 0; i < 2 * take; ++i) {
            const u32 x = src[i];
            if (x >= h->cap) return set_err(GCC_E_INVALID, "vertex id %u >= id_capacity %u", x, h->cap);
            dst[i] = x;
        }
        h->staged += take;
        done += take;
        if (h->staged == gcc_forest::kStageEdges) {
            rc = submit_slot(h, h->staged);
            if (rc) return rc;
        }
    }
    h->host_valid = false;
    ++h->version;
    return flush_fold(h);
}

int gcc_forest_fold_device(gcc_forest* h, const uint32_t* d_pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(d_pairs || n_edges == 0, "d_pairs is null");
    DeviceGuard g(h->device);
    int rc = flush_staged(h);
    if (rc) return rc;
    return launch_fold(h, d_pairs, n_edges);
}

// Pinned host batch (the JNI / FFM direct-buffer path): chunks (tune.pin_chunk edges) go H2D on the handle's copy
// stream into two device slots while the previous chunk folds on the handle's stream; ids are validated on the
// device (edge_ok). Each chunk is one batch of the fold pipeline. Asynchronous: `pairs` must stay valid until the
// next synchronising call.

int gcc_forest_fold_pinned(gcc_forest* h, const uint32_t* pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(pairs || n_edges == 0, "pairs is null");
    DeviceGuard g(h->device);
    int rc = flush_staged(h);
    if (rc) return rc;
    if (n_edges == 0) return GCC_OK;
    const u64 chunk = std::min<u64>(n_edges, std::max<u64>(1024, h->tune.pin_chunk));
    if (!h->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
    if (!h->pin_copied[0]) {
        for (int s = 0; s < 2; ++s) {
            HIP_TRY(hipEventCreateWithFlags(&h->pin_copied[s], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&h->pin_folded[s], hipEventDisableTiming));
            HIP_TRY(hipEventRecord(h->pin_folded[s], h->stream));
        }
    }
    if (h->pin_cap < chunk) {  // grow the slots (both streams idle first: a slot may still be read)
        HIP_TRY(hipStreamSynchronize(h->stream));
        HIP_TRY(hipStreamSynchronize(h->copy_stream));
        for (int s = 0; s < 2; ++s) {
            if (h->d_pin[s]) HIP_TRY(hipFree(h->d_pin[s]));
            h->d_pin[s] = nullptr;
        }
        h->pin_cap = 0;
        for (int s = 0; s < 2; ++s) HIP_TRY(hipMalloc((void**)&h->d_pin[s], (size_t)chunk * 2 * sizeof(u32)));
        h->pin_cap = chunk;
    }
    for (u64 b = 0, k = 0; b < n_edges; b += chunk, ++k) {
        const int s = (int)(k & 1);
        const u64 m = std::min<u64>(chunk, n_edges - b);
        HIP_TRY(hipStreamWaitEvent(h->copy_stream, h->pin_folded[s], 0));  // the slot's last fold is done
        HIP_TRY(hipMemcpyAsync(h->d_pin[s], pairs + 2 * b, (size_t)m * 2 * sizeof(u32), hipMemcpyHostToDevice,
                               h->copy_stream));
        HIP_TRY(hipEventRecord(h->pin_copied[s], h->copy_stream));
        HIP_TRY(hipStreamWaitEvent(h->stream, h->pin_copied[s], 0));
        rc = launch_fold(h, h->d_pin[s], m);
        if (rc) return rc;
        HIP_TRY(hipEventRecord(h->pin_folded[s], h->stream));
    }
    h->host_valid = false;
    ++h->version;
    return GCC_OK;
}

int gcc_forest_flush(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    return flush_fold(h);
}

int gcc_forest_sync(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = flush_fold(h);
    if (!rc) rc = pipe_labels_ready(h);  // and the last window's scan
    if (rc) return rc;
    return stream_sync_checked(h);
}

int gcc_forest_merge_labels_device(gcc_forest* into, const uint32_t* d_labels, uint32_t n) {
    CHECK_ARG(into, "null forest");
    CHECK_ARG(d_labels || n == 0, "d_labels is null");
    CHECK_ARG(n <= into->cap, "labels longer than id_capacity");
    DeviceGuard g(into->device);
    int rc = flush(into);
    if (rc) return rc;
    if (n == 0) return GCC_OK;
    hipLaunchKernelGGL(merge_labels_kernel, dim3(grid_for(n, kMaxGrid)), dim3(kBlock), 0, into->stream, into->d_parent,
                       d_labels, n, into->cap, into->d_err);
    HIP_TRY(hipGetLastError());
    into->host_valid = false;
    ++into->version;
    into->compressed = false;
    into->rec_all = false;
    into->delta_armed = false;
    return GCC_OK;
}

int gcc_forest_merge(gcc_forest* into, gcc_forest* from) {
    CHECK_ARG(into && from, "null forest");
    if (into == from) return GCC_OK;
    CHECK_ARG(from->cap <= into->cap, "merge source has a larger id range than the target");
    {
        DeviceGuard g(from->device);
        int rc = flush(from);
        if (rc) return rc;
    }
    DeviceGuard g(into->device);
    int rc = flush(into);
    if (rc) return rc;
    // Two events, each created on the device whose stream records it: ev_from orders into's stream after everything
    // queued on from's stream; ev_into orders from's stream after the merge has read from's parent[] (from must
    // not be mutated before). Both are destroyed on every path.
    hipEvent_t ev_from = nullptr, ev_into = nullptr;
    auto done = [&](int code) {
        if (ev_from) {
            DeviceGuard gf(from->device);
            (void)hipEventDestroy(ev_from);
        }
        if (ev_into) (void)hipEventDestroy(ev_into);
        return code;
    };
    auto hip = [&](hipError_t e, const char* what) {
        return e == hipSuccess ? GCC_OK : set_err(GCC_E_HIP, "gcc_forest_merge: %s: %s", what, hipGetErrorString(e));
    };
    {
        DeviceGuard gf(from->device);
        rc = hip(hipEventCreateWithFlags(&ev_from, hipEventDisableTiming), "event (from)");
        if (!rc) rc = hip(hipEventRecord(ev_from, from->stream), "record (from)");
    }
    if (!rc) rc = hip(hipEventCreateWithFlags(&ev_into, hipEventDisableTiming), "event (into)");
    if (!rc) rc = hip(hipStreamWaitEvent(into->stream, ev_from, 0), "wait (into)");
    if (rc) return done(rc);
    const u32* src = from->d_parent;
    if (from->device != into->device) {
        if (!into->d_scratch) rc = hip(hipMalloc((void**)&into->d_scratch, (size_t)into->cap * sizeof(u32)), "scratch");
        if (!rc)
            rc = hip(hipMemcpyPeerAsync(into->d_scratch, into->device, from->d_parent, from->device,
                                        (size_t)from->cap * sizeof(u32), into->stream), "peer copy");
        src = into->d_scratch;
    }
    if (!rc) rc = gcc_forest_merge_labels_device(into, src, from->cap);
    // whatever was enqueued on into's stream, from waits for it before its next mutation
    int rc2 = hip(hipEventRecord(ev_into, into->stream), "record (into)");
    if (!rc2) {
        DeviceGuard gf(from->device);
        rc2 = hip(hipStreamWaitEvent(from->stream, ev_into, 0), "wait (from)");
    }
    return done(rc ? rc : rc2);
}

uint64_t gcc_msg_bytes(uint32_t id_capacity, uint64_t cap_others) {
    return GCC_MSG_HEADER_BYTES + (((u64)id_capacity + 63) / 64) * sizeof(u64) + cap_others * 2 * sizeof(u32);
}

int gcc_forest_encode(gcc_forest* h, void* d_msg, uint64_t cap_others) {
    CHECK_ARG(h && d_msg, "null argument");
    CHECK_ARG((reinterpret_cast<uintptr_t>(d_msg) & 15) == 0, "message buffer must be 16-byte aligned");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    u32* hdr = reinterpret_cast<u32*>(d_msg);
    u64* bits = reinterpret_cast<u64*>(static_cast<char*>(d_msg) + GCC_MSG_HEADER_BYTES);
    const u64 nw = ((u64)h->cap + 63) / 64;
    u32* others = reinterpret_cast<u32*>(bits + nw);
    const u32 nb = (u32)((nw + kMsgWordsPerBlock - 1) / kMsgWordsPerBlock);
    if (!h->d_witness) HIP_TRY(hipMalloc((void**)&h->d_witness, kMaxPeers * sizeof(u32)));
    if ((rc = ensure_msg_scratch(h))) return rc;
    u32* cnt = reinterpret_cast<u32*>(h->d_msg_oth + nw);
    u32* base = cnt + nb;
    // An uncompressed forest is compressed first, by a compress that also writes the others' masks (one pass
    // over parent[]), so the encode only reads the 8-B masks. Without the giant filter (no masks from the
    // compress), it is encoded from its parent pointers (read-only finds). Either way the forest's
    // tracked-component bitmap and root end up exactly what the encode saw, so an absorb right after it can take
    // "seen" = bitmap | the others' masks without loading parent[].
    bool masks = false;
    if (!h->compressed && h->filter_enabled()) {
        rc = compress_now(h, "compress", h->d_msg_oth, &masks);
        if (rc) return rc;
    } else if (h->compressed && h->mask_version == h->version) {
        masks = true;  // the last compress (a bucketed fold's closing one) wrote them and nothing changed since
    }
    const bool find = !h->compressed;
    const bool track = h->has_giant && h->d_bits && h->d_giant;
    hipLaunchKernelGGL(msg_header_kernel, dim3(1), dim3(kMaxPeers), 0, h->stream, hdr,
                       h->d_giant ? h->d_giant + h->giant_slot : hdr, h->has_giant ? 1u : 0u, h->cap, h->d_witness,
                       (const u32*)h->d_parent, track ? h->d_giant + (h->giant_slot ^ 1) : nullptr);
    if ((rc = msg_launched(h, "msg_header_kernel"))) return rc;
    h->witness_armed = true;
    u64* mine = track ? h->d_bits : nullptr;
    const u32* gprev = track ? (const u32*)(h->d_giant + h->giant_slot) : nullptr;
    if (masks && track) {
        hipLaunchKernelGGL(msg_cnt_kernel, dim3(nb), dim3(kBlock), 0, h->stream, (const u64*)h->d_msg_oth,
                           (const u64*)h->d_bits, bits, nw, cnt);
        if ((rc = msg_launched(h, "msg_cnt_kernel"))) return rc;
    }
    else if (find) {
        hipLaunchKernelGGL(msg_count_kernel<true>, dim3(nb), dim3(kMsgBlock), 0, h->stream, (const u32*)h->d_parent,
                           h->cap, (const u32*)hdr, gprev, bits, mine, h->d_msg_oth, cnt);
        if ((rc = msg_launched(h, "msg_count_kernel"))) return rc;
    }
    else {
        hipLaunchKernelGGL(msg_count_kernel<false>, dim3(nb), dim3(kMsgBlock), 0, h->stream, (const u32*)h->d_parent,
                           h->cap, (const u32*)hdr, gprev, bits, mine, h->d_msg_oth, cnt);
        if ((rc = msg_launched(h, "msg_count_kernel"))) return rc;
    }
    hipLaunchKernelGGL(msg_scan_kernel, dim3(1), dim3(kScanBlock), 0, h->stream, (const u32*)cnt, nb, base, hdr);
    if ((rc = msg_launched(h, "msg_scan_kernel"))) return rc;
    if (find) {
        hipLaunchKernelGGL(msg_write_kernel<true>, dim3(nb), dim3(kBlock), 0, h->stream, (const u32*)h->d_parent, h->cap,
                           (const u64*)h->d_msg_oth, (const u32*)base, (const u32*)hdr, gprev, others, (u64)cap_others);
        if ((rc = msg_launched(h, "msg_write_kernel"))) return rc;
    }
    else {
        hipLaunchKernelGGL(msg_write_kernel<false>, dim3(nb), dim3(kBlock), 0, h->stream, (const u32*)h->d_parent, h->cap,
                           (const u64*)h->d_msg_oth, (const u32*)base, (const u32*)hdr, gprev, others, (u64)cap_others);
        if ((rc = msg_launched(h, "msg_write_kernel"))) return rc;
    }
    HIP_TRY(hipGetLastError());
    if (track) h->giant_slot ^= 1;  // the header kernel stored the tracked component's current root there
    h->enc_version = h->version;
    return GCC_OK;
}

int gcc_forest_absorb_many(gcc_forest* h, const void* d_msgs, uint64_t stride_bytes, uint32_t count, uint32_t skip,
                           uint64_t cap_others) {
    CHECK_ARG(h && (d_msgs || count == 0), "null argument");
    CHECK_ARG(((reinterpret_cast<uintptr_t>(d_msgs) | stride_bytes) & 15) == 0, "messages must be 16-byte aligned");
    CHECK_ARG(count <= 1 || stride_bytes >= gcc_msg_bytes(h->cap, cap_others), "stride smaller than a message");
    CHECK_ARG(count <= kMaxPeers, "at most 64 messages per call");
    if (h->tune.fail_absorb > 0 && --h->tune.fail_absorb == 0)
        return set_err(GCC_E_INTERNAL, "gcc_forest_absorb_many: injected failure (tune key fail_absorb)");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    if (count == 0 || (count == 1 && skip == 0)) return GCC_OK;
    const u64 nw = ((u64)h->cap + 63) / 64;
    const bool tracked = h->has_giant && h->d_bits;
    const u64* mine = tracked ? h->d_bits : nullptr;
    const char* msgs = static_cast<const char*>(d_msgs);
    if (tracked) {
        if (!h->d_witness) HIP_TRY(hipMalloc((void**)&h->d_witness, kMaxPeers * sizeof(u32)));
        if (!h->witness_armed) HIP_TRY(hipMemsetAsync(h->d_witness, 0xFF, kMaxPeers * sizeof(u32), h->stream));
        h->witness_armed = false;
        hipLaunchKernelGGL(msg_overlap_kernel, dim3(grid_for((u64)count * ((nw + 63) / 64) * 64, kMaxGrid)), dim3(kBlock),
                           0, h->stream, msgs, (u64)stride_bytes, count, skip, h->cap, mine, h->d_witness);
        if ((rc = msg_launched(h, "msg_overlap_kernel"))) return rc;
    }
    // one list entry per lane; with no tracked component every giant goes id by id too (one word per wave)
    const u64 lists = std::max<u64>((u64)count * cap_others, 1);
    const u64 work = tracked ? std::max<u64>(lists, 64 * kBlock) : std::max<u64>(nw * 64, lists);
    // With the encode's masks (this forest's seen ids outside T), the new ids above R are not stored one by one:
    // they go into `newbits` (the masks' words, overwritten) and the compress that follows right here labels them
    // with R's root as it writes every label anyway (one pass over parent[] less). Until that compress the forest
    // is not a valid forest: it runs before this call returns.
    const bool masks = tracked && h->d_msg_oth && h->enc_version == h->version;
    u64* newbits = (masks && h->filter_enabled()) ? h->d_msg_oth : nullptr;
    const u32* troot = tracked ? (const u32*)(h->d_giant + h->giant_slot) : nullptr;
    if (tracked) {
        hipLaunchKernelGGL(msg_absorb_bits_kernel, dim3(grid_for(nw * 64, kMaxGrid)), dim3(kBlock), 0, h->stream,
                           h->d_parent, msgs, (u64)stride_bytes, count, skip, h->cap, mine, troot,
                           (const u32*)h->d_witness, masks ? (const u64*)h->d_msg_oth : nullptr, newbits);
        if ((rc = msg_launched(h, "msg_absorb_bits_kernel"))) return rc;
    }
    hipLaunchKernelGGL(msg_absorb_kernel, dim3(grid_for(work, kMaxGrid)), dim3(kBlock), 0, h->stream, h->d_parent, msgs,
                       (u64)stride_bytes, count, skip, (u64)cap_others, h->cap, tracked,
                       tracked ? (const u32*)h->d_witness : nullptr, (const u64*)newbits, troot);
    if ((rc = msg_launched(h, "msg_absorb_kernel"))) return rc;
    HIP_TRY(hipGetLastError());
    mark_mutated(h);
    if (newbits) return compress_now(h, "compress", nullptr, nullptr, newbits);
    return GCC_OK;
}

// ---- the delta merge (round 6; include/gelly_cc.h) ---------------------------------------------------
uint64_t gcc_delta_msg_bytes(uint64_t cap_pairs) { return GCC_MSG_HEADER_BYTES + 8 * cap_pairs; }

int gcc_forest_delta_arm(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    if (!h->d_delta_cnt) HIP_TRY(hipMalloc((void**)&h->d_delta_cnt, (kDeltaStripes + 1) * sizeof(u32)));
    if (!h->delta_cnt_zero) HIP_TRY(hipMemsetAsync(h->d_delta_cnt, 0, (kDeltaStripes + 1) * sizeof(u32), h->stream));
    h->delta_cnt_zero = true;
    h->delta_need = 0;
    h->delta_edges = 0;
    h->delta_armed = !h->pending_reset;  // a pending reset is a mutation no list records
    return GCC_OK;
}

int gcc_forest_encode_delta(gcc_forest* h, void* d_msg, uint64_t cap_pairs) {
    CHECK_ARG(h && d_msg, "null argument");
    CHECK_ARG((reinterpret_cast<uintptr_t>(d_msg) & 15) == 0, "message buffer must be 16-byte aligned");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    const bool armed = h->delta_armed && h->d_delta && h->d_delta_cnt;
    const u64 bound = armed ? std::min<u64>(cap_pairs, (u64)kDeltaStripes * h->delta_subcap) : 0;
    hipLaunchKernelGGL(delta_encode_kernel, dim3(grid_for(std::max<u64>(bound, 1), kMaxGrid)), dim3(kBlock), 0, h->stream,
                       (const u32*)h->d_parent, (const u32*)h->d_delta, (const u32*)h->d_delta_cnt, h->delta_subcap,
                       static_cast<u32*>(d_msg), (u64)cap_pairs, h->cap,
                       (u32)std::min<u64>(h->delta_edges, 0xFFFFFFFFull), armed ? 1u : 0u);
    return msg_launched(h, "delta_encode_kernel");
}

int gcc_forest_absorb_delta_many(gcc_forest* h, const void* d_msgs, uint64_t stride_bytes, uint32_t count, uint32_t skip,
                                 uint64_t cap_pairs) {
    CHECK_ARG(h && (d_msgs || count == 0), "null argument");
    CHECK_ARG(((reinterpret_cast<uintptr_t>(d_msgs) | stride_bytes) & 15) == 0, "messages must be 16-byte aligned");
    CHECK_ARG(count <= 1 || stride_bytes >= gcc_delta_msg_bytes(cap_pairs), "stride smaller than a message");
    if (h->tune.fail_absorb > 0 && --h->tune.fail_absorb == 0)
        return set_err(GCC_E_INTERNAL, "gcc_forest_absorb_delta_many: injected failure (tune key fail_absorb)");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    // the unions keep the incremental compress's bloom complete when it is (rec_all): the next compress stays incremental
    const bool bloom = h->rec_all && h->d_bloom && inc_forest(h);
    const u64 work = std::max<u64>((u64)count * cap_pairs, 1);
    if (bloom)
        hipLaunchKernelGGL(delta_absorb_kernel<true>, dim3(grid_for(work, kMaxGrid)), dim3(kBlock), 0, h->stream, h->d_parent,
                           static_cast<const char*>(d_msgs), (u64)stride_bytes, count, skip, (u64)cap_pairs, h->cap,
                           h->bloom(h->bloom_cur), h->d_delta_cnt, h->d_err);
    else
        hipLaunchKernelGGL(delta_absorb_kernel<false>, dim3(grid_for(work, kMaxGrid)), dim3(kBlock), 0, h->stream,
                           h->d_parent, static_cast<const char*>(d_msgs), (u64)stride_bytes, count, skip, (u64)cap_pairs,
                           h->cap, (u32*)nullptr, h->d_delta_cnt, h->d_err);
    if ((rc = msg_launched(h, "delta_absorb_kernel"))) return rc;
    mark_mutated(h, bloom);
    h->delta_armed = false;  // the caller arms it again once the merge is complete (gcc_forest_delta_arm)
    if (h->d_delta_cnt) h->delta_cnt_zero = true;  // the absorb zeroed this forest's stripe counters
    return GCC_OK;
}

int gcc_forest_absorb(gcc_forest* h, const void* d_msg, uint64_t cap_others) {
    return gcc_forest_absorb_many(h, d_msg, 0, 1, UINT32_MAX, cap_others);
}

// ---- serialized summary (Merger.snapshotState / restoreState; the bytes Kryo ships for a DisjointSet) ----------
// Layout (include/gelly_cc.h): a 32-byte header {magic, version, id_capacity, kind, n_seen, payload bytes}, then
// kind 1: n_seen (v, label) u32 pairs in id order; kind 2: the compact merge message with cap_others = its count.
// serialize picks the smaller form (the message when one component dominates: ~V/8 bytes + the other ids).
struct SerHeader {
    u32 magic, version, id_capacity, kind;
    u64 n_seen, payload;
};
static_assert(sizeof(SerHeader) == GCC_SER_HEADER_BYTES, "serialized header");

static int ser_plan(gcc_forest* h, u32* kind, u64* n_seen, u64* n_others, u64* payload) {
    unsigned long long c[2];
    int rc = counts(h, c);  // flush + exact #seen
    if (rc) return rc;
    *n_seen = c[0];
    rc = compress_async(h);
    if (rc) return rc;
    // the message's true list length: an encode with capacity 0 still counts every other id into its header
    const u64 hdr_only = gcc_msg_bytes(h->cap, 0);
    u8* tmp = nullptr;
    HIP_TRY(hipMalloc((void**)&tmp, (size_t)hdr_only));
    rc = gcc_forest_encode(h, tmp, 0);
    u32 hdr[4] = {0, 0, 0, 0};
    if (!rc) {
        hipError_t e = hipMemcpyAsync(hdr, tmp, sizeof(hdr), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) rc = set_err(GCC_E_HIP, "serialize: %s", hipGetErrorString(e));
    }
    (void)hipFree(tmp);
    if (rc) return rc;
    *n_others = hdr[1];
    const u64 msg = gcc_msg_bytes(h->cap, *n_others), pairs = 8ull * *n_seen;
    *kind = (h->has_giant && msg < pairs) ? 2u : 1u;
    *payload = *kind == 2 ? msg : pairs;
    return GCC_OK;
}

int gcc_forest_serialized_size(gcc_forest* h, uint64_t* bytes) {
    CHECK_ARG(h && bytes, "null argument");
    DeviceGuard g(h->device);
    u32 kind;
    u64 n_seen, n_others, payload;
    int rc = ser_plan(h, &kind, &n_seen, &n_others, &payload);
    if (rc) return rc;
    *bytes = GCC_SER_HEADER_BYTES + payload;
    return GCC_OK;
}

int gcc_forest_serialize(gcc_forest* h, void* out, uint64_t size, uint64_t* written) {
    CHECK_ARG(h && out, "null argument");
    DeviceGuard g(h->device);
    u32 kind;
    u64 n_seen, n_others, payload;
    int rc = ser_plan(h, &kind, &n_seen, &n_others, &payload);
    if (rc) return rc;
    if (size < GCC_SER_HEADER_BYTES + payload)
        return set_err(GCC_E_INVALID, "serialize: buffer of %llu bytes, need %llu", (unsigned long long)size,
                       (unsigned long long)(GCC_SER_HEADER_BYTES + payload));
    SerHeader hd{GCC_SER_MAGIC, 1u, h->cap, kind, n_seen, payload};
    std::memcpy(out, &hd, sizeof(hd));
    u8* body = static_cast<u8*>(out) + GCC_SER_HEADER_BYTES;
    if (kind == 2) {  // the message, straight from the device
        u8* d = nullptr;
        HIP_TRY(hipMalloc((void**)&d, (size_t)payload));
        rc = gcc_forest_encode(h, d, n_others);
        hipError_t e = hipSuccess;
        if (!rc) e = hipMemcpyAsync(body, d, (size_t)payload, hipMemcpyDeviceToHost, h->stream);
        if (!rc && e == hipSuccess) e = hipStreamSynchronize(h->stream);
        (void)hipFree(d);
        if (rc) return rc;
        if (e != hipSuccess) return set_err(GCC_E_HIP, "serialize: %s", hipGetErrorString(e));
    } else {  // (v, label) of every seen id, in id order
        rc = refresh_host(h);
        if (rc) return rc;
        u32* p = reinterpret_cast<u32*>(body);
        u64 k = 0;
        for (u32 v = 0; v < h->cap && k < n_seen; ++v)
            if (h->host_labels[v] != UNSEEN) {
                p[2 * k] = v;
                p[2 * k + 1] = h->host_labels[v];
                ++k;
            }
    }
    if (written) *written = GCC_SER_HEADER_BYTES + payload;
    return GCC_OK;
}

int gcc_forest_deserialize(gcc_forest* h, const void* in, uint64_t size) {
    CHECK_ARG(h && in, "null argument");
    CHECK_ARG(size >= GCC_SER_HEADER_BYTES, "serialized summary shorter than its header");
    SerHeader hd;
    std::memcpy(&hd, in, sizeof(hd));
    CHECK_ARG(hd.magic == GCC_SER_MAGIC && hd.version == 1, "not a serialized gelly summary (magic / version)");
    CHECK_ARG(hd.id_capacity <= h->cap, "serialized summary has a larger id range than the forest");
    // compared without arithmetic on the untrusted fields (a wrapped n_seen or payload must not pass)
    CHECK_ARG(hd.payload <= size - GCC_SER_HEADER_BYTES, "serialized summary truncated");
    DeviceGuard g(h->device);
    const u8* body = static_cast<const u8*>(in) + GCC_SER_HEADER_BYTES;
    if (hd.kind == 1) {
        CHECK_ARG(hd.payload % 8 == 0 && hd.n_seen == hd.payload / 8 && hd.n_seen <= (u64)hd.id_capacity,
                  "serialized pairs: bad length");
        return gcc_forest_fold_host(h, reinterpret_cast<const u32*>(body), hd.n_seen);  // ids validated there
    }
    CHECK_ARG(hd.kind == 2, "serialized summary: unknown kind");
    CHECK_ARG(hd.id_capacity == h->cap, "a serialized message restores into a forest of the same id range only");
    CHECK_ARG(hd.payload >= GCC_MSG_HEADER_BYTES, "serialized message: bad length");
    u32 mh[4];
    std::memcpy(mh, body, sizeof(mh));
    const u64 n_others = mh[1];
    CHECK_ARG(mh[2] == h->cap && hd.payload == gcc_msg_bytes(h->cap, n_others) &&
                  (mh[0] == UNSEEN || mh[0] < h->cap),
              "serialized message: inconsistent header");
    u8* d = nullptr;
    HIP_TRY(hipMalloc((void**)&d, (size_t)hd.payload));
    hipError_t e = hipMemcpyAsync(d, body, (size_t)hd.payload, hipMemcpyHostToDevice, h->stream);
    int rc = e == hipSuccess ? gcc_forest_absorb(h, d, n_others) : set_err(GCC_E_HIP, "%s", hipGetErrorString(e));
    if (!rc) rc = stream_sync_checked(h);  // the staging buffer is freed below
    (void)hipFree(d);
    return rc;
}

int gcc_forest_compress(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    // lazy emission (FoldTune::emit_div): in the plain regime the forest itself is the emitted summary until the edges
    // folded since the last compress reach id_capacity / emit_div
    if (h->tune.emit_div > 0 && !h->pipe && !h->compressed && (!h->filter_enabled() || h->filter_off) &&
        h->edges_since_compress * (u64)h->tune.emit_div < (u64)h->cap)
        return flush_fold(h);
    if (h->tune.emit_filtered && !h->pipe && !h->compressed && h->filter_enabled() && !h->filter_off && h->has_giant) {
        int rc = flush_fold(h);
        return rc ? rc : refresh_now(h);
    }
    return compress_async(h, false);
}

int gcc_forest_labels(gcc_forest* h, uint32_t* out, uint32_t n) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(out || n == 0, "out is null");
    CHECK_ARG(n <= h->cap, "n exceeds id_capacity");
    DeviceGuard g(h->device);
    int rc = refresh_host(h);
    if (rc) return rc;
    std::memcpy(out, h->host_labels.data(), (size_t)n * sizeof(u32));
    return GCC_OK;
}

int gcc_forest_raw_parent(gcc_forest* h, uint32_t* out, uint32_t n) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(out || n == 0, "out is null");
    CHECK_ARG(n <= h->cap, "n exceeds id_capacity");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, h->d_parent, (size_t)n * sizeof(u32), hipMemcpyDeviceToHost, h->stream));
    return stream_sync_checked(h);
}

int gcc_forest_find(gcc_forest* h, uint32_t v, uint32_t* root) {
    CHECK_ARG(h && root, "null argument");
    if (v >= h->cap) {
        *root = UNSEEN;  // outside the id range: never seen (DisjointSet.find returns null)
        return GCC_OK;
    }
    DeviceGuard g(h->device);
    int rc = refresh_host(h);
    if (rc) return rc;
    *root = h->host_labels[v];
    return GCC_OK;
}

int gcc_forest_size(gcc_forest* h, uint64_t* n_seen) {
    CHECK_ARG(h && n_seen, "null argument");
    DeviceGuard g(h->device);
    unsigned long long c[2];
    int rc = counts(h, c);
    if (rc) return rc;
    *n_seen = c[0];
    return GCC_OK;
}

int gcc_forest_count_components(gcc_forest* h, uint64_t* n_components) {
    CHECK_ARG(h && n_components, "null argument");
    DeviceGuard g(h->device);
    unsigned long long c[2];
    int rc = counts(h, c);
    if (rc) return rc;
    *n_components = c[1];
    return GCC_OK;
}

int gcc_forest_import_pairs(gcc_forest* h, const uint32_t* pairs, uint64_t n_pairs) {
    return gcc_forest_fold_host(h, pairs, n_pairs);
}

int gcc_forest_enable_timing(gcc_forest* h, int enable) {
    CHECK_ARG(h, "null forest");
    h->timing = enable < 0 ? 0 : (enable > 2 ? 2 : enable);
    return GCC_OK;
}

int gcc_forest_tune(gcc_forest* h, const char* key, double value) {
    CHECK_ARG(h && key, "null argument");
    if (h->pipe) {  // a knob may change the regime: the pipelined emission ends first
        DeviceGuard g(h->device);
        if (int rc = pipe_exit(h)) return rc;
    }
    FoldTune& t = h->tune;
    const std::string k(key);
    if (k == "filter") t.filter = value != 0;
    else if (k == "filter_min_batch") t.filter_min_batch = (u64)value;
    else if (k == "sample_first") t.sample_first = (u64)value;
    else if (k == "sample_growth") t.sample_growth = (u64)value;
    else if (k == "sample_div") t.sample_div = (u64)value;
    else if (k == "sample_min") t.sample_min = (u64)value;
    else if (k == "refresh_min_batch") t.refresh_min_batch = (u64)value;
    else if (k == "refresh1") t.refresh[0] = value;
    else if (k == "refresh2") t.refresh[1] = value;
    else if (k == "refresh3") t.refresh[2] = value;
    else if (k == "depth") t.depth = (int)value == 8 ? 8 : 4;
    else if (k == "seed") t.seed = value != 0;
    else if (k == "hook") t.hook = value != 0;
    else if (k == "lds_edges_per_word") t.lds_edges_per_word = std::max(0.0, value);
    else if (k == "drain_at") t.drain_at = (u32)std::max(1.0, std::min(64.0, value));
    else if (k == "seed_nt") t.seed_nt = value != 0;
    else if (k == "seed_global") t.seed_global = value != 0;
    else if (k == "seed_passes") t.seed_passes = std::max(0, std::min(16, (int)value));
    else if (k == "seed_div") t.seed_div = std::max<u64>(1, (u64)value);
    else if (k == "seed_div1") t.seed_div1 = std::max<u64>(1, (u64)value);
    else if (k == "seed_refresh") t.seed_refresh = value;
    else if (k == "seed_fuse") t.seed_fuse = value != 0;
    else if (k == "share_async") t.share_async = value != 0;
    else if (k == "filter_min_share") t.filter_min_share = value;
    else if (k == "incremental") t.incremental = value != 0;
    else if (k == "inc_inplace") t.inc_inplace = value != 0;
    else if (k == "refresh_labels") t.refresh_labels = value != 0;
    else if (k == "inc_min_ids") t.inc_min_ids = (u64)value;
    else if (k == "inc_div") t.inc_div = std::max<u64>(1, (u64)value);
    else if (k == "inc_check") t.inc_check = value != 0;
    else if (k == "experimental") t.experimental = value != 0;
    else if (k == "inc_split") {
        if (value != 0 && !t.experimental)
            return set_err(GCC_E_INVALID, "inc_split = 1 can produce wrong labels (DESIGN.md §3); set 'experimental' first");
        t.inc_split = value != 0;
    }
    else if (k == "fold_release") t.fold_release = (int)value;
    else if (k == "post_check") t.post_check = std::max(0, std::min(2, (int)value));
    else if (k == "fail_absorb") t.fail_absorb = std::max(0, (int)value);
    else if (k == "compress_split") t.compress_split = value != 0;
    else if (k == "fold_split") t.fold_split = value != 0;
    else if (k == "inc_pipe") t.inc_pipe = std::max(0, std::min(2, (int)value));
    else if (k == "emit_div") t.emit_div = std::max(0, std::min(1 << 20, (int)value));
    else if (k == "emit_rec") t.emit_rec = value != 0;
    else if (k == "emit_filtered") t.emit_filtered = value != 0;
    else if (k == "pin_chunk") t.pin_chunk = (u64)value;
    else if (k == "bucket_p1") t.bucket_p1 = std::max(0, std::min(3, (int)value));
    else if (k == "bucket_p2_per") t.bucket_p2_per = (int)value == 12 ? 12 : 8;
    else if (k == "bucket_p2_vw") t.bucket_p2_vw = (int)value == 8 ? 8 : 4;
    else if (k == "scratch_realloc") t.scratch_realloc = std::max(0, std::min(3, (int)value));
    else if (k == "bucket_chunk") t.bucket_chunk = std::max(0, std::min((int)bk::kMaxChunk, (int)value));
    else if (k == "bucket_windows") t.bucket_windows = value != 0;
    else if (k == "bucket_items") t.bucket_items = std::max(1, std::min(64, (int)value));
    else if (k == "bucket_items_p3") t.bucket_items_p3 = std::max(1, std::min(64, (int)value));
    else if (k == "bucket_slow2") t.bucket_slow2 = value != 0.0;
    else if (k == "bucket_defer") t.bucket_defer = value != 0.0;
    else if (k == "bucket_defer_c") t.bucket_defer_c = std::max(0, std::min(2, (int)value));
    else if (k == "bucket") t.bucket = value != 0;
    else if (k == "bucket_min_batch") t.bucket_min_batch = (u64)value;
    else if (k == "bucket_min_ids") t.bucket_min_ids = (u64)value;
    else if (k == "bucket_levels") t.bucket_levels = std::max(0, std::min(6, (int)value));
    else if (k == "bucket_sample") t.bucket_sample = std::max(0.0, std::min(1.0, value));
    else if (k == "bucket_sample_sparse") t.bucket_sample_sparse = std::max(0.0, std::min(1.0, value));
    else if (k == "bucket_hub_sample") t.bucket_hub_sample = std::max(0.0, std::min(1.0, value));
    else return set_err(GCC_E_INVALID, "unknown tuning key '%s'", key);
    return GCC_OK;
}

int gcc_forest_fold_profile(gcc_forest* h, char* buf, uint64_t size) {
    CHECK_ARG(h && buf && size > 0, "null argument");
    buf[0] = 0;
    if (h->klog.empty()) return GCC_OK;  // nothing logged
    DeviceGuard g(h->device);
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->pipe_stream) HIP_TRY(hipStreamSynchronize(h->pipe_stream));
    std::string out;
    char line[160];
    // per kernel: "name ms edges"; per fold: a "begin" line first and, after its kernels, "fold_span ms edges" =
    // first kernel start -> last kernel stop (the fold's device time including the gaps between its launches)
    int first = -1, last = -1;
    u64 fold_edges = 0;
    auto close_fold = [&]() {
        if (first >= 0 && last >= 0) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, h->kev[first].first, h->kev[last].second);
            snprintf(line, sizeof line, "fold_span %.5f %llu\n", ms, (unsigned long long)fold_edges);
            out += line;
        }
        first = last = -1;
        fold_edges = 0;
    };
    bool in_fold = false;
    for (const auto& k : h->klog) {
        if (k.ev < 0) {  // a fold starts
            if (in_fold) close_fold();
            in_fold = true;
            out += "begin 0 0\n";
            continue;
        }
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, h->kev[k.ev].first, h->kev[k.ev].second));
        snprintf(line, sizeof line, "%s %.5f %llu\n", k.name, ms, (unsigned long long)k.edges);
        out += line;
        if (in_fold && std::strcmp(k.name, "compress") != 0 && std::strcmp(k.name, "compress_inc") != 0 &&
            std::strcmp(k.name, "resolve") != 0 && std::strcmp(k.name, "compress_pipe") != 0) {  // this fold's
            if (first < 0) first = k.ev;
            last = k.ev;
            if (!std::strcmp(k.name, "filtered") || !std::strcmp(k.name, "plain") || !std::strcmp(k.name, "sample") ||
                !std::strcmp(k.name, "bucket") || !std::strcmp(k.name, "plain_pipe"))  // P1: every edge once
                fold_edges += k.edges;
        } else if (in_fold) {
            close_fold();
            in_fold = false;
        }
    }
    if (in_fold) close_fold();
    h->klog.clear();  // drained: the event pairs are reused
    h->kev_used = 0;
    h->last_fold_first = h->last_fold_last = -1;
    for (size_t r = 0; r < h->slow_rounds.size(); ++r) {
        unsigned long long sum = 0;
        for (u32 b = 0; b < h->slow_rounds[r]; ++b) sum += h->h_segcount[r * kMaxGrid + b];
        snprintf(line, sizeof line, "slow_edges 0 %llu\n", sum);
        out += line;
    }
    h->slow_rounds.clear();
    if (out.size() + 1 > size) return set_err(GCC_E_INVALID, "profile buffer too small (%zu bytes needed)", out.size() + 1);
    snprintf(buf, size, "%s", out.c_str());
    return GCC_OK;
}

int gcc_step_mark(void* hip_stream) {
    hipLaunchKernelGGL(gcc_step_mark_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(hip_stream));
    HIP_TRY(hipGetLastError());
    return GCC_OK;
}

int gcc_forest_inc_check_stats(gcc_forest* h, uint64_t* checks, uint64_t* bad_labels, uint64_t* lost_marks) {
    CHECK_ARG(h && checks && bad_labels && lost_marks, "null argument");
    *checks = h->inc_checks;
    *bad_labels = h->inc_bad_labels;
    *lost_marks = h->inc_lost_marks;
    return GCC_OK;
}

int gcc_forest_post_check_stats(gcc_forest* h, uint64_t* checks, uint64_t* offenders, uint32_t* records,
                                uint32_t n_records) {
    CHECK_ARG(h && checks && offenders, "null argument");
    *checks = 0;
    *offenders = 0;
    if (!h->d_post) return GCC_OK;
    DeviceGuard g(h->device);
    u32 d[64];
    HIP_TRY(hipMemcpyAsync(d, h->d_post, sizeof(d), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *checks = d[1];
    *offenders = d[0];
    if (records)
        for (u32 k = 0; k < std::min<u32>(n_records, std::min<u32>(d[0], kPostRecs)); ++k)
            std::memcpy(records + 8 * k, d + 16 + 8 * k, 8 * sizeof(u32));
    return GCC_OK;
}

int gcc_forest_last_fold_ms(gcc_forest* h, float* ms) {
    CHECK_ARG(h && ms, "null argument");
    CHECK_ARG(h->last_fold_first >= 0, "no timed fold recorded (call gcc_forest_enable_timing first)");
    DeviceGuard g(h->device);
    HIP_TRY(hipEventSynchronize(h->kev[h->last_fold_last].second));
    HIP_TRY(hipEventElapsedTime(ms, h->kev[h->last_fold_first].first, h->kev[h->last_fold_last].second));
    return GCC_OK;
}

}  // extern "C"
