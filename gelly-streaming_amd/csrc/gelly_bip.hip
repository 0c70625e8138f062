// gelly_bip.hip — gfx950 signed forest: the device summary of BipartitenessCheck (include/gelly_cc.h, gcc_signed_*).
//
// What it replaces (`…/` = src/main/java/org/apache/flink/graph/streaming/):
//   Candidates (Tuple2<Boolean, TreeMap<Long, Map<Long, SignedVertex>>>)   …/summaries/Candidates.java:27-197
//   BipartitenessCheck.updateFunction.foldEdges = candidates.merge(edgeToCandidate(v1, v2))
//                                                                         …/library/BipartitenessCheck.java:54-61, :93-95
//   BipartitenessCheck.combineFunction.reduce  = c1.merge(c2)            :128-130
// A Candidates object is a set of components, each a map vertex -> sign with the two ends of every edge on
// opposite signs, plus a success flag that turns false (for good) once an edge closes an odd cycle. Signs are
// only defined up to one flip per component (Candidates.merge reverses the input side to match), so the parity
// contract observes, per vertex: its component's minimum id and its sign relative to that vertex, plus the flag.
//
// Device representation: one u32 word[id_capacity] per forest + one fail word.
//   word[v] == GCC_UNSEEN          -> v is not in any component
//   word[v] == (p << 1) | q        -> v hangs under p with sign(v) = sign(p) XOR q   (q = parity bit)
//   p == v (then q == 0)           -> v is a root
// Invariant p <= v (min-id hooking, as the CC forest): roots are component minima, and a compress leaves
// (min id << 1) | parity-to-min, which IS the canonical output. Ids must be < 2^31 - 1 (word range).
// Concurrency follows the CC forest (gelly_cc.hip header): a word only ever points to an ancestor, with the
// parity of the path to it, so a stale read is historically valid; roots leave root state only through CAS;
// path-splitting plain stores only target non-roots. The parity of a vertex relative to any ancestor is a
// fact of the constraints, never changed by later writes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "abi_common.h"
#include "gelly_cc.h"
#include "signed_bucket_api.h"  // the bucketed fold (gelly_cc.hip, signed_bucket.h)
#include "signed_uf.h"  // find / seen / unite, shared with the host replay (tests/cpp/test_signed_uf.cpp)

namespace {

typedef uint32_t u32;
typedef uint64_t u64;
constexpr u32 kUnseen = GCC_UNSEEN;
constexpr u32 kMaxSignedId = 0x7FFFFFFEu;  // (id << 1) | 1 must stay below GCC_UNSEEN
constexpr unsigned kMaxGrid = 2048;

__device__ __forceinline__ u32 sw_parent(u32 w) { return suf::parent_of(w); }
__device__ __forceinline__ u32 sw_par(u32 w) { return suf::parity_of(w); }
__device__ __forceinline__ u32 sfind(u32* word, u32 x, u32 wx, u32& par) { return suf::find(word, x, wx, par); }
__device__ __forceinline__ u32 sseen(u32* word, u32 v) { return suf::seen(word, v); }
__device__ __forceinline__ void sunite(u32* word, u32 u, u32 v, u32 q, u32* fail) { suf::unite(word, u, v, q, fail); }

__global__ __launch_bounds__(256) void signed_fold_kernel(u32* __restrict__ word, const u64* __restrict__ edges, u64 n,
                                                         u32* __restrict__ fail) {
    const u64 stride = (u64)gridDim.x * 256;
    u32 it = 0;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride, ++it) {
        // A failed summary is final: Candidates.merge answers fail() as soon as either side has failed (:78-81), so
        // no later edge changes the emitted value (false, {}). Stop folding; a stale read only delays the exit.
        // The words of a failed forest are not part of the contract (bipartite.py: getMap() == {}).
        if ((it & 7) == 0 && suf::ld(fail)) return;
        const u64 e = __builtin_nontemporal_load(edges + i);
        sunite(word, (u32)e, (u32)(e >> 32), 1u, fail);
    }
}

// ---- the giant-filtered fold (a skewed batch: kron / R-MAT hubs) ----
// A plain fold of a hub-heavy batch contends on the hubs' roots (C4's 2^27-edge share: 24.7 ms, 5.3 G edges/s).
// As the CC forest's filtered fold (gelly_cc.hip fold_filtered_kernel), most of such a batch lies inside one
// component C: fold a prefix sample, vote C's root over sampled edges' roots, and snapshot per id two bits — in C,
// and the parity to C's root (a find per seen id, as the compress; skipped, bits all 0, when no component holds
// min_share of the samples: C3's random graph). Then an edge with both ends in
// the snapshot's C is a pure check: the constraint sign(u) XOR sign(v) = 1 holds iff the parities differ (the
// parity of a vertex to an ancestor is a fact, never changed by later writes), else the batch has an odd cycle
// and the summary fails (Candidates.merge -> fail(), Candidates.java:77-139). It needs no forest access. Every
// other edge takes the plain unite; an edge with one end in C also adds the other end to C (its parity from the
// edge). A self loop inside C only adds its vertex: skipped.
constexpr u32 kVoteSamples = 4096;
constexpr u32 kVoteSlots = 8192;  // LDS hash of the sampled labels (a power of two)

// one block: the most frequent root over kVoteSamples sampled edges' first ends of the folded prefix; vote[0] =
// that root (or kUnseen), vote[1] = its count
__global__ __launch_bounds__(1024) void signed_vote_kernel(u32* __restrict__ word, const u64* __restrict__ edges,
                                                          u64 s, u32* __restrict__ vote) {
    __shared__ u32 key[kVoteSlots], cnt[kVoteSlots];
    __shared__ unsigned long long best;
    for (u32 i = threadIdx.x; i < kVoteSlots; i += 1024) {
        key[i] = kUnseen;
        cnt[i] = 0;
    }
    if (threadIdx.x == 0) best = 0;
    __syncthreads();
    for (u32 k = threadIdx.x; k < kVoteSamples; k += 1024) {
        const u64 e = edges[(u64)k * s / kVoteSamples];
        const u32 w = suf::ld(&word[(u32)e]);
        if (w == kUnseen) continue;
        u32 par;
        const u32 lab = sfind(word, (u32)e, w, par);
        u32 h = (lab * 0x9E3779B1u) >> 19;  // 13 bits
        while (true) {
            const u32 o = atomicCAS(&key[h], kUnseen, lab);
            if (o == kUnseen || o == lab) break;
            h = (h + 1) & (kVoteSlots - 1);
        }
        atomicAdd(&cnt[h], 1u);
    }
    __syncthreads();
    for (u32 i = threadIdx.x; i < kVoteSlots; i += 1024)
        if (cnt[i]) atomicMax(&best, ((unsigned long long)cnt[i] << 32) | key[i]);
    __syncthreads();
    if (threadIdx.x == 0) {
        vote[0] = (u32)best;
        vote[1] = (u32)(best >> 32);
    }
}

// 2 bits per id, 16 ids per word: bit 2j = id 16w+j in the voted root's component, bit 2j+1 = its parity to the root.
// No component when the vote's share is below 1/min_share_inv of the samples (a batch without a dominant one). One id
// per lane (coalesced plain loads: the sample fold has completed), 16 lanes' bits OR-ed into a word by shuffles
// (round 5: a lane per word read its 16 ids with 16 coherent loads 64 B apart: 239 us at 2^26 ids).
__global__ __launch_bounds__(256) void signed_snapshot_kernel(u32* __restrict__ word, u32 n, const u32* __restrict__ vote,
                                                             u32 min_count, u32* __restrict__ gbits) {
    const bool on = vote[1] >= min_count;
    const u32 r = vote[0];
    const u32 nw = (n + 15) / 16;
    const u64 ids = (u64)nw * 16;
    const u64 stride = (u64)gridDim.x * 256;
    const u32 lane = threadIdx.x % 64;
    constexpr int kU = 4;  // ids per lane per iteration, their loads in flight together
    for (u64 i0 = (u64)blockIdx.x * 256 + threadIdx.x; i0 - lane < ids; i0 += kU * stride) {
        u32 wk[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const u64 i = i0 + k * stride;
            wk[k] = on && i < n ? word[i] : kUnseen;
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const u64 i = i0 + k * stride;
            if (i - lane >= ids) break;  // whole waves (the shuffles): ids past the range contribute nothing
            const u32 v = (u32)i;
            u32 b = 0;
            if (wk[k] != kUnseen) {
                u32 par = 0;
                const u32 root = sw_parent(wk[k]) == v ? v : sfind(word, v, wk[k], par);
                if (root == r) b = (1u | par << 1) << (2 * (v & 15));
            }
            b |= __shfl_xor(b, 1, 64);
            b |= __shfl_xor(b, 2, 64);
            b |= __shfl_xor(b, 4, 64);
            b |= __shfl_xor(b, 8, 64);
            if ((v & 15) == 0 && i < ids) gbits[v >> 4] = b;
        }
    }
}

// one edge of the giant-filtered fold; bu / bv: the two ends' snapshot bits (bit 0 in C, bit 1 parity to r).
// Returns whether the edge needs a unite.
__device__ __forceinline__ bool giant_edge(u32* __restrict__ word, u32* __restrict__ gbits, u32* __restrict__ fail, u32 r,
                                           u32 u, u32 v, u32 bu, u32 bv) {
    if (bu & bv & 1u) {  // both in C: a check, no forest access
        if (u != v && !((bu ^ bv) & 2u)) suf::st(fail, 1u);
        return false;
    }
    if (!((bu ^ bv) & 1u)) return true;  // neither end in C
    // one end in C: the other, x, joins C with the opposite parity (the edge's constraint); later edges on x are
    // checks. Every bit is the parity the processed edges imply (snapshot: the forest's; derived: an edge that is
    // united in the forest), so a check compares forest parities; two derivations that disagree are an
    // odd cycle among forest edges, which the forest's unites report (fail), and a failed summary's bits no longer
    // matter. A stale read of a bit only sends an edge to the unite.
    const u32 x = (bu & 1u) ? v : u, px = (((bu & 1u) ? bu : bv) >> 1 & 1u) ^ 1u;
    atomicOr(&gbits[x >> 4], (1u | px << 1) << (2 * (x & 15)));
    // x unseen (its first edge: most of a kron batch's non-checks): hang it under r, C's root at the snapshot, an
    // ancestor of every C member for good, with that parity — one CAS, no walks. Min-id hooking allows it when
    // r < x; otherwise (or x seen) the unite.
    return !(r < x && suf::ld(&word[x]) == kUnseen && suf::cas(&word[x], kUnseen, (r << 1) | px) == kUnseen);
}

// U edges per lane per step (i, i + stride, ...): their loads and bit lookups in flight together
template <int U>
__global__ __launch_bounds__(256) void signed_fold_giant_kernel(u32* __restrict__ word, const u64* __restrict__ edges, u64 n,
                                                               u32* __restrict__ gbits, const u32* __restrict__ vote,
                                                               u32 min_count, u32* __restrict__ fail) {
    const u32 r = vote[0];  // C's root at the snapshot (no bit is set when the vote found no C)
    const u64 stride = (u64)gridDim.x * 256;
    u32 it = 0;
    if (vote[1] < min_count) {  // no C (the snapshot is empty): the plain fold, without the bit lookups
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride, ++it) {
            if ((it & 7) == 0 && suf::ld(fail)) return;
            const u64 e = __builtin_nontemporal_load(edges + i);
            sunite(word, (u32)e, (u32)(e >> 32), 1u, fail);
        }
        return;
    }
    for (u64 i0 = (u64)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += U * stride, ++it) {
        if ((it & (U >= 8 ? 0 : 8 / U - 1)) == 0 && suf::ld(fail)) return;  // a failed summary is final
        u64 e[U];
        u32 bu[U], bv[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const u64 j = i0 + k * stride;
            e[k] = __builtin_nontemporal_load(edges + (j < n ? j : n - 1));  // clamped: countable loads
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            bu[k] = gbits[(u32)e[k] >> 4];
            bv[k] = gbits[(u32)(e[k] >> 32) >> 4];
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const u32 u = (u32)e[k], v = (u32)(e[k] >> 32);
            const bool want = i0 + k * stride < n &&
                              giant_edge(word, gbits, fail, r, u, v, bu[k] >> (2 * (u & 15)), bv[k] >> (2 * (v & 15)));
            // the unite inline: deferring them to a list and a second pass (per-block regions, wave-aggregated LDS
            // appends) measured slower, 4.3 + 5.3 ms against 7.0 on C4's share (profiles/r4u_bip_*)
            if (want) sunite(word, u, v, 1u, fail);
        }
    }
}

// ---- the XCD-partitioned giant fold (round 5) ----
// The giant kernel above is bound by random 64-B line fetches of the 2-bit snapshot (16 MiB at C4's 2^26 ids: 1.7 L2
// misses per edge, profiles/r4u_bip_pmc_*). Here the batch is first split by the SOURCE id into 8 parts of the id
// range (one per XCD), and the blocks that serve part x all run on one XCD (blocks are dealt round-robin over the 8
// XCDs: block b serves part b % 8 — a placement used for speed only, never for correctness), so the source's
// snapshot lookups stay inside 1/8 of the snapshot (2 MiB at C4), which that XCD's 4 MiB L2 holds; the target's
// stay random. The split is a one-level multi-split (kXcdParts lists, chunked reservations from a sampled layout, an
// overflow list for a part whose estimate was low: still exact, the overflow edges take the kernel above).
constexpr u32 kXcdParts = 8;
constexpr int kSpBlock = 1024, kSpPer = 8;                    // split tiles of 8K edges (8 per thread, 4 x 16-B loads)
constexpr u32 kSpTile = (u32)kSpBlock * kSpPer;
constexpr u32 kSpChunk = 8192;                                // entries per chunk reservation
constexpr u32 kSpSample = 1u << 16;                           // the layout's sample: 64 runs of 1024 edges
struct XcdMeta {
    u64 base[kXcdParts];  // part x: entries [base[x], base[x] + cap[x]) of the split buffer
    u32 cap[kXcdParts];
    u32 cur[kXcdParts];   // reservation cursor (may pass cap: the rest went to the overflow list)
    u32 ovf_cur;          // overflow list cursor
    u32 shift;            // part of a source id u: min(u >> shift, kXcdParts - 1)
};
__device__ __forceinline__ u32 xcd_part(u32 u, u32 shift) { const u32 x = u >> shift; return x < kXcdParts ? x : kXcdParts - 1; }

// one block: capacities from a strided sample (1.25 x the estimate + one chunk per splitting block + slack, rounded
// to 16 entries), their prefix sums; the cursors reset
__global__ __launch_bounds__(1024) void xcd_layout_kernel(const u64* __restrict__ edges, u64 n, u32 shift, u32 blocks,
                                                         XcdMeta* __restrict__ m) {
    __shared__ u32 s_cnt[kXcdParts];
    if (threadIdx.x < kXcdParts) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    const u64 n_smp = n < kSpSample ? n : kSpSample, stride = n / 64;
    for (u32 r = 0; r < 64; ++r) {
        const u64 k = n <= kSpSample ? threadIdx.x + (u64)r * 1024 : (u64)r * stride + threadIdx.x;
        if (k < n && threadIdx.x + (u64)r * 1024 < n_smp) atomicAdd(&s_cnt[xcd_part((u32)edges[k], shift)], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 b = 0;
        for (u32 x = 0; x < kXcdParts; ++x) {
            const u64 est = (u64)s_cnt[x] * n / (n_smp ? n_smp : 1);
            const u64 c = (est + est / 4 + 4096 + (u64)blocks * kSpChunk + 15) / 16 * 16;
            m->base[x] = b;
            m->cap[x] = (u32)(c < 0xFFFFFFF0ull ? c : 0xFFFFFFF0ull);
            m->cur[x] = 0;
            b += m->cap[x];
        }
        m->ovf_cur = 0;
        m->shift = shift;
    }
}

// the split: per tile, an LDS counting sort by part, then each part's run written contiguously into the block's
// current chunk of that part (a new chunk from the part's cursor when it runs out); past the capacity, the overflow
// list. The unused tail of every chunk is written ~0 at exit (the giant kernel skips it).
__global__ __launch_bounds__(kSpBlock) void xcd_split_kernel(const u64* __restrict__ edges, u64 n, XcdMeta* __restrict__ m,
                                                            u64* __restrict__ out, u64* __restrict__ ovf, u32 ovf_cap) {
    __shared__ u64 s_t[kSpTile];
    __shared__ u32 s_cnt[kXcdParts], s_start[kXcdParts], s_cpos[kXcdParts], s_cend[kXcdParts];
    __shared__ u32 s_p1[kXcdParts], s_l1[kXcdParts], s_p2[kXcdParts], s_l2[kXcdParts];
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u32 shift = m->shift;
    if (threadIdx.x < kXcdParts) s_cpos[threadIdx.x] = s_cend[threadIdx.x] = 0;
    const u64 ntiles = (n + kSpTile - 1) / kSpTile;
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        if (threadIdx.x < kXcdParts) s_cnt[threadIdx.x] = 0;
        __syncthreads();  // (1) counters clear, the previous tile's write-out done
        u64 e[kSpPer];
        u32 rk[kSpPer];
        const u64 t0 = t * kSpTile;
#pragma unroll
        for (int k = 0; k < kSpPer / 2; ++k) {  // two edges per 16-B load, coalesced
            const u64 j = t0 + 2 * ((u64)k * kSpBlock + threadIdx.x);
            if (j + 1 < n) {
                const u4 q = __builtin_nontemporal_load(reinterpret_cast<const u4*>(edges + j));
                e[2 * k] = ((u64)q.y << 32) | q.x;
                e[2 * k + 1] = ((u64)q.w << 32) | q.z;
            } else {
                e[2 * k] = j < n ? edges[j] : ~0ull;
                e[2 * k + 1] = ~0ull;
            }
        }
#pragma unroll
        for (int k = 0; k < kSpPer; ++k)
            if (e[k] != ~0ull) rk[k] = atomicAdd(&s_cnt[xcd_part((u32)e[k], shift)], 1u);
        __syncthreads();  // (2) counts
        if (threadIdx.x == 0) {  // part starts in the tile, and each part's run reserved (chunked)
            u32 st = 0;
            for (u32 x = 0; x < kXcdParts; ++x) {
                s_start[x] = st;
                const u32 c = s_cnt[x];
                st += c;
                const u32 have = s_cend[x] - s_cpos[x], a = c < have ? c : have;
                s_p1[x] = s_cpos[x];
                s_l1[x] = a;
                s_cpos[x] += a;
                s_l2[x] = 0;
                if (c > a) {
                    const u32 need = c - a, size = ((need > kSpChunk ? need : kSpChunk) + 15) / 16 * 16;
                    const u32 g = atomicAdd(&m->cur[x], size), cap = m->cap[x];
                    const u32 beg = g < cap ? g : cap, end = g >= cap ? cap : ((u64)g + size > cap ? cap : g + size);
                    const u32 b2 = need < end - beg ? need : end - beg;
                    s_p2[x] = beg;
                    s_l2[x] = b2;
                    s_cpos[x] = beg + b2;
                    s_cend[x] = end;
                }
            }
        }
        __syncthreads();  // (3) starts and runs
#pragma unroll
        for (int k = 0; k < kSpPer; ++k)
            if (e[k] != ~0ull) s_t[s_start[xcd_part((u32)e[k], shift)] + rk[k]] = e[k];
        __syncthreads();  // (4) the tile in part order
        const u32 tot = s_start[kXcdParts - 1] + s_cnt[kXcdParts - 1];
        for (u32 i = threadIdx.x; i < tot; i += kSpBlock) {
            const u64 x64 = s_t[i];
            const u32 x = xcd_part((u32)x64, shift), r = i - s_start[x];
            u64 pos = ~0ull;
            if (r < s_l1[x]) pos = m->base[x] + s_p1[x] + r;
            else if (r - s_l1[x] < s_l2[x]) pos = m->base[x] + s_p2[x] + (r - s_l1[x]);
            if (pos != ~0ull) {
                out[pos] = x64;
            } else {  // the part is full (its estimate was low): the overflow list (the kernel above folds it)
                const u32 o = atomicAdd(&m->ovf_cur, 1u);
                if (o < ovf_cap) ovf[o] = x64;
            }
        }
    }
    __syncthreads();
    for (u32 x = 0; x < kXcdParts; ++x)  // the unused tails of this block's chunks
        for (u32 i = s_cpos[x] + threadIdx.x; i < s_cend[x]; i += kSpBlock) out[m->base[x] + i] = ~0ull;
}

// the giant kernel over the split batch: block b serves part b % 8 (its XCD, under round-robin placement), the
// part's entries grid-strided over the gridDim.x / 8 blocks of that part; ~0 entries (chunk tails) skipped
__global__ __launch_bounds__(256) void signed_fold_giant_xcd_kernel(u32* __restrict__ word, const u64* __restrict__ split,
                                                                   const XcdMeta* __restrict__ m, u32* __restrict__ gbits,
                                                                   const u32* __restrict__ vote, u32 min_count,
                                                                   u32* __restrict__ fail) {
    const u32 r = vote[0];
    const bool none = vote[1] < min_count;  // no C (the snapshot is empty): unites without the bit lookups
    const u32 x = blockIdx.x % kXcdParts, nb = gridDim.x / kXcdParts, bi = blockIdx.x / kXcdParts;
    const u64 len = m->cur[x] < m->cap[x] ? m->cur[x] : m->cap[x];
    const u64* part = split + m->base[x];
    const u64 stride = (u64)nb * 256;
    u32 it = 0;
    for (u64 i = (u64)bi * 256 + threadIdx.x; i < len; i += stride, ++it) {
        if ((it & 7) == 0 && suf::ld(fail)) return;  // a failed summary is final
        const u64 e = __builtin_nontemporal_load(part + i);
        if (e == ~0ull) continue;
        const u32 u = (u32)e, v = (u32)(e >> 32);
        if (none) {
            sunite(word, u, v, 1u, fail);
            continue;
        }
        const u32 bu = gbits[u >> 4], bv = gbits[v >> 4];
        if (giant_edge(word, gbits, fail, r, u, v, bu >> (2 * (u & 15)), bv >> (2 * (v & 15)))) sunite(word, u, v, 1u, fail);
    }
}

// the split's overflow list (a part whose estimate was low), and the whole batch again if even that list overflowed:
// the giant rule per edge (exact: a check, a bit set or a unite done twice changes nothing)
__global__ __launch_bounds__(256) void signed_fold_rest_kernel(u32* __restrict__ word, const u64* __restrict__ ovf,
                                                              const XcdMeta* __restrict__ m, u32 ovf_cap,
                                                              const u64* __restrict__ edges, u64 n,
                                                              u32* __restrict__ gbits, const u32* __restrict__ vote,
                                                              u32 min_count, u32* __restrict__ fail) {
    const u32 r = vote[0];
    const bool none = vote[1] < min_count;
    const u64 stride = (u64)gridDim.x * 256;
    const u64 no = m->ovf_cur < ovf_cap ? m->ovf_cur : ovf_cap;
    auto one = [&](u64 e) {
        const u32 u = (u32)e, v = (u32)(e >> 32);
        if (none) {
            sunite(word, u, v, 1u, fail);
            return;
        }
        const u32 bu = gbits[u >> 4], bv = gbits[v >> 4];
        if (giant_edge(word, gbits, fail, r, u, v, bu >> (2 * (u & 15)), bv >> (2 * (v & 15)))) sunite(word, u, v, 1u, fail);
    };
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < no; i += stride) one(ovf[i]);
    if (m->ovf_cur > ovf_cap)
        for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) one(edges[i]);
}

// into ∪= the signed partition of `other` (any forest of the same id range, compressed or not): the triple
// (v, parent, parity) of every seen v is the constraint sign(v) XOR sign(parent) = parity. A failed input
// fails the result (Candidates.merge :78-81).
__global__ __launch_bounds__(256) void signed_merge_kernel(u32* __restrict__ word, const u32* __restrict__ other, u32 n,
                                                          u32* __restrict__ fail, const u32* __restrict__ other_fail) {
    if (other_fail && blockIdx.x == 0 && threadIdx.x == 0 && *other_fail) *fail = 1u;
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 v = (u64)blockIdx.x * 256 + threadIdx.x; v < n; v += stride) {
        const u32 w = other[v];
        if (w == kUnseen) continue;
        const u32 p = sw_parent(w);
        if (p == (u32)v) {
            (void)sseen(word, (u32)v);
            continue;
        }
        sunite(word, (u32)v, p, sw_par(w), fail);
    }
}

// canonical words, out of place (as the CC compress): (min id << 1) | parity to it, UNSEEN stays UNSEEN
__global__ __launch_bounds__(256) void signed_compress_kernel(u32* __restrict__ word, u32* __restrict__ out, u32 n) {
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 v = (u64)blockIdx.x * 256 + threadIdx.x; v < n; v += stride) {
        const u32 w = word[v];
        if (w == kUnseen || sw_parent(w) == (u32)v) {  // a separate launch: no stale reads of word[v] itself
            out[v] = w;
            continue;
        }
        u32 par;
        const u32 r = sfind(word, (u32)v, w, par);
        out[v] = (r << 1) | par;
    }
}

}  // namespace

struct gcc_signed {
    int device = 0;
    u32 cap = 0;
    u32* d_word = nullptr;
    u32* d_spare = nullptr;
    u32* d_fail = nullptr;
    u32* d_stage = nullptr;  // host-fed edges
    u64 stage_cap = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    bool compressed = true;
    u32* d_gbits = nullptr;  // the giant-filtered fold's snapshot (2 bits per id) + 2 vote words
    int giant = 1;           // gcc_signed_tune "giant": the giant-filtered fold for big batches
    int sample_shift = 6;    // "sample_shift": its prefix sample = batch >> shift (at least 2^20 edges)
    double min_share = 0.25; // "min_share": the voted component's share of the sampled edges, else the plain fold
    int unroll = 1;          // "unroll": edges per lane per step of the giant-filtered fold (1, 2, 4, 8)
    // "xcd": the giant-filtered fold over the batch split by source part, one part per XCD. Measured (round 5,
    // profiles/r5f_ab_bip_xcd.txt, interleaved on one box): C4's share mapped bipartite 7.13-7.15 ms without the split,
    // 8.0-8.3 ms with it — the split's pass is not paid back: the target lookups and the new members' bit updates
    // still miss, and the wave divergence around the unites stays. Off; kept as a tested knob
    int xcd = 0;
    u64 xcd_min = 1ull << 25; // "xcd_min": ... for batches (past the sample) of at least this many edges
    XcdMeta* d_xm = nullptr;  // its layout
    u64* d_split = nullptr;   // the split batch (+ the overflow list behind it)
    u64 split_cap = 0;        // entries
    // "bucket" (round 5): the giant-filtered fold BUCKETED — both snapshot lookups of an edge in LDS (signed_bucket.h),
    // for batches (past the sample) of at least "bucket_min" edges when the vote found a component; "bucket_levels":
    // filter levels before the rest (1 or 2)
    int bucket = 1;
    u64 bucket_min = 1ull << 22;
    int bucket_levels = 2;
    int bucket_items = 2;              // "bucket_items": work items (slice parts) per CU of its filter / check kernels (a slice load each: 2 beat 1, 4, 8, 16 — profiles/r5ao_sweep_bip_items.txt)
    gcc_forest* bk_scratch = nullptr;  // a CC forest of the same id range: its bucket storage (P1) only
    u32* d_n2 = nullptr;               // 2 bits per id + the 8 counter words behind them
    u64* d_lists = nullptr;            // the emit list and two slow lists
    u64 list_cap = 0;                  // entries per list
    u64 last_counts[6] = {0, 0, 0, 0, 0, 0};  // the last bucketed fold's emitted / slow entries per level (diagnostics)
    std::vector<u32> host_words;
    bool host_valid = false;
};

static int signed_compress(gcc_signed* h) {
    if (h->compressed) return GCC_OK;
    hipLaunchKernelGGL(signed_compress_kernel, dim3(grid_for_n(h->cap, kMaxGrid)), dim3(256), 0, h->stream, h->d_word,
                       h->d_spare, h->cap);
    HIP_TRY(hipGetLastError());
    std::swap(h->d_word, h->d_spare);
    h->compressed = true;
    return GCC_OK;
}

static int signed_fold_plain(gcc_signed* h, const u64* edges, u64 n);

// The bucketed giant-filtered fold of the batch's rest (the snapshot and the vote made, a component found): gelly_cc.hip
// gcc_internal_signed_bucket. It ends with the closing compress (deferred members are labelled from the bits).
static int signed_fold_bucketed(gcc_signed* h, const u64* edges, u64 n, const u32* vote) {
    const u64 nw = ((u64)h->cap + 15) / 16;
    if (!h->bk_scratch) {
        int rc = gcc_forest_create(h->device, h->cap, &h->bk_scratch);
        if (rc) return rc;
        HIP_TRY(hipMalloc((void**)&h->d_n2, (nw + 8 + 6 * 512) * sizeof(u32)));  // N2, ctr, hist (2 per level)
        HIP_TRY(hipMemsetAsync(h->d_n2, 0, (nw + 8) * sizeof(u32), h->stream));
    }
    if (h->list_cap < n) {
        if (h->d_lists) {
            HIP_TRY(hipStreamSynchronize(h->stream));
            HIP_TRY(hipFree(h->d_lists));
            h->d_lists = nullptr;
        }
        const u64 c = (n + 15) / 16 * 16;
        HIP_TRY(hipMalloc((void**)&h->d_lists, 3 * c * sizeof(u64)));
        h->list_cap = c;
    }
    GccSignedBucketArgs a{};
    a.stream = h->stream;
    a.word = h->d_word;
    a.out = h->d_spare;
    a.gbits = h->d_gbits;
    a.n2 = h->d_n2;
    a.vote = vote;
    a.fail = h->d_fail;
    a.edges = edges;
    a.n = n;
    a.cap = h->cap;
    a.emit = h->d_lists;
    a.slow0 = h->d_lists + h->list_cap;
    a.slow1 = h->d_lists + 2 * h->list_cap;
    a.ctr = h->d_n2 + nw;
    a.hist = h->d_n2 + nw + 8;
    a.levels = h->bucket_levels;
    a.items_per_cu = h->bucket_items;
    const char* stats = std::getenv("GELLY_BUCKET_STATS");
    a.want_counts = stats && *stats && *stats != '0';
    int rc = gcc_internal_signed_bucket(h->bk_scratch, &a);
    if (rc) {  // N2 must be zero before the next batch (sb_join clears it on the normal path): clear it here
        (void)hipMemsetAsync(h->d_n2, 0, nw * sizeof(u32), h->stream);
        return rc;
    }
    std::memcpy(h->last_counts, a.counts, sizeof(a.counts));
    if (a.want_counts)
        std::fprintf(stderr, "[signed-bucket] n=%llu level 1: emitted %llu slow %llu; level 2: emitted %llu slow %llu; level 3: emitted %llu slow %llu\n",
                     (unsigned long long)n, (unsigned long long)a.counts[0], (unsigned long long)a.counts[1],
                     (unsigned long long)a.counts[2], (unsigned long long)a.counts[3], (unsigned long long)a.counts[4],
                     (unsigned long long)a.counts[5]);
    std::swap(h->d_word, h->d_spare);  // the closing compress wrote the canonical words
    h->compressed = true;
    h->host_valid = false;
    return GCC_OK;
}

// a batch of at least 2^22 edges and a quarter of the id range (the snapshot's O(ids) passes amortised): the
// giant-filtered fold (above signed_vote_kernel)
static int signed_fold(gcc_signed* h, const u32* d_pairs, u64 n) {
    const u64* edges = reinterpret_cast<const u64*>(d_pairs);
    if (!h->giant || n < (1ull << 22) || n < h->cap / 4) return signed_fold_plain(h, edges, n);
    const u64 s = std::min<u64>(n, std::max<u64>(1ull << 20, n >> h->sample_shift) & ~1ull);  // even: 16-B aligned rest
    int rc = signed_fold_plain(h, edges, s);
    if (rc) return rc;
    const u64 nw = ((u64)h->cap + 15) / 16;
    if (!h->d_gbits) HIP_TRY(hipMalloc((void**)&h->d_gbits, (nw + 2) * sizeof(u32)));  // + the vote
    u32* vote = h->d_gbits + nw;
    hipLaunchKernelGGL(signed_vote_kernel, dim3(1), dim3(1024), 0, h->stream, h->d_word, edges, s, vote);
    HIP_TRY(hipGetLastError());
    const u32 min_count = (u32)std::max(1.0, h->min_share * kVoteSamples);
    hipLaunchKernelGGL(signed_snapshot_kernel, dim3(grid_for_n(nw * 16, kMaxGrid)), dim3(256), 0, h->stream, h->d_word, h->cap,
                       vote, min_count, h->d_gbits);
    HIP_TRY(hipGetLastError());
    // id ranges up to 2^27 (past 2^27 the bucketing takes untested shapes — 6-B emit entries, 12K-edge P1
    // tiles — so those ranges keep the giant-filtered fold)
    if (n > s && h->bucket && n - s >= h->bucket_min && h->cap <= (1u << 27) &&
        ((reinterpret_cast<uintptr_t>(edges + s) & 15) == 0)) {
        u32 hv[2];  // the vote: a component to filter against, or the plain fold (no bucketing for it)
        HIP_TRY(hipMemcpyAsync(hv, vote, sizeof(hv), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        if (hv[1] >= min_count) return signed_fold_bucketed(h, edges + s, n - s, vote);
    }
    if (n > s && h->xcd && n - s >= h->xcd_min && ((reinterpret_cast<uintptr_t>(edges + s) & 15) == 0)) {
        // the split: capacities from a sample, chunked reservations, the overflow list after the parts
        const u64 m_edges = n - s;
        int nb = 256;
        (void)hipDeviceGetAttribute(&nb, hipDeviceAttributeMultiprocessorCount, h->device);
        const u64 need = m_edges + m_edges / 4 + kXcdParts * (4096 + (u64)nb * kSpChunk + 16);
        const u32 ovf_cap = (u32)std::min<u64>(m_edges / 8 + 65536, 0xFFFFFFF0ull);
        if (h->split_cap < need + ovf_cap) {
            if (h->d_split) {
                HIP_TRY(hipStreamSynchronize(h->stream));
                HIP_TRY(hipFree(h->d_split));
                h->d_split = nullptr;
                h->split_cap = 0;
            }
            HIP_TRY(hipMalloc((void**)&h->d_split, (need + ovf_cap) * sizeof(u64)));
            h->split_cap = need + ovf_cap;
        }
        if (!h->d_xm) HIP_TRY(hipMalloc((void**)&h->d_xm, sizeof(XcdMeta)));
        u32 bits = 0;
        while (bits < 32 && ((u64)1 << bits) < h->cap) ++bits;
        const u32 shift = bits > 3 ? bits - 3 : 0;  // 8 parts of the id range (by the top 3 bits of an id)
        u64* ovf = h->d_split + need;
        hipLaunchKernelGGL(xcd_layout_kernel, dim3(1), dim3(1024), 0, h->stream, edges + s, m_edges, shift, (u32)nb, h->d_xm);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(xcd_split_kernel, dim3(nb), dim3(kSpBlock), 0, h->stream, edges + s, m_edges, h->d_xm,
                           h->d_split, ovf, ovf_cap);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(signed_fold_giant_xcd_kernel, dim3(8 * (u32)nb), dim3(256), 0, h->stream, h->d_word, h->d_split,
                           h->d_xm, h->d_gbits, vote, min_count, h->d_fail);
        HIP_TRY(hipGetLastError());
        hipLaunchKernelGGL(signed_fold_rest_kernel, dim3(nb), dim3(256), 0, h->stream, h->d_word, (const u64*)ovf, h->d_xm,
                           ovf_cap, edges + s, m_edges, h->d_gbits, vote, min_count, h->d_fail);
        HIP_TRY(hipGetLastError());
    } else if (n > s) {
        const dim3 g(grid_for_n(n - s, kMaxGrid));
        auto k = h->unroll >= 8 ? signed_fold_giant_kernel<8>
                 : h->unroll >= 4 ? signed_fold_giant_kernel<4>
                 : h->unroll >= 2 ? signed_fold_giant_kernel<2> : signed_fold_giant_kernel<1>;
        hipLaunchKernelGGL(k, g, dim3(256), 0, h->stream, h->d_word, edges + s, n - s, h->d_gbits, vote, min_count,
                           h->d_fail);
        HIP_TRY(hipGetLastError());
    }
    h->compressed = false;
    h->host_valid = false;
    return GCC_OK;
}

// the plain fold. The first launches are small and grow geometrically: while the hubs of a skewed stream are still
// unhooked, few threads contend on their roots (the CC forest's sampled start, gelly_cc.hip).
static int signed_fold_plain(gcc_signed* h, const u64* edges, u64 n) {
    u64 b = 0;
    for (u64 c = 4096; b < n; c *= 4) {
        // past 2^20 edges the rest in one launch (to_bipartite(C3): 4M + 3.9M-edge tail launches 1.04 ms, one 8.2M
        // launch after the 1M-edge prefix 0.92 ms, profiles/r4u_bip_r6r_*)
        const u64 e = c >= (1ull << 20) ? n : std::min(n, b + c);
        hipLaunchKernelGGL(signed_fold_kernel, dim3(grid_for_n(e - b, kMaxGrid)), dim3(256), 0, h->stream, h->d_word,
                           edges + b, e - b, h->d_fail);
        HIP_TRY(hipGetLastError());
        b = e;
    }
    h->compressed = false;
    h->host_valid = false;
    return GCC_OK;
}

extern "C" {

int gcc_signed_create(int device, uint32_t id_capacity, gcc_signed** out) {
    CHECK_ARG(out, "out is null");
    *out = nullptr;
    CHECK_ARG(id_capacity >= 1 && id_capacity <= kMaxSignedId + 1, "id_capacity must be in [1, 2^31 - 1]");
    int rc = gcc_check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    gcc_signed* h = new gcc_signed();
    h->device = device;
    h->cap = id_capacity;
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_word, (size_t)id_capacity * sizeof(u32));
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_spare, (size_t)id_capacity * sizeof(u32));
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_fail, sizeof(u32));
    if (e != hipSuccess) {
        gcc_signed_destroy(h);
        return gcc_set_err(e == hipErrorOutOfMemory ? GCC_E_OOM : GCC_E_HIP, "gcc_signed_create: %s",
                           hipGetErrorString(e));
    }
    h->stream = h->own_stream;
    rc = gcc_signed_reset(h);
    if (rc) {
        gcc_signed_destroy(h);
        return rc;
    }
    *out = h;
    return GCC_OK;
}

int gcc_signed_destroy(gcc_signed* h) {
    if (!h) return GCC_OK;
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->d_word) (void)hipFree(h->d_word);
    if (h->d_spare) (void)hipFree(h->d_spare);
    if (h->d_fail) (void)hipFree(h->d_fail);
    if (h->d_gbits) (void)hipFree(h->d_gbits);
    if (h->d_split) (void)hipFree(h->d_split);
    if (h->d_xm) (void)hipFree(h->d_xm);
    if (h->d_stage) (void)hipFree(h->d_stage);
    if (h->d_n2) (void)hipFree(h->d_n2);
    if (h->d_lists) (void)hipFree(h->d_lists);
    if (h->bk_scratch) (void)gcc_forest_destroy(h->bk_scratch);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return GCC_OK;
}

int gcc_signed_set_stream(gcc_signed* h, void* hip_stream, int use_own) {
    CHECK_ARG(h, "null handle");
    DeviceGuard g(h->device);
    hipStream_t next = use_own ? h->own_stream : (hipStream_t)hip_stream;
    if (next != h->stream) {
        hipEvent_t ev;
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev, h->stream));
        HIP_TRY(hipStreamWaitEvent(next, ev, 0));
        HIP_TRY(hipEventDestroy(ev));
        h->stream = next;
    }
    return GCC_OK;
}

int gcc_signed_reset(gcc_signed* h) {
    CHECK_ARG(h, "null handle");
    DeviceGuard g(h->device);
    HIP_TRY(hipMemsetAsync(h->d_word, 0xFF, (size_t)h->cap * sizeof(u32), h->stream));
    HIP_TRY(hipMemsetAsync(h->d_fail, 0, sizeof(u32), h->stream));
    h->compressed = true;
    h->host_valid = false;
    return GCC_OK;
}

int gcc_signed_fold_device(gcc_signed* h, const uint32_t* d_pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null handle");
    CHECK_ARG(d_pairs || n_edges == 0, "d_pairs is null");
    if (n_edges == 0) return GCC_OK;
    DeviceGuard g(h->device);
    return signed_fold(h, d_pairs, n_edges);
}

int gcc_signed_fold_host(gcc_signed* h, const uint32_t* pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null handle");
    CHECK_ARG(pairs || n_edges == 0, "pairs is null");
    if (n_edges == 0) return GCC_OK;
    for (u64 i = 0; i < 2 * n_edges; ++i)  // a bad id would be an out-of-bounds device access
        if (pairs[i] >= h->cap) return gcc_set_err(GCC_E_INVALID, "vertex id %u >= id_capacity %u", pairs[i], h->cap);
    DeviceGuard g(h->device);
    if (h->stage_cap < n_edges) {
        if (h->d_stage) {
            HIP_TRY(hipStreamSynchronize(h->stream));
            HIP_TRY(hipFree(h->d_stage));
            h->d_stage = nullptr;
        }
        HIP_TRY(hipMalloc((void**)&h->d_stage, n_edges * 2 * sizeof(u32)));
        h->stage_cap = n_edges;
    }
    HIP_TRY(hipMemcpyAsync(h->d_stage, pairs, n_edges * 2 * sizeof(u32), hipMemcpyHostToDevice, h->stream));
    int rc = signed_fold(h, h->d_stage, n_edges);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));  // pageable source: consumed before returning
    return GCC_OK;
}

int gcc_signed_merge(gcc_signed* into, gcc_signed* from) {
    CHECK_ARG(into && from, "null handle");
    if (into == from) return GCC_OK;
    CHECK_ARG(from->cap <= into->cap, "merge source has a larger id range than the target");
    CHECK_ARG(from->device == into->device, "signed forests must live on one device");
    DeviceGuard g(into->device);
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(ev, from->stream));
    HIP_TRY(hipStreamWaitEvent(into->stream, ev, 0));
    hipLaunchKernelGGL(signed_merge_kernel, dim3(grid_for_n(from->cap, kMaxGrid)), dim3(256), 0, into->stream,
                       into->d_word, from->d_word, from->cap, into->d_fail, from->d_fail);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev, into->stream));
    HIP_TRY(hipStreamWaitEvent(from->stream, ev, 0));  // from must not change before the merge has read it
    HIP_TRY(hipEventDestroy(ev));
    into->compressed = false;
    into->host_valid = false;
    return GCC_OK;
}

int gcc_signed_tune(gcc_signed* h, const char* key, double value) {
    CHECK_ARG(h && key, "null argument");
    const std::string k(key);
    if (k == "giant") h->giant = value != 0;
    else if (k == "sample_shift") {
        CHECK_ARG(value >= 0 && value <= 20, "sample_shift must be in [0, 20]");
        h->sample_shift = (int)value;
    } else if (k == "unroll") {
        CHECK_ARG(value == 1 || value == 2 || value == 4 || value == 8, "unroll must be 1, 2, 4 or 8");
        h->unroll = (int)value;
    } else if (k == "xcd") {
        h->xcd = value != 0;
    } else if (k == "xcd_min") {
        CHECK_ARG(value >= 0, "xcd_min must be >= 0");
        h->xcd_min = (u64)value;
    } else if (k == "bucket") {
        h->bucket = value != 0;
    } else if (k == "bucket_min") {
        CHECK_ARG(value >= 0, "bucket_min must be >= 0");
        h->bucket_min = (u64)value;
    } else if (k == "bucket_items") {
        CHECK_ARG(value >= 1 && value <= 64, "bucket_items must be in [1, 64]");
        h->bucket_items = (int)value;
    } else if (k == "bucket_levels") {
        CHECK_ARG(value >= 1 && value <= 3, "bucket_levels must be 1, 2 or 3");
        h->bucket_levels = (int)value;
    } else if (k == "min_share") {
        CHECK_ARG(value > 0 && value <= 1, "min_share must be in (0, 1]");
        h->min_share = value;
    } else return gcc_set_err(GCC_E_INVALID, "gcc_signed_tune: unknown key '%s'", key);
    return GCC_OK;
}

int gcc_signed_compress(gcc_signed* h) {
    CHECK_ARG(h, "null handle");
    DeviceGuard g(h->device);
    return signed_compress(h);
}

int gcc_signed_device_words(gcc_signed* h, const uint32_t** d_words) {
    CHECK_ARG(h && d_words, "null argument");
    *d_words = h->d_word;
    return GCC_OK;
}

int gcc_signed_merge_words(gcc_signed* into, const uint32_t* d_words, uint32_t n, int other_failed) {
    CHECK_ARG(into, "null handle");
    CHECK_ARG(d_words || n == 0, "d_words is null");
    CHECK_ARG(n <= into->cap, "n exceeds id_capacity");
    DeviceGuard g(into->device);
    if (other_failed) HIP_TRY(hipMemsetAsync(into->d_fail, 1, 1, into->stream));  // fail() is absorbing (:78-81)
    if (n) {
        // the other forest's (v, parent, parity) triples as constraints; its fail word is the flag above
        hipLaunchKernelGGL(signed_merge_kernel, dim3(grid_for_n(n, kMaxGrid)), dim3(256), 0, into->stream, into->d_word,
                           d_words, n, into->d_fail, nullptr);  // other_failed: the memset above
        HIP_TRY(hipGetLastError());
    }
    into->compressed = false;
    into->host_valid = false;
    return GCC_OK;
}

int gcc_signed_words(gcc_signed* h, uint32_t* out, uint32_t n) {
    CHECK_ARG(h, "null handle");
    CHECK_ARG(out || n == 0, "out is null");
    CHECK_ARG(n <= h->cap, "n exceeds id_capacity");
    DeviceGuard g(h->device);
    if (!h->host_valid) {
        int rc = signed_compress(h);
        if (rc) return rc;
        h->host_words.resize(h->cap);
        HIP_TRY(hipMemcpyAsync(h->host_words.data(), h->d_word, (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToHost,
                               h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        if ((rc = gcc_internal_take_err(h->bk_scratch, h->stream))) return rc;  // the bucketed fold's skipped ids
        h->host_valid = true;
    }
    std::memcpy(out, h->host_words.data(), (size_t)n * sizeof(u32));
    return GCC_OK;
}

int gcc_signed_success(gcc_signed* h, int* success) {
    CHECK_ARG(h && success, "null argument");
    DeviceGuard g(h->device);
    u32 f = 0;
    HIP_TRY(hipMemcpyAsync(&f, h->d_fail, sizeof(u32), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *success = f ? 0 : 1;
    return gcc_internal_take_err(h->bk_scratch, h->stream);  // the bucketed fold's skipped ids
}

int gcc_signed_capacity(gcc_signed* h, uint32_t* id_capacity) {
    CHECK_ARG(h && id_capacity, "null argument");
    *id_capacity = h->cap;
    return GCC_OK;
}

}  // extern "C"
