// bucket_fold.h — the bucketed fold of a FRESH forest over a big id range (DESIGN.md §4 "bucketed fold").
// Included by gelly_cc.hip after its kernels (uses UF, edge_ok, ring_push / unite_entry, hub_elect).
//
// Why: the giant filter of fold_filtered_kernel looks both endpoints of every edge up in a bitmap of the tracked
// component. At C4 (V = 2^26) that bitmap is 8 MiB — bigger than an XCD's 4 MiB L2 — and the random lookups, not
// HBM, bound the pass (63 G edges/s for 2 lookups per edge, 824 G edges/s for the same stream with the lookups in
// LDS; profiles/r2_probe_bucket.log). So the batch is first split by the source id's SLICE (2^19 ids = a 64 KiB
// slice of the bitmap), and every later pass over an edge finds its bitmap slice in LDS:
//   bucket_kernel        P1: multi-split of the batch into per-slice buckets (tile-local LDS counting sort, one
//                        global cursor add per (tile, bucket)); histograms the target ids' slices too
//   slice_filter_kernel  P2: per bucket, the slice of C in LDS: u in C -> v joins the v-list of v's slice (a 4-B
//                        multi-split), else (FINAL) the edge takes the union path (per-wave LDS ring)
//   slice_hook_kernel    P3: per v-list, the slice of C in LDS: v not in C -> SEED: v joins C (LDS bit, OR-ed
//                        back into the global bitmap); FINAL: v is hooked under g (the edge (u, v) = (g, v))
// Seeding (C = the component of a hub h, grown over a sample of every bucket by a few P2 + P3 levels), then
// parent[v] := v in C ? g = min C : UNSEEN (bucket_init_kernel), then P2 + P3 over ALL bucketed edges, then the
// overflow list (edges a bucket had no room for) and, only if even that list overflowed, the whole batch again
// (bucket_rest_kernel). Every edge of the batch is folded exactly once by a union or lies inside C, which is one
// component of the batch: the result is the partition of the batch, whatever the sample or the level count.
#pragma once

namespace bk {

constexpr u32 kSliceBits = 19;                  // ids per slice: 2^19 -> a 64 KiB bitmap slice in LDS
constexpr u32 kSliceIds = 1u << kSliceBits;
constexpr u32 kSliceWords = kSliceIds / 32;     // u32 words per slice (16384)
// v-lists (P2's output, P3's input) are split by TARGET slices of 2^kVSliceBits ids (round 3: 2^20, a 128 KiB bitmap
// slice in P3's LDS, which holds nothing else): half as many lists as buckets, so P2 keeps half as many write streams
// open (2 per list: lo, hi), counts and scans half as many runs per round and writes them twice as long
#ifndef GCC_VSLICE_BITS
#define GCC_VSLICE_BITS 20
#endif
constexpr u32 kVSliceBits = GCC_VSLICE_BITS;
constexpr u32 kVSliceWords = (1u << kVSliceBits) / 32;
__host__ __device__ inline u32 vslices(u32 cap) { return (u32)(((u64)cap + (1u << kVSliceBits) - 1) >> kVSliceBits); }
// P1 geometry (tune.bucket_p1): 0 = 512 threads x 16 edges (8192-edge tiles, 2 blocks per CU), 1 = 1024 x 16
// (16384-edge tiles, one block per CU: runs twice as long per (tile, bucket))
constexpr int kP1Block = 512;
constexpr int kP1Per = 16;                      // edges per thread per tile
constexpr u32 kP1Tile = kP1Block * kP1Per;      // the smallest tile (bucket_applies: a batch of >= 2 tiles)
constexpr int kP2Block = 1024;
// P2 entries per thread per round (tune bucket_p2_per: 8 or 12): a round of kP2Block * PER entries, and at most that
// many v's in the round's LDS tile + up to 3 padding slots per v-list (kMaxVLists)
constexpr u32 p2_round(int per) { return (u32)kP2Block * per; }
// + up to VW - 1 padding slots per v-list (kMaxVLists): VW = entries per lane in the write-out (4, or 8 since round 4)
constexpr u32 p2_tile(int per, int vw = 4) { return p2_round(per) + (u32)(vw - 1) * 256; }
// id ranges up to 2^28 (larger: the unbucketed fold): at most 512 buckets (2^19-id source slices) and 256 v-lists
// (2^20-id target slices). P1's per-bucket LDS state is sized per instantiation (P1 MAXB: 256 up to 2^27 ids, 512
// beyond, with a smaller tile); P2 / P3 keep per-v-list state only
constexpr u32 kMaxBuckets = 512;
constexpr u32 kMaxVLists = 256;
static_assert(((u64)kMaxBuckets << kSliceBits) == ((u64)kMaxVLists << kVSliceBits), "the same id range");
constexpr int kP3Block = 1024;
constexpr u32 kMaxP2Blocks = 1024;

// Per-forest metadata (device): per bucket (kMaxBuckets) and per v-list (kMaxVLists).
struct Meta {
    u64 bk_base[kMaxBuckets];  // bucket s: edges [bk_base[s], bk_base[s] + bk_cap[s]) of the bucket storage
    u32 bk_cap[kMaxBuckets];
    u32 bk_cur[kMaxBuckets];   // reservation cursor (may pass bk_cap: the rest went to the overflow list)
    u64 vl_base[kMaxVLists];   // v-list s (targets in slice s): entries [vl_base[s], vl_base[s] + vl_cap[s])
    u32 vl_cap[kMaxVLists];
    // per pass (seeding levels, FINAL, the second level: kVlPasses), may pass vl_cap: those v's were hooked inline
    // (FINAL) or dropped (SEED). One array per pass, all zeroed by the layout (round 5: no memset between passes)
    u32 vl_cur[8][kMaxVLists];
    u32 work[16];                // per-launch dequeue counters
    u32 ovf_cur;                 // overflow list cursor (may pass its capacity: then `spill`)
    u32 spill;                   // 1: some edge fit neither its bucket nor the overflow list
    u32 gmin;                    // min C (seeding)
    u32 nseg;                    // FINAL P2: slow-list segments recorded (SlowSeg table)
    u32 ring_used;               // FINAL P2 united some slow edges itself (its region was full): see bucket_join_kernel
    u32 chunk;                   // entries per chunk reservation (chunk_entries)
    u32 slow_cnt[kMaxP2Blocks];  // FINAL P2: slow edges (source not in C) each block listed in its own region
    u64 n_list;                  // the batch size when the layout took it from the device (bucket_kernel: n = ~0)
};
constexpr u32 kVlPasses = 8;  // Meta::vl_cur: seeding levels 0..5, FINAL (6), the second level (7)
constexpr u32 kVlFinal = 6, kVlLevel2 = 7;

// A run of one P2 block's slow list whose edges share a source slice (one P2 item's slow edges): the second
// filter level (slice_filter_kernel<true, true>) takes these runs as its items. off is even (runs padded to pairs).
struct SlowSeg {
    u64 off;  // first entry, in the whole slow array
    u32 sl;   // source slice
    u32 len;  // entries (a ~0 tail entry pads an odd run)
};

__device__ __forceinline__ u32 lds_bit(const u32* s, u32 x) { return (s[x >> 5] >> (x & 31)) & 1u; }

// Phase timing (diagnostic builds only: -DGCC_PHASES): every wave accumulates clock64() deltas per phase of P1's tile
// loop (kernel 0) and FINAL P2's round loop (kernel 1), summed over the owner waves (0-1) and the others apart;
// GELLY_BUCKET_STATS prints them.
#ifdef GCC_PHASES
__device__ unsigned long long gcc_phase_acc[2][16];
struct PhaseClock {
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t = 0;
    __device__ __forceinline__ void start() { t = clock64(); }
    __device__ __forceinline__ void mark(int k) {
        const unsigned long long n = clock64();
        acc[k] += n - t;
        t = n;
    }
    __device__ __forceinline__ void flush(int kern) {  // lane 0 of every wave: waves 0-1 (the lists' owners) in
        if ((threadIdx.x & 63) == 0)                     // slots 0-7, the other waves in slots 8-15
            for (int k = 0; k < 8; ++k) atomicAdd(&gcc_phase_acc[kern][k + (threadIdx.x < 128 ? 0 : 8)], acc[k]);
    }
};
#define GCC_PH_START(pc) (pc).start()
#define GCC_PH_MARK(pc, k) (pc).mark(k)
#define GCC_PH_FLUSH(pc, kern) (pc).flush(kern)
// ... and every block's start and end on the device's constant-rate clock (wall_clock64, 100 MHz), per kernel kind:
// 0 P1, 1 FINAL P2, 2 the second level's P2, 3 FINAL P3, 4 the second level's P3, 5 a seeding P2, 6 a seeding P3,
// 7 the slow kernel (the last launch of a kind wins): how long each block worked against the kernel's span
constexpr int kBtKinds = 8, kBtBlocks = 1024;
__device__ unsigned long long gcc_blk_time[kBtKinds][kBtBlocks][2];
#define GCC_BT(kind, which)                                                                       \
    do {                                                                                          \
        if (threadIdx.x == 0 && blockIdx.x < kBtBlocks) gcc_blk_time[kind][blockIdx.x][which] = wall_clock64(); \
    } while (0)
#else
#define GCC_BT(kind, which) (void)0
struct PhaseClock {};
#define GCC_PH_START(pc) (void)0
#define GCC_PH_MARK(pc, k) (void)0
#define GCC_PH_FLUSH(pc, kern) (void)0
#endif
typedef u64 u64x2 __attribute__((ext_vector_type(2)));
typedef uint16_t u16;
typedef u16 u16x4 __attribute__((ext_vector_type(4)));

// ---- bucket entries: 6 bytes (round 3; round 2 stored the u64 edge). The bucket (= source slice s) already names
// the source's high bits, so an entry holds the target v (< 2^28: ns <= 512 slices of 2^19 ids) and the source's
// 19 slice-local bits ul, in two parallel arrays of the same index: lo (u32) = v | ul[3:0] << 28, hi (u16) =
// ul[18:4] (15 bits). hi = 0xFFFF (never 15 bits) marks a padding slot or an unused chunk tail. P1 writes and P2
// reads 6 B per edge instead of 8: 25 % of both passes' bucket traffic.
constexpr u32 kTgtBits = 28;
constexpr u32 kTgtMask = (1u << kTgtBits) - 1;
constexpr u16 kPadHi = 0xFFFF;

// e = (v << 32) | u, or ~0 (padding)
__device__ __forceinline__ u32 bk_lo_of(u64 e) {
    return e == ~0ull ? 0xFFFFFFFFu : (u32)(e >> 32) | (((u32)e & (kSliceIds - 1)) << kTgtBits);
}
__device__ __forceinline__ u16 bk_hi_of(u64 e) {
    return e == ~0ull ? kPadHi : (u16)(((u32)e & (kSliceIds - 1)) >> (32 - kTgtBits));
}

// the source (slice base sbase | ul) and target of an entry; false for padding
__device__ __forceinline__ bool bk_decode(u32 lo, u16 hi, u32 sbase, u32& u, u32& v) {
    u = sbase | ((u32)hi << (32 - kTgtBits)) | (lo >> kTgtBits);
    v = lo & kTgtMask;
    return hi != kPadHi;
}

// Bucket bases 2 MiB-aligned (the lo array; hi 1 MiB) for batches of >= 2^26 edges: every capacity is rounded up
// to 2^19 entries. The lists' write frontiers advance in step, and their relative placement matters (a hashed
// stagger of the bases cost P2 +0.8 ms, profiles/r3af_ab_stagger.log); aligned buckets: C4 9.64 -> 9.52 ms on two
// boxes (P1 and P2 -0.05 ms each; aligning the v-lists as well: no further change; profiles/r3ag_*, r3ah_*)
constexpr u64 kBkAlign = 1ull << 19;  // entries
__host__ __device__ inline bool bk_aligned(u64 n) { return n >= (1ull << 26); }

// ---- v-list entries: 3 bytes (round 3; round 2 stored the u32 target). A v-list belongs to one target slice, so an
// entry holds the target's kVSliceBits slice-local bits: lo (u16) = x[15:0], hi (u8) = x[kVSliceBits-1:16]; hi = 0xFF
// marks padding or an unused chunk tail. P2 writes and P3 reads 3 B per listed edge instead of 4.
typedef uint8_t u8;
constexpr u8 kPadV = 0xFF;
struct VList {
    u16* lo;
    u8* hi;
};
__host__ __device__ inline u64 vl_entries(u64 storage) { return (storage + 15) / 16 * 16; }
__host__ __device__ inline u64 vl_bytes(u64 storage) { return 3 * vl_entries(storage); }

// the bucket storage of S entries (S a multiple of 2^19): lo at the start, hi right after (1 MiB-aligned)
__host__ __device__ inline u64 bk_entries(u64 storage) { return (storage + kBkAlign - 1) / kBkAlign * kBkAlign; }
__host__ __device__ inline u64 bk_bytes(u64 storage) { return 6 * bk_entries(storage); }

// Internal consistency checks: every id a kernel takes from an internal list (buckets, slow and overflow lists) and
// uses to index GLOBAL memory must be < cap. It always is; if one were not, the entry is skipped (never
// dereferenced) and its flag is OR-ed into the forest's error word, which the next synchronising call reports as
// GCC_E_INTERNAL naming the list. Ids that only index a block's LDS (P2's sources, P3's targets) are not checked:
// LDS accesses cannot fault, and a full check there cost P2 + P3 0.6 ms of C4's 12 (profiles/r2_ab_guards.log).
constexpr u32 kErrP2 = 2, kErrSlow = 8, kErrOvf = 16;
__device__ __forceinline__ void flag_err(u32* err, u32 f) { atomicOr(err, f); }

// ---- layout from a strided sample: capacity = 1.25 x the estimated count + slack, for the buckets (by source
// slice) and the v-lists (by target slice). One block. The sums are bounded by storage_edges() (host) whatever
// the sample says; a batch the sample misjudges only overflows (overflow list / inline hooks: still exact).
constexpr u32 kSample = 1u << 16;
constexpr u32 kSlack = 1u << 12;
// Writers reserve space in a bucket / v-list a CHUNK at a time per (block, slice) — one global atomic per chunk,
// not per tile — and mark the unused tail of their last chunk with UNSEEN at exit (readers skip UNSEEN entries).
// Each list's capacity therefore carries one chunk per writing block of slack, and so do the lists' reads: C4's
// 1/8 share carried 21M tail entries of 1024-entry chunks over 128 x 256 (bucket, block) pairs. The chunk is chosen
// per batch (Meta::chunk, host: chunk_entries): 1024 entries from 2^29 edges up, 512 below (round 4, A/B in
// profiles/r4k_*: the share and C4's 2^27-edge windows gain, C4 in one batch loses with 512)
constexpr u32 kMaxChunk = 4096;
__host__ __device__ inline u32 chunk_entries(u64 n, u32 tuned) {
    const u32 c = tuned ? tuned : (n >= (1ull << 29) ? 1024u : 512u);
    return c < 64 ? 64u : c > kMaxChunk ? kMaxChunk : (c + 15) / 16 * 16;
}


// The entries `nl` lists of an n-edge batch can claim (each list's capacity rounded up to 16); `aligned`: the buckets'
// capacities of a batch of >= 2^26 edges are also rounded up to kBkAlign (the v-lists' are not).
__host__ __device__ inline u64 storage_edges(u64 n, u32 nl, u32 blocks, bool aligned, u32 chunk) {
    return n + n / 4 + (u64)nl * (kSlack + 64 + (u64)blocks * chunk) + 64 + (aligned ? (u64)nl * kBkAlign : 0);
}

__device__ __forceinline__ u32 est_cap(u32 hits, u64 n, u64 n_smp, u32 blocks, u32 chunk) {
    const u64 est = (u64)hits * n / (n_smp ? n_smp : 1);
    const u64 c = ((est + est / 4 + kSlack + (u64)blocks * chunk) + 15) / 16 * 16;  // 16-entry multiples: aligned
    return (u32)(c < 0xFFFFFFF0ull ? c : 0xFFFFFFF0ull);
}

// Chunked reservation of this round's run of `c` entries of slice s by the block (one thread per slice): the rest
// of the block's current chunk [cpos, cend) first, then (if needed) a new chunk of max(chunk, rest) entries from
// the list's global cursor, clamped to the capacity. The run's first l1 entries go to p1.., the next l2 to p2..,
// the remaining c - l1 - l2 (capacity exhausted) overflow. Positions are list-relative.
struct Runs {
    u32* cpos;
    u32* cend;
    u32* p1;
    u32* l1;
    u32* p2;
    u32* l2;
};

__device__ __forceinline__ void reserve_run(const Runs& r, u32 s, u32 c, u32* cursor, u32 cap, u32 chunk) {
    const u32 have = r.cend[s] - r.cpos[s];
    const u32 a = c < have ? c : have;
    r.p1[s] = r.cpos[s];
    r.l1[s] = a;
    r.cpos[s] += a;
    r.l2[s] = 0;
    if (c > a) {
        const u32 need = c - a;
        const u32 size = ((need > chunk ? need : chunk) + 15) / 16 * 16;
        const u32 g = atomicAdd(cursor, size);
        const u32 end = g >= cap ? cap : ((u64)g + size > cap ? cap : g + size);
        const u32 beg = g < cap ? g : cap;
        const u32 b = need < end - beg ? need : end - beg;
        r.p2[s] = beg;
        r.l2[s] = b;
        r.cpos[s] = beg + b;
        r.cend[s] = end;
    }
}

// The list position of entry i of slice s's run this round, or 0xFFFFFFFF (overflow).
__device__ __forceinline__ u32 run_pos(const Runs& r, u32 s, u32 i) {
    if (i < r.l1[s]) return r.p1[s] + i;
    i -= r.l1[s];
    return i < r.l2[s] ? r.p2[s] + i : 0xFFFFFFFFu;
}

// exclusive prefix of cap[0..ns) into base[] (1024 threads, ns <= 1024)
__device__ __forceinline__ void block_prefix(const u32* cap, u64* base, u32 ns, u64* s_scan) {
    const u64 loc = threadIdx.x < ns ? cap[threadIdx.x] : 0;
    s_scan[threadIdx.x] = loc;
    __syncthreads();
    for (u32 o = 1; o < 1024; o <<= 1) {  // inclusive scan (Hillis-Steele; 1024 entries, once per batch)
        const u64 y = threadIdx.x >= o ? s_scan[threadIdx.x - o] : 0;
        __syncthreads();
        s_scan[threadIdx.x] += y;
        __syncthreads();
    }
    if (threadIdx.x < ns) base[threadIdx.x] = s_scan[threadIdx.x] - loc;
    __syncthreads();
}

// n_dev / exact (the signed forest's bucketed fold, signed_bucket.h): the batch's size from the device (a list a
// kernel appended; bucket_kernel then takes n = ~0 and reads m->n_list) and its exact per-bucket counts, no sample.
__global__ __launch_bounds__(1024) void bucket_layout_kernel(const u64* __restrict__ edges, u64 n, u32 ns, u32 cap,
                                                              Meta* __restrict__ m, u32 bk_blocks, u32 vl_blocks,
                                                              u32 chunk, const u32* __restrict__ n_dev,
                                                              const u32* __restrict__ exact) {
    trace_start(kTrBkLayout);
    __shared__ u32 s_cu[kMaxBuckets], s_cv[kMaxVLists];
    __shared__ u64 s_scan[1024];
    const u32 nvs = vslices(cap);
    if (n_dev) n = *n_dev < n ? *n_dev : n;
    for (u32 s = threadIdx.x; s < ns; s += 1024) {
        s_cu[s] = exact ? exact[s] : 0u;
        if (s < nvs) s_cv[s] = 0;
    }
    if (threadIdx.x == 0) m->n_list = n;
    __syncthreads();
    const u64 n_smp = exact ? n : n < kSample ? n : kSample;
    // the sample: kSample / 1024 = 64 runs of 1024 CONSECUTIVE edges spread evenly over the batch (coalesced, 64
    // pages; single edges kSample apart touched 64K pages and took this one block 0.12 ms on C4), 32 loads in
    // flight per thread (64 would spill)
    constexpr u32 kPer = kSample / 1024, kBatch = 32;
    const u64 run_stride = n / kPer;  // >= 1024 whenever n >= kSample; below that the sample is the batch
    for (u32 b = 0; b < (exact ? 0u : kPer); b += kBatch) {
        u64 e[kBatch];
#pragma unroll
        for (u32 i = 0; i < kBatch; ++i) {
            const u64 k = n <= kSample ? threadIdx.x + (u64)(b + i) * 1024 : (u64)(b + i) * run_stride + threadIdx.x;
            e[i] = k < n ? edges[k] : ~0ull;
        }
#pragma unroll
        for (u32 i = 0; i < kBatch; ++i) {
            const u32 u = (u32)e[i], v = (u32)(e[i] >> 32);
            if (u < cap && v < cap) {
                atomicAdd(&s_cu[u >> kSliceBits], 1u);
                atomicAdd(&s_cv[v >> kVSliceBits], 1u);
            }
        }
    }
    __syncthreads();
    for (u32 s = threadIdx.x; s < ns; s += 1024) {
        m->bk_cap[s] = est_cap(s_cu[s], n, n_smp, bk_blocks, chunk);
        if (bk_aligned(n)) m->bk_cap[s] = (u32)((m->bk_cap[s] + kBkAlign - 1) / kBkAlign * kBkAlign);
        m->bk_cur[s] = 0;
        if (s < nvs) {
            m->vl_cap[s] = est_cap(s_cv[s], n, n_smp, vl_blocks, chunk);
#pragma unroll
            for (u32 p = 0; p < kVlPasses; ++p) m->vl_cur[p][s] = 0;  // every pass's cursors (round 5: no memsets)
        }
    }
    __syncthreads();
    block_prefix(m->bk_cap, m->bk_base, ns, s_scan);
    block_prefix(m->vl_cap, m->vl_base, nvs, s_scan);
    if (threadIdx.x < 16) m->work[threadIdx.x] = 0;
    if (threadIdx.x == 0) m->nseg = 0;
    if (threadIdx.x == 0) m->ring_used = 0;
    if (threadIdx.x == 0) m->chunk = chunk;
    if (threadIdx.x == 0) {
        m->ovf_cur = 0;
        m->spill = 0;
    }
}

// Runs are padded to a multiple of W entries (W = 4 or 8): padw.
template <u32 W>
__device__ __forceinline__ u32 padw(u32 c) { return (c + W - 1) & ~(W - 1); }

// Exclusive scan of the padded counts padw<W>(cnt[0..ns)) into start[], by wave 0 alone (lane l: lists
// [l * per, l * per + per), per = ceil(ns / 64)), no barrier inside: the caller's next barrier publishes start[].
// Round 4: the block-wide form (round 3) cost every round an extra barrier and, in wave w, w dependent LDS loads of
// the other waves' sums, while only the first ns threads held counts.
template <u32 W>
__device__ __forceinline__ void wave_scan(const u32* cnt, u32* start, u32 ns) {
    const u32 lane = threadIdx.x & 63;
    const u32 per = (ns + 63) >> 6;
    u32 loc = 0;
    for (u32 j = 0; j < per; ++j) {
        const u32 s = lane * per + j;
        loc += s < ns ? padw<W>(cnt[s]) : 0;
    }
    u32 inc = loc;
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(inc, o, 64);
        if (lane >= (u32)o) inc += y;
    }
    u32 run = inc - loc;
    for (u32 j = 0; j < per; ++j) {
        const u32 s = lane * per + j;
        if (s < ns) {
            start[s] = run;
            run += padw<W>(cnt[s]);
        }
    }
}

// ---- P1: the multi-split -------------------------------------------------------------------------------------
// Persistent; a tile of kP1Tile edges is counted per bucket in LDS (atomicAdd returns each edge's rank in its
// bucket), the block reserves each bucket's run with ONE global atomicAdd, scatters the tile into LDS in bucket
// order and writes every run out contiguously (runs of ~kP1Tile / ns edges). The next tile's loads are in flight
// meanwhile. Bad ids: skipped + *err. The odd last edge of an odd-length batch and every edge past its bucket's
// capacity go to the overflow list.
// P1's dynamic LDS: the tile in bucket order, every bucket's run padded to a multiple of 4 — up to three slots per
// slice beyond the tile. (Round 2 first sized it to the tile alone: a full tile's last padded slots fell past the
// allocation and relied on the LDS allocation's rounding slack; a 1024 x 8 geometry with less slack lost edges.)
// W (round 4): entries per lane in the write-out, every run padded to a multiple of W. W = 4: 16 B of lo and 8 B of hi
// per lane; W = 8: 2 x 16 B of lo and 16 B of hi (8-B stores run at 0.54-0.70x the 16-B rate, MI355X_MICROARCH.md)
constexpr size_t p1_lds(int block, int per, u32 maxb = 256, u32 w = 4) {
    return ((size_t)block * per + (w - 1) * maxb) * sizeof(u64);
}

// KEYONLY (the signed fold's emit lists, signed_bucket.h): the second id is a parity bit, so an entry is 4 B — the
// key's slice-local bits | second << kSliceBits in lo, no hi array (padding: lo = ~0)
template <int P1B, int P1P, u32 MAXB = 256, u32 W = 4, bool KEYONLY = false>
__global__ __launch_bounds__(P1B, (P1B == 512 ? 4 : 4)) void bucket_kernel(const u64* __restrict__ edges, u64 n, u32 ns, u32 cap,
                                                          Meta* __restrict__ m, u32* __restrict__ bk_lo,
                                                          u16* __restrict__ bk_hi, u64* __restrict__ ovf, u32 ovf_cap,
                                                          u32* __restrict__ err, u32* __restrict__ reset) {
    trace_start(kTrBkP1);
    if (n == ~0ull) n = m->n_list;  // the layout took it from the device
    GCC_BT(0, 0);
    // the tile in bucket order: dynamic LDS (p1_lds: P1B * P1P + 3 MAXB u64, 66 / 130 KiB), set up like every
    // kernel's LDS beyond 64 KiB (gelly_cc.hip set_lds_attrs_impl); the per-bucket state below is static (MAXB >= ns)
    static_assert(MAXB <= kMaxBuckets, "Meta holds kMaxBuckets buckets");
    extern __shared__ __attribute__((aligned(16))) u64 s_srt[];
    // counts double-buffered by tile parity: a tile counts into one buffer while slower waves may still read the
    // other (the previous tile's write-out); 3 barriers per tile (round 3: 6)
    __shared__ u32 s_cntb[2 * MAXB], s_start[MAXB], s_cap[MAXB];
    __shared__ u32 s_cpos[MAXB], s_cend[MAXB], s_p1[MAXB], s_l1[MAXB], s_p2[MAXB], s_l2[MAXB];
    __shared__ u64 s_base[MAXB];
    const Runs runs{s_cpos, s_cend, s_p1, s_l1, s_p2, s_l2};
    const u32 chunk = m->chunk;
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u4* body = reinterpret_cast<const u4*>(edges);  // 16-B aligned (bucket_applies checks)
    for (u32 s = threadIdx.x; s < ns; s += P1B) {  // the layout, once per block (not a global load per edge)
        s_cap[s] = m->bk_cap[s];
        s_base[s] = m->bk_base[s];
        s_cpos[s] = s_cend[s] = 0;  // no chunk yet
        s_cntb[s] = s_cntb[MAXB + s] = 0;
    }
    // Every thread reads every slice's state below — in the tile loop after its barriers, but a block with no
    // tile goes straight to the chunk-tail loop at the end. Without this barrier such a block read s_cpos / s_cend
    // / s_base before their owner threads had written them: LDS left over from the previous kernel on the CU, a
    // wild store address, and (intermittently, small batches only: C4 gives every block tiles) a GPU memory fault.
    __syncthreads();
    const u64 n2 = n / 2;                                  // whole pairs
    const u64 ntiles = (n2 * 2 + (P1B * P1P) - 1) / (P1B * P1P);
    constexpr int kQ = P1P / 2;
    // reset (round 5): a fresh forest's lazy reset, parent[] := UNSEEN, spread over the tiles: tile t stores its
    // 1/ntiles of the id range behind the next tile's loads (P1 never reads parent[]; the waves mostly wait for their
    // loads). It replaces bucket_init_kernel's 4 B per id of its own launch: C is deferred like N (bucket_join_kernel)
    const u64 rq = reset ? (u64)cap / 4 : 0;  // whole 16-B quads; the last cap % 4 ids here:
    if (reset && blockIdx.x == 0 && threadIdx.x < (cap & 3u)) reset[4 * rq + threadIdx.x] = GCC_UNSEEN_DEV;
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {  // the odd last edge
        u32 a = (u32)edges[n - 1], b = (u32)(edges[n - 1] >> 32);
        if (edge_ok(a, b, cap, err)) {
            const u32 o = atomicAdd(&m->ovf_cur, 1u);
            if (o < ovf_cap) ovf[o] = ((u64)b << 32) | a;
            else m->spill = 1u;
        }
    }
    auto load_tile = [&](u64 t, u4 (&q)[kQ]) {
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            const u64 j = t * ((P1B * P1P) / 2) + (u64)k * P1B + threadIdx.x;
            q[k] = __builtin_nontemporal_load(body + (j < n2 ? j : n2 - 1));  // clamped: countable loads
        }
    };
    u4 q[kQ];
    u64 t = blockIdx.x;
    if (t < ntiles) load_tile(t, q);
    [[maybe_unused]] PhaseClock phc;
    GCC_PH_START(phc);
    u32 rb = 0;  // tile parity: the count buffer in use
    for (; t < ntiles; t += gridDim.x) {
        u32* s_cnt = s_cntb + rb * MAXB;
        u32 ua[P1P], va[P1P], rk[P1P];
        bool ok[P1P];
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            const u64 j = t * ((P1B * P1P) / 2) + (u64)k * P1B + threadIdx.x;
            ua[2 * k] = q[k].x;
            va[2 * k] = q[k].y;
            ua[2 * k + 1] = q[k].z;
            va[2 * k + 1] = q[k].w;
            ok[2 * k] = ok[2 * k + 1] = j < n2;
        }
        if (t + gridDim.x < ntiles) load_tile(t + gridDim.x, q);  // the next tile streams in meanwhile
        if (reset) {
            const u4 un = {GCC_UNSEEN_DEV, GCC_UNSEEN_DEV, GCC_UNSEEN_DEV, GCC_UNSEEN_DEV};
            for (u64 x = rq * t / ntiles + threadIdx.x; x < rq * (t + 1) / ntiles; x += P1B)
                reinterpret_cast<u4*>(reset)[x] = un;
        }
        GCC_PH_MARK(phc, 0);  // waited for this tile's loads
#pragma unroll
        for (int k = 0; k < P1P; ++k) {
            if (ok[k]) ok[k] = edge_ok(ua[k], va[k], cap, err);
            if (ok[k]) rk[k] = atomicAdd(&s_cnt[ua[k] >> kSliceBits], 1u);
        }
        GCC_PH_MARK(phc, 1);  // LDS counting
        __syncthreads();  // (1) the tile's counts are complete; every wave has left the previous tile's write-out
        GCC_PH_MARK(phc, 2);
        // every bucket's run is padded to a multiple of W with ~0 entries (P2 skips them), so that runs, tile slots
        // and list positions stay multiples of W and the write-out moves W entries per lane (4: 16 B of lo, 8 of hi)
        if (threadIdx.x < 64) wave_scan<W>(s_cnt, s_start, ns);
        for (u32 s = threadIdx.x; s < ns; s += P1B) s_cntb[(rb ^ 1) * MAXB + s] = 0;  // the next tile's buffer
        GCC_PH_MARK(phc, 3);  // scan
        __syncthreads();  // (2) starts
        GCC_PH_MARK(phc, 4);
        // the reservations (their global atomics) overlap the other waves' scatter
        for (u32 s = threadIdx.x; s < ns; s += P1B) {
            const u32 pc = padw<W>(s_cnt[s]);
            if (pc) reserve_run(runs, s, pc, &m->bk_cur[s], s_cap[s], chunk);
            for (u32 j = s_cnt[s]; j < pc; ++j) s_srt[s_start[s] + j] = ~0ull;
        }
#pragma unroll
        for (int k = 0; k < P1P; ++k)
            if (ok[k]) s_srt[s_start[ua[k] >> kSliceBits] + rk[k]] = ((u64)va[k] << 32) | ua[k];
        GCC_PH_MARK(phc, 5);  // reservations + scatter
        __syncthreads();  // (3) the tile in bucket order, the runs reserved
        GCC_PH_MARK(phc, 6);
        const u32 totw = (s_start[ns - 1] + padw<W>(s_cnt[ns - 1])) / W;
        for (u32 xw = threadIdx.x; xw < totw; xw += P1B) {
            u64 e[W];
#pragma unroll
            for (u32 k = 0; k < W / 2; ++k) {  // slot W xw is never padding
                const u64x2 ek = reinterpret_cast<const u64x2*>(s_srt)[(W / 2) * xw + k];
                e[2 * k] = ek.x;
                e[2 * k + 1] = ek.y;
            }
            const u32 s = (u32)e[0] >> kSliceBits;
            const u32 off = run_pos(runs, s, W * xw - s_start[s]);  // a multiple of W: all W in one chunk
            if (KEYONLY && off != 0xFFFFFFFFu) {
                auto key_of = [](u64 x) -> u32 {
                    return x == ~0ull ? 0xFFFFFFFFu : ((u32)x & (kSliceIds - 1)) | ((u32)(x >> 32) << kSliceBits);
                };
#pragma unroll
                for (u32 k = 0; k < W / 4; ++k) {
                    const u4 lo = {key_of(e[4 * k]), key_of(e[4 * k + 1]), key_of(e[4 * k + 2]), key_of(e[4 * k + 3])};
                    *reinterpret_cast<u4*>(bk_lo + s_base[s] + off + 4 * k) = lo;
                }
            } else if (off != 0xFFFFFFFFu) {
#pragma unroll
                for (u32 k = 0; k < W / 4; ++k) {  // 16-B aligned (bases: 16-entry multiples)
                    const u4 lo = {bk_lo_of(e[4 * k]), bk_lo_of(e[4 * k + 1]), bk_lo_of(e[4 * k + 2]), bk_lo_of(e[4 * k + 3])};
                    *reinterpret_cast<u4*>(bk_lo + s_base[s] + off + 4 * k) = lo;
                }
                if constexpr (W == 8) {
                    typedef u16 u16x8 __attribute__((ext_vector_type(8)));
                    const u16x8 hi = {bk_hi_of(e[0]), bk_hi_of(e[1]), bk_hi_of(e[2]), bk_hi_of(e[3]),
                                      bk_hi_of(e[4]), bk_hi_of(e[5]), bk_hi_of(e[6]), bk_hi_of(e[7])};
                    *reinterpret_cast<u16x8*>(bk_hi + s_base[s] + off) = hi;  // 16-B aligned
                } else {
                    const u16x4 hi = {bk_hi_of(e[0]), bk_hi_of(e[1]), bk_hi_of(e[2]), bk_hi_of(e[3])};
                    *reinterpret_cast<u16x4*>(bk_hi + s_base[s] + off) = hi;  // 8-B aligned
                }
            } else {  // the bucket is full (its estimate was low): the overflow list (folded at the end)
                u32 k = 1;
#pragma unroll
                for (u32 i = 1; i < W; ++i) k += e[i] != ~0ull;  // padding only at the end
                const u32 o = atomicAdd(&m->ovf_cur, k);
                for (u32 i = 0; i < k; ++i)
                    if (o + i < ovf_cap) ovf[o + i] = e[i];
                if (o + k > ovf_cap) m->spill = 1u;  // -> bucket_rest: the whole batch again
            }
        }
        GCC_PH_MARK(phc, 7);  // write-out
        rb ^= 1;  // the next tile's barrier (1) orders this write-out before its scan and scatter
    }
    GCC_PH_FLUSH(phc, 0);
    // the unused tails of this block's chunks: padding entries (P2 skips them)
    for (u32 s = 0; s < ns; ++s)
        for (u32 i = s_cpos[s] + threadIdx.x; i < s_cend[s]; i += P1B) {
            if (KEYONLY) bk_lo[s_base[s] + i] = 0xFFFFFFFFu;
            else bk_hi[s_base[s] + i] = kPadHi;
        }
    GCC_BT(0, 1);
}

// Work items of P2 / P3: item i -> (slice i / cps, part i % cps) of a list of `len` entries; the part's range.
__device__ __forceinline__ void item_range(u64 len, u32 part, u32 cps, u64& lo, u64& hi) {
    lo = len * part / cps;
    hi = len * (part + 1) / cps;
}

// Load slice s of the bitmap (WORDS u32: kSliceWords for a bucket, kVSliceWords for a v-list) into LDS (16-B loads,
// 8 in flight per thread).
template <int BLOCK, u32 WORDS = kSliceWords>
__device__ __forceinline__ void load_slice(u32* s_bits, const u32* __restrict__ bits, u32 s, u32 nwords32) {
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u32 w0 = s * WORDS;
    const u32 nw = w0 + WORDS <= nwords32 ? WORDS : (w0 < nwords32 ? nwords32 - w0 : 0);
    if (nw == WORDS) {
        lds_fill<BLOCK>(reinterpret_cast<u4*>(s_bits), reinterpret_cast<const u4*>(bits + w0), WORDS / 4);
    } else {  // the last, partial slice
        for (u32 w = threadIdx.x; w < WORDS; w += BLOCK) s_bits[w] = w < nw ? bits[w0 + w] : 0u;
    }
}

// The hook of an edge (u, v) with u in C, i.e. union(g, v): unite_entry's hook form — one atomicMin, a union only
// if v already hung under some other id.
__device__ __forceinline__ void hook_g(u32* parent, u32 g, u32 v) {
    NoCount c;
    if (v > g) {
        const u32 old = atomicMin(&parent[v], g);
        if (old != GCC_UNSEEN_DEV && old != v && old != g) UF::unite(parent, g, old, c);
    } else if (v != g) {
        UF::unite(parent, g, v, c);
    }
}

// ---- P2: filter by the source slice --------------------------------------------------------------------------
// u in C -> v into the v-lists (SEED: only the first `frac` (16.16 fixed point) of every bucket: the sample).
// FINAL: an edge whose u is not in C is a SLOW edge: listed in the block's own region of the slow list (no global
// atomics; past the region's capacity it is united right here through the per-wave LDS ring). A full v-list (its
// capacity came from a sample): FINAL hooks v under g right here, SEED drops it (seeding is only a heuristic).
// Rounds of kP2Round edges, the next round's loads in flight; counters double-buffered (3 barriers per round).
// LDS: slice (64 KiB) + v tile (kP2Round u32) + counters + layout + rings (FINAL).
// hub_only (SEED): the first level, C = {h} (m->gmin): only the items of h's slice are streamed.
// SEG (second level, FINAL only): the items are the slow-list runs the FINAL pass recorded (`segs`, m->nseg of
// them; `bk` = the slow array), C is then C | N, and its own slow edges go to `slow` (the bucket storage, free
// by then). FINAL without SEG records those runs into `segs` (one per item with slow edges; null: none).
template <bool FINAL, bool SEG = false, int PER = 8, int VW = 4>
__global__ __launch_bounds__(kP2Block) void slice_filter_kernel(u32* __restrict__ parent, const u32* __restrict__ bk_lo,
                                                                const u16* __restrict__ bk_hi, const u64* __restrict__ bk,
                                                                const u32* __restrict__ bits, u32 nwords32, u32 ns,
                                                                Meta* __restrict__ m, VList vl, u32 cps,
                                                                u32 frac, u32 work_slot, u32 drain_at, u32 hub_only,
                                                                const u32* __restrict__ giant, u64* __restrict__ slow,
                                                                u32 slow_cap, u32 cap, u32* __restrict__ err,
                                                                SlowSeg* __restrict__ segs, u32 pass) {
    static_assert(FINAL || !SEG, "the second level is a FINAL pass");
    trace_start(FINAL ? kTrBkP2 : kTrBkP2Seed);
    GCC_BT(FINAL ? (SEG ? 2 : 1) : 5, 0);
    extern __shared__ __attribute__((aligned(16))) u32 s_dyn[];
    u32* s_bits = s_dyn;                                   // kSliceWords
    u32* s_vt = s_dyn + kSliceWords;                       // p2_tile(PER, VW): the round's targets + run padding
    // per v-list state, kMaxVLists entries each
    u32* s_cnt2 = s_vt + p2_tile(PER, VW);                 // 2 x (double-buffered counts)
    u32* s_start = s_cnt2 + 2 * kMaxVLists;
    u32* s_vcap = s_start + kMaxVLists;
    u32* s_run = s_vcap + kMaxVLists;                      // 6 x: the chunk state (Runs)
    u64* s_vbase = reinterpret_cast<u64*>(s_run + 6 * kMaxVLists);
    u64* ring = s_vbase + kMaxVLists + (threadIdx.x >> 6) * kRing;  // FINAL only
    __shared__ u32 s_item, s_slow;
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    constexpr int kQ = PER / 2;
    const u32 lane = threadIdx.x & 63;
    const u32 g = FINAL ? *giant : 0u;
    u64* my_slow = slow + (u64)blockIdx.x * slow_cap;
    u32 wq = 0, wd = 0;  // this wave's ring cursors (FINAL)
    u32 cur_slice = 0xFFFFFFFFu;
    u32 rb = 0;  // round parity: the counter buffer in use
    for (u32 s = threadIdx.x; s < 2 * kMaxVLists; s += kP2Block) s_cnt2[s] = 0;
    const u32 chunk = m->chunk;
    const Runs runs{s_run, s_run + kMaxVLists, s_run + 2 * kMaxVLists, s_run + 3 * kMaxVLists,
                    s_run + 4 * kMaxVLists, s_run + 5 * kMaxVLists};
    const u32 nvs = vslices(cap);  // v-lists: target slices of 2^kVSliceBits ids
    for (u32 s = threadIdx.x; s < nvs; s += kP2Block) {  // the v-list layout, once per block
        s_vcap[s] = m->vl_cap[s];
        s_vbase[s] = m->vl_base[s];
        runs.cpos[s] = runs.cend[s] = 0;
    }
    if (threadIdx.x == 0) s_slow = 0;
    [[maybe_unused]] PhaseClock phc;
    GCC_PH_START(phc);
    // the first seeding level (hub_only): C = {h}, so only h's slice has sources in C: its sample alone, in cps
    // parts (the other 127 of C4's 128 sample buckets would be streamed for nothing)
    const u32 hub_sl = (!FINAL && hub_only) ? (m->gmin >> kSliceBits) : 0u;
    const u32 n_items = SEG ? m->nseg : ((!FINAL && hub_only) ? (hub_sl < ns ? cps : 0u) : ns * cps);
    // thread 0: the open slow-list run of the current item (FINAL, recording)
    u32 seg_sl = 0xFFFFFFFFu, seg_start = 0;
    auto close_seg = [&]() {  // thread 0, after a barrier (every wave's slow stores of the item are done)
        if (!FINAL || SEG || !segs || seg_sl == 0xFFFFFFFFu) return;
        u32 end = s_slow;
        if (end & 1u) {  // pad to a pair: the next run starts 16-B aligned
            if (end < slow_cap) my_slow[end] = ~0ull;
            s_slow = ++end;
        }
        end = end < slow_cap ? end : slow_cap;
        if (end > seg_start) {
            const u32 k = atomicAdd(&m->nseg, 1u);
            segs[k] = SlowSeg{(u64)blockIdx.x * slow_cap + seg_start, seg_sl, end - seg_start};
        }
        seg_sl = 0xFFFFFFFFu;
    };
    while (true) {
        __syncthreads();
        if (threadIdx.x == 0) {
            close_seg();
            seg_start = s_slow;  // stable here: the item's waves add to s_slow only after the next barrier
            s_item = atomicAdd(&m->work[work_slot], 1u);
        }
        __syncthreads();
        const u32 item = s_item;
        if (item >= n_items) break;
        u32 sl;
        u64 len, lo, hi;
        const u64* src = bk;
        u64 ebase = 0;
        if constexpr (SEG) {
            const SlowSeg sg = segs[item];
            sl = sg.sl;
            src = bk + sg.off;
            lo = 0;
            hi = len = sg.len;
        } else {
            const bool hub = !FINAL && hub_only;
            sl = hub ? hub_sl : item / cps;
            len = m->bk_cur[sl] < m->bk_cap[sl] ? m->bk_cur[sl] : m->bk_cap[sl];
            if (!FINAL) len = len * frac >> 16;
            item_range(len, hub ? item : item % cps, cps, lo, hi);
            ebase = m->bk_base[sl];
        }
        if (lo >= hi) continue;
        if (threadIdx.x == 0) seg_sl = sl;
        if (sl != cur_slice) {
            load_slice<kP2Block>(s_bits, bits, sl, nwords32);
            cur_slice = sl;
            __syncthreads();
        }
        const u32 sbase = sl << kSliceBits;
        // SEG: u64 pairs [lo / 2, ceil(hi / 2)) of the slow list; buckets: 4-entry groups [lo / 4, ceil(hi / 4)) of the
        // 6-B entries. Either way entries outside [lo, hi) are masked (a part may start or end mid-pair / mid-group).
        const u64 plo = SEG ? lo / 2 : lo / 4;
        const u32 np = SEG ? (u32)((hi + 1) / 2 - plo) : (u32)((hi + 3) / 4 - plo);
        const u4* ep = reinterpret_cast<const u4*>(src) + plo;                        // SEG: pairs (16-B aligned)
        const u4* elo = reinterpret_cast<const u4*>(bk_lo + ebase) + plo;             // buckets: 16-B aligned
        const u64* ehi = reinterpret_cast<const u64*>(bk_hi + ebase) + plo;           // 8-B aligned
        constexpr u32 kRoundItems = SEG ? p2_round(PER) / 2 : p2_round(PER) / 4;  // pairs or groups per round
        constexpr int kL = SEG ? kQ : PER / 4;                        // loads (of each stream) per thread
        u4 q[kL];
        u64 qh[kL];
        auto load_round = [&](u32 p0) {
#pragma unroll
            for (int k = 0; k < kL; ++k) {
                const u32 j = p0 + (u32)k * kP2Block + threadIdx.x;
                const u32 jc = j < np ? j : np - 1;  // clamped: countable loads
                if constexpr (SEG) {
                    q[k] = __builtin_nontemporal_load(ep + jc);
                } else {
                    q[k] = __builtin_nontemporal_load(elo + jc);
                    qh[k] = __builtin_nontemporal_load(ehi + jc);
                }
            }
        };
        load_round(0);
        for (u32 p0 = 0; p0 < np; p0 += kRoundItems) {
            GCC_PH_MARK(phc, 7);  // (previous round's write-out / item switch)
            u32* s_cnt = s_cnt2 + rb * kMaxVLists;
            u32 ua[PER], va[PER], rk[PER];
            // per-entry flags as bit k of a VGPR (round 4: bool arrays became lane-mask SGPR pairs, 70 SGPRs
            // spilled at PER = 12)
            u32 in_m = 0;
            if constexpr (SEG) {
                const bool skip_first = lo & 1, skip_last = hi & 1;  // the part starts / ends in the middle of a pair
#pragma unroll
                for (int k = 0; k < kQ; ++k) {
                    const u32 j = p0 + (u32)k * kP2Block + threadIdx.x;
                    ua[2 * k] = q[k].x;
                    va[2 * k] = q[k].y;
                    ua[2 * k + 1] = q[k].z;
                    va[2 * k + 1] = q[k].w;
                    in_m |= (u32)(j < np && !(skip_first && j == 0) && ua[2 * k] != 0xFFFFFFFFu) << (2 * k);  // UNSEEN: a pad
                    in_m |= (u32)(j < np && !(skip_last && j == np - 1) && ua[2 * k + 1] != 0xFFFFFFFFu) << (2 * k + 1);
                }
            } else {
#pragma unroll
                for (int k = 0; k < kL; ++k) {
                    const u32 j = p0 + (u32)k * kP2Block + threadIdx.x;
                    const u64 e0 = 4 * (plo + j);  // the group's first entry index in the bucket
                    const u32 lv[4] = {q[k].x, q[k].y, q[k].z, q[k].w};
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const u16 h16 = (u16)(qh[k] >> (16 * c));
                        const bool real = bk_decode(lv[c], h16, sbase, ua[4 * k + c], va[4 * k + c]);
                        in_m |= (u32)(j < np && real && e0 + c >= lo && e0 + c < hi) << (4 * k + c);
                    }
                }
            }
            u32 bad = 0;
#pragma unroll
            for (int k = 0; k < PER; ++k) {  // the target indexes global lists (v-lists, parent[]): < cap
                const u32 big = (u32)(va[k] >= cap) & (in_m >> k);
                bad |= big;
                in_m &= ~(big << k);
            }
            if (bad) flag_err(err, kErrP2);
            GCC_PH_MARK(phc, 0);  // waited for this round's loads, decoded
            if (p0 + kRoundItems < np) load_round(p0 + kRoundItems);  // next round in flight
            u32 emit_m = 0;  // edges whose source is in C, bit k
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if ((in_m >> k) & 1u) emit_m |= lds_bit(s_bits, ua[k] - sbase) << k;
            if constexpr (SEG) {
                // (round 4) the second level's other direction: an edge whose source is not in C | N but whose
                // target is (the global bitmap: C | N, written by the join before this pass) hooks the SOURCE — it
                // goes to the v-lists as u (P3 adds it to N', the join hooks it) instead of the slow list, where 3/4
                // of C4's and the share's slow-kernel input were such hooks, profiles/r4j_stats_*.log)
                u32 gw[PER];
#pragma unroll
                for (int k = 0; k < PER; ++k) gw[k] = ((in_m & ~emit_m) >> k) & 1u ? bits[va[k] >> 5] : 0u;
#pragma unroll
                for (int k = 0; k < PER; ++k)
                    if ((gw[k] >> (va[k] & 31)) & 1u) {
                        va[k] = ua[k];
                        emit_m |= 1u << k;
                    }
            }
            const u32 slow_m = in_m & ~emit_m;  // FINAL: this lane's slow edges (neither rule applies), bit k
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if ((emit_m >> k) & 1u) rk[k] = atomicAdd(&s_cnt[va[k] >> kVSliceBits], 1u);
            GCC_PH_MARK(phc, 1);  // source lookups + LDS counting
            if constexpr (FINAL) {  // the slow edges: into this block's region of the slow list, one LDS add per wave
                // positions from one ballot per entry slot k (k-major: the lanes of one store are consecutive);
                // round 3 scanned the lanes' counts with 6 cross-lane shuffles every round, slow edges or not
                u32 tot = 0;
#pragma unroll
                for (int k = 0; k < PER; ++k) tot += (u32)__popcll(__ballot((slow_m >> k) & 1u));
                if (tot) {  // wave-uniform
                    u32 base = 0;
                    if (lane == 0) base = atomicAdd(&s_slow, tot);
                    base = __builtin_amdgcn_readfirstlane(base);
                    u32 spill_m = 0;
#pragma unroll
                    for (int k = 0; k < PER; ++k) {
                        const u64 b = __ballot((slow_m >> k) & 1u);
                        if (b) {
                            const u32 pos = base + __builtin_amdgcn_mbcnt_hi((u32)(b >> 32), __builtin_amdgcn_mbcnt_lo((u32)b, 0u));
                            if ((slow_m >> k) & 1u) {
                                if (pos < slow_cap) my_slow[pos] = ((u64)va[k] << 32) | ua[k];
                                else spill_m |= 1u << k;
                            }
                            base += (u32)__popcll(b);
                        }
                    }
                    if (__ballot(spill_m != 0)) {  // past the region (never at the default sizes): united right here
                        if (lane == 0) atomicOr(&m->ring_used, 1u);
#pragma unroll
                        for (int k = 0; k < PER; ++k)
                            ring_push((spill_m >> k) & 1u, ua[k], va[k], ring, wq, wd, parent, drain_at, 0xFFFFFFFFu);
                    }
                }
            }
            GCC_PH_MARK(phc, 2);  // slow-list stores
            __syncthreads();  // (1) counts of this round complete
            GCC_PH_MARK(phc, 3);
            constexpr u32 kHm = (1u << (kVSliceBits - 16)) - 1;  // the local id's bits above 16
            // runs padded to a multiple of VW with UNSEEN (P3 skips it): a lane writes VW targets per store
            if (threadIdx.x < 64) wave_scan<VW>(s_cnt, s_start, nvs);
            for (u32 s = threadIdx.x; s < nvs; s += kP2Block) s_cnt2[(rb ^ 1) * kMaxVLists + s] = 0;  // next round's
            __syncthreads();  // (2) starts
            GCC_PH_MARK(phc, 4);
            // the reservations (their global atomics) overlap the other waves' scatter
            for (u32 s = threadIdx.x; s < nvs; s += kP2Block) {
                const u32 pc = padw<VW>(s_cnt[s]);
                if (pc) reserve_run(runs, s, pc, &m->vl_cur[pass][s], s_vcap[s], chunk);
                for (u32 j = s_cnt[s]; j < pc; ++j) s_vt[s_start[s] + j] = 0xFFFFFFFFu;
            }
#pragma unroll
            for (int k = 0; k < PER; ++k)
                if ((emit_m >> k) & 1u) s_vt[s_start[va[k] >> kVSliceBits] + rk[k]] = va[k];
            GCC_PH_MARK(phc, 5);
            __syncthreads();  // (3) tile in bucket order
            GCC_PH_MARK(phc, 6);
            const u32 totw = (s_start[nvs - 1] + padw<VW>(s_cnt[nvs - 1])) / VW;
            auto hib = [](u32 x) { return x == 0xFFFFFFFFu ? (u32)kPadV : (x >> 16 & kHm); };
            for (u32 xw = threadIdx.x; xw < totw; xw += kP2Block) {
                u32 v[VW];
#pragma unroll
                for (int k = 0; k < VW / 4; ++k) {  // slot VW xw is never padding
                    const u4 q4 = reinterpret_cast<const u4*>(s_vt)[(VW / 4) * xw + k];
                    v[4 * k] = q4.x;
                    v[4 * k + 1] = q4.y;
                    v[4 * k + 2] = q4.z;
                    v[4 * k + 3] = q4.w;
                }
                const u32 s = v[0] >> kVSliceBits;
                const u32 off = run_pos(runs, s, VW * xw - s_start[s]);  // a multiple of VW: one chunk
                if (off != 0xFFFFFFFFu) {  // bases: 16-entry multiples, off: VW
                    if constexpr (VW == 8) {  // 16-B lo / 8-B hi stores
                        typedef u16 u16x8 __attribute__((ext_vector_type(8)));
                        const u16x8 lo = {(u16)v[0], (u16)v[1], (u16)v[2], (u16)v[3],
                                          (u16)v[4], (u16)v[5], (u16)v[6], (u16)v[7]};
                        const u64 hi = (u64)(hib(v[0]) | hib(v[1]) << 8 | hib(v[2]) << 16 | hib(v[3]) << 24) |
                                       (u64)(hib(v[4]) | hib(v[5]) << 8 | hib(v[6]) << 16 | hib(v[7]) << 24) << 32;
                        *reinterpret_cast<u16x8*>(vl.lo + s_vbase[s] + off) = lo;
                        *reinterpret_cast<u64*>(vl.hi + s_vbase[s] + off) = hi;
                    } else {  // 8-B lo / 4-B hi stores
                        const u16x4 lo = {(u16)v[0], (u16)v[1], (u16)v[2], (u16)v[3]};
                        const u32 hi = hib(v[0]) | hib(v[1]) << 8 | hib(v[2]) << 16 | hib(v[3]) << 24;
                        *reinterpret_cast<u16x4*>(vl.lo + s_vbase[s] + off) = lo;
                        *reinterpret_cast<u32*>(vl.hi + s_vbase[s] + off) = hi;
                    }
                } else if (FINAL) {  // the v-list is full: (u in C, v) = union(g, v) now
#pragma unroll
                    for (int k = 0; k < VW; ++k)
                        if (v[k] != 0xFFFFFFFFu) hook_g(parent, g, v[k]);
                }
            }
            rb ^= 1;  // the write-out above is done before anyone passes the next round's barrier (1)
        }
    }
    __syncthreads();
    if constexpr (FINAL && !SEG) GCC_PH_FLUSH(phc, 1);
    // the unused tails of this block's chunks: UNSEEN (P3 skips them)
    for (u32 s = 0; s < nvs; ++s)
        for (u32 i = runs.cpos[s] + threadIdx.x; i < runs.cend[s]; i += kP2Block) vl.hi[s_vbase[s] + i] = kPadV;
    if constexpr (FINAL) {  // the rest of this wave's ring; the block's slow count
        for (; wd < wq; wd += 64) {
            if (lane < wq - wd) {
                const u64 e = ring[(wd + lane) & (kRing - 1)];
                unite_entry(parent, (u32)e, (u32)(e >> 32), 0xFFFFFFFFu);
            }
        }
        if (threadIdx.x == 0) m->slow_cnt[blockIdx.x] = s_slow < slow_cap ? s_slow : slow_cap;
    }
    GCC_BT(FINAL ? (SEG ? 2 : 1) : 5, 1);
}

// ---- P3: the target slice ------------------------------------------------------------------------------------
// Every v of the slice's v-list that is not in C (LDS slice) is reached from C: it joins the block's LDS copy of
// the slice (atomicOr). When the block leaves a slice its new members are OR-ed into `out` (one atomicOr per
// changed word): SEED: out = the bitmap of C itself (C grows for the next level; the block's minimum new id goes
// to m->gmin); FINAL: out = N, the bitmap of the ids reached from C (bucket_hook_kernel hooks them under g, once
// each). The v-list streams 16 B per lane, kP3Q loads in flight.
#ifndef GCC_P3Q
#define GCC_P3Q 8
#endif
constexpr int kP3Q = GCC_P3Q;  // 4-entry groups per thread per iteration: 8 beat 4 and 2 (C4 P3 0.69 / 0.75 / 0.85 ms, profiles/r3p_ab_p3_loads.log)
template <bool FINAL>
__global__ __launch_bounds__(kP3Block) void slice_hook_kernel(u32* __restrict__ bits, u32* __restrict__ out,
                                                              u32 nwords32, u32 ns, Meta* __restrict__ m,
                                                              VList vl, u32 cps, u32 work_slot,
                                                              u32 cap, u32* __restrict__ err, u32 pass) {
    trace_start(FINAL ? kTrBkP3 : kTrBkP3Seed);
    GCC_BT(FINAL ? (pass == kVlLevel2 ? 4 : 3) : 6, 0);
    extern __shared__ __attribute__((aligned(16))) u32 s_bits[];  // kVSliceWords
    __shared__ u32 s_item, s_min;
    u32 cur_slice = 0xFFFFFFFFu;
    const u32 n_items = ns * cps;  // ns: the v-list count (vslices)
    u32 lmin = 0xFFFFFFFFu;
    auto flush_slice = [&]() {  // this block's new members of cur_slice -> out
        if (cur_slice == 0xFFFFFFFFu) return;
        const u32 w0 = cur_slice * kVSliceWords;
        // 8 words' global loads in flight together (round 5: a word per iteration waited out a load latency per word,
        // 32 per thread per flush; the signed fold's flush gained 60 us a check kernel from the same change)
        constexpr int kPer = 8;
        for (u32 wb = 0; wb < kVSliceWords; wb += kPer * kP3Block) {
            u32 g[kPer], o[kPer];
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const u32 w = wb + k * kP3Block + threadIdx.x;
                const bool in = w < kVSliceWords && w0 + w < nwords32;
                g[k] = in ? bits[w0 + w] : ~0u;
                o[k] = FINAL && in ? out[w0 + w] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kPer; ++k) {
                const u32 w = wb + k * kP3Block + threadIdx.x;
                if (w >= kVSliceWords || w0 + w >= nwords32) continue;
                const u32 nw = s_bits[w] & ~g[k];
                if (nw && (!FINAL || (nw & ~o[k]))) atomicOr(&out[w0 + w], nw);
            }
        }
    };
    auto visit = [&](u32 x, u32 sbase) {  // x: the slice-local target (19 bits: only indexes this block's LDS slice)
        const u32 msk = 1u << (x & 31);
        if (s_bits[x >> 5] & msk) return;                  // already in C (or taken by this block)
        if (atomicOr(&s_bits[x >> 5], msk) & msk) return;  // another lane of the block took it
        if (!FINAL) lmin = (sbase | x) < lmin ? (sbase | x) : lmin;
    };
    while (true) {
        __syncthreads();
        if (threadIdx.x == 0) s_item = atomicAdd(&m->work[work_slot], 1u);
        __syncthreads();
        const u32 item = s_item;
        if (item >= n_items) break;
        const u32 sl = item / cps;
        const u64 len = m->vl_cur[pass][sl] < m->vl_cap[sl] ? m->vl_cur[pass][sl] : m->vl_cap[sl];
        u64 lo, hi;
        item_range(len, item % cps, cps, lo, hi);
        if (lo >= hi) continue;
        if (sl != cur_slice) {
            flush_slice();
            __syncthreads();
            load_slice<kP3Block, kVSliceWords>(s_bits, bits, sl, nwords32);
            cur_slice = sl;
            __syncthreads();
        }
        const u64* vlo = reinterpret_cast<const u64*>(vl.lo + m->vl_base[sl]);  // 4 entries per 8 B (aligned)
        const u32* vhi = reinterpret_cast<const u32*>(vl.hi + m->vl_base[sl]);  // 4 entries per 4 B
        const u32 sbase = sl << kVSliceBits;
        const u64 qlo = lo / 4, qhi = (hi + 3) / 4;  // 4-entry groups; entries outside [lo, hi) masked
        for (u64 b = qlo; b < qhi; b += (u64)kP3Q * kP3Block) {
            u64 rl[kP3Q];
            u32 rh[kP3Q];
#pragma unroll
            for (int k = 0; k < kP3Q; ++k) {
                const u64 j = b + (u64)k * kP3Block + threadIdx.x;
                const u64 jc = j < qhi ? j : qhi - 1;  // clamped: countable loads
                rl[k] = __builtin_nontemporal_load(vlo + jc);
                rh[k] = __builtin_nontemporal_load(vhi + jc);
            }
#pragma unroll
            for (int k = 0; k < kP3Q; ++k) {
                const u64 j = b + (u64)k * kP3Block + threadIdx.x;
                if (j >= qhi) continue;
                const u64 e = 4 * j;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const u32 h8 = (rh[k] >> (8 * c)) & 0xFFu;
                    if (h8 != kPadV && e + c >= lo && e + c < hi)  // padding: a P2 run pad or chunk tail
                        visit((h8 << 16) | (u32)((rl[k] >> (16 * c)) & 0xFFFFu), sbase);
                }
            }
        }
    }
    __syncthreads();
    flush_slice();
    if constexpr (!FINAL) {
        for (int o = 32; o > 0; o >>= 1) lmin = min(lmin, (u32)__shfl_down(lmin, o, 64));
        if (threadIdx.x == 0) s_min = 0xFFFFFFFFu;
        __syncthreads();
        if ((threadIdx.x & 63) == 0 && lmin != 0xFFFFFFFFu) atomicMin(&s_min, lmin);
        __syncthreads();
        if (threadIdx.x == 0 && s_min != 0xFFFFFFFFu) atomicMin(&m->gmin, s_min);
    }
    GCC_BT(FINAL ? (pass == kVlLevel2 ? 4 : 3) : 6, 1);
}

// N (ids reached from C by the FINAL pass) joins g's tree, each id once: a new id above g by a plain store (in this
// kernel nothing else writes an UNSEEN slot: the hooks below only touch seen ids and roots), anything else by
// hook_g. The tracked component's bitmap becomes C | N (one component: g's), N is cleared for the next batch.
__global__ __launch_bounds__(kBlock) void bucket_hook_kernel(u32* __restrict__ parent, u32* __restrict__ bits,
                                                             u32* __restrict__ nbits, u32 nwords32,
                                                             const u32* __restrict__ giant) {
    trace_start(kTrBkHook);
    const u32 g = *giant;
    for (u64 w = (u64)blockIdx.x * kBlock + threadIdx.x; w < nwords32; w += (u64)gridDim.x * kBlock) {
        u32 d = nbits[w];
        if (!d) continue;
        nbits[w] = 0;
        d &= ~bits[w];
        if (!d || g == GCC_UNSEEN_DEV) continue;
        bits[w] |= d;
        while (d) {
            const u32 k = (u32)__builtin_ctz(d);
            d &= d - 1;
            const u32 v = (u32)(w * 32 + k);
            if (v > g && parent[v] == GCC_UNSEEN_DEV) parent[v] = g;
            else hook_g(parent, g, v);
        }
    }
}

// Deferred N (tune.bucket_defer): C |= N word by word, and N stays in nbits, UNSEEN in parent[], until the fold's
// closing compress labels it g's root (compress_bits_kernel's newbits) — no per-id store — except the ids below g,
// hooked here (each may become the component's root). Every later pass of
// the fold treats an edge with one end in C | N as the hook of its other end (slow, rest), so nothing unions an
// id of N directly; only FINAL P2's in-kernel ring unions (a full slow region, m->ring_used) could have made one
// seen, and then every seen id of N is hooked under g here. later (a later window, round 4): ids of N may be seen
// already, members of other components: every seen id of N is hooked under g here, only the new ones are deferred.
// defer_c (a fresh forest, round 5): C itself is deferred the same way — P1 reset parent[] to UNSEEN and no kernel
// stored g into C's slots (bucket_init_kernel's job until round 4), so nbits := C | N here, for the closing compress,
// and with ring_used the seen ids of C are hooked too (a ring union may have made one seen, under another root).
__global__ __launch_bounds__(kBlock) void bucket_join_kernel(u32* __restrict__ parent, u32* __restrict__ bits,
                                                             u32* __restrict__ nbits, u32 nwords32,
                                                             const u32* __restrict__ giant, const Meta* __restrict__ m,
                                                             u32 later, u32 defer_c) {
    trace_start(kTrBkHook);
    const u32 g = *giant;
    const bool ring = m->ring_used != 0 || later;
    for (u64 w = (u64)blockIdx.x * kBlock + threadIdx.x; w < nwords32; w += (u64)gridDim.x * kBlock) {
        u32 d = nbits[w];
        const u32 cw = defer_c ? bits[w] : 0u;
        if (defer_c) {
            if (!(d | cw)) continue;
            if (~d & cw) nbits[w] = d | cw;
            if (ring) d |= cw;  // the seen ids of C too
        } else if (!d) {
            continue;
        }
        bits[w] |= d;
        if (g == GCC_UNSEEN_DEV) continue;
        // an id below g is hooked now: it becomes the component's root, which the compress must find
        const u64 w0 = w * 32;
        const u32 low = w0 >= g ? 0u : (w0 + 31 < g ? d : d & ((1u << (u32)(g - w0)) - 1u));
        u32 todo = ring ? d : low;
        while (todo) {
            const u32 k = (u32)__builtin_ctz(todo);
            todo &= todo - 1;
            const u32 v = (u32)(w0 + k);
            if (v < g || parent[v] != GCC_UNSEEN_DEV) hook_g(parent, g, v);
        }
    }
}

// The slow list (FINAL P2: edges whose source was not in C) against C | N: both ends in it -> already connected to
// g; one end -> the other hooked under g; neither -> united. Block b takes part b % kSlowSplit of P2 block
// (b / kSlowSplit)'s region, only up to that region's count (a grid-stride over every region's capacity read the
// count for each of C4's 134M slots, most of them empty).
constexpr u32 kSlowSplit = 8;
__global__ __launch_bounds__(kBlock) void bucket_slow_kernel(u32* __restrict__ parent, const u64* __restrict__ slow,
                                                             u32 slow_cap, const Meta* __restrict__ m, u32 nblocks,
                                                             const u32* __restrict__ bits, const u32* __restrict__ giant,
                                                             u32 cap, u32* __restrict__ err) {
    trace_start(kTrBkSlow);
    GCC_BT(7, 0);
    const u32 g = *giant;
    NoCount c;
    const u32 r = blockIdx.x / kSlowSplit, part = blockIdx.x % kSlowSplit;
    if (r >= nblocks) {
        GCC_BT(7, 1);
        return;
    }
    const u32 cnt = m->slow_cnt[r];
    const u64* list = slow + (u64)r * slow_cap;
    for (u32 k = part * kBlock + threadIdx.x; k < cnt; k += kSlowSplit * kBlock) {
        const u64 e = list[k];
        if (e == ~0ull) continue;  // a run's pad entry (slice_filter_kernel's close_seg)
        const u32 a = (u32)e, b = (u32)(e >> 32);
        if (a >= cap || b >= cap) {
            flag_err(err, kErrSlow);
            continue;
        }
        const u32 ia = lds_bit(bits, a), ib = lds_bit(bits, b);
        if (ia & ib) continue;
        if (ia) hook_g(parent, g, b);
        else if (ib) hook_g(parent, g, a);
        else UF::unite(parent, a, b, c);
    }
    GCC_BT(7, 1);
}

// Seeding start: clear the bitmap (done by the host's memset), elect the hub h of the batch's first edges (the
// same deterministic election as the seeded fold), C := {h}, gmin := h. One block.
__global__ __launch_bounds__(kHubBlock) void bucket_hub_kernel(const u64* __restrict__ edges, u64 n, u32 cap,
                                                               u32* __restrict__ bits, Meta* __restrict__ m) {
    trace_start(kTrBkHub);
    extern __shared__ __attribute__((aligned(16))) u32 s_tab[];
    u64 e[kHubPer];
    hub_sample(edges, n < kHubSample ? n : kHubSample, e);
    const u32 h = hub_elect(e, s_tab, cap);
    if (threadIdx.x == 0) {
        m->gmin = h;
        if (h != GCC_UNSEEN_DEV) bits[h >> 5] = 1u << (h & 31);
    }
}

// giant := g = min C, the component's representative (a fresh forest whose C is deferred: P1 did the reset).
__global__ void bucket_root_kernel(const Meta* __restrict__ m, u32* __restrict__ giant) {
    trace_start(kTrBkInit);
    *giant = m->gmin;
}

// parent[v] := v in C ? g : UNSEEN over the whole id range (the reset and all of C's unions in one write);
// giant := g. 4 ids per lane, 16-B stores. (With bucket_defer: P1's reset + bucket_root_kernel instead.)
__global__ __launch_bounds__(kBlock) void bucket_init_kernel(u32* __restrict__ parent, u32 n,
                                                             const u32* __restrict__ bits, const Meta* __restrict__ m,
                                                             u32* __restrict__ giant) {
    trace_start(kTrBkInit);
    const u32 g = m->gmin;
    if (blockIdx.x == 0 && threadIdx.x == 0) *giant = g;
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u64 nq = ((u64)n + 3) / 4;
    for (u64 q = (u64)blockIdx.x * kBlock + threadIdx.x; q < nq; q += (u64)gridDim.x * kBlock) {
        const u32 w = bits[q >> 3] >> ((q & 7) * 4);
        const u64 v = 4 * q;
        if (v + 3 < n) {
            u4 o;
            o.x = (w & 1u) ? g : GCC_UNSEEN_DEV;
            o.y = (w & 2u) ? g : GCC_UNSEEN_DEV;
            o.z = (w & 4u) ? g : GCC_UNSEEN_DEV;
            o.w = (w & 8u) ? g : GCC_UNSEEN_DEV;
            reinterpret_cast<u4*>(parent)[q] = o;
        } else {
            for (u32 k = 0; k < 4; ++k)
                if (v + k < n) parent[v + k] = ((w >> k) & 1u) ? g : GCC_UNSEEN_DEV;
        }
    }
}

// The overflow list (edges their bucket had no room for): united, skipped when both ends are in C. If the list
// itself overflowed (spill), the WHOLE batch is united again: exact (union is idempotent), only slow.
// An edge with one end in C | N (g's component) is the hook of its other end, and with both ends there nothing:
// the overflow list and the whole-batch fallback take the slow kernel's rule, so they never union an id of C | N
// directly (with the deferred N, such an id may still be UNSEEN: bucket_join_kernel).
__device__ __forceinline__ void bucket_edge(u32* parent, const u32* bits, u32 g, u32 a, u32 b) {
    NoCount c;
    const u32 ia = lds_bit(bits, a), ib = lds_bit(bits, b);
    if (ia & ib) return;
    if (ia) hook_g(parent, g, b);
    else if (ib) hook_g(parent, g, a);
    else UF::unite(parent, a, b, c);
}

__global__ __launch_bounds__(kBlock) void bucket_rest_kernel(u32* __restrict__ parent, const u64* __restrict__ ovf,
                                                             u32 ovf_cap, const Meta* __restrict__ m,
                                                             const u32* __restrict__ bits,
                                                             const u64* __restrict__ edges, u64 n, u32 cap,
                                                             u32* __restrict__ err, const u32* __restrict__ giant) {
    trace_start(kTrBkRest);
    const u32 g = *giant;
    const u64 stride = (u64)gridDim.x * kBlock;
    const u64 no = m->ovf_cur < ovf_cap ? m->ovf_cur : ovf_cap;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < no; i += stride) {
        const u64 e = ovf[i];
        const u32 a = (u32)e, b = (u32)(e >> 32);
        if (a >= cap || b >= cap) {
            flag_err(err, kErrOvf);
            continue;
        }
        bucket_edge(parent, bits, g, a, b);
    }
    if (m->spill) {
        for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
            const u64 e = edges[i];
            u32 a = (u32)e, b = (u32)(e >> 32);
            if (!edge_ok(a, b, cap, err)) continue;
            bucket_edge(parent, bits, g, a, b);
        }
    }
}

}  // namespace bk
