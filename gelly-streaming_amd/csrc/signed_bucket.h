// signed_bucket.h — the BUCKETED giant-filtered fold of the signed forest (BipartitenessCheck's summary, gelly_bip.hip),
// round 5. Included by gelly_cc.hip after bucket_fold.h, whose P1 (bucket_kernel: the batch split
// by the first id's 2^19-id slice into 6-B entries) it reuses as a plain partition; the host side is
// gcc_internal_signed_bucket in gelly_cc.hip, called by gelly_bip.hip's signed_fold.
//
// The giant-filtered fold (gelly_bip.hip signed_fold_giant_kernel) looks up two 2-bit snapshot entries per edge — in
// C (the voted component), and the parity to C's root r — in a 16 MiB array at 2^26 ids, beyond an XCD's L2: random
// 64-B line fetches bound it (1.7 misses per edge). Here both lookups find their slice of the snapshot in LDS:
//   sb_filter_kernel   per source-slice bucket, the slice's 2 bits per id in LDS (128 KiB): u in C -> the pair
//                      (v, parity(u) ^ 1) joins the EMIT list (v must carry that parity); else the edge joins the SLOW
//                      list with its ends swapped (block-aggregated appends: one global add per list per 16K
//                      entries), and counts both lists' entries per slice of their first id (the next P1's exact layout)
//   bucket_kernel      the emit list split by v's slice (the same P1, KEYONLY: 4-B entries, v's slice-local bits |
//                      parity << 19)
//   sb_check_kernel    per target-slice bucket, the slice in LDS: v in C -> its parity must be the pair's, else the
//                      batch has an odd cycle (fail); v not in C -> v joins the block's LDS copy with that parity (a
//                      lane that finds it added with the other parity: fail); at the end of its items a block ORs
//                      its new members into N2, 2 bits per id: "reached with parity 0", "with parity 1"
//   sb_join_low_kernel the new members below r united with r first (each makes C's root a smaller id)
//   sb_join_kernel     C |= N2 (both parities: fail); a new member already seen in the forest (the sample's fold made
//                      it seen in another tree) is united with C's root R (found once per block) with its parity; the
//                      others stay UNSEEN in the forest — DEFERRED, as the CC fold's N (bucket_join_kernel)
// then the same again over the slow list against C | N (a second level; `levels`: up to 3) — by the edges' OTHER ends:
// a bipartite stream's sources and targets can be disjoint sets (to_bipartite: even -> odd ids), and N holds targets —
// and the remaining edges by
//   sb_rest_kernel     the giant kernel's rule with deferred members: an edge with one end x outside C unites x with
//                      r (never with the deferred end itself); neither end in C: the signed union
//   sb_compress_kernel the closing compress: a member of C is labelled (root(r) << 1) | (its parity ^ r's parity to
//                      root(r)) straight from the bits (the deferred ones need no forest entry); the others by find.
// Every parity a bit holds is implied by edges of the batch (the snapshot's by the forest, the rest by an edge from a
// member), so two bits that disagree are an odd cycle: the summary fails, as the reference's Candidates.merge does at
// the edge that closes it (…/summaries/Candidates.java:77-139; a failed summary's words are not part of the contract).
#pragma once

#include "signed_uf.h"

namespace sb {

using bk::kSliceBits;
constexpr u32 kSliceW = (1u << kSliceBits) / 16;  // 2-bit words of a slice: 32768 (128 KiB of LDS)
constexpr int kBlock = 1024;
constexpr u32 kMask2 = 0x55555555u;               // bit 2j of every 2-bit pair
constexpr int kGroups = 4;                         // 4-entry groups per lane per filter round

__device__ __forceinline__ u32 pair2(u32 w, u32 x) { return (w >> (2 * (x & 15))) & 3u; }

// the slice's 2-bit words of the snapshot into LDS (beyond the id range: zero). 16-B loads, all of a thread's in flight
// before its LDS stores (a word per iteration waited out one load latency per word: 32 per thread per slice)
__device__ __forceinline__ void load_slice2(u32* s, const u32* __restrict__ g, u32 sl, u32 nw16) {
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u32 w0 = sl * kSliceW;
    if (w0 + kSliceW <= nw16 && blockDim.x == kBlock) {  // a whole slice: 8 x 16 B per thread
        constexpr int kPer = kSliceW / 4 / kBlock;
        const u4* q = reinterpret_cast<const u4*>(g + w0);
        u4 v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) v[k] = q[k * kBlock + threadIdx.x];
#pragma unroll
        for (int k = 0; k < kPer; ++k) reinterpret_cast<u4*>(s)[k * kBlock + threadIdx.x] = v[k];
        return;
    }
    for (u32 w = threadIdx.x; w < kSliceW; w += blockDim.x) s[w] = w0 + w < nw16 ? g[w0 + w] : 0u;
}

// Block-aggregated appends of this round's entries (K per lane: entry c goes to list 0 if bit c of m0 is set, to
// list 1 if bit c of m1) to two global lists: a wave's counts by ballots, the block's by one scan in LDS, ONE global
// add per list per round.
struct Appender {
    u32* s_wc;    // [16 waves][2 lists]
    u32* s_base;  // [2]
};
template <int K>
__device__ __forceinline__ void append2(const Appender& ap, u32* cursors, u64* l0, u64* l1, u32 m0, u32 m1,
                                        const u64 (&e)[K]) {
    const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    u32 c0 = 0, c1 = 0;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        c0 += (u32)__popcll(__ballot((m0 >> c) & 1u));
        c1 += (u32)__popcll(__ballot((m1 >> c) & 1u));
    }
    if (lane == 0) {
        ap.s_wc[2 * wv] = c0;
        ap.s_wc[2 * wv + 1] = c1;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        u32 tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            const u32 c = ap.s_wc[2 * w + threadIdx.x];
            ap.s_wc[2 * w + threadIdx.x] = tot;
            tot += c;
        }
        ap.s_base[threadIdx.x] = tot ? atomicAdd(&cursors[threadIdx.x], tot) : 0u;
    }
    __syncthreads();
    u32 p0 = ap.s_base[0] + ap.s_wc[2 * wv], p1 = ap.s_base[1] + ap.s_wc[2 * wv + 1];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const u64 b0 = __ballot((m0 >> c) & 1u), b1 = __ballot((m1 >> c) & 1u);
        const u32 r0 = __builtin_amdgcn_mbcnt_hi((u32)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((u32)b0, 0u));
        const u32 r1 = __builtin_amdgcn_mbcnt_hi((u32)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((u32)b1, 0u));
        if ((m0 >> c) & 1u) l0[p0 + r0] = e[c];
        if ((m1 >> c) & 1u) l1[p1 + r1] = e[c];
        p0 += (u32)__popcll(b0);
        p1 += (u32)__popcll(b1);
    }
}

// Work items: (slice, part) of the buckets, dequeued from ctr[0]. Every round of a block takes 4 entries per lane.
// ctr[1] / ctr[2]: the emit / slow cursors.
__global__ __launch_bounds__(kBlock) void sb_filter_kernel(const u32* __restrict__ bk_lo, const bk::u16* __restrict__ bk_hi,
                                                           const bk::Meta* __restrict__ m, u32 ns, u32 cps,
                                                           u32* __restrict__ ctr, const u32* __restrict__ gbits, u32 nw16,
                                                           u64* __restrict__ emit, u64* __restrict__ slow, u32 cap,
                                                           u32* __restrict__ hist_e, u32* __restrict__ hist_s,
                                                           u32* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) u32 s_bits[];  // kSliceW
    __shared__ u32 s_item, s_wc[2 * (kBlock / 64)], s_base[2];
    // the lists' entries per slice of their first id (the emitted target, the slow edge's other end): the next P1's
    // exact layout (no sample; bucket_layout_kernel `exact`)
    __shared__ u32 s_he[bk::kMaxBuckets], s_hs[bk::kMaxBuckets];
    const Appender ap{s_wc, s_base};
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    for (u32 s = threadIdx.x; s < ns; s += kBlock) s_he[s] = s_hs[s] = 0;
    const u32 n_items = ns * cps;
    u32 cur = 0xFFFFFFFFu;
    while (true) {
        __syncthreads();
        if (threadIdx.x == 0) s_item = atomicAdd(&ctr[0], 1u);
        __syncthreads();
        const u32 item = s_item;
        if (item >= n_items) break;
        const u32 sl = item / cps;
        const u64 len = m->bk_cur[sl] < m->bk_cap[sl] ? m->bk_cur[sl] : m->bk_cap[sl];
        u64 lo, hi;
        bk::item_range(len, item % cps, cps, lo, hi);
        if (lo >= hi) continue;
        if (sl != cur) {
            load_slice2(s_bits, gbits, sl, nw16);
            cur = sl;
            __syncthreads();
        }
        const u32 sbase = sl << kSliceBits;
        const u64 base = m->bk_base[sl];
        const u64 g0 = lo / 4, g1 = (hi + 3) / 4;  // 4-entry groups (bases: 16-entry multiples)
        // a round: kGroups 4-entry groups per lane, all loads issued first (one block per CU — the slice takes 128 KiB
        // of LDS —, so a round's latency is not hidden by other blocks: 4 entries per lane measured 0.6 ms at level 1)
        for (u64 gb = g0; gb < g1; gb += kGroups * kBlock) {  // block-uniform
            u32 em = 0, smk = 0, bad = 0;
            u64 val[4 * kGroups];
            u4 l4[kGroups];
            u64 h4[kGroups];
#pragma unroll
            for (int k = 0; k < kGroups; ++k) {
                const u64 g = gb + (u64)k * kBlock + threadIdx.x;
                l4[k] = g < g1 ? *reinterpret_cast<const u4*>(bk_lo + base + 4 * g) : u4{0, 0, 0, 0};
                h4[k] = g < g1 ? *reinterpret_cast<const u64*>(bk_hi + base + 4 * g) : ~0ull;
            }
#pragma unroll
            for (int k = 0; k < kGroups; ++k) {
                const u64 g = gb + (u64)k * kBlock + threadIdx.x;
                const u32 lv[4] = {l4[k].x, l4[k].y, l4[k].z, l4[k].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int j = 4 * k + c;
                    u32 u, v;
                    const u64 e = 4 * g + c;
                    val[j] = 0;
                    if (!bk::bk_decode(lv[c], (bk::u16)(h4[k] >> (16 * c)), sbase, u, v) || e < lo || e >= hi) continue;
                    if (v >= cap) {
                        bad = 1;
                        continue;
                    }
                    const u32 b = pair2(s_bits[(u - sbase) >> 4], u);
                    if (b & 1u) {  // u in C: v must take the other parity (a self loop in C: nothing to do)
                        if (u != v) {
                            val[j] = (u64)v | ((u64)(((b >> 1) & 1u) ^ 1u) << 32);
                            em |= 1u << j;
                            atomicAdd(&s_he[v >> kSliceBits], 1u);
                        }
                    } else {  // slow: listed with its ends SWAPPED, so that the next level looks at the other end
                        val[j] = ((u64)u << 32) | v;
                        smk |= 1u << j;
                        atomicAdd(&s_hs[v >> kSliceBits], 1u);
                    }
                }
            }
            if (bad) bk::flag_err(err, bk::kErrP2);
            append2<4 * kGroups>(ap, ctr + 1, emit, slow, em, smk, val);
        }
    }
    __syncthreads();
    for (u32 s = threadIdx.x; s < ns; s += kBlock) {
        if (s_he[s]) atomicAdd(&hist_e[s], s_he[s]);
        if (s_hs[s]) atomicAdd(&hist_s[s], s_hs[s]);
    }
}

// The new members of the block's slice copy (set in LDS, not in the snapshot) into N2: bit 2j "reached with parity
// 0", bit 2j + 1 "with parity 1" (memory-side ORs; the join reads them in a later kernel)
__device__ __forceinline__ void flush_slice2(const u32* s, const u32* __restrict__ gbits, u32* __restrict__ n2, u32 sl,
                                             u32 nw16) {
    const u32 w0 = sl * kSliceW;
    constexpr int kPer = 8;  // the snapshot's words of a batch of 8 LDS words in flight together
    for (u32 wb = 0; wb < kSliceW; wb += kPer * kBlock) {
        u32 g[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const u32 w = wb + k * kBlock + threadIdx.x;
            g[k] = w < kSliceW && w0 + w < nw16 ? gbits[w0 + w] : ~0u;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const u32 w = wb + k * kBlock + threadIdx.x;
            if (w >= kSliceW || w0 + w >= nw16) continue;
            const u32 lw = s[w];
            const u32 nm = lw & ~g[k] & kMask2;  // members this block added
            if (!nm) continue;
            const u32 p1 = (lw >> 1) & nm;
            atomicOr(&n2[w0 + w], (nm & ~p1) | (p1 << 1));
        }
    }
}

// Work items over the emit list's buckets (entries: v, parity p): see the header comment. ctr[0]: the item counter.
template <bool KEYONLY>
__global__ __launch_bounds__(kBlock) void sb_check_kernel(const u32* __restrict__ bk_lo, const bk::u16* __restrict__ bk_hi,
                                                          const bk::Meta* __restrict__ m, u32 ns, u32 cps,
                                                          u32* __restrict__ ctr, const u32* __restrict__ gbits, u32 nw16,
                                                          u32* __restrict__ n2, u32 cap, u32* __restrict__ fail,
                                                          u32* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) u32 s_bits[];  // kSliceW
    __shared__ u32 s_item;
    typedef u32 u4 __attribute__((ext_vector_type(4)));
    const u32 n_items = ns * cps;
    u32 cur = 0xFFFFFFFFu;
    u32 odd = 0;
    while (true) {
        __syncthreads();
        if (threadIdx.x == 0) s_item = atomicAdd(&ctr[0], 1u);
        __syncthreads();
        const u32 item = s_item;
        if (item >= n_items) break;
        const u32 sl = item / cps;
        const u64 len = m->bk_cur[sl] < m->bk_cap[sl] ? m->bk_cur[sl] : m->bk_cap[sl];
        u64 lo, hi;
        bk::item_range(len, item % cps, cps, lo, hi);
        if (lo >= hi) continue;
        if (sl != cur) {
            if (cur != 0xFFFFFFFFu) flush_slice2(s_bits, gbits, n2, cur, nw16);
            __syncthreads();
            load_slice2(s_bits, gbits, sl, nw16);
            cur = sl;
            __syncthreads();
        }
        const u32 sbase = sl << kSliceBits;
        const u64 base = m->bk_base[sl];
        const u64 g0 = lo / 4, g1 = (hi + 3) / 4;
        for (u64 g = g0 + threadIdx.x; g < g1; g += kBlock) {
            const u4 l4 = *reinterpret_cast<const u4*>(bk_lo + base + 4 * g);
            const u64 h4 = KEYONLY ? 0ull : *reinterpret_cast<const u64*>(bk_hi + base + 4 * g);
            const u32 lv[4] = {l4.x, l4.y, l4.z, l4.w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                u32 x, p;
                const u64 e = 4 * g + c;
                if (KEYONLY) {  // 4-B entries: x's slice-local bits | p << kSliceBits (bucket_fold.h KEYONLY); ~0 = padding
                    if (lv[c] == 0xFFFFFFFFu || e < lo || e >= hi) continue;
                    x = sbase | (lv[c] & (bk::kSliceIds - 1));
                    p = lv[c] >> kSliceBits;
                } else if (!bk::bk_decode(lv[c], (bk::u16)(h4 >> (16 * c)), sbase, x, p) || e < lo || e >= hi) {
                    continue;
                }
                if (x >= cap || p > 1u) {
                    bk::flag_err(err, bk::kErrP2);
                    continue;
                }
                const u32 xl = x - sbase, sh = 2 * (xl & 15);
                const u32 b = (s_bits[xl >> 4] >> sh) & 3u;
                if (b & 1u) {  // a member (of C, or added by this block): the parities must agree
                    odd |= (b >> 1) != p;
                } else {
                    const u32 o = (atomicOr(&s_bits[xl >> 4], (1u | p << 1) << sh) >> sh) & 3u;
                    odd |= (o & 1u) && (o >> 1) != p;  // another lane added it with the other parity
                }
            }
        }
    }
    __syncthreads();
    if (cur != 0xFFFFFFFFu) flush_slice2(s_bits, gbits, n2, cur, nw16);
    if (odd) suf::st(fail, 1u);
}

// A list of pairs (v, p) checked against the GLOBAL snapshot, new members straight into N2: the emit bucketing's
// overflow list (m: its count is m->ovf_cur, and a spill — P1's overflow list overflowed, entries lost — sets ctr[3]: the
// final sb_rest_kernel pass then takes the whole batch again), or a short emit list that was not worth a P1.
__global__ __launch_bounds__(256) void sb_check_list_kernel(const u64* __restrict__ list, u32 n, const bk::Meta* __restrict__ m,
                                                            const u32* __restrict__ gbits, u32* __restrict__ n2, u32 cap,
                                                            u32* __restrict__ fail, u32* __restrict__ ctr) {
    if (m) {
        if (blockIdx.x == 0 && threadIdx.x == 0 && m->spill) ctr[3] = 1u;
        n = m->ovf_cur < n ? m->ovf_cur : n;
    }
    for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const u64 e = list[i];
        const u32 x = (u32)e, p = (u32)(e >> 32);
        if (x >= cap || p > 1u) continue;
        const u32 b = pair2(gbits[x >> 4], x);
        if (b & 1u) {
            if ((b >> 1) != p) suf::st(fail, 1u);
        } else {
            atomicOr(&n2[x >> 4], 1u << (2 * (x & 15) + p));
        }
    }
}

// The new members below r first (sb_join_low_kernel: the words below r's; each hooks C's root under a smaller id), so
// that sb_join_kernel's unites of seen members start at a stable root: C's root R = root(r) found once per block, each
// seen member united with R (parity composed with r's to R). Round 5: every unite walked from r, and the below-r hooks
// made that walk a chain of successively smaller roots — the seen members' 706K unites cost the share's two joins
// ~0.24 ms (a timing build without them: 73 against 195 us per join).
__global__ __launch_bounds__(256) void sb_join_low_kernel(u32* __restrict__ word, const u32* __restrict__ n2,
                                                          const u32* __restrict__ vote, u32* __restrict__ fail) {
    const u32 r = vote[0];
    for (u32 w = blockIdx.x * 256 + threadIdx.x; 16ull * w < r; w += gridDim.x * 256) {
        const u32 h = n2[w];
        const u32 h1 = (h >> 1) & kMask2;
        for (u32 d = (h | h1) & kMask2; d; d &= d - 1) {
            const u32 j = (u32)__builtin_ctz(d) >> 1, x = w * 16 + j;
            if (x < r) suf::unite(word, x, r, (h1 >> (2 * j)) & 1u, fail);
        }
    }
}

// C |= N2 (see the header comment). r = vote[0], C's root at the snapshot. N2 is cleared for the next level.
__global__ __launch_bounds__(256) void sb_join_kernel(u32* __restrict__ word, u32* __restrict__ gbits, u32* __restrict__ n2,
                                                      u32 nw16, const u32* __restrict__ vote, u32* __restrict__ fail) {
    __shared__ u32 s_R, s_pr;
    const u32 r = vote[0];
    if (threadIdx.x == 0) {
        u32 pr = 0;
        s_R = suf::find_ro(word, r, suf::ld(&word[r]), pr);
        s_pr = pr;
    }
    __syncthreads();
    const u32 R = s_R, pr = s_pr;  // a unite with R is exact whatever R has become meanwhile (the unite finds)
    const u32 stride = gridDim.x * 256;
    constexpr int kU = 4;  // words per lane per iteration, their loads in flight together
    for (u32 w0 = blockIdx.x * 256 + threadIdx.x; w0 < nw16; w0 += kU * stride) {
      u32 hk[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) hk[k] = w0 + k * stride < nw16 ? n2[w0 + k * stride] : 0u;
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const u32 w = w0 + k * stride, h = hk[k];
        if (!h) continue;
        atomicExch(&n2[w], 0u);  // memory-side: the next level's ORs follow in later kernels
        const u32 h0 = h & kMask2, h1 = (h >> 1) & kMask2;
        if (h0 & h1) suf::st(fail, 1u);  // reached with both parities: an odd cycle
        const u32 nm = h0 | h1;
        atomicOr(&gbits[w], nm | (h1 << 1));
        for (u32 d = nm; d; d &= d - 1) {
            const u32 j = (u32)__builtin_ctz(d) >> 1, x = w * 16 + j;
            if (x >= r && suf::ld(&word[x]) != suf::kUnseen)  // (below r: sb_join_low_kernel)
                suf::unite(word, x, R, ((h1 >> (2 * j)) & 1u) ^ pr, fail);
        }
      }
    }
}

// The remaining edges (the last level's slow list, every source bucketing's overflow list — n_dev: its count, and
// spill_meta: a spill there sets ctr[3]; the whole batch again when a bucketing spilled: `needs_spill`, then only when
// ctr[3] is set) by the giant kernel's rule, deferred-safe.
__global__ __launch_bounds__(256) void sb_rest_kernel(u32* __restrict__ word, const u64* __restrict__ edges, u64 n,
                                                      const u32* __restrict__ n_dev, u32 needs_spill,
                                                      const bk::Meta* __restrict__ spill_meta, u32* __restrict__ gbits,
                                                      const u32* __restrict__ vote, u32 cap, u32* __restrict__ fail,
                                                      u32* __restrict__ ctr) {
    if (needs_spill && !ctr[3]) return;
    if (spill_meta && blockIdx.x == 0 && threadIdx.x == 0 && spill_meta->spill) ctr[3] = 1u;
    if (n_dev) n = *n_dev < n ? *n_dev : n;
    const u32 r = vote[0];
    const u64 stride = (u64)gridDim.x * 256;
    for (u64 i = (u64)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const u64 e = edges[i];
        if (e == ~0ull) continue;
        const u32 u = (u32)e, v = (u32)(e >> 32);
        if (u >= cap || v >= cap) continue;
        const u32 bu = pair2(suf::ld(&gbits[u >> 4]), u), bv = pair2(suf::ld(&gbits[v >> 4]), v);
        if (bu & bv & 1u) {  // both in C: a check
            if (u != v && !((bu ^ bv) & 2u)) suf::st(fail, 1u);
            continue;
        }
        if ((bu ^ bv) & 1u) {  // one end in C: the other end x joins C under r, with the parity the edge implies
            const u32 x = (bu & 1u) ? v : u, px = ((((bu & 1u) ? bu : bv) >> 1) & 1u) ^ 1u;
            atomicOr(&gbits[x >> 4], (1u | px << 1) << (2 * (x & 15)));
            if (!(r < x && suf::ld(&word[x]) == suf::kUnseen &&
                  suf::cas(&word[x], suf::kUnseen, (r << 1) | px) == suf::kUnseen))
                suf::unite(word, x, r, px, fail);
            continue;
        }
        suf::unite(word, u, v, 1u, fail);
    }
}

// The closing compress (out of place): C's members from the bits, the rest by find (gelly_bip.hip
// signed_compress_kernel's rule).
__global__ __launch_bounds__(256) void sb_compress_kernel(u32* __restrict__ word, u32* __restrict__ out, u32 n,
                                                          const u32* __restrict__ gbits, const u32* __restrict__ vote) {
    __shared__ u32 s_rf, s_pr;
    if (threadIdx.x == 0) {
        const u32 r = vote[0];
        u32 pr = 0;
        s_rf = suf::find_ro(word, r, suf::ld(&word[r]), pr);
        s_pr = pr;
    }
    __syncthreads();
    const u32 rf = s_rf, pr = s_pr;
    const u64 stride = (u64)gridDim.x * 256;
    constexpr int kU = 4;  // ids per lane per iteration, their loads in flight together
    for (u64 i0 = (u64)blockIdx.x * 256 + threadIdx.x; i0 < n; i0 += kU * stride) {
        u32 bw[kU], ww[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const u64 i = i0 + k * stride;
            bw[k] = i < n ? gbits[i >> 4] : 0u;
            ww[k] = i < n ? word[i] : suf::kUnseen;
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const u64 i = i0 + k * stride;
            if (i >= n) break;
            const u32 v = (u32)i;
            const u32 b = pair2(bw[k], v);
            const u32 w = ww[k];
            if (b & 1u) {
                out[v] = (rf << 1) | (((b >> 1) & 1u) ^ pr);
            } else if (w == suf::kUnseen || suf::parent_of(w) == v) {
                out[v] = w;
            } else {
                u32 par;
                const u32 root = suf::find_ro(word, v, w, par);
                out[v] = (root << 1) | par;
            }
        }
    }
}

}  // namespace sb
