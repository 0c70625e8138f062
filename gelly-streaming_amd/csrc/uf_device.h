// uf_device.h — union-find primitives over a u32 parent[] forest (min-id hooking), shared by the product kernels
// (gelly_cc.hip, bucket_fold.h), the measurement probes (tools/probe_fold.hip) and the HOST replay harness
// (tests/cpp/test_uf_replay.cpp), which runs these exact functions on host threads with relaxed atomics and
// injected stale loads. Compiled by hipcc (device + host) and by g++ (host only: no HIP headers).
//
// Forest encoding: parent[v] == UNSEEN -> v not in the key set; parent[v] == v -> root; parent[v] < v otherwise.
// Reference semantics restated: DisjointSet.makeSet/find/union (…/summaries/DisjointSet.java:58-123); see
// gelly_cc.hip's header for the memory-model argument (stale reads are historically valid, CAS returns fresh).
#pragma once
#include <stdint.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define UF_HD __host__ __device__ __forceinline__
#define UF_UNROLL _Pragma("unroll")
#else
#define UF_HD inline
#define UF_UNROLL
#endif

#define GCC_UNSEEN_DEV 0xFFFFFFFFu
// The optimistic first CAS of unite (round 4 experiment, OFF): 1 = an unseen endpoint hangs under the other's
// observed parent (no find first); 2 = also two seen endpoints' observed parents hooked directly. Measured against 0
// (profiles/r4g_ab_*, r4h_ab_*, interleaved builds on one box): level 2 C3 one window -2.6 %, C5's windows +7 % in the
// fold (the CAS fails whenever an observed parent was hooked earlier in the window, and a failed atomic costs more
// than the load it saves); level 1 C5 +6.6 %, C3 equal. So 0: the find runs first.
#ifndef GCC_UNITE_OPT
#define GCC_UNITE_OPT 0
#endif

namespace gcc {

typedef uint32_t u32;
typedef uint64_t u64;

// ---- word-level memory operations: device intrinsics, or (host replay) relaxed __atomic builtins ----------------
#if !defined(__HIP_DEVICE_COMPILE__)
// Host replay only (tests/cpp/test_uf_replay.cpp): a scheduling point before every memory operation (a controlled
// scheduler interleaves the threads there), the value a plain load returns (a stale but historically valid one may
// be injected), and a note of every value a store or atomic wrote (the history loads may be answered from).
struct ReplayHooks {
    virtual void before(const u32* p) = 0;
    virtual u32 load(const u32* p, u32 fresh) = 0;
    virtual void wrote(const u32* p, u32 v) = 0;
    // a PLAIN store (not an atomic): the model may let it land again later, after the next kernel's writes (round 4:
    // a plain store of one kernel can become visible after stores of the next one)
    virtual void stored(u32* p, u32 v) { (void)p, (void)v; }
    // a memory-side ATOMIC changed the word (CAS success, atomicMin lowering it, atomicOr): the model decides whether
    // a late plain store issued before it may still land over it
    virtual void atomic(const u32* p) { (void)p; }
};
inline ReplayHooks* replay = nullptr;  // null: plain relaxed atomics (product host code never sets it)
#define UF_REPLAY_BEFORE(p) \
    if (replay) replay->before(p)
#define UF_REPLAY_WROTE(p, v) \
    if (replay) replay->wrote(p, v)
#define UF_REPLAY_ATOMIC(p) \
    if (replay) replay->atomic(p)
#endif

UF_HD u32 ld(const u32* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return *p;  // global_load: L1 -> L2 (may be stale inside a kernel: historically valid)
#else
    UF_REPLAY_BEFORE(p);
    const u32 fresh = __atomic_load_n(p, __ATOMIC_RELAXED);
    return replay ? replay->load(p, fresh) : fresh;
#endif
}
UF_HD void st(u32* p, u32 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    *p = v;  // a plain (vector) store
#else
    UF_REPLAY_BEFORE(p);
    __atomic_store_n(p, v, __ATOMIC_RELAXED);
    UF_REPLAY_WROTE(p, v);
    if (replay) replay->stored(p, v);
#endif
}
// A WRITE-THROUGH store (agent-scope relaxed atomic store: global_store ... sc1 on gfx950, which leaves no dirty line in
// the XCD's L2 — MI355X_MICROARCH.md, store flavours). The in-place incremental compress writes its labels with it:
// a plain store there could land over the same slot's label of the next in-place compress two kernels later (the late
// plain stores of DESIGN.md §3; the replay models it as an atomic write).
UF_HD void st_through(u32* p, u32 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    UF_REPLAY_BEFORE(p);
    __atomic_store_n(p, v, __ATOMIC_RELAXED);
    UF_REPLAY_WROTE(p, v);
    UF_REPLAY_ATOMIC(p);
#endif
}
UF_HD u32 cas(u32* p, u32 cmp, u32 val) {  // returns the old value (fresh: executed at the memory side)
#if defined(__HIP_DEVICE_COMPILE__)
    return atomicCAS(p, cmp, val);
#else
    UF_REPLAY_BEFORE(p);
    if (__atomic_compare_exchange_n(p, &cmp, val, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        UF_REPLAY_WROTE(p, val);
        UF_REPLAY_ATOMIC(p);
    }
    return cmp;
#endif
}
UF_HD u32 amin(u32* p, u32 v) {  // returns the old value
#if defined(__HIP_DEVICE_COMPILE__)
    return atomicMin(p, v);
#else
    UF_REPLAY_BEFORE(p);
    u32 old = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (old > v && !__atomic_compare_exchange_n(p, &old, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
    if (old > v) {
        UF_REPLAY_WROTE(p, v);
        UF_REPLAY_ATOMIC(p);
    }
    return old;
#endif
}
UF_HD void aor(u32* p, u32 m) {
#if defined(__HIP_DEVICE_COMPILE__)
    atomicOr(p, m);
#else
    UF_REPLAY_BEFORE(p);
    __atomic_fetch_or(p, m, __ATOMIC_RELAXED);
    UF_REPLAY_ATOMIC(p);
#endif
}

// load policies for parent[] reads
struct LoadPlain {  // global_load: L1 -> L2 (host replay: relaxed load + optional stale injection)
    static UF_HD u32 ld(const u32* p) { return gcc::ld(p); }
};
#if defined(__HIPCC__)
struct LoadAgent {  // relaxed agent-scope atomic load (sc1): bypasses the CU's L1, served by the XCD's L2
    static __device__ __forceinline__ u32 ld(const u32* p) {
        return __hip_atomic_load(const_cast<u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};
struct LoadSystem {  // relaxed system-scope atomic load (sc0 sc1)
    static __device__ __forceinline__ u32 ld(const u32* p) {
        return __hip_atomic_load(const_cast<u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
};
#endif

// optional per-thread event counters (probe builds only)
struct NoCount {
    UF_HD void cas() {}
    UF_HD void cas_fail() {}
    UF_HD void step() {}
    UF_HD void store() {}
};
struct Count {
    u32 n_cas = 0, n_fail = 0, n_step = 0, n_store = 0;
    UF_HD void cas() { ++n_cas; }
    UF_HD void cas_fail() { ++n_fail; }
    UF_HD void step() { ++n_step; }
    UF_HD void store() { ++n_store; }
};

// Mutation recorder for the incremental compress (gelly_cc.hip compress_inc_kernel). Between two compresses,
// every id that LEAVES root state (a successful hook CAS) is marked in a bloom filter of kBloomBits bits. Every
// parent value is an id that was a root at some time since the last compress (parent[] was compressed then, and
// every value written since is a root returned by find, or a copy of a parent value in path splitting; a stale
// UNSEEN read only stops a find at an id reached through a parent pointer, so at such an id). So an unmarked id
// p that is some id's parent is still a root: that id's label is p, no find needed. Ids that leave UNSEEN need
// no mark: one hung straight under a root never becomes a parent value, one made a root is marked if hooked.
constexpr u32 kBloomBits = 1u << 20;  // 128 KiB: one CU's LDS copy in the incremental compress
// A BLOCKED bloom filter (round 3): a mark sets kBloomK bits of ONE 32-bit word, so marking is one memory-side
// atomicOr and a test one LDS read. Round 2's filter set 2 bits
// in 2 words: two atomics per hook in the fold (the fold of a short window is bound by memory-side atomics) and a
// 1.4 % false-hit rate at C5's 65K marks per window; 4 bits in one of 32K words: ~0.8 %.
// One multiply per test (round 3): the incremental compress tests every id of the forest, and with three 32-bit
// multiplies per test (a quarter-rate VALU op each) it was bound by the VALU, not by its 16-B stream. The word is
// the product's top 15 bits and the kBloomK bit positions its next 15 bits (5 each); bit i of x * K depends on bits
// 0..i of x only, so the low 2 bits are left out.
constexpr int kBloomK = 3;
constexpr u32 kBloomMul = 0x9E3779B1u;
UF_HD u32 bloom_word(u32 x) { return (x * kBloomMul) >> 17; }  // 15 bits: one of kBloomBits / 32 words
UF_HD u32 bloom_mask(u32 x) {
    const u32 h = x * kBloomMul;
    return (1u << ((h >> 12) & 31)) | (1u << ((h >> 7) & 31)) | (1u << ((h >> 2) & 31));
}
UF_HD bool bloom_test(const u32* bloom, u32 x) {
    const u32 m = bloom_mask(x);
    return (bloom[bloom_word(x)] & m) == m;
}
// A fold's recording policy: mark(x) when root x is hooked (x leaves root state), born(x) when x leaves UNSEEN.
struct NoRec {
    UF_HD void mark(u32) const {}
    UF_HD void born(u32) const {}
};
struct BloomRec {
    u32* bloom;
    UF_HD void mark(u32 x) const { aor(&bloom[bloom_word(x)], bloom_mask(x)); }
    UF_HD void born(u32) const {}
};
// The pipelined emission's fold (gelly_cc.hip fold_pipe_kernel, round 5): the bloom mark, and every touched id exact
// in `touched`, two u32 words per 32 ids — [2 w] the hooked roots, [2 w + 1] the new ids — which the window's
// resolve kernel reads (and clears) to snapshot their roots before the next window's fold runs.
struct PipeRec {
    u32* bloom;
    u32* touched;
    UF_HD void mark(u32 x) const {
        aor(&bloom[bloom_word(x)], bloom_mask(x));
        aor(&touched[2 * (x >> 5)], 1u << (x & 31));
    }
    UF_HD void born(u32 x) const { aor(&touched[2 * (x >> 5) + 1], 1u << (x & 31)); }
};

// The delta merge's recorder (round 6; gelly_cc.hip fold_kernel<.., DELTA>, gcc_forest_encode_delta): every id whose
// slot one of this fold's memory-side atomics changed — a root hooked (mark) or an id that left UNSEEN (born) — is
// noted in the lane's event buffer; the fold kernel appends each wave's events to the forest's delta lists after the
// unite. Those ids are the whole difference between the forest and the partition it held when the delta was armed:
// that partition plus {(x, root(x))} for the noted x is the forest's partition. A unite notes at most
// 3 (born lo, born hi, mark hi); kLaneEvents slots, a lane past them flags the delta as unusable.
constexpr u32 kLaneEvents = 4;
struct LaneEvents {
    u32 x[kLaneEvents];
    u32 n = 0;
    UF_HD void note(u32 v) {
        if (n < kLaneEvents) x[n] = v;
        ++n;
    }
};
struct DeltaRec {
    LaneEvents* ev;
    UF_HD void mark(u32 x) const { ev->note(x); }
    UF_HD void born(u32 x) const { ev->note(x); }
};
struct BloomDeltaRec {  // both recorders: the incremental compress's bloom and the delta
    u32* bloom;
    LaneEvents* ev;
    UF_HD void mark(u32 x) const {
        aor(&bloom[bloom_word(x)], bloom_mask(x));
        ev->note(x);
    }
    UF_HD void born(u32 x) const { ev->note(x); }
};

template <class L, bool SPLIT, class C = NoCount>
struct UnionFind {
    // makeSet-on-first-sight (DisjointSet.union :99-104): an observed parent of v that is not UNSEEN
    static UF_HD u32 seen_parent(u32* parent, u32 v, C& c) {
        u32 p = L::ld(&parent[v]);
        if (p == GCC_UNSEEN_DEV) {
            c.cas();
            const u32 old = gcc::cas(&parent[v], GCC_UNSEEN_DEV, v);
            p = (old == GCC_UNSEEN_DEV) ? v : old;
        }
        return p;
    }

    // find (DisjointSet.find :71-85) from x with observed parent p; optional path splitting (plain stores of
    // grandparents into non-root slots). p >= x means x is a root (or p is a stale UNSEEN).
    static UF_HD u32 find_from(u32* parent, u32 x, u32 p, C& c) {
        if (p >= x) return x;
        u32 prev = x, cur = p;
        while (true) {
            c.step();
            const u32 next = L::ld(&parent[cur]);
            if (next >= cur) break;
            if (SPLIT) {
                gcc::st(&parent[prev], next);
                c.store();
            }
            prev = cur;
            cur = next;
        }
        return cur;
    }

    // union (DisjointSet.union :97-123), min-id hooking with a CAS on the larger root.
    // An unseen endpoint v joining a component whose root r < v is made seen AND hung under r by ONE CAS
    // (UNSEEN -> r): the common case of a stream (a new vertex attaching to an existing component).
    // Optimistic first CAS (round 4, GCC_UNITE_OPT >= 2): the endpoints' observed parents pu, pv are tried as if they
    // were the roots — right after a compress they are — before any find: CAS(parent[hi], hi, lo), {lo, hi} = {pu, pv}.
    // It succeeds only if hi is a root at that moment; then hi roots one endpoint's tree and lo < hi lies in the
    // other's (a root is its tree's minimum, so lo cannot be in hi's tree: no cycle), and hanging hi under lo is the
    // union — lo need not be a root (the invariant parent < self holds, and lo was a root at some time of the window
    // or at its start, which is all the bloom of the incremental compress needs). Likewise an unseen v hangs under
    // pu < v directly (GCC_UNITE_OPT >= 1). A failed CAS returns hi's fresh parent and the general path below goes on
    // from there. Saves the dependent load of parent[pu] per edge.
    template <class R = NoRec>
    static UF_HD void unite(u32* parent, u32 u, u32 v, C& c, const R& rec = R()) {
        u32 pu = L::ld(&parent[u]);
        if (u == v) {  // self loop: makeSet only
            if (pu == GCC_UNSEEN_DEV) {
                c.cas();
                if (gcc::cas(&parent[u], GCC_UNSEEN_DEV, u) == GCC_UNSEEN_DEV) rec.born(u);
            }
            return;
        }
        u32 pv = L::ld(&parent[v]);
        if (pu == pv && pu != GCC_UNSEEN_DEV) return;  // same parent: same tree (flat-forest fast path)
        if (pu == GCC_UNSEEN_DEV) {  // keep the unseen endpoint (if any) in v
            u32 t = u; u = v; v = t;
            t = pu; pu = pv; pv = t;
        }
#if GCC_UNITE_OPT
        if (pu != GCC_UNSEEN_DEV) {
            if (GCC_UNITE_OPT >= 2 && pv != GCC_UNSEEN_DEV) {  // both seen: the observed parents as roots
                const u32 lo = pu < pv ? pu : pv, hi = pu < pv ? pv : pu;
                c.cas();
                const u32 old = gcc::cas(&parent[hi], hi, lo);
                if (old == hi) {
                    rec.mark(hi);
                    return;
                }
                c.cas_fail();
                // hi was not a root: its fresh parent replaces it as that endpoint's observed parent
                if (hi == pu) pu = old;
                else pv = old;
            } else if (pu < v) {  // v unseen: hang it under u's observed parent (a node of u's tree, below v)
                c.cas();
                const u32 o = gcc::cas(&parent[v], GCC_UNSEEN_DEV, pu);
                if (o == GCC_UNSEEN_DEV) {
                    rec.born(v);
                    return;
                }
                pv = o;  // v became seen meanwhile
            }
        }
#endif
        if (pu == GCC_UNSEEN_DEV) {  // both unseen: make the smaller one seen (a root unless raced)
            const u32 lo = u < v ? u : v, hi = u < v ? v : u;
            c.cas();
            const u32 o = gcc::cas(&parent[lo], GCC_UNSEEN_DEV, lo);
            if (o == GCC_UNSEEN_DEV) rec.born(lo);
            u = lo;
            pu = (o == GCC_UNSEEN_DEV) ? lo : o;
            v = hi;
        }
        u32 ru = find_from(parent, u, pu, c);
        if (pv == GCC_UNSEEN_DEV) {
            c.cas();
            if (ru < v) {
                const u32 o = gcc::cas(&parent[v], GCC_UNSEEN_DEV, ru);
                if (o == GCC_UNSEEN_DEV) {  // v seen and hooked under ru in one step
                    rec.born(v);
                    return;
                }
                pv = o;
            } else {
                const u32 o = gcc::cas(&parent[v], GCC_UNSEEN_DEV, v);
                if (o == GCC_UNSEEN_DEV) rec.born(v);
                pv = (o == GCC_UNSEEN_DEV) ? v : o;
            }
        }
        u32 rv = find_from(parent, v, pv, c);
        while (ru != rv) {
            const u32 lo = ru < rv ? ru : rv;
            const u32 hi = ru < rv ? rv : ru;
            c.cas();
            u32 old = gcc::cas(&parent[hi], hi, lo);
            if (old == hi) {
                rec.mark(hi);
                return;
            }
            c.cas_fail();
            if (old == GCC_UNSEEN_DEV) {  // unreachable for seen roots; keeps the loop finite regardless
                old = gcc::cas(&parent[hi], GCC_UNSEEN_DEV, lo);
                if (old == GCC_UNSEEN_DEV) {
                    rec.born(hi);
                    rec.mark(hi);
                    return;
                }
            }
            ru = find_from(parent, hi, old, c);
            rv = find_from(parent, lo, L::ld(&parent[lo]), c);
        }
    }
};

typedef UnionFind<LoadPlain, true> UF;       // the fold's union (path splitting)
typedef UnionFind<LoadPlain, false> UFRead;  // read-only finds (compress)
// The RECORDING fold's union (fold_kernel<true>, before an incremental compress): no path splitting, so the fold writes
// parent[] only with memory-side atomics. A plain store of a kernel can land after the next kernel's stores on gfx950
// (round 4: tools/stress_inc.py, profiles/r4a_stress_*): a split store landing after the in-place compress rewrote its
// slot put back a root hooked in that window (a wrong label, counts intact). With no plain store in the fold, every
// value the compress writes stays written. (tests/cpp/test_uf_replay.cpp models such late stores.)
typedef UnionFind<LoadPlain, false> UFRec;

// ---- the per-id and per-edge steps of the other kernels, shared with the host replay ------------------------

// The filtered fold's direct hook of an edge (g, b) with g in the tracked component and b > g outside it
// (gelly_cc.hip filter_round), in its two halves: the atomicMin, issued for a whole round first, and its check
// ("settle") one round later: old = UNSEEN (b was new), b (b was a root) or g: b now hangs under g, done;
// otherwise b left the tree of old (or already hung lower), and union(g, old) restores the connection.
UF_HD u32 hook_min(u32* parent, u32 b, u32 g) { return amin(&parent[b], g); }
UF_HD bool hook_needs_union(u32 old, u32 b, u32 g) { return old != GCC_UNSEEN_DEV && old != b && old != g; }

// A ring entry of the filtered fold (gelly_cc.hip unite_entry): (g, x) with x > g takes the hook form in one step.
UF_HD void unite_entry(u32* parent, u32 a, u32 b, u32 g) {
    NoCount c;
    if (a == g && b > g) {
        const u32 old = hook_min(parent, b, g);
        if (hook_needs_union(old, b, g)) UF::unite(parent, g, old, c);
    } else {
        UF::unite(parent, a, b, c);
    }
}

// msg_absorb_bits_kernel: an id x of a peer's giant, outside this forest's tracked component T (root R), joins R.
// A new id above R by ONE CAS (UNSEEN -> R), anything else by the union. (Rounds 1-3 used a plain store — in that
// kernel x has no other writer — but the next kernel, msg_absorb_kernel, may CAS the same slot, and a plain store can
// land after the next kernel's memory-side atomics on gfx950: DESIGN.md §3.)
UF_HD void absorb_join(u32* parent, u32 x, u32 R) {
    NoCount c;
    if (x > R && ld(&parent[x]) == GCC_UNSEEN_DEV && cas(&parent[x], GCC_UNSEEN_DEV, R) == GCC_UNSEEN_DEV) return;
    UF::unite(parent, x, R, c);
}

// compress_kernel's per-id step (out of place): labels[v] = root(v), UNSEEN stays UNSEEN. Read-only find (round 5:
// compress_bits_kernel<false>; a split store into the old buffer could land over the labels written into it two
// kernels later, after the buffers swap back).
UF_HD u32 compress_label(u32* parent, u32 v) {
    NoCount c;
    const u32 p = ld(&parent[v]);
    return (p >= v) ? p : UFRead::find_from(parent, v, p, c);
}

// compress_inc_kernel's per-id step: after a compress, parent[] IS the label array; an unmarked parent p is
// still a root (BloomRec), so labels[v] = p without a find; a marked one takes a read-only find.
UF_HD u32 inc_label(const u32* parent, const u32* bloom, u32 v, u32 p) {
    if (p >= v) return p;  // root (p == v) or UNSEEN
    if (!bloom_test(bloom, p)) return p;
    NoCount c;
    return UFRead::find_from(const_cast<u32*>(parent), v, p, c);
}

// The pipelined emission's per-id steps (gelly_cc.hip pipe_resolve_kernel / compress_pipe_kernel, round 5; shared
// with the host replay's "pipe" pipeline). pipe_root: the root of a touched id in the quiescent forest (after the
// window's folds, before the next window's). pipe_label: v's label after window w from its label l after window w-1,
// whether v is new in w, the window's bloom and its roots snapshot: a new id takes its root; a label marked in the
// bloom takes roots[l] unless that is UNSEEN (a false positive never touched since the mode started: l stays; one
// touched two or more windows ago of the same parity was new then and has been a root since: roots[l] = l).
// pipe_root also shortcuts the touched id to that root (a memory-side atomicMin: the root is the smallest id on the
// path, and the forest's only writes stay atomics) — the mode writes labels elsewhere, so without it parent[] would
// only deepen, window after window.
UF_HD u32 pipe_root(u32* parent, u32 x) {
    NoCount c;
    const u32 p = ld(&parent[x]);
    const u32 r = UFRead::find_from(parent, x, p, c);
    if (r < p) amin(&parent[x], r);
    return r;
}
// The scan's per-id test, then (batched: compress_pipe_kernel queues the hits) the roots lookup and the label. A new id
// (no label yet: l = UNSEEN) looks up its own root; a marked label its root's.
UF_HD bool pipe_hit(const u32* bloom, u32 l, bool born) { return born || (l != GCC_UNSEEN_DEV && bloom_test(bloom, l)); }
UF_HD u32 pipe_key(u32 v, u32 l) { return l == GCC_UNSEEN_DEV ? v : l; }
UF_HD u32 pipe_settle(u32 l, u32 q) { return l == GCC_UNSEEN_DEV ? q : (q == GCC_UNSEEN_DEV ? l : q); }
UF_HD u32 pipe_label(const u32* bloom, const u32* roots, u32 v, u32 l, bool born) {
    return pipe_hit(bloom, l, born) ? pipe_settle(l, ld(&roots[pipe_key(v, l)])) : l;
}

}  // namespace gcc
