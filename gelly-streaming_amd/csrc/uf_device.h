// uf_device.h — device union-find primitives over a u32 parent[] forest (min-id hooking), shared by the
// product kernels (gelly_cc.hip) and the measurement probes (tools/probe_fold.hip).
//
// Forest encoding: parent[v] == UNSEEN -> v not in the key set; parent[v] == v -> root; parent[v] < v otherwise.
// Reference semantics restated: DisjointSet.makeSet/find/union (…/summaries/DisjointSet.java:58-123); see
// gelly_cc.hip's header for the memory-model argument (stale reads are historically valid, CAS returns fresh).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GCC_UNSEEN_DEV 0xFFFFFFFFu

namespace gcc {

typedef uint32_t u32;
typedef uint64_t u64;

// load policies for parent[] reads
struct LoadPlain {  // global_load: L1 -> L2
    static __device__ __forceinline__ u32 ld(const u32* p) { return *p; }
};
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

// optional per-thread event counters (probe builds only)
struct NoCount {
    __device__ __forceinline__ void cas() {}
    __device__ __forceinline__ void cas_fail() {}
    __device__ __forceinline__ void step() {}
    __device__ __forceinline__ void store() {}
};
struct Count {
    u32 n_cas = 0, n_fail = 0, n_step = 0, n_store = 0;
    __device__ __forceinline__ void cas() { ++n_cas; }
    __device__ __forceinline__ void cas_fail() { ++n_fail; }
    __device__ __forceinline__ void step() { ++n_step; }
    __device__ __forceinline__ void store() { ++n_store; }
};

// Mutation recorder for the incremental compress (gelly_cc.hip compress_inc_kernel). Between two compresses,
// every id that LEAVES root state (a successful hook CAS) is marked in a bloom filter of kBloomBits bits. Every
// parent value is an id that was a root at some time since the last compress (parent[] was compressed then, and
// every value written since is a root returned by find, or a copy of a parent value in path splitting; a stale
// UNSEEN read only stops a find at an id reached through a parent pointer, so at such an id). So an unmarked id
// p that is some id's parent is still a root: that id's label is p, no find needed. Ids that leave UNSEEN need
// no mark: one hung straight under a root never becomes a parent value, one made a root is marked if hooked.
constexpr u32 kBloomBits = 1u << 20;  // 128 KiB: one CU's LDS copy in the incremental compress
__host__ __device__ __forceinline__ u32 bloom_slot(u32 x) { return (x * 0x9E3779B1u) >> 12; }
struct NoRec {
    __device__ __forceinline__ void mark(u32) const {}
};
struct BloomRec {
    u32* bloom;
    __device__ __forceinline__ void mark(u32 x) const {
        const u32 s = bloom_slot(x);
        atomicOr(&bloom[s >> 5], 1u << (s & 31));
    }
};

template <class L, bool SPLIT, class C = NoCount>
struct UnionFind {
    // makeSet-on-first-sight (DisjointSet.union :99-104): an observed parent of v that is not UNSEEN
    static __device__ __forceinline__ u32 seen_parent(u32* parent, u32 v, C& c) {
        u32 p = L::ld(&parent[v]);
        if (p == GCC_UNSEEN_DEV) {
            c.cas();
            const u32 old = atomicCAS(&parent[v], GCC_UNSEEN_DEV, v);
            p = (old == GCC_UNSEEN_DEV) ? v : old;
        }
        return p;
    }

    // find (DisjointSet.find :71-85) from x with observed parent p; optional path splitting (plain stores of
    // grandparents into non-root slots). p >= x means x is a root (or p is a stale UNSEEN).
    static __device__ __forceinline__ u32 find_from(u32* parent, u32 x, u32 p, C& c) {
        if (p >= x) return x;
        u32 prev = x, cur = p;
        while (true) {
            c.step();
            const u32 next = L::ld(&parent[cur]);
            if (next >= cur) break;
            if (SPLIT) {
                parent[prev] = next;
                c.store();
            }
            prev = cur;
            cur = next;
        }
        return cur;
    }

    // union (DisjointSet.union :97-123), min-id hooking with atomicCAS on the larger root.
    // An unseen endpoint v joining a component whose root r < v is made seen AND hung under r by ONE CAS
    // (UNSEEN -> r): the common case of a stream (a new vertex attaching to an existing component).
    template <class R = NoRec>
    static __device__ __forceinline__ void unite(u32* parent, u32 u, u32 v, C& c, const R& rec = R()) {
        u32 pu = L::ld(&parent[u]);
        if (u == v) {  // self loop: makeSet only
            if (pu == GCC_UNSEEN_DEV) {
                c.cas();
                atomicCAS(&parent[u], GCC_UNSEEN_DEV, u);
            }
            return;
        }
        u32 pv = L::ld(&parent[v]);
        if (pu == pv && pu != GCC_UNSEEN_DEV) return;  // same parent: same tree (flat-forest fast path)
        if (pu == GCC_UNSEEN_DEV) {  // keep the unseen endpoint (if any) in v
            u32 t = u; u = v; v = t;
            t = pu; pu = pv; pv = t;
        }
        if (pu == GCC_UNSEEN_DEV) {  // both unseen: make the smaller one seen (a root unless raced)
            const u32 lo = u < v ? u : v, hi = u < v ? v : u;
            c.cas();
            const u32 o = atomicCAS(&parent[lo], GCC_UNSEEN_DEV, lo);
            u = lo;
            pu = (o == GCC_UNSEEN_DEV) ? lo : o;
            v = hi;
        }
        u32 ru = find_from(parent, u, pu, c);
        if (pv == GCC_UNSEEN_DEV) {
            c.cas();
            if (ru < v) {
                const u32 o = atomicCAS(&parent[v], GCC_UNSEEN_DEV, ru);
                if (o == GCC_UNSEEN_DEV) return;  // v seen and hooked under ru in one step
                pv = o;
            } else {
                const u32 o = atomicCAS(&parent[v], GCC_UNSEEN_DEV, v);
                pv = (o == GCC_UNSEEN_DEV) ? v : o;
            }
        }
        u32 rv = find_from(parent, v, pv, c);
        while (ru != rv) {
            const u32 lo = ru < rv ? ru : rv;
            const u32 hi = ru < rv ? rv : ru;
            c.cas();
            u32 old = atomicCAS(&parent[hi], hi, lo);
            if (old == hi) {
                rec.mark(hi);
                return;
            }
            c.cas_fail();
            if (old == GCC_UNSEEN_DEV) {  // unreachable for seen roots; keeps the loop finite regardless
                old = atomicCAS(&parent[hi], GCC_UNSEEN_DEV, lo);
                if (old == GCC_UNSEEN_DEV) {
                    rec.mark(hi);
                    return;
                }
            }
            ru = find_from(parent, hi, old, c);
            rv = find_from(parent, lo, L::ld(&parent[lo]), c);
        }
    }
};

}  // namespace gcc
