// signed_uf.h — the signed union-find of BipartitenessCheck's summary (gelly_bip.hip), as __host__ __device__
// code: the device kernels and the host replay test (tests/cpp/test_signed_uf.cpp, real threads + atomics)
// run the same functions. Encoding and invariants: gelly_bip.hip header.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SUF_HD __host__ __device__ __forceinline__
#else
#define SUF_HD static inline
#endif

namespace suf {

typedef uint32_t u32;
constexpr u32 kUnseen = 0xFFFFFFFFu;

// relaxed loads/stores and a compare-and-swap that return the previous value, on both sides. On gfx950 a plain
// load may return a STALE value (a CU's L1 is not coherent with other CUs' writes): every value it can return is
// one the word held at some earlier time, UNSEEN included. The host replay injects exactly that (ld_hook).
#if !defined(__HIPCC__) || !defined(__HIP_DEVICE_COMPILE__)
extern u32 (*ld_hook)(const u32* p, u32 fresh);  // host replay only: may return an older value of *p
#endif
SUF_HD u32 ld(const u32* p) {
    const u32 v = __atomic_load_n(p, __ATOMIC_RELAXED);
#if !defined(__HIPCC__) || !defined(__HIP_DEVICE_COMPILE__)
    if (ld_hook) return ld_hook(p, v);
#endif
    return v;
}
SUF_HD void st(u32* p, u32 v) { __atomic_store_n(p, v, __ATOMIC_RELAXED); }
SUF_HD u32 cas(u32* p, u32 expected, u32 desired) {
    __atomic_compare_exchange_n(p, &expected, desired, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
    return expected;  // the value found (== the old expected on success)
}

SUF_HD u32 parent_of(u32 w) { return w >> 1; }
SUF_HD u32 parity_of(u32 w) { return w & 1u; }

// root of x and the parity of x relative to it; wx = an observed word of x. Path splitting: each visited slot
// is pointed at its grandparent with the composed parity (plain store, non-root slots only).
// A parent >= the node means a root OR a stale UNSEEN (parent_of(UNSEEN) = 0x7FFFFFFF > every id): the walk then
// stops at a true ancestor with the true parity to it, so an equality / parity verdict between two walks is
// still a fact, and a hook of a node that is not really a root fails its CAS (callers retry).
SUF_HD u32 find(u32* word, u32 x, u32 wx, u32& par) {
    u32 acc = parity_of(wx), cur = parent_of(wx), prev = x, prev_par = parity_of(wx);
    if (cur >= x) {
        par = 0;
        return x;
    }
    while (true) {
        const u32 wc = ld(&word[cur]);
        const u32 nxt = parent_of(wc);
        if (nxt >= cur) break;  // cur is a root (or a stale UNSEEN was read)
        st(&word[prev], (nxt << 1) | (prev_par ^ parity_of(wc)));
        acc ^= parity_of(wc);
        prev = cur;
        prev_par = parity_of(wc);
        cur = nxt;
    }
    par = acc;
    return cur;
}

// find without path splitting (read-only): a compress that writes its labels into the other buffer (the late-store
// model of the CC forest, DESIGN.md §3: a split store into the old buffer could land over the labels written into it
// when the buffers swap back)
SUF_HD u32 find_ro(const u32* word, u32 x, u32 wx, u32& par) {
    u32 acc = parity_of(wx), cur = parent_of(wx);
    if (cur >= x) {
        par = 0;
        return x;
    }
    while (true) {
        const u32 wc = ld(&word[cur]);
        const u32 nxt = parent_of(wc);
        if (nxt >= cur) break;
        acc ^= parity_of(wc);
        cur = nxt;
    }
    par = acc;
    return cur;
}

// makeSet on first sight: the observed word of v, v made a root if it was unseen
SUF_HD u32 seen(u32* word, u32 v) {
    u32 w = ld(&word[v]);
    if (w == kUnseen) {
        const u32 o = cas(&word[v], kUnseen, v << 1);
        w = (o == kUnseen) ? (v << 1) : o;
    }
    return w;
}

// the constraint sign(u) XOR sign(v) == q (an edge: q = 1; a merged (v, parent, parity) triple: q = parity).
// A violated constraint inside one component sets *fail (an odd cycle: Candidates.merge -> fail()).
// Both words are loaded before anything depends on them (round 4, as the CC forest's unite, uf_device.h):
//   * both hang under the same parent p (a compressed forest, or one end is the other's parent): the constraint is
//     a check of the two parities to p, no walk;
//   * an unseen end v joining u's tree: ONE CAS hangs it under u's root ru with its parity (pu ^ q) when ru < v
//     (min-id hooking), instead of a makeSet CAS and a hook CAS;
//   * both unseen: the smaller becomes a root, the larger hangs under it.
// A word read stale is one the slot held earlier: it points to an ancestor with the parity to it (facts), and
// UNSEEN read stale is answered by the CAS's fresh value.
SUF_HD void unite(u32* word, u32 u, u32 v, u32 q, u32* fail) {
    u32 wu = ld(&word[u]);
    if (u == v) {  // a self loop only adds its vertex (edgeToCandidate ignores add()'s result)
        if (wu == kUnseen) (void)cas(&word[u], kUnseen, u << 1);
        return;
    }
    u32 wv = ld(&word[v]);
    if (wu != kUnseen && wv != kUnseen && parent_of(wu) == parent_of(wv)) {
        if ((parity_of(wu) ^ parity_of(wv)) != q) st(fail, 1u);
        return;
    }
    if (wu == kUnseen) {  // keep the unseen end (if any) in v
        u32 t = u; u = v; v = t;
        t = wu; wu = wv; wv = t;
    }
    if (wu == kUnseen) {  // both unseen: the smaller one seen (a root unless raced)
        const u32 lo = u < v ? u : v, hi = u < v ? v : u;
        const u32 o = cas(&word[lo], kUnseen, lo << 1);
        u = lo;
        wu = (o == kUnseen) ? (lo << 1) : o;
        v = hi;
    }
    u32 pu, pv;
    u32 ru = find(word, u, wu, pu);
    if (wv == kUnseen) {
        if (ru < v) {
            const u32 o = cas(&word[v], kUnseen, (ru << 1) | (pu ^ q));
            if (o == kUnseen) return;  // v seen and hung under ru in one step
            wv = o;
        } else {
            const u32 o = cas(&word[v], kUnseen, v << 1);
            wv = (o == kUnseen) ? (v << 1) : o;
        }
    }
    while (true) {
        const u32 rv = find(word, v, wv, pv);
        if (ru == rv) {
            if ((pu ^ pv) != q) st(fail, 1u);
            return;
        }
        const u32 lo = ru < rv ? ru : rv, hi = ru < rv ? rv : ru;
        const u32 x = pu ^ pv ^ q;  // parity of hi relative to lo that satisfies the constraint
        const u32 o = cas(&word[hi], hi << 1, (lo << 1) | x);
        if (o == (hi << 1)) return;
        wu = seen(word, u);  // hi was hooked meanwhile: walk again; seen() answers a stale UNSEEN with the CAS's
        wv = seen(word, v);  // fresh value, so a stale line cannot spin this loop
        ru = find(word, u, wu, pu);
    }
}

}  // namespace suf
