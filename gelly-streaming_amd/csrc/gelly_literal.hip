// gelly_literal.hip — BipartitenessCheck's Candidates summary AS WRITTEN (include/gelly_cc.h, gcc_literal_*).
//
// gelly_bip.hip's signed forest is the bipartiteness summary with the intended semantics (bipartite iff no odd
// cycle). The reference's own Candidates.merge (…/summaries/Candidates.java:77-192; `…/` =
// src/main/java/org/apache/flink/graph/streaming/) is not a partition join, and a job that switches to this
// library may depend on what it really emits. This translation unit reproduces it, step for step:
//   merge(input)       :77-139  input components in key order (TreeMap); per component the self components that
//                               share a vertex, EXCEPT one with exactly the same vertex set (:91-95); none: add the
//                               component as is (:108-111, add()'s false ignored); else _merge into the smallest
//                               (:113-121, a failure fails the whole result), then every other one into
//                               min(inputKey, first) (:123-134: the result of that _merge is dropped) and removed
//   _merge             :142-192 reversal from the first common vertex in vertex order, every common vertex checked,
//                               then the input's vertices (reversed or not) added in vertex order under
//                               min(inputKey, selfKey) (:176-189: the self component is NOT moved there), stopping
//                               at the first sign conflict
//   add                :61-74   a vertex already present with the other sign: false, nothing changed
//   edgeToCandidate    …/library/BipartitenessCheck.java:54-61 ({min: true, max: false}; a self loop: {v: true})
//   fail()             :194-196 (false, {})
// The summary's state is a device array of entries (component key << 32 | vertex << 1 | sign). The semantics are
// sequential by definition (every step depends on the state the previous one left, in TreeMap iteration order),
// so ONE wavefront runs each fold / merge in order; its 64 lanes share every scan of the state (set membership
// via per-vertex mark arrays, ballots for "first conflict" and for compaction). This is a compatibility mode for
// parity with the reference's own output, not a throughput path: the signed forest is that.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "abi_common.h"
#include "gelly_cc.h"

namespace {

typedef uint32_t u32;
typedef uint64_t u64;
constexpr u64 kDead = ~0ull;
constexpr u32 kNone = 0xFFFFFFFFu;
constexpr u32 kMaxLitId = 0x7FFFFFFEu;  // vertex << 1 | sign stays below 2^32

enum : u32 { kErrCap = 1, kErrNoCommon = 2 };

struct LitDev {  // device header of one Candidates
    u32 success;
    u32 n;    // entries used (dead ones included until the end-of-launch compaction)
    u32 err;  // kErr*: the launch stopped (capacity), or the reference itself would have thrown
    u32 pad;
};

// Per-handle scratch, indexed by vertex / component key (< id capacity), all zero between steps.
struct Scratch {
    u32* mk_in;   // 1 + sign of the input component's vertices
    u32* mk_c;    // 1 + sign of one self component's vertices
    u32* cnt_in;  // per self key: its vertices inside the input component
    u32* cnt_sz;  // per touched self key: its size
    u32* keys;    // touched keys, then the merge list (mergeWith)
    u64* tmp;     // a component's entries (gathered), then sorted by vertex
    u64* tmp2;
    u32 cap_tmp;
};

__device__ __forceinline__ u32 ld(const u32* p) {  // agent-scope load: L1 bypassed, lanes see each other's stores
    return __hip_atomic_load(const_cast<u32*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld(const u64* p) {
    return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __syncthreads();
}
__device__ __forceinline__ u32 e_key(u64 e) { return (u32)(e >> 32); }
__device__ __forceinline__ u32 e_v(u64 e) { return (u32)e >> 1; }
__device__ __forceinline__ u32 e_s(u64 e) { return (u32)e & 1u; }
__device__ __forceinline__ u64 mk_e(u32 key, u32 v, u32 s) { return ((u64)key << 32) | ((u64)v << 1) | s; }

struct Lit {
    LitDev* hd;
    u64* ent;
    u32 cap;
    Scratch sc;
    u32 lane;

    __device__ u32 n() const { return ld(&hd->n); }

    // mark[v] = 1 + sign for every entry of component `key` (value 0 clears)
    __device__ void mark_comp(u32* mark, u32 key, bool set) {
        const u32 nn = n();
        for (u32 i = lane; i < nn; i += 64) {
            const u64 e = ld(&ent[i]);
            if (e != kDead && e_key(e) == key) mark[e_v(e)] = set ? 1u + e_s(e) : 0u;
        }
        sync();
    }

    // a component's entries (key) gathered into sc.tmp and sorted by vertex into sc.tmp2 (a TreeMap's order);
    // returns the count (kNone: more than the scratch holds)
    __device__ u32 gather_sorted(const u64* src, u32 nsrc, u32 key) {
        __shared__ u32 s_cnt;
        if (lane == 0) s_cnt = 0;
        sync();
        for (u32 b = 0; b < nsrc; b += 64) {
            const u32 i = b + lane;
            const u64 e = i < nsrc ? ld(&src[i]) : kDead;
            const bool take = e != kDead && e_key(e) == key;
            const u64 m = __ballot(take);
            const u32 base = s_cnt;
            if (take) {
                const u32 pos = base + (u32)__popcll(m & ((1ull << lane) - 1));
                if (pos < sc.cap_tmp) sc.tmp[pos] = e;
            }
            sync();
            if (lane == 0) s_cnt = base + (u32)__popcll(m);
            sync();
        }
        const u32 cnt = s_cnt;
        if (cnt > sc.cap_tmp) return kNone;
        for (u32 i = lane; i < cnt; i += 64) {  // rank sort (vertices of one component are distinct)
            const u64 e = ld(&sc.tmp[i]);
            u32 r = 0;
            for (u32 j = 0; j < cnt; ++j) r += e_v(ld(&sc.tmp[j])) < e_v(e);
            sc.tmp2[r] = e;
        }
        sync();
        return cnt;
    }

    // add(common, v, sign') for the sorted input vertices `inv` (sign' = sign ^ rev) in order, stopping at the
    // first conflict (Candidates.add :61-74). mk_c holds component `common`. Returns false at a conflict.
    __device__ bool add_in_order(const u64* inv, u32 m, u32 common, u32 rev) {
        __shared__ u32 s_stop, s_n;
        if (lane == 0) {
            s_stop = 0;
            s_n = n();
        }
        sync();
        for (u32 b = 0; b < m; b += 64) {
            const u32 j = b + lane;
            u32 v = 0, s = 0, have = 0;
            if (j < m) {
                const u64 e = ld(&inv[j]);
                v = e_v(e);
                s = e_s(e) ^ rev;
                have = ld(&sc.mk_c[v]);
            }
            const bool conflict = j < m && have && have - 1 != s;
            const u64 cm = __ballot(conflict);
            const u32 first = cm ? (u32)__builtin_ctzll(cm) : 64u;  // lanes at or past it add nothing
            const bool add = j < m && !have && lane < first;
            const u64 am = __ballot(add);
            const u32 base = s_n;
            if (add) {
                const u32 pos = base + (u32)__popcll(am & ((1ull << lane) - 1));
                if (pos < cap) ent[pos] = mk_e(common, v, s);
            }
            sync();
            if (lane == 0) {
                const u32 nn = base + (u32)__popcll(am);
                if (nn > cap) hd->err |= kErrCap;
                s_n = nn < cap ? nn : cap;
                if (cm) s_stop = 1;
            }
            sync();
            if (s_stop || (ld(&hd->err) & kErrCap)) break;
        }
        if (lane == 0) hd->n = s_n;
        sync();
        return s_stop == 0;
    }

    // Candidates._merge(input, this, inKey, selfKey) with the input component's sorted vertices `inv`
    // (:142-192). Leaves mk_c clear.
    __device__ bool merge_into(const u64* inv, u32 m, u32 in_key, u32 self_key) {
        __shared__ u32 s_first, s_rev, s_bad;
        mark_comp(sc.mk_c, self_key, true);
        if (lane == 0) {
            s_first = kNone;
            s_bad = 0;
        }
        sync();
        // the first common vertex in the input's (vertex) order decides the reversal (:156-158)
        for (u32 b = 0; b < m && s_first == kNone; b += 64) {
            const u32 j = b + lane;
            const bool common = j < m && ld(&sc.mk_c[e_v(ld(&inv[j]))]) != 0;
            const u64 cmask = __ballot(common);
            if (lane == 0 && cmask) {
                const u32 f = b + (u32)__builtin_ctzll(cmask);
                const u64 e = ld(&inv[f]);
                s_first = f;
                s_rev = e_s(e) != ld(&sc.mk_c[e_v(e)]) - 1;
            }
            sync();
        }
        if (s_first == kNone) {  // mergeBy.get(0) on an empty list: the reference throws here
            if (lane == 0) hd->err |= kErrNoCommon;
            mark_comp(sc.mk_c, self_key, false);
            return false;
        }
        const u32 rev = s_rev;
        for (u32 j = lane; j < m; j += 64) {  // every common vertex consistent with the reversal (:162-173)
            const u64 e = ld(&inv[j]);
            const u32 h = ld(&sc.mk_c[e_v(e)]);
            if (h && ((e_s(e) ^ rev) != h - 1)) s_bad = 1;
        }
        sync();
        if (s_bad) {
            mark_comp(sc.mk_c, self_key, false);
            return false;
        }
        const u32 common = in_key < self_key ? in_key : self_key;  // :176
        if (common != self_key) {
            mark_comp(sc.mk_c, self_key, false);
            mark_comp(sc.mk_c, common, true);
        }
        const bool ok = add_in_order(inv, m, common, rev);
        mark_comp(sc.mk_c, common, false);
        return ok;
    }

    __device__ void fail() {
        if (lane == 0) {
            hd->success = 0;
            hd->n = 0;
        }
        sync();
    }

    __device__ void kill_comp(u32 key) {
        const u32 nn = n();
        for (u32 i = lane; i < nn; i += 64)
            if (e_key(ld(&ent[i])) == key) ent[i] = kDead;
        sync();
    }

    // one input component (key in_key, sorted vertices inv[0..m)) against this (:84-135); false: fail()
    __device__ bool merge_component(const u64* inv, u32 m, u32 in_key) {
        __shared__ u32 s_nt, s_nmw;
        for (u32 j = lane; j < m; j += 64) {
            const u64 e = ld(&inv[j]);
            sc.mk_in[e_v(e)] = 1u + e_s(e);
        }
        if (lane == 0) s_nt = 0;
        sync();
        const u32 nn = n();
        for (u32 i = lane; i < nn; i += 64) {  // the self components sharing a vertex with the input's
            const u64 e = ld(&ent[i]);
            if (e == kDead || !ld(&sc.mk_in[e_v(e)])) continue;
            if (atomicAdd(&sc.cnt_in[e_key(e)], 1u) == 0) sc.keys[atomicAdd(&s_nt, 1u)] = e_key(e);
        }
        sync();
        const u32 nt = s_nt;
        if (nt) {
            for (u32 i = lane; i < nn; i += 64) {  // and their sizes (the identical-set test, :91-95)
                const u64 e = ld(&ent[i]);
                if (e != kDead && ld(&sc.cnt_in[e_key(e)])) atomicAdd(&sc.cnt_sz[e_key(e)], 1u);
            }
            sync();
        }
        // mergeWith (:86-106): touched keys whose vertex set differs from the input's; then sorted (:114)
        if (lane == 0) {
            u32 k = 0;
            for (u32 t = 0; t < nt; ++t) {
                const u32 key = ld(&sc.keys[t]);
                const bool same = ld(&sc.cnt_in[key]) == m && ld(&sc.cnt_sz[key]) == m;
                if (!same) sc.keys[k++] = key;
            }
            s_nmw = k;
        }
        sync();
        // clear the counters of every touched key (the touched list was compacted in place above: by a scan of
        // the entries instead). The counters are only ever written by memory-side atomics, never by plain stores:
        // a dirty L2 copy of a counter line could be written back over a later atomic's result
        for (u32 i = lane; i < nn; i += 64) {
            const u64 e = ld(&ent[i]);
            if (e != kDead && ld(&sc.cnt_in[e_key(e)])) {
                atomicExch(&sc.cnt_in[e_key(e)], 0u);
                atomicExch(&sc.cnt_sz[e_key(e)], 0u);
            }
        }
        const u32 nmw = s_nmw;
        // sort the merge list (insertion sort by lane 0: a few keys)
        if (lane == 0)
            for (u32 a = 1; a < nmw; ++a) {
                const u32 x = ld(&sc.keys[a]);
                u32 b = a;
                while (b > 0 && ld(&sc.keys[b - 1]) > x) {
                    sc.keys[b] = ld(&sc.keys[b - 1]);
                    --b;
                }
                sc.keys[b] = x;
            }
        sync();
        bool ok = true;
        if (nmw == 0) {
            mark_comp(sc.mk_c, in_key, true);  // this.add(inKey, vertices): add()'s false ignored (:111)
            (void)add_in_order(inv, m, in_key, 0u);
            mark_comp(sc.mk_c, in_key, false);
        } else {
            const u32 first = ld(&sc.keys[0]);
            ok = merge_into(inv, m, in_key, first);
            const u32 f2 = in_key < first ? in_key : first;  // :123
            for (u32 i = 1; ok && i < nmw; ++i) {
                const u32 k = ld(&sc.keys[i]);
                const u32 cnt = gather_sorted(ent, n(), k);  // inputComponent = this.getMap().get(k), in vertex order
                if (cnt == kNone) {
                    if (lane == 0) hd->err |= kErrCap;
                    sync();
                    break;
                }
                (void)merge_into(sc.tmp2, cnt, k, f2);  // :128-131: a failure is dropped
                kill_comp(k);                            // :133
                if (ld(&hd->err)) break;
            }
        }
        for (u32 j = lane; j < m; j += 64) sc.mk_in[e_v(ld(&inv[j]))] = 0;
        sync();
        return ok;
    }

    __device__ void compact() {  // drop dead entries, keeping the order
        __shared__ u32 s_w;
        if (lane == 0) s_w = 0;
        sync();
        const u32 nn = n();
        for (u32 b = 0; b < nn; b += 64) {
            const u32 i = b + lane;
            const u64 e = i < nn ? ld(&ent[i]) : kDead;
            const u64 m = __ballot(e != kDead);
            const u32 base = s_w;
            sync();
            if (e != kDead) ent[base + (u32)__popcll(m & ((1ull << lane) - 1))] = e;
            sync();
            if (lane == 0) s_w = base + (u32)__popcll(m);
            sync();
        }
        if (lane == 0) hd->n = s_w;
        sync();
    }
};

// updateFunction.foldEdges per edge, in stream order: candidates = candidates.merge(edgeToCandidate(u, v))
__global__ __launch_bounds__(64) void literal_fold_kernel(LitDev* hd, u64* ent, u32 cap, Scratch sc, const u64* edges,
                                                          u64 n_edges) {
    Lit L{hd, ent, cap, sc, threadIdx.x};
    __shared__ u64 s_in[2];
    for (u64 i = 0; i < n_edges; ++i) {
        if (!ld(&hd->success) || ld(&hd->err)) break;  // merge() of a failed summary: fail() again (:78-81)
        const u64 e = ld(&edges[i]);
        const u32 a = (u32)e, b = (u32)(e >> 32);
        const u32 src = a < b ? a : b, trg = a < b ? b : a;
        if (threadIdx.x == 0) {
            s_in[0] = mk_e(src, src, 1u);
            s_in[1] = mk_e(src, trg, 0u);  // a self loop: add() refuses (trg, false) (BipartitenessCheck.java:58-59)
        }
        __syncthreads();
        if (!L.merge_component(s_in, src == trg ? 1u : 2u, src)) L.fail();
        if ((i & 63) == 63) L.compact();
    }
    L.compact();
}

// combineFunction.reduce / the Merger: this = this.merge(input) with input's entries `in` (any order)
__global__ __launch_bounds__(64) void literal_merge_kernel(LitDev* hd, u64* ent, u32 cap, Scratch sc, const u64* in,
                                                           u32 n_in, u32 in_success) {
    Lit L{hd, ent, cap, sc, threadIdx.x};
    __shared__ u32 s_key;
    if (!in_success || !ld(&hd->success)) {  // :78-81
        L.fail();
        return;
    }
    // the input's components in key order (TreeMap): the smallest key above the last one, each time
    u32 last = 0;
    bool started = false;
    for (;;) {
        u32 best = kNone;
        for (u32 i = threadIdx.x; i < n_in; i += 64) {
            const u32 k = e_key(ld(&in[i]));
            if ((!started || k > last) && k < best) best = k;
        }
        for (int o = 32; o > 0; o >>= 1) {
            const u32 y = __shfl_xor(best, o, 64);
            best = y < best ? y : best;
        }
        if (best == kNone) break;
        if (threadIdx.x == 0) s_key = best;
        __syncthreads();
        const u32 key = s_key;
        started = true;
        last = key;
        const u32 m = L.gather_sorted(in, n_in, key);
        if (m == kNone) {
            if (threadIdx.x == 0) hd->err |= kErrCap;
            break;
        }
        // the input's sorted component sits in sc.tmp2; merge_component's second level reuses tmp / tmp2, so it is
        // copied to the upper half of tmp2 first
        u64* inv = sc.tmp2 + sc.cap_tmp;
        for (u32 j = threadIdx.x; j < m; j += 64) inv[j] = ld(&sc.tmp2[j]);
        sync();
        if (!L.merge_component(inv, m, key)) {
            L.fail();
            break;
        }
        if (ld(&hd->err)) break;
        L.compact();
    }
    L.compact();
}

}  // namespace

struct gcc_literal {
    int device = 0;
    u32 cap_ids = 0;
    u32 cap_ent = 0;
    hipStream_t stream = nullptr;
    LitDev* d_hd = nullptr;
    u64* d_ent = nullptr;
    Scratch sc{};
    u64* d_in = nullptr;  // staging: edges or another summary's entries
    u64 in_cap = 0;
};

static int lit_check(gcc_literal* h) {
    LitDev hd;
    HIP_TRY(hipMemcpyAsync(&hd, h->d_hd, sizeof(hd), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (hd.err & kErrCap)
        return gcc_set_err(GCC_E_OOM, "literal Candidates: more than %u entries (entry_capacity)", h->cap_ent);
    if (hd.err & kErrNoCommon)
        return gcc_set_err(GCC_E_INVALID, "literal Candidates: _merge found no common vertex (the reference throws "
                                          "IndexOutOfBoundsException at Candidates.java:156)");
    return GCC_OK;
}

static int lit_stage(gcc_literal* h, u64 n) {
    if (h->in_cap >= n) return GCC_OK;
    if (h->d_in) HIP_TRY(hipFree(h->d_in));
    h->d_in = nullptr;
    h->in_cap = 0;
    HIP_TRY(hipMalloc((void**)&h->d_in, std::max<u64>(n, 64) * sizeof(u64)));
    h->in_cap = std::max<u64>(n, 64);
    return GCC_OK;
}

extern "C" {

int gcc_literal_create(int device, uint32_t id_capacity, uint32_t entry_capacity, gcc_literal** out) {
    CHECK_ARG(out, "out is null");
    *out = nullptr;
    CHECK_ARG(id_capacity > 0 && id_capacity <= kMaxLitId, "id_capacity must be in [1, 2^31 - 2]");
    CHECK_ARG(entry_capacity >= 64, "entry_capacity must be >= 64");
    int rc = gcc_check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    gcc_literal* h = new gcc_literal();
    h->device = device;
    h->cap_ids = id_capacity;
    h->cap_ent = entry_capacity;
    const size_t V = id_capacity;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_hd, sizeof(LitDev));
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_ent, (size_t)entry_capacity * sizeof(u64));
    u32* marks = nullptr;
    if (e == hipSuccess) e = hipMalloc((void**)&marks, 5 * V * sizeof(u32));
    h->sc.cap_tmp = entry_capacity;
    if (e == hipSuccess) e = hipMalloc((void**)&h->sc.tmp, 3 * (size_t)entry_capacity * sizeof(u64));
    if (e == hipSuccess) e = hipMemsetAsync(marks, 0, 5 * V * sizeof(u32), h->stream);
    if (e == hipSuccess) {
        h->sc.mk_in = marks;
        h->sc.mk_c = marks + V;
        h->sc.cnt_in = marks + 2 * V;
        h->sc.cnt_sz = marks + 3 * V;
        h->sc.keys = marks + 4 * V;
        h->sc.tmp2 = h->sc.tmp + entry_capacity;  // tmp2 spans two halves (merge input copy above)
        LitDev hd{1u, 0u, 0u, 0u};                 // new Candidates(true) (:31-34)
        e = hipMemcpyAsync(h->d_hd, &hd, sizeof(hd), hipMemcpyHostToDevice, h->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        if (marks) (void)hipFree(marks);
        h->sc.mk_in = nullptr;
        gcc_literal_destroy(h);
        return gcc_set_err(e == hipErrorOutOfMemory ? GCC_E_OOM : GCC_E_HIP, "gcc_literal_create: %s", hipGetErrorString(e));
    }
    *out = h;
    return GCC_OK;
}

int gcc_literal_destroy(gcc_literal* h) {
    if (!h) return GCC_OK;
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->d_hd) (void)hipFree(h->d_hd);
    if (h->d_ent) (void)hipFree(h->d_ent);
    if (h->sc.mk_in) (void)hipFree(h->sc.mk_in);
    if (h->sc.tmp) (void)hipFree(h->sc.tmp);
    if (h->d_in) (void)hipFree(h->d_in);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return GCC_OK;
}

int gcc_literal_reset(gcc_literal* h) {
    CHECK_ARG(h, "handle is null");
    DeviceGuard g(h->device);
    LitDev hd{1u, 0u, 0u, 0u};
    HIP_TRY(hipMemcpyAsync(h->d_hd, &hd, sizeof(hd), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return GCC_OK;
}

int gcc_literal_fold_host(gcc_literal* h, const uint32_t* pairs, uint64_t n_edges) {
    CHECK_ARG(h, "handle is null");
    CHECK_ARG(pairs || n_edges == 0, "pairs is null");
    if (n_edges == 0) return GCC_OK;
    for (u64 i = 0; i < 2 * n_edges; ++i)
        CHECK_ARG(pairs[i] < h->cap_ids, "an edge id is >= id_capacity");
    DeviceGuard g(h->device);
    int rc = lit_stage(h, n_edges);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h->d_in, pairs, n_edges * sizeof(u64), hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(literal_fold_kernel, dim3(1), dim3(64), 0, h->stream, h->d_hd, h->d_ent, h->cap_ent, h->sc,
                       (const u64*)h->d_in, (u64)n_edges);
    HIP_TRY(hipGetLastError());
    return lit_check(h);
}

int gcc_literal_merge(gcc_literal* into, gcc_literal* from) {
    CHECK_ARG(into && from, "handle is null");
    CHECK_ARG(into != from, "merge of a summary with itself");
    CHECK_ARG(into->cap_ids == from->cap_ids && into->device == from->device,
              "summaries of different id capacities or devices");
    DeviceGuard g(into->device);
    LitDev fh;
    HIP_TRY(hipStreamSynchronize(into->stream));
    HIP_TRY(hipMemcpyAsync(&fh, from->d_hd, sizeof(fh), hipMemcpyDeviceToHost, from->stream));
    HIP_TRY(hipStreamSynchronize(from->stream));
    hipLaunchKernelGGL(literal_merge_kernel, dim3(1), dim3(64), 0, into->stream, into->d_hd, into->d_ent, into->cap_ent,
                       into->sc, (const u64*)from->d_ent, fh.n, fh.success);
    HIP_TRY(hipGetLastError());
    return lit_check(into);
}

int gcc_literal_success(gcc_literal* h, int* success) {
    CHECK_ARG(h && success, "null argument");
    DeviceGuard g(h->device);
    LitDev hd;
    HIP_TRY(hipMemcpyAsync(&hd, h->d_hd, sizeof(hd), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *success = hd.success ? 1 : 0;
    return GCC_OK;
}

int gcc_literal_entries(gcc_literal* h, uint64_t* out, uint64_t cap, uint64_t* n) {
    CHECK_ARG(h && n, "null argument");
    DeviceGuard g(h->device);
    LitDev hd;
    HIP_TRY(hipMemcpyAsync(&hd, h->d_hd, sizeof(hd), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *n = hd.n;
    if (!out) return GCC_OK;
    CHECK_ARG(cap >= hd.n, "out holds fewer entries than the summary (call with out = NULL for the count)");
    if (hd.n) HIP_TRY(hipMemcpy(out, h->d_ent, (size_t)hd.n * sizeof(u64), hipMemcpyDeviceToHost));
    return GCC_OK;
}

}  // extern "C"
