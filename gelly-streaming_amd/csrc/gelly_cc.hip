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

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gelly_cc.h"
#include "edge_gen.h"

typedef uint32_t u32;
typedef uint64_t u64;

#define UNSEEN GCC_UNSEEN

// ------------------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------------------
static thread_local std::string g_last_error;

static int set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            return set_err(e_ == hipErrorOutOfMemory ? GCC_E_OOM : GCC_E_HIP, "%s failed: %s (%s:%d)", \
                           #expr, hipGetErrorString(e_), __FILE__, __LINE__);                          \
        }                                                                                              \
    } while (0)

#define CHECK_ARG(cond, msg)                               \
    do {                                                   \
        if (!(cond)) return set_err(GCC_E_INVALID, "%s", msg); \
    } while (0)

// ------------------------------------------------------------------------------------------------
// device union-find primitives
// ------------------------------------------------------------------------------------------------

// makeSet-on-first-sight (DisjointSet.union :99-104): returns an observed parent of v that is not UNSEEN.
__device__ __forceinline__ u32 seen_parent(u32* parent, u32 v) {
    u32 p = parent[v];
    if (p == UNSEEN) {
        const u32 old = atomicCAS(&parent[v], UNSEEN, v);
        p = (old == UNSEEN) ? v : old;
    }
    return p;
}

// find (DisjointSet.find :71-85) from x whose observed parent is p, with path splitting: every visited
// non-root slot is re-pointed at its grandparent (plain store; see the memory-model note at the top).
__device__ __forceinline__ u32 find_from(u32* parent, u32 x, u32 p) {
    // p >= x: x is a root, or p is a stale UNSEEN (an L1 line older than x's makeSet CAS): treat x as a root —
    // a later CAS on it compares against the real value
    if (p >= x) return x;
    u32 prev = x, cur = p;
    while (true) {
        const u32 next = parent[cur];
        if (next >= cur) break;  // cur is a root (next == cur); a stale UNSEEN reads as root too
        parent[prev] = next;
        prev = cur;
        cur = next;
    }
    return cur;
}

// union (DisjointSet.union :97-123) with min-id hooking instead of union-by-rank.
__device__ __forceinline__ void unite(u32* parent, u32 u, u32 v) {
    const u32 pu = seen_parent(parent, u);
    if (u == v) return;  // self loop: makeSet only (DisjointSet.union with e1 == e2)
    const u32 pv = seen_parent(parent, v);
    u32 ru = find_from(parent, u, pu);
    u32 rv = find_from(parent, v, pv);
    while (ru != rv) {
        const u32 lo = ru < rv ? ru : rv;
        const u32 hi = ru < rv ? rv : ru;
        u32 old = atomicCAS(&parent[hi], hi, lo);
        if (old == hi) return;  // hooked
        if (old == UNSEEN) {    // not reachable for seen roots; kept so the loop can never spin
            old = atomicCAS(&parent[hi], UNSEEN, lo);
            if (old == UNSEEN) return;
        }
        // hi was hooked by someone else meanwhile: old is its (fresh) parent, strictly < hi
        ru = find_from(parent, hi, old);
        rv = find_from(parent, lo, parent[lo]);
    }
}

// ------------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------------
constexpr int kBlock = 256;

// Fold a batch of edges (interleaved u32 pairs) into the forest: one edge per lane per iteration,
// 8 B/lane coalesced stream; the parent lookups are the random part.
__global__ __launch_bounds__(kBlock) void fold_kernel(u32* __restrict__ parent, const uint2* __restrict__ edges,
                                                      u64 n_edges) {
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n_edges; i += stride) {
        // the edge stream is read once: non-temporal, so it does not evict parent[] lines from L2
        const u64 e = __builtin_nontemporal_load(reinterpret_cast<const u64*>(edges) + i);
        unite(parent, (u32)e, (u32)(e >> 32));
    }
}

// Merge: into ∪ {(v, labels[v])}. labels may be any parent array of a forest over the same id range
// (compressed or not) — its (key, parent) pairs generate its partition (DisjointSet.merge :132-136).
__global__ __launch_bounds__(kBlock) void merge_labels_kernel(u32* __restrict__ parent, const u32* __restrict__ labels,
                                                              u32 n) {
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 vv = (u64)blockIdx.x * kBlock + threadIdx.x; vv < n; vv += stride) {
        const u32 v = (u32)vv;
        const u32 l = labels[v];
        if (l == UNSEEN) continue;
        unite(parent, v, l);
    }
}

// Canonicalise: labels[v] := root(v) = min id of v's component, UNSEEN stays UNSEEN (multi-level pointer
// jumping). Out of place on purpose: the path-splitting stores that let all threads collapse a deep chain
// together (O(log d) instead of O(d) per thread) write intermediate ancestors into parent[], and such a store
// can land after another thread's final root store — in place that would leave a vertex pointing at a
// non-root. labels[] is written exactly once per slot, by its own thread, so it is race-free; parent[] only
// needs to stay a valid forest (every store is an ancestor, roots never move: no hook is in flight).
// Algorithmic traffic: 4 B read + 4 B write per id (chain reads hit L2).
__global__ __launch_bounds__(kBlock) void compress_kernel(u32* __restrict__ parent, u32* __restrict__ labels, u32 n) {
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 vv = (u64)blockIdx.x * kBlock + threadIdx.x; vv < n; vv += stride) {
        const u32 v = (u32)vv;
        const u32 p = parent[v];
        labels[v] = (p >= v) ? p : find_from(parent, v, p);  // root / UNSEEN: itself
    }
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

__global__ __launch_bounds__(kBlock) void gen_kernel(gcc_gen_params prm, u64 first, u64 count, uint2* __restrict__ out) {
    const u64 stride = (u64)gridDim.x * kBlock;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < count; i += stride) {
        u32 u, v;
        gcc_gen_edge(&prm, first + i, &u, &v);
        out[i] = make_uint2(u, v);
    }
}

static inline unsigned grid_for(u64 n, unsigned max_blocks) {
    u64 b = (n + kBlock - 1) / kBlock;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (unsigned)b;
}

// 256 CUs x 8 resident 256-thread blocks
constexpr unsigned kMaxGrid = 2048;

// ------------------------------------------------------------------------------------------------
// host-side forest handle
// ------------------------------------------------------------------------------------------------
struct gcc_forest {
    int device = 0;
    u32 cap = 0;
    // two id-range buffers: d_parent (the working forest) and d_spare; compress writes the canonical labels
    // into d_spare and the two swap roles, so after a compress d_parent IS the label array
    u32* d_parent = nullptr;
    u32* d_spare = nullptr;
    bool own_bufs = true;
    bool compressed = false;  // d_parent holds canonical labels (no mutation since the last compress)
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    // pinned double-buffered staging for host-fed edges (per-edge foldEdges appends here)
    static constexpr u64 kStageEdges = 1ull << 20;  // 8 MiB per slot
    u32* h_stage[2] = {nullptr, nullptr};
    u32* d_stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    int slot = 0;
    u64 staged = 0;

    // scratch for cross-device merges
    u32* d_scratch = nullptr;

    unsigned long long* d_counts = nullptr;

    // lazy host view of the labels (getMatches()/find() consumers)
    std::vector<u32> host_labels;
    bool host_valid = false;

    bool timing = false;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    bool t_recorded = false;
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

static int check_device(int device) {
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

static int launch_fold(gcc_forest* h, const u32* d_pairs, u64 n) {
    if (n == 0) return GCC_OK;
    if (h->timing) HIP_TRY(hipEventRecord(h->t0, h->stream));
    hipLaunchKernelGGL(fold_kernel, dim3(grid_for(n, kMaxGrid)), dim3(kBlock), 0, h->stream, h->d_parent,
                       reinterpret_cast<const uint2*>(d_pairs), n);
    HIP_TRY(hipGetLastError());
    if (h->timing) {
        HIP_TRY(hipEventRecord(h->t1, h->stream));
        h->t_recorded = true;
    }
    h->host_valid = false;
    h->compressed = false;
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

static int flush(gcc_forest* h) {
    if (h->staged == 0) return GCC_OK;
    return submit_slot(h, h->staged);
}

static int compress_async(gcc_forest* h) {
    int rc = flush(h);
    if (rc) return rc;
    if (h->compressed) return GCC_OK;
    hipLaunchKernelGGL(compress_kernel, dim3(grid_for(h->cap, kMaxGrid)), dim3(kBlock), 0, h->stream, h->d_parent,
                       h->d_spare, h->cap);
    HIP_TRY(hipGetLastError());
    std::swap(h->d_parent, h->d_spare);
    h->compressed = true;
    return GCC_OK;
}

static int refresh_host(gcc_forest* h) {
    if (h->host_valid) return GCC_OK;
    int rc = compress_async(h);
    if (rc) return rc;
    h->host_labels.resize(h->cap);
    HIP_TRY(hipMemcpyAsync(h->host_labels.data(), h->d_parent, (size_t)h->cap * sizeof(u32), hipMemcpyDeviceToHost,
                           h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->host_valid = true;
    return GCC_OK;
}

static int counts(gcc_forest* h, unsigned long long out[2]) {
    int rc = flush(h);
    if (rc) return rc;
    if (!h->d_counts) HIP_TRY(hipMalloc((void**)&h->d_counts, 2 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(h->d_counts, 0, 2 * sizeof(unsigned long long), h->stream));
    hipLaunchKernelGGL(count_kernel, dim3(grid_for(h->cap, kMaxGrid)), dim3(kBlock), 0, h->stream, h->d_parent, h->cap,
                       h->d_counts);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, h->d_counts, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return GCC_OK;
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
extern "C" {

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
    int rc = check_device(device);
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

static int forest_create_impl(int device, uint32_t id_capacity, uint32_t* d_buf0, uint32_t* d_buf1,
                              gcc_forest** out) {
    CHECK_ARG(out, "out is null");
    *out = nullptr;
    CHECK_ARG(id_capacity >= 1 && id_capacity <= UNSEEN, "id_capacity must be in [1, 0xFFFFFFFF]");
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    gcc_forest* h = new gcc_forest();
    h->device = device;
    h->cap = id_capacity;
    auto fail = [&](int code) {
        gcc_forest_destroy(h);
        return code;
    };
    hipError_t e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return fail(set_err(GCC_E_HIP, "hipStreamCreate: %s", hipGetErrorString(e)));
    h->stream = h->own_stream;
    if (d_buf0) {
        h->d_parent = d_buf0;
        h->d_spare = d_buf1;
        h->own_bufs = false;
    } else {
        e = hipMalloc((void**)&h->d_parent, (size_t)id_capacity * sizeof(u32));
        if (e == hipSuccess) e = hipMalloc((void**)&h->d_spare, (size_t)id_capacity * sizeof(u32));
        if (e != hipSuccess) return fail(set_err(GCC_E_OOM, "hipMalloc 2 x u32[%u]: %s", id_capacity, hipGetErrorString(e)));
    }
    e = hipEventCreate(&h->t0);
    if (e == hipSuccess) e = hipEventCreate(&h->t1);
    if (e != hipSuccess) return fail(set_err(GCC_E_HIP, "hipEventCreate: %s", hipGetErrorString(e)));
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
    return forest_create_impl(device, id_capacity, d_buf0, d_buf1, out);
}

int gcc_forest_destroy(gcc_forest* h) {
    if (!h) return GCC_OK;
    DeviceGuard g(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
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
    if (h->d_counts) (void)hipFree(h->d_counts);
    if (h->t0) (void)hipEventDestroy(h->t0);
    if (h->t1) (void)hipEventDestroy(h->t1);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
    return GCC_OK;
}

int gcc_forest_set_stream(gcc_forest* h, void* hip_stream) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    hipStream_t next = hip_stream ? (hipStream_t)hip_stream : h->own_stream;
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

int gcc_forest_device_ptr(gcc_forest* h, uint32_t** d_parent) {
    CHECK_ARG(h && d_parent, "null argument");
    *d_parent = h->d_parent;
    return GCC_OK;
}

int gcc_forest_reset(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    h->staged = 0;
    HIP_TRY(hipMemsetAsync(h->d_parent, 0xFF, (size_t)h->cap * sizeof(u32), h->stream));
    h->host_valid = false;
    h->compressed = true;  // all UNSEEN is canonical
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
    return flush(h);
}

int gcc_forest_fold_device(gcc_forest* h, const uint32_t* d_pairs, uint64_t n_edges) {
    CHECK_ARG(h, "null forest");
    CHECK_ARG(d_pairs || n_edges == 0, "d_pairs is null");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    return launch_fold(h, d_pairs, n_edges);
}

int gcc_forest_flush(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    return flush(h);
}

int gcc_forest_sync(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    int rc = flush(h);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(h->stream));
    return GCC_OK;
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
                       d_labels, n);
    HIP_TRY(hipGetLastError());
    into->host_valid = false;
    into->compressed = false;
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
    // order into's stream after everything queued on from's stream
    hipEvent_t ev;
    {
        DeviceGuard gf(from->device);
        HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ev, from->stream));
    }
    HIP_TRY(hipStreamWaitEvent(into->stream, ev, 0));
    const u32* src = from->d_parent;
    if (from->device != into->device) {
        if (!into->d_scratch) HIP_TRY(hipMalloc((void**)&into->d_scratch, (size_t)into->cap * sizeof(u32)));
        HIP_TRY(hipMemcpyPeerAsync(into->d_scratch, into->device, from->d_parent, from->device,
                                   (size_t)from->cap * sizeof(u32), into->stream));
        src = into->d_scratch;
    }
    rc = gcc_forest_merge_labels_device(into, src, from->cap);
    // from must not be mutated before the merge has read it
    HIP_TRY(hipEventRecord(ev, into->stream));
    {
        DeviceGuard gf(from->device);
        HIP_TRY(hipStreamWaitEvent(from->stream, ev, 0));
    }
    HIP_TRY(hipEventDestroy(ev));
    return rc;
}

int gcc_forest_compress(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    DeviceGuard g(h->device);
    return compress_async(h);
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
    HIP_TRY(hipStreamSynchronize(h->stream));
    return GCC_OK;
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
    h->timing = enable != 0;
    h->t_recorded = false;
    return GCC_OK;
}

int gcc_forest_last_fold_ms(gcc_forest* h, float* ms) {
    CHECK_ARG(h && ms, "null argument");
    CHECK_ARG(h->t_recorded, "no timed fold recorded (call gcc_forest_enable_timing first)");
    DeviceGuard g(h->device);
    HIP_TRY(hipEventSynchronize(h->t1));
    HIP_TRY(hipEventElapsedTime(ms, h->t0, h->t1));
    return GCC_OK;
}

}  // extern "C"
