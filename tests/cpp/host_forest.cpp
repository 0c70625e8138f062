// host_forest.cpp — TEST INFRASTRUCTURE ONLY: the forest half of the C ABI (include/gelly_cc.h) that the cross-GPU
// group merge (gelly-streaming_amd/csrc/gelly_group.cpp) calls, restated on the host, so that the product's merge
// protocol — gcc_forest_group_merge with nranks > 1: speculative compact rounds, agree(), failed-status headers, the
// label fallback — runs in CPU processes over the shared-memory RCCL stand-in (tests/cpp/shm_rccl.cpp) and is
// checked against the oracle every window (tests/test_group_protocol.py). Linked with gelly_group.cpp and the
// hipmock header into tests/cpp/build/libgelly_group_host.so; nothing under gelly-streaming_amd/ uses it.
//
// The forest is a min-id union-find (the device forest's partition rule: every root is its component's minimum
// id, so a full compress is the canonical label array). The message layout is include/gelly_cc.h's: header
// {g, n_others, id_capacity, status}, the bitmap of label == g, then (v, label) of the other seen ids; n_others is
// the true count even past cap_others (only cap_others pairs written). A message whose id_capacity differs is
// ignored, as on the device (a failed-status header has id_capacity 0).
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <unordered_map>
#include <vector>

#include "abi_common.h"

typedef uint32_t u32;
typedef uint64_t u64;

struct gcc_forest {
    u32 cap = 0;
    std::vector<u32> parent;  // UNSEEN, or a smaller id (roots: parent[v] == v)
    std::vector<u32> labels;  // canonical labels after compress (what gcc_forest_labels_device hands out)
    int fail_absorb = 0;
    bool bad_label = false;  // an out-of-range label was skipped (reported by the next sync, as on the device)
    // the delta merge (round 6): while armed, the folds list every id whose slot they change (a hooked root, a new
    // id), as the device fold's delta lists do; any other mutation disarms
    bool armed = false;
    std::vector<u32> delta;
    u64 delta_edges = 0;
};

namespace {
thread_local std::string g_err;

u32 find(gcc_forest* h, u32 v) {
    u32 r = v;
    while (h->parent[r] != r) r = h->parent[r];
    while (h->parent[v] != r) {  // full compression
        const u32 n = h->parent[v];
        h->parent[v] = r;
        v = n;
    }
    return r;
}

void unite(gcc_forest* h, u32 a, u32 b, bool record = false) {
    std::vector<u32>* ev = record && h->armed ? &h->delta : nullptr;
    if (!record) h->armed = false;
    if (h->parent[a] == GCC_UNSEEN) {  // makeSet on sight (DisjointSet.java:99-104)
        h->parent[a] = a;
        if (ev) ev->push_back(a);
    }
    if (h->parent[b] == GCC_UNSEEN) {
        h->parent[b] = b;
        if (ev) ev->push_back(b);
    }
    const u32 ra = find(h, a), rb = find(h, b);
    const u32 lo = ra < rb ? ra : rb, hi = ra < rb ? rb : ra;
    if (lo != hi) {
        h->parent[hi] = lo;
        // a new id hung straight under the other's root is one event, as on the device (one CAS UNSEEN -> root)
        if (ev && !(ev->size() && ev->back() == hi)) ev->push_back(hi);
    }
}

void compress(gcc_forest* h) {
    for (u32 v = 0; v < h->cap; ++v) h->labels[v] = h->parent[v] == GCC_UNSEEN ? GCC_UNSEEN : find(h, v);
}
}  // namespace

int gcc_set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
int gcc_check_device(int device) { return device == 0 ? GCC_OK : gcc_set_err(GCC_E_NODEV, "host forest: device 0 only"); }
const char* gcc_fault_note(hipError_t) { return ""; }

extern "C" {

const char* gcc_last_error(void) { return g_err.c_str(); }

int gcc_forest_create(int device, uint32_t id_capacity, gcc_forest** out) {
    CHECK_ARG(out && id_capacity > 0, "null argument");
    (void)device;
    gcc_forest* h = new gcc_forest();
    h->cap = id_capacity;
    h->parent.assign(id_capacity, GCC_UNSEEN);
    h->labels.assign(id_capacity, GCC_UNSEEN);
    *out = h;
    return GCC_OK;
}
int gcc_forest_destroy(gcc_forest* h) {
    delete h;
    return GCC_OK;
}
int gcc_forest_fold_host(gcc_forest* h, const uint32_t* pairs, uint64_t n) {
    CHECK_ARG(h && (pairs || !n), "null argument");
    for (u64 i = 0; i < n; ++i) {
        CHECK_ARG(pairs[2 * i] < h->cap && pairs[2 * i + 1] < h->cap, "id >= id_capacity");
        unite(h, pairs[2 * i], pairs[2 * i + 1], true);
    }
    h->delta_edges += n;
    return GCC_OK;
}
int gcc_forest_labels(gcc_forest* h, uint32_t* out, uint32_t n) {
    CHECK_ARG(h && out && n <= h->cap, "bad argument");
    if (h->bad_label) {
        h->bad_label = false;
        return gcc_set_err(GCC_E_INVALID, "a label >= id_capacity was skipped");
    }
    compress(h);
    for (u32 v = 0; v < n; ++v) out[v] = h->labels[v];
    return GCC_OK;
}
int gcc_forest_device(gcc_forest* h, int* dev) {
    CHECK_ARG(h && dev, "null argument");
    *dev = 0;
    return GCC_OK;
}
int gcc_forest_capacity(gcc_forest* h, uint32_t* cap) {
    CHECK_ARG(h && cap, "null argument");
    *cap = h->cap;
    return GCC_OK;
}
int gcc_forest_get_stream(gcc_forest* h, void** s) {
    CHECK_ARG(h && s, "null argument");
    *s = nullptr;
    return GCC_OK;
}
int gcc_forest_sync(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    return GCC_OK;
}
int gcc_forest_compress(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    compress(h);
    return GCC_OK;
}
int gcc_forest_labels_device(gcc_forest* h, const uint32_t** d) {
    CHECK_ARG(h && d, "null argument");
    compress(h);
    *d = h->labels.data();
    return GCC_OK;
}
int gcc_forest_merge_labels_device(gcc_forest* into, const uint32_t* lab, uint32_t n) {
    CHECK_ARG(into && (lab || !n) && n <= into->cap, "bad argument");
    into->armed = false;  // a mutation no delta list records (as on the device)
    std::vector<u32> copy(lab, lab + n);  // lab may be into's own label buffer
    for (u32 v = 0; v < n; ++v) {
        if (copy[v] == GCC_UNSEEN) continue;
        if (copy[v] >= into->cap) {
            into->bad_label = true;
            continue;
        }
        unite(into, v, copy[v]);
    }
    return GCC_OK;
}
int gcc_forest_merge(gcc_forest* into, gcc_forest* from) {
    CHECK_ARG(into && from && from->cap <= into->cap, "bad argument");
    compress(from);
    return gcc_forest_merge_labels_device(into, from->labels.data(), from->cap);
}
uint64_t gcc_msg_bytes(uint32_t id_capacity, uint64_t cap_others) {
    return GCC_MSG_HEADER_BYTES + (((u64)id_capacity + 63) / 64) * 8 + cap_others * 8;
}
int gcc_forest_encode(gcc_forest* h, void* d_msg, uint64_t cap_others) {
    CHECK_ARG(h && d_msg, "null argument");
    compress(h);
    std::unordered_map<u32, u64> count;
    for (u32 v = 0; v < h->cap; ++v)
        if (h->labels[v] != GCC_UNSEEN) ++count[h->labels[v]];
    u32 g = GCC_UNSEEN;
    u64 best = 0;
    for (auto& kv : count)
        if (kv.second > best || (kv.second == best && kv.first < g)) g = kv.first, best = kv.second;
    u32* hdr = static_cast<u32*>(d_msg);
    u64* bits = reinterpret_cast<u64*>(static_cast<char*>(d_msg) + GCC_MSG_HEADER_BYTES);
    const u64 nw = ((u64)h->cap + 63) / 64;
    u32* oth = reinterpret_cast<u32*>(bits + nw);
    for (u64 w = 0; w < nw; ++w) bits[w] = 0;
    u64 n = 0;
    for (u32 v = 0; v < h->cap; ++v) {
        const u32 l = h->labels[v];
        if (l == GCC_UNSEEN) continue;
        if (l == g) {
            bits[v / 64] |= 1ull << (v % 64);
        } else {
            if (n < cap_others) oth[2 * n] = v, oth[2 * n + 1] = l;
            ++n;
        }
    }
    hdr[0] = g;
    hdr[1] = (u32)n;
    hdr[2] = h->cap;
    hdr[3] = 0;
    return GCC_OK;
}
int gcc_forest_absorb_many(gcc_forest* h, const void* d_msgs, uint64_t stride, uint32_t count, uint32_t skip,
                           uint64_t cap_others) {
    CHECK_ARG(h && (d_msgs || !count), "null argument");
    CHECK_ARG(count <= 1 || stride >= gcc_msg_bytes(h->cap, cap_others), "stride smaller than a message");
    if (h->fail_absorb > 0 && --h->fail_absorb == 0)
        return gcc_set_err(GCC_E_INTERNAL, "gcc_forest_absorb_many: injected failure (tune key fail_absorb)");
    const u64 nw = ((u64)h->cap + 63) / 64;
    h->armed = false;
    for (u32 p = 0; p < count; ++p) {
        if (p == skip) continue;
        const char* m = static_cast<const char*>(d_msgs) + (u64)p * stride;
        const u32* hdr = reinterpret_cast<const u32*>(m);
        if (hdr[2] != h->cap) continue;  // another id range, or a failed-status header
        const u64* bits = reinterpret_cast<const u64*>(m + GCC_MSG_HEADER_BYTES);
        const u32 g = hdr[0];
        if (g < h->cap)
            for (u64 w = 0; w < nw; ++w)
                for (u64 b = bits[w]; b; b &= b - 1) unite(h, (u32)(64 * w + __builtin_ctzll(b)), g);
        const u32* oth = reinterpret_cast<const u32*>(bits + nw);
        const u64 k = hdr[1] < cap_others ? hdr[1] : cap_others;
        for (u64 i = 0; i < k; ++i) {
            if (oth[2 * i] >= h->cap || oth[2 * i + 1] >= h->cap) {
                h->bad_label = true;
                continue;
            }
            unite(h, oth[2 * i], oth[2 * i + 1]);
        }
    }
    return GCC_OK;
}
uint64_t gcc_delta_msg_bytes(uint64_t cap_pairs) { return GCC_MSG_HEADER_BYTES + 8 * cap_pairs; }
int gcc_forest_delta_arm(gcc_forest* h) {
    CHECK_ARG(h, "null forest");
    h->armed = true;
    h->delta.clear();
    h->delta_edges = 0;
    return GCC_OK;
}
int gcc_forest_encode_delta(gcc_forest* h, void* d_msg, uint64_t cap_pairs) {
    CHECK_ARG(h && d_msg, "null argument");
    u32* hdr = static_cast<u32*>(d_msg);
    u32* pairs = hdr + GCC_MSG_HEADER_BYTES / sizeof(u32);
    hdr[0] = (u32)h->delta_edges;
    hdr[1] = h->armed ? (u32)h->delta.size() : 0;
    hdr[2] = h->cap;
    hdr[3] = h->armed ? 0 : GCC_DELTA_STATUS_UNARMED;
    if (h->armed)
        for (u64 k = 0; k < h->delta.size() && k < cap_pairs; ++k) {
            pairs[2 * k] = h->delta[k];
            pairs[2 * k + 1] = find(h, h->delta[k]);
        }
    return GCC_OK;
}
int gcc_forest_absorb_delta_many(gcc_forest* h, const void* d_msgs, uint64_t stride, uint32_t count, uint32_t skip,
                                 uint64_t cap_pairs) {
    CHECK_ARG(h && (d_msgs || !count), "null argument");
    CHECK_ARG(count <= 1 || stride >= gcc_delta_msg_bytes(cap_pairs), "stride smaller than a message");
    if (h->fail_absorb > 0 && --h->fail_absorb == 0)
        return gcc_set_err(GCC_E_INTERNAL, "gcc_forest_absorb_delta_many: injected failure (tune key fail_absorb)");
    for (u32 p = 0; p < count; ++p) {
        if (p == skip) continue;
        const u32* hdr = reinterpret_cast<const u32*>(static_cast<const char*>(d_msgs) + (u64)p * stride);
        if (hdr[2] != h->cap || hdr[3] != 0) continue;
        const u32* pairs = hdr + GCC_MSG_HEADER_BYTES / sizeof(u32);
        for (u64 k = 0; k < hdr[1] && k < cap_pairs; ++k) {
            if (pairs[2 * k] >= h->cap || pairs[2 * k + 1] >= h->cap) {
                h->bad_label = true;
                continue;
            }
            unite(h, pairs[2 * k], pairs[2 * k + 1]);
        }
    }
    h->armed = false;
    return GCC_OK;
}
int gcc_forest_tune(gcc_forest* h, const char* key, double value) {
    CHECK_ARG(h && key, "null argument");
    if (std::string(key) != "fail_absorb") return gcc_set_err(GCC_E_INVALID, "host forest: unknown key '%s'", key);
    h->fail_absorb = value > 0 ? (int)value : 0;
    return GCC_OK;
}

}  // extern "C"
