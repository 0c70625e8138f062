// gelly_idmap.cpp — host side of the boundary for wide vertex ids (include/gelly_cc.h, "id dictionary").
//
// The reference's summary is DisjointSet<Long> (…/summaries/DisjointSet.java:30-34: HashMap<R,R> keyed by the
// vertex id itself), so a Flink job may carry any Java Long as a vertex id. The device forest works on dense
// u32 ids. This dictionary assigns dense ids in first-seen order (an open-addressing table of int64 keys) and
// turns a forest's labels over dense ids back into the reference's canonical form: label = the minimum
// ORIGINAL id of the component, in Java Long (signed) order. Dense order is not id order, so the per-component
// minimum is taken explicitly (one pass over the seen ids) instead of being read off the min-id roots.
// Host-only code: no device calls, so it is testable without a GPU.

#include <stdint.h>

#include <cstring>
#include <new>
#include <vector>

#include "gelly_cc.h"

int gcc_set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

struct gcc_idmap {
    uint32_t capacity = 0;
    uint64_t mask = 0;
    std::vector<int64_t> keys;   // table slots (valid where used[s])
    std::vector<uint32_t> vals;  // dense id of the slot's key
    std::vector<uint8_t> used;
    std::vector<int64_t> orig;   // orig[d] = original id of dense id d
};

static inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

extern "C" {

int gcc_idmap_create(uint32_t capacity, gcc_idmap** out) {
    if (!out || capacity == 0 || capacity == GCC_UNSEEN)
        return gcc_set_err(GCC_E_INVALID, "gcc_idmap_create: capacity must be in [1, 0xFFFFFFFE] and out non-null");
    gcc_idmap* m = new (std::nothrow) gcc_idmap;
    if (!m) return gcc_set_err(GCC_E_OOM, "gcc_idmap_create: out of host memory");
    uint64_t slots = 16;
    while (slots < 2ull * capacity) slots <<= 1;  // load factor <= 1/2
    try {
        m->keys.resize(slots);
        m->vals.resize(slots);
        m->used.assign(slots, 0);
        m->orig.reserve(capacity < (1u << 20) ? capacity : (1u << 20));
    } catch (...) {
        delete m;
        return gcc_set_err(GCC_E_OOM, "gcc_idmap_create: out of host memory for %u ids", capacity);
    }
    m->capacity = capacity;
    m->mask = slots - 1;
    *out = m;
    return GCC_OK;
}

int gcc_idmap_destroy(gcc_idmap* m) {
    delete m;
    return GCC_OK;
}

int gcc_idmap_size(gcc_idmap* m, uint64_t* n) {
    if (!m || !n) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_size: null argument");
    *n = m->orig.size();
    return GCC_OK;
}

int gcc_idmap_map(gcc_idmap* m, const int64_t* ids, uint64_t n, uint32_t* dense_out) {
    if (!m || ((!ids || !dense_out) && n)) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_map: null argument");
    // All or nothing: a batch whose new ids do not all fit leaves the dictionary as it was (a caller that retries or
    // fails the batch must not find dense ids that were never submitted). The slots this call filled are undone in
    // reverse order, which restores the linear-probing table exactly (no entry placed earlier probed past them).
    const uint64_t first_new = m->orig.size();
    std::vector<uint64_t> filled;
    auto undo = [&]() {
        for (auto it = filled.rbegin(); it != filled.rend(); ++it) m->used[*it] = 0;
        m->orig.resize(first_new);
    };
    for (uint64_t i = 0; i < n; ++i) {
        const int64_t k = ids[i];
        uint64_t s = mix64((uint64_t)k) & m->mask;
        while (m->used[s] && m->keys[s] != k) s = (s + 1) & m->mask;
        if (!m->used[s]) {  // first sight: the next dense id
            if (m->orig.size() >= m->capacity) {
                undo();
                return gcc_set_err(GCC_E_INVALID, "gcc_idmap_map: more than %u distinct vertex ids (the batch was not mapped)",
                                   m->capacity);
            }
            try {
                filled.push_back(s);
                m->orig.push_back(k);
            } catch (...) {
                undo();
                return gcc_set_err(GCC_E_OOM, "gcc_idmap_map: out of host memory");
            }
            m->used[s] = 1;
            m->keys[s] = k;
            m->vals[s] = (uint32_t)(m->orig.size() - 1);
        }
        dense_out[i] = m->vals[s];
    }
    return GCC_OK;
}

int gcc_idmap_lookup(gcc_idmap* m, int64_t id, uint32_t* dense) {
    if (!m || !dense) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_lookup: null argument");
    uint64_t s = mix64((uint64_t)id) & m->mask;
    while (m->used[s] && m->keys[s] != id) s = (s + 1) & m->mask;
    *dense = m->used[s] ? m->vals[s] : GCC_UNSEEN;
    return GCC_OK;
}

int gcc_idmap_ids(gcc_idmap* m, int64_t* out, uint64_t n) {
    if (!m || (!out && n)) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_ids: null argument");
    if (n > m->orig.size()) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_ids: %llu > %llu mapped ids",
                                               (unsigned long long)n, (unsigned long long)m->orig.size());
    if (n) std::memcpy(out, m->orig.data(), n * sizeof(int64_t));
    return GCC_OK;
}

int gcc_idmap_canonical(gcc_idmap* m, const uint32_t* dense_labels, uint64_t n, int64_t* out, int64_t unseen) {
    if (!m || ((!dense_labels || !out) && n)) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_canonical: null argument");
    if (n > m->orig.size()) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_canonical: %llu labels for %llu mapped ids",
                                               (unsigned long long)n, (unsigned long long)m->orig.size());
    // minimum original id per component root (roots are dense ids < n; labels of unseen ids are GCC_UNSEEN)
    std::vector<int64_t> best;
    std::vector<uint8_t> has;
    try {
        best.resize(n);
        has.assign(n, 0);
    } catch (...) {
        return gcc_set_err(GCC_E_OOM, "gcc_idmap_canonical: out of host memory");
    }
    for (uint64_t d = 0; d < n; ++d) {
        const uint32_t r = dense_labels[d];
        if (r == GCC_UNSEEN) continue;
        if (r >= n) return gcc_set_err(GCC_E_INVALID, "gcc_idmap_canonical: label %u of id %llu out of range", r,
                                       (unsigned long long)d);
        const int64_t o = m->orig[d];
        if (!has[r] || o < best[r]) {
            best[r] = o;
            has[r] = 1;
        }
    }
    for (uint64_t d = 0; d < n; ++d) {
        const uint32_t r = dense_labels[d];
        out[d] = r == GCC_UNSEEN ? unseen : best[r];
    }
    return GCC_OK;
}

}  // extern "C"
