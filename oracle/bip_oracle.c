/*
 * bip_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of gelly-streaming's BipartitenessCheck summary (`…/` = src/main/java/org/apache/flink/graph/
 * streaming/): Candidates (…/summaries/Candidates.java:27-197) folded by updateFunction / combined by
 * combineFunction (…/library/BipartitenessCheck.java:54-61, :93-95, :128-130) over the SummaryBulkAggregation
 * window topology (…/SummaryBulkAggregation.java:76-83, Merger …/SummaryAggregation.java:107-119).
 *
 * What a Candidates value means, and what is restated:
 *   components        Candidates.f1: component -> {vertex -> sign}. Candidates.merge joins the components that
 *                     share a vertex and reverses the input side's signs to match (:84-135, :142-192). That is
 *                     a union-find with a parity per vertex: sign(v) XOR sign(u) = 1 for every edge (u, v)
 *                     (edgeToCandidate puts min(v1,v2) on + and max on -, :54-61). bo_t keeps, per vertex,
 *                     (parent, parity to parent) in an open-addressing table; bo_union applies one constraint.
 *   success           Candidates.f0: false for good once a constraint contradicts the component's signs, i.e.
 *                     an odd cycle (:65-69 add -> false, :118-121 merge -> fail()); fail() empties the map (:194-196).
 *   self loops        edgeToCandidate(v, v) adds (v,+) then (v,-) to one component and ignores add()'s false
 *                     (:58-59): the vertex is added, success unchanged. Restated as makeSet only.
 *   canonical output  (not in the reference: its signs depend on which side a merge reversed) per vertex:
 *                     (min vertex of its component << 1) | (sign differs from the minimum's), UNSEEN if absent.
 *                     tests/golden/make_golden_bip.py pins this against a literal Python restatement of
 *                     Candidates.merge and the reference's BipartitenessCheckTest / NonBipartitnessCheckTest.
 *   one deviation     Candidates.merge drops the fail() of a second-level merge (:128-131 call fail() without
 *                     returning it); a conflict there is reported here (and on the GPU) as a failure.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BO_UNSEEN 0xFFFFFFFFu
#define BO_EMPTY 0xFFFFFFFFFFFFFFFFull

typedef struct {
    uint64_t* keys;
    uint64_t* parent;
    uint8_t* par; /* parity to parent */
    uint64_t cap, size;
    int fail;
} bo_t;

static inline uint64_t bo_mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

static int bo_alloc(bo_t* d, uint64_t cap) {
    d->keys = (uint64_t*)malloc(cap * sizeof(uint64_t));
    d->parent = (uint64_t*)malloc(cap * sizeof(uint64_t));
    d->par = (uint8_t*)malloc(cap);
    if (!d->keys || !d->parent || !d->par) return -1;
    memset(d->keys, 0xFF, cap * sizeof(uint64_t));
    d->cap = cap;
    d->size = 0;
    return 0;
}

bo_t* bo_new(void) {
    bo_t* d = (bo_t*)calloc(1, sizeof(bo_t));
    if (!d || bo_alloc(d, 64)) abort();
    return d;
}

void bo_free(bo_t* d) {
    if (!d) return;
    free(d->keys);
    free(d->parent);
    free(d->par);
    free(d);
}

static inline uint64_t bo_slot(const bo_t* d, uint64_t key) {
    uint64_t m = d->cap - 1, i = bo_mix(key) & m;
    while (d->keys[i] != BO_EMPTY && d->keys[i] != key) i = (i + 1) & m;
    return i;
}

static void bo_grow(bo_t* d) {
    bo_t n;
    if (bo_alloc(&n, d->cap * 2)) abort();
    for (uint64_t i = 0; i < d->cap; ++i) {
        if (d->keys[i] == BO_EMPTY) continue;
        uint64_t j = bo_slot(&n, d->keys[i]);
        n.keys[j] = d->keys[i];
        n.parent[j] = d->parent[i];
        n.par[j] = d->par[i];
    }
    n.size = d->size;
    n.fail = d->fail;
    free(d->keys);
    free(d->parent);
    free(d->par);
    *d = n;
}

/* add v as its own component with sign + if absent; returns its slot */
static uint64_t bo_make(bo_t* d, uint64_t v) {
    if (2 * (d->size + 1) > d->cap) bo_grow(d);
    uint64_t i = bo_slot(d, v);
    if (d->keys[i] == BO_EMPTY) {
        d->keys[i] = v;
        d->parent[i] = v;
        d->par[i] = 0;
        d->size++;
    }
    return i;
}

/* root of the key in slot i and the parity of that key to it (iterative, full path compression) */
static uint64_t bo_find(bo_t* d, uint64_t i, int* parity) {
    uint64_t r = i;
    int p = 0;
    while (d->parent[r] != d->keys[r]) {
        p ^= d->par[r];
        r = bo_slot(d, d->parent[r]);
    }
    /* compress: every node on the path points at the root with its own parity to it */
    int q = p;
    uint64_t x = i;
    while (d->parent[x] != d->keys[x]) {
        uint64_t nx = bo_slot(d, d->parent[x]);
        int px = d->par[x];
        d->parent[x] = d->keys[r];
        d->par[x] = (uint8_t)q;
        q ^= px;
        x = nx;
    }
    *parity = p;
    return r;
}

/* constraint sign(u) XOR sign(v) == q; a contradiction inside one component is an odd cycle */
void bo_union(bo_t* d, uint64_t u, uint64_t v, int q) {
    bo_make(d, u);
    if (u == v) return; /* self loop: the vertex only (edgeToCandidate :58-59) */
    bo_make(d, v);
    int pu, pv;
    uint64_t ru = bo_find(d, bo_slot(d, u), &pu), rv = bo_find(d, bo_slot(d, v), &pv);
    if (ru == rv) {
        if ((pu ^ pv) != q) d->fail = 1;
        return;
    }
    /* hang the root with the larger key under the smaller (any choice gives the same canonical output) */
    uint64_t lo = d->keys[ru] < d->keys[rv] ? ru : rv, hi = lo == ru ? rv : ru;
    d->parent[hi] = d->keys[lo];
    d->par[hi] = (uint8_t)(pu ^ pv ^ q);
}

/* Candidates.merge (:77-139): every vertex of `other` with its parity to its root joins this summary */
void bo_merge(bo_t* d, bo_t* other) {
    if (other->fail) d->fail = 1; /* :78-81 */
    for (uint64_t i = 0; i < other->cap; ++i) {
        if (other->keys[i] == BO_EMPTY) continue;
        int p;
        uint64_t r = bo_find(other, i, &p);
        bo_union(d, other->keys[i], other->keys[r], p);
    }
}

int bo_success(const bo_t* d) { return !d->fail; }
uint64_t bo_size(const bo_t* d) { return d->size; }

/* canonical words over ids [0, V); -1 if a key is >= V */
int bo_words(bo_t* d, uint32_t V, uint32_t* out) {
    for (uint64_t v = 0; v < V; ++v) out[v] = BO_UNSEEN;
    uint32_t* minv = (uint32_t*)malloc((size_t)V * sizeof(uint32_t));
    uint8_t* minpar = (uint8_t*)malloc((size_t)V);
    if (!minv || !minpar) abort();
    for (uint64_t v = 0; v < V; ++v) minv[v] = BO_UNSEEN;
    int rc = 0;
    for (uint64_t i = 0; i < d->cap; ++i) { /* per root: its minimum key and that key's parity to the root */
        uint64_t k = d->keys[i];
        if (k == BO_EMPTY) continue;
        if (k >= V) {
            rc = -1;
            continue;
        }
        int p;
        uint64_t r = d->keys[bo_find(d, i, &p)];
        if (r >= V) {
            rc = -1;
            continue;
        }
        if (k < minv[r]) {
            minv[r] = (uint32_t)k;
            minpar[r] = (uint8_t)p;
        }
    }
    for (uint64_t i = 0; i < d->cap; ++i) {
        uint64_t k = d->keys[i];
        if (k == BO_EMPTY || k >= V) continue;
        int p;
        uint64_t r = d->keys[bo_find(d, i, &p)];
        if (r < V) out[k] = (minv[r] << 1) | (uint32_t)(p ^ minpar[r]);
    }
    free(minv);
    free(minpar);
    return rc;
}

/*
 * The BipartitenessCheck summary over an edge stream: per window, each of n_partitions contiguous chunks is folded
 * into a fresh Candidates (updateFunction), the partials are combined in partition order (combineFunction), and the
 * Merger folds the window into the running summary (transientState = false). Outputs per window (NULL = skip):
 * emitted[w], success[w], words[w*V .. w*V+V). Returns 0, or -1 if an id is >= V.
 */
int bo_stream(const uint32_t* pairs, const uint64_t* window_starts, uint32_t n_windows, uint32_t n_partitions,
              uint32_t V, uint8_t* emitted, uint8_t* success, uint32_t* words) {
    if (n_partitions < 1) n_partitions = 1;
    bo_t* summary = bo_new();
    int rc = 0;
    for (uint32_t w = 0; w < n_windows; ++w) {
        const uint64_t b = window_starts[w], e = window_starts[w + 1];
        if (emitted) emitted[w] = e > b;
        if (e > b) {
            bo_t* acc = NULL;
            const uint64_t len = e - b;
            for (uint32_t p = 0; p < n_partitions; ++p) {
                const uint64_t pb = b + len * p / n_partitions, pe = b + len * (p + 1) / n_partitions;
                if (pe == pb) continue;
                bo_t* part = bo_new();
                for (uint64_t i = pb; i < pe; ++i) bo_union(part, pairs[2 * i], pairs[2 * i + 1], 1);
                if (!acc) {
                    acc = part;
                } else {
                    bo_merge(acc, part);
                    bo_free(part);
                }
            }
            bo_merge(acc, summary); /* Merger: summary = combine.reduce(window, summary) */
            bo_free(summary);
            summary = acc;
        }
        if (success) success[w] = (uint8_t)bo_success(summary);
        if (words && bo_words(summary, V, words + (uint64_t)w * V)) rc = -1;
    }
    bo_free(summary);
    return rc;
}
