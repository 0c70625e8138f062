/*
 * gelly_cc.h — C ABI of the MI355X-native streaming connected-components summary.
 *
 * This is the drop-in boundary for gelly-streaming's one data-parallel hot path:
 *   SimpleEdgeStream.aggregate(new ConnectedComponents(mergeWindowTime))
 *   -> SummaryBulkAggregation: fold DisjointSet.union over each edge partition per window,
 *      combine the partial forests with CombineCC (DisjointSet.merge), running summary in Merger.
 * Reference files (relative to the reference repo, `…/` = src/main/java/org/apache/flink/graph/streaming/):
 *   …/summaries/DisjointSet.java        (makeSet :58-61, find :71-85, union :97-123, merge :132-136,
 *                                         getMatches :49-51, toString :139-153)
 *   …/library/ConnectedComponents.java  (UpdateCC.foldEdges :83-86, CombineCC.reduce :116-125)
 *   …/SummaryBulkAggregation.java       (PartialAgg.fold :121-123, timeWindowAll.reduce :81-82)
 *   …/SummaryAggregation.java           (Merger.flatMap :107-119, snapshotState/restoreState :127-135)
 * Each entry point below names the reference method it replaces. A JNI / Panama-FFM binding for the
 * Java side is given in INTEGRATION.md.
 *
 * Conventions
 *  - Vertex ids are u32 in [0, id_capacity); id_capacity <= 0xFFFFFFFF. GCC_UNSEEN (0xFFFFFFFF) marks a
 *    vertex that is not in the summary's key set (DisjointSet.getMatches().containsKey(v) == false).
 *  - Canonical labels: label[v] = min{u : u ~ v} over the edges folded so far, GCC_UNSEEN if unseen.
 *    Partition parity with the reference is defined on these labels (union-by-rank roots are not part
 *    of the contract; DisjointSet.java:113-122 only changes which root is chosen).
 *  - Edge batches are interleaved u32 pairs (src0, dst0, src1, dst1, ...), 8 bytes per edge.
 *  - Every function returns 0 on success or a negative GCC_E* code; gcc_last_error() returns a
 *    thread-local message for the last failure on the calling thread. No C++ exception crosses the ABI.
 *  - Threading: one forest handle is used by one thread at a time (a Flink task thread calls fold /
 *    reduce / flatMap serially on one accumulator); different handles may be used concurrently.
 *  - Each forest owns (or is given, gcc_forest_set_stream) one hipStream_t; all device work of the
 *    handle is ordered on it. Reads that return data to the host synchronise that stream first.
 */
#ifndef GELLY_CC_H
#define GELLY_CC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GCC_UNSEEN 0xFFFFFFFFu

/* error codes */
#define GCC_OK 0
#define GCC_E_INVALID (-1) /* bad argument (null handle, id out of range, size mismatch) */
#define GCC_E_HIP (-2)     /* a HIP runtime call failed */
#define GCC_E_NODEV (-3)   /* no usable gfx950 device */
#define GCC_E_OOM (-4)     /* device or pinned-host allocation failed */
#define GCC_E_INTERNAL (-5) /* a device-side consistency check failed (a bug: the message names the kernel) */

/* ---- generator parameters (synthetic edge streams; see gelly-streaming_amd/csrc/edge_gen.h) ---- */
enum {
    GCC_GEN_EXAMPLE = 1,     /* ConnectedComponentsExample default data (…/example/ConnectedComponentsExample.java:121-133) */
    GCC_GEN_RMAT = 2,        /* R-MAT / Kronecker (0.57, 0.19, 0.19, 0.05) */
    GCC_GEN_GNM = 3,         /* uniform G(n, m) */
    GCC_GEN_ADVERSARIAL = 4, /* shuffled long path + stars */
};

typedef struct gcc_gen_params {
    uint32_t kind;       /* GCC_GEN_* */
    uint32_t scale;      /* RMAT: log2(V); ADVERSARIAL: path bits P */
    uint64_t n_vertices; /* GNM: n */
    uint64_t n_edges;    /* RMAT / GNM: number of edges */
    uint64_t seed;
    uint32_t n_stars;    /* ADVERSARIAL: number of stars S */
    uint32_t star_size;  /* ADVERSARIAL: ids per star L (hub + L-1 leaves) */
    uint32_t permute;    /* RMAT: 1 = seeded vertex permutation */
    uint32_t reserved;
} gcc_gen_params;

typedef struct gcc_forest gcc_forest; /* opaque: one device-resident union-find forest (one DisjointSet) */

/* ---- process / device ---- */
const char* gcc_last_error(void);
int gcc_version(void); /* ABI version, 1 */
int gcc_device_count(int* n);
int gcc_init(int device); /* select + warm up one device (optional; create does it lazily) */

/* ---- generators (no reference counterpart: synthetic inputs for the benchmark configs) ---- */
int gcc_gen_info(const gcc_gen_params* p, uint64_t* n_edges, uint64_t* n_vertices);
int gcc_gen_host(const gcc_gen_params* p, uint64_t first, uint64_t count, uint32_t* out_pairs);
int gcc_gen_device(const gcc_gen_params* p, uint64_t first, uint64_t count, uint32_t* d_out_pairs, void* hip_stream);

/* ---- forest lifetime: `new DisjointSet<>()` (DisjointSet.java:36-39) ---- */
int gcc_forest_create(int device, uint32_t id_capacity, gcc_forest** out);
/* same, over two caller-owned device buffers of id_capacity u32 each (e.g. torch tensors; not freed by
 * destroy). The forest works in one and compress writes the canonical labels into the other, after which they
 * swap roles: gcc_forest_device_ptr tells which one currently holds the forest / labels. Both must be 16-byte
 * aligned (GCC_E_INVALID otherwise). */
int gcc_forest_create_ext(int device, uint32_t id_capacity, uint32_t* d_buf0, uint32_t* d_buf1, gcc_forest** out);
int gcc_forest_destroy(gcc_forest* h);
/* order the handle's work on hip_stream (taken literally: NULL = the null stream, e.g. torch's default
 * stream), or back on the handle's own non-blocking stream if use_own != 0 */
int gcc_forest_set_stream(gcc_forest* h, void* hip_stream, int use_own);
int gcc_forest_get_stream(gcc_forest* h, void** hip_stream);
int gcc_forest_capacity(gcc_forest* h, uint32_t* id_capacity);
int gcc_forest_device(gcc_forest* h, int* device);
/* current forest buffer (= labels after compress); the caller may WRITE through it, so every cached view of the
 * forest is dropped (the next read compresses again) */
int gcc_forest_device_ptr(gcc_forest* h, uint32_t** d_parent);
/* compress (async) and return the canonical labels' device buffer, READ-ONLY (valid until the handle's next
 * mutation): the send side of a cross-GPU label exchange */
int gcc_forest_labels_device(gcc_forest* h, const uint32_t** d_labels);
/* back to the initial value (SummaryAggregation.Merger transientState reset, :113-115; fresh fold value) */
int gcc_forest_reset(gcc_forest* h);

/* ---- fold: UpdateCC.foldEdges -> DisjointSet.union (ConnectedComponents.java:83-86, DisjointSet.java:97-123) ---- */
int gcc_forest_union(gcc_forest* h, uint32_t u, uint32_t v); /* one edge, appended to pinned staging */
int gcc_forest_make_set(gcc_forest* h, uint32_t v);          /* DisjointSet.makeSet (:58-61) = union(v, v) */
int gcc_forest_staging(gcc_forest* h, uint32_t** pairs, uint64_t* cap_edges); /* pinned host staging buffer */
int gcc_forest_submit(gcc_forest* h, uint64_t n_edges);      /* fold the first n_edges of staging (async) */
int gcc_forest_fold_host(gcc_forest* h, const uint32_t* pairs, uint64_t n_edges); /* pageable host pairs */
/* pairs in HBM, async. Ids are validated on the device: an edge with an id >= id_capacity is skipped (never
 * dereferenced) and the next synchronising call on the handle (labels / find / size / sync / ...) returns
 * GCC_E_INVALID once for it; the batch's other edges are folded. */
int gcc_forest_fold_device(gcc_forest* h, const uint32_t* d_pairs, uint64_t n_edges);
/* pairs in PINNED host memory (hipHostMalloc / hipHostRegister / a JNI direct ByteBuffer's registered pages), async:
 * chunked H2D on the handle's copy stream overlapped with the folds, ids validated on the device as above. The
 * buffer must stay valid and unmodified until the next synchronising call (e.g. gcc_forest_sync). */
int gcc_forest_fold_pinned(gcc_forest* h, const uint32_t* pairs, uint64_t n_edges);
int gcc_forest_flush(gcc_forest* h); /* launch any staged single-edge unions */
int gcc_forest_sync(gcc_forest* h);  /* flush + wait for the handle's stream */

/* ---- combine: CombineCC.reduce / DisjointSet.merge (ConnectedComponents.java:116-125, DisjointSet.java:132-136) ---- */
int gcc_forest_merge(gcc_forest* into, gcc_forest* from); /* into := into ∪ from (any two devices) */
/* into := into ∪ {(v, labels[v]) : labels[v] != GCC_UNSEEN}; d_labels: n u32 in HBM of into's device,
 * ordered on into's stream (the receive side of the cross-GPU merge). A label >= id_capacity is skipped (never
 * dereferenced) and reported by the next synchronising call as GCC_E_INVALID, like an id of a device batch */
int gcc_forest_merge_labels_device(gcc_forest* into, const uint32_t* d_labels, uint32_t n);

/* ---- cross-GPU merge message: the partial forest as the RCCL payload (replaces the Kryo-serialised
 * DisjointSet that SummaryBulkAggregation.java:81-83 ships to the one task running timeWindowAll.reduce).
 * Layout (one device buffer, gcc_msg_bytes(id_capacity, cap_others) bytes):
 *   u32 header[4] = { g, n_others, id_capacity, status }   status 0; GCC_MSG_STATUS_FAILED: the sender's merge
 *                                          failed (header only, id_capacity 0: absorbed as nothing; every rank's
 *                                          gcc_forest_group_merge then returns an error)
 *   u64 bits[ceil(id_capacity / 64)]      bit v set <=> label[v] == g   (g = the tracked giant's root)
 *   u32 others[2 * cap_others]            (v, label[v]) for every other seen v (n_others of them, any order)
 * The partition it encodes is exactly the forest's: {(v, g) : bit v} ∪ {(v, label[v]) : others}. */
#define GCC_MSG_HEADER_BYTES 16
#define GCC_MSG_STATUS_FAILED 1u
uint64_t gcc_msg_bytes(uint32_t id_capacity, uint64_t cap_others);
/* compress, then write the message into d_msg (async on h's stream); the header's n_others is the true
 * count even when it exceeds cap_others (then only cap_others entries are written: re-encode larger) */
int gcc_forest_encode(gcc_forest* h, void* d_msg, uint64_t cap_others);
/* h := h ∪ the message's partition (async); cap_others = the layout the message was written with, and its
 * n_others must not exceed it. The sender must have the same id_capacity (else the message is ignored). */
int gcc_forest_absorb(gcc_forest* h, const void* d_msg, uint64_t cap_others);
/* the same for `count` messages at d_msgs + i * stride_bytes (i != skip: this rank's own), in one launch —
 * the receive side of the all_gather; stride_bytes >= gcc_msg_bytes(id_capacity, cap_others), 16-B aligned */
int gcc_forest_absorb_many(gcc_forest* h, const void* d_msgs, uint64_t stride_bytes, uint32_t count, uint32_t skip,
                           uint64_t cap_others);

/* ---- the DELTA merge message (round 6): only what a forest changed since the last merge, shaped like the reference's
 * per-window partials (…/SummaryBulkAggregation.java:80 folds each window into a fresh partial, so the all-window
 * reduce moves only that window's unions, :81-83). After a group merge every rank holds the same partition P; the
 * rank arms its delta (gcc_forest_delta_arm) and its next plain folds list every id whose slot they change (a root
 * hooked, an id seen for the first time). The forest's partition is then P ∪ {(x, root(x)) : x listed}: at most 2
 * pairs per edge folded, 8 B each, instead of the forest. Any other mutation (a filtered / seeded / bucketed fold, a
 * merge, a reset, a device-pointer write) disarms it.
 * Layout (one device buffer, gcc_delta_msg_bytes(cap_pairs) bytes):
 *   u32 header[4] = { edges folded since arming, n_pairs, id_capacity, status }
 *                   status 0; GCC_MSG_STATUS_FAILED (as above); GCC_DELTA_STATUS_UNARMED: the sender's changes were not
 *                   all listed; GCC_DELTA_STATUS_OVERFLOW: its lists overflowed — either way the merge needs the compact
 *                   message. n_pairs is the true count even past cap_pairs (only cap_pairs written: send again larger)
 *   u32 pairs[2 * cap_pairs]            (x, root(x)) */
#define GCC_DELTA_STATUS_UNARMED 2u
#define GCC_DELTA_STATUS_OVERFLOW 3u
uint64_t gcc_delta_msg_bytes(uint64_t cap_pairs);
/* the forest's current partition becomes the base of its delta (after a merge every rank holds the same one) */
int gcc_forest_delta_arm(gcc_forest* h);
int gcc_forest_encode_delta(gcc_forest* h, void* d_msg, uint64_t cap_pairs); /* async on h's stream */
/* h := h ∪ the partition of each of `count` delta messages at d_msgs + i * stride_bytes (i != skip), async; a message
 * whose status is not 0 or whose id_capacity differs is ignored. Leaves the delta disarmed (the caller arms it). */
int gcc_forest_absorb_delta_many(gcc_forest* h, const void* d_msgs, uint64_t stride_bytes, uint32_t count, uint32_t skip,
                                 uint64_t cap_pairs);

/* ---- cross-GPU group merge (gelly_group.cpp): replaces timeWindowAll(t).reduce(CombineCC) + the parallelism-1
 * Merger (…/SummaryBulkAggregation.java:81-83, …/SummaryAggregation.java:107-119). One communicator per GPU over
 * RCCL (xGMI); every rank's forest becomes the union of all ranks' forests — ONE all_gather of the compact messages
 * above (label arrays when no component dominates), each rank absorbing the others itself. RCCL is loaded at run
 * time (dlopen librccl.so.1; a process that already mapped one, e.g. torch's, shares it; the environment variable
 * GELLY_RCCL_LIB names another library with RCCL's ABI instead — the tests' shared-memory stand-in). */
typedef struct gcc_comm gcc_comm;
#define GCC_COMM_ID_BYTES 128 /* = the RCCL unique id */
/* rank 0 creates the id and hands its bytes to every rank over any channel (torch.distributed, the JVM, a file) */
int gcc_comm_unique_id(void* id_out);
int gcc_comm_init(int device, int nranks, int rank, const void* id, gcc_comm** out); /* one process per GPU */
int gcc_comm_init_all(int ndev, const int* devices, gcc_comm** comms_out);           /* one process, ndev GPUs */
int gcc_comm_destroy(gcc_comm* c);
/* nranks, rank, and the bytes each rank contributed to the last merge's all_gather (any may be NULL) */
int gcc_comm_info(gcc_comm* c, int* nranks, int* rank, uint64_t* last_bytes);
/* the last gcc_forest_group_merge: its all_gathers (compact rounds, + 1 for the label exchange), whether it ended with
 * the label exchange, and the speculative list capacity the next merge starts from (any may be NULL) */
int gcc_comm_last_merge(gcc_comm* c, int* rounds, int* labels, uint64_t* cap_others);
/* the last merge's kind (0 compact message, 1 label exchange, 2 delta), the bytes each rank contributed over all of its
 * all_gathers (a failed delta round included) and the delta capacity (pairs) the next merge starts from */
int gcc_comm_last_merge_kind(gcc_comm* c, int* kind, uint64_t* bytes_per_rank, uint64_t* cap_delta);
/* collective over the communicator's ranks (every rank calls it with its forest, same id_capacity); synchronises
 * the forest's stream. Afterwards every rank's forest holds the global partition (compressed, unless the forest's
 * lazy emission defers it: tune key emit_every) and its delta is armed. Round 6: the delta messages first (above), the
 * compact rounds when a rank's delta is unusable or too large (GELLY_GROUP_DELTA=0: compact rounds only). */
int gcc_forest_group_merge(gcc_forest* h, gcc_comm* c);
/* single process: hs[0..n) := their union. Forests on one device need no comms (NULL); forests on several devices
 * need comms[i] = rank i of a gcc_comm_init_all group on hs[i]'s device. Synchronises every forest's stream. */
int gcc_group_merge(gcc_forest** hs, int n, gcc_comm** comms);

/* ---- BipartitenessCheck's summary: Candidates (…/summaries/Candidates.java:27-197) as a signed forest ----
 * BipartitenessCheck(mergeWindowTime) = SummaryBulkAggregation(updateFunction, combineFunction, new Candidates(true),
 * mergeWindowTime, false) (…/library/BipartitenessCheck.java:50-52). Per vertex the canonical word is
 * (min id of its component << 1) | (its sign differs from that vertex's), GCC_UNSEEN if unseen; the success flag
 * turns 0 for good once an edge closes an odd cycle (Candidates.fail, :194-196). Ids < 2^31 - 1. */
typedef struct gcc_signed gcc_signed;
int gcc_signed_create(int device, uint32_t id_capacity, gcc_signed** out); /* new Candidates(true) (:31-34) */
int gcc_signed_destroy(gcc_signed* h);
int gcc_signed_set_stream(gcc_signed* h, void* hip_stream, int use_own);
int gcc_signed_capacity(gcc_signed* h, uint32_t* id_capacity);
int gcc_signed_reset(gcc_signed* h);
/* updateFunction.foldEdges = merge(edgeToCandidate(v1, v2)) per edge (BipartitenessCheck.java:54-61, :93-95) */
int gcc_signed_fold_host(gcc_signed* h, const uint32_t* pairs, uint64_t n_edges);
int gcc_signed_fold_device(gcc_signed* h, const uint32_t* d_pairs, uint64_t n_edges);
/* combineFunction.reduce = Candidates.merge (BipartitenessCheck.java:128-130, Candidates.java:77-139) */
int gcc_signed_merge(gcc_signed* into, gcc_signed* from);
/* the same across processes (combineFunction over a transport; bipartite.merge_group): into ∪= the signed partition
 * held in d_words[0, n) — another forest's words in device memory of into's device, compressed or not (a rank's
 * gcc_signed_words / gcc_signed_device_words, sent); other_failed != 0: that summary had failed, so into fails.
 * Asynchronous on into's stream: d_words must stay valid until that stream has run the merge. */
int gcc_signed_merge_words(gcc_signed* into, const uint32_t* d_words, uint32_t n, int other_failed);
/* the forest's own device words (valid until the next fold / compress / merge on h, which may swap buffers) */
int gcc_signed_device_words(gcc_signed* h, const uint32_t** d_words);
/* speed-only knobs (results identical): "giant" (1/0: the giant-filtered fold for batches of >= 2^22 edges and
 * >= id_capacity / 4), "sample_shift" (its prefix sample = batch >> shift), "min_share" (the voted component's
 * share of sampled edges below which the batch takes the plain fold), "unroll" (1/2/4/8 edges per lane per step of
 * the giant-filtered fold), "xcd" (1/0: that fold over the batch split into 8 parts by source id, one part per XCD)
 * and "xcd_min" (the edges past the sample from which the split is used), "bucket" (1/0: that fold bucketed by the
 * ids' 2^19-id slices, both snapshot lookups in LDS — round 5, the default for id ranges up to 2^27; one host
 * synchronisation per batch, for the vote; it keeps a scratch CC forest (8 B per id) and three lists of 8 B per edge
 * of the largest batch for the handle's lifetime), "bucket_min" (the edges past the sample from which it is used),
 * "bucket_levels" (1, 2 or 3 filter levels before the rest), "bucket_items" (work items per CU of its filter / check
 * kernels; 2). An id >= id_capacity in a bucketed batch is skipped and reported (GCC_E_INVALID) by the next
 * gcc_signed_words / gcc_signed_success. GCC_E_INVALID for an unknown key. */
int gcc_signed_tune(gcc_signed* h, const char* key, double value);
/* the emission on the device: the canonical words replace the forest (asynchronous on the forest's stream; what
 * gcc_signed_words copies out). After a failure the words are unspecified (the emitted value is (false, {})). */
int gcc_signed_compress(gcc_signed* h);
int gcc_signed_words(gcc_signed* h, uint32_t* out, uint32_t n); /* canonical words of ids [0, n) */
int gcc_signed_success(gcc_signed* h, int* success);              /* Candidates.getSuccess (:44-46) */

/* ---- Candidates AS WRITTEN (reference-literal mode; csrc/gelly_literal.hip) ----
 * The signed forest above implements the intended semantics. Candidates.merge itself is not a partition join: it
 * skips components with identical vertex sets (Candidates.java:91-95), drops a failed second-level merge
 * (:128-131) and files the input's vertices under min(inputKey, selfKey) without moving the self component
 * (:176-189). This summary reproduces that output exactly (the state is the TreeMap itself: entries
 * (component key << 32) | (vertex << 1) | sign), for a job that depends on it. Sequential by definition: one
 * wavefront runs each fold / merge in the reference's order. Ids < 2^31 - 1; entry_capacity bounds the entries
 * (a vertex may sit in several components): GCC_E_OOM past it. */
typedef struct gcc_literal gcc_literal;
int gcc_literal_create(int device, uint32_t id_capacity, uint32_t entry_capacity, gcc_literal** out);
int gcc_literal_destroy(gcc_literal* h);
int gcc_literal_reset(gcc_literal* h); /* new Candidates(true) (:31-34) */
/* per edge, in order: this = this.merge(edgeToCandidate(v1, v2)) (BipartitenessCheck.java:54-61, :93-95) */
int gcc_literal_fold_host(gcc_literal* h, const uint32_t* pairs, uint64_t n_edges);
/* into = into.merge(from) (combineFunction.reduce :128-130; the Merger's reduce(window, summary)) */
int gcc_literal_merge(gcc_literal* into, gcc_literal* from);
int gcc_literal_success(gcc_literal* h, int* success); /* Candidates.getSuccess (:44-46) */
/* the TreeMap's entries, (key << 32) | (vertex << 1) | sign, in no particular order; out = NULL: the count only */
int gcc_literal_entries(gcc_literal* h, uint64_t* out, uint64_t cap, uint64_t* n);

/* ---- summary reads (DisjointSet.find :71-85, getMatches :49-51; the emitted summary per window) ---- */
/* async: the emission of everything folded so far (canonical labels); afterwards gcc_forest_device_ptr = labels.
 * Short windows over a big forest (the incremental regime, tune key inc_pipe, round 5) take the PIPELINED emission:
 * the label scan runs on the forest's second stream and the handle's stream does not wait for it, so the next window's
 * fold overlaps it. Every label read of this API (gcc_forest_labels_device / labels / find / size / digest, sync)
 * waits for it; a device pointer kept from before must be fetched again with gcc_forest_labels_device. */
int gcc_forest_compress(gcc_forest* h);
int gcc_forest_labels(gcc_forest* h, uint32_t* out, uint32_t n); /* compress + copy n labels to host */
int gcc_forest_find(gcc_forest* h, uint32_t v, uint32_t* root); /* canonical root; GCC_UNSEEN = Java null */
/* the raw parent array as it stands (no compress): diagnostics and tests of forest invariants */
int gcc_forest_raw_parent(gcc_forest* h, uint32_t* out, uint32_t n);
int gcc_forest_size(gcc_forest* h, uint64_t* n_seen);            /* getMatches().size() */
int gcc_forest_count_components(gcc_forest* h, uint64_t* n_components);
/* restore / deserialize: fold (key, parent) pairs (Merger.restoreState :132-135 + Kryo path) */
int gcc_forest_import_pairs(gcc_forest* h, const uint32_t* pairs, uint64_t n_pairs);

/* ---- serialized summary: the checkpoint / wire form of a DisjointSet (Merger.snapshotState / restoreState,
 * …/SummaryAggregation.java:127-135, and the Kryo bytes a partial is shipped as, …/SummaryBulkAggregation.java:81).
 * Little-endian bytes:
 *   header (GCC_SER_HEADER_BYTES): u32 magic GCC_SER_MAGIC, u32 version 1, u32 id_capacity, u32 kind,
 *                                  u64 n_seen (getMatches().size()), u64 payload bytes
 *   kind 1 (pairs):   n_seen x {u32 v, u32 canonical label}, ascending v
 *   kind 2 (message): the compact merge message above with cap_others = its n_others (a dominant component:
 *                     ~id_capacity/8 bytes instead of 8 per seen id)
 * serialize writes whichever is smaller into a HOST buffer (size from gcc_forest_serialized_size, which
 * synchronises); deserialize folds a summary INTO h (restore = reset + deserialize: the same partition). */
#define GCC_SER_MAGIC 0x53434347u /* "GCCS" */
#define GCC_SER_HEADER_BYTES 32
int gcc_forest_serialized_size(gcc_forest* h, uint64_t* bytes);
int gcc_forest_serialize(gcc_forest* h, void* out, uint64_t size, uint64_t* written);
int gcc_forest_deserialize(gcc_forest* h, const void* in, uint64_t size);

/* parity helper: compress (like gcc_forest_labels) and return, computed on the device, the digest of the canonical
 * label array, sum over every id v of splitmix64((label[v] << 32) | v) mod 2^64 (GCC_UNSEEN labels included: the
 * formula of tests/golden/stream_digests.json), plus #seen and #components (either pointer may be null).
 * Synchronises. */
int gcc_forest_label_digest(gcc_forest* h, uint64_t* digest, uint64_t* n_seen, uint64_t* n_components);

/* ---- measurement: duration of the last fold launch (HIP events on the handle's stream) ---- */
int gcc_forest_enable_timing(gcc_forest* h, int enable); /* 0 off, 1 events, 2 events + slow-edge counts */
int gcc_forest_last_fold_ms(gcc_forest* h, float* ms);
/* measurement only (timing mode): drains the per-phase event log of every fold since the last call, as
 * "phase ms edges" lines; each fold starts with a "begin" line (+ "slow_edges 0 n" lines in mode 2).
 * Recording never synchronises, so a timed region stays sync-free; this call synchronises. */
int gcc_forest_fold_profile(gcc_forest* h, char* buf, uint64_t size);
/* measurement only: one empty kernel (gcc_step_mark_kernel) on hip_stream (NULL = the null stream). bench.py
 * --step-marker launches it once per step, so a rocprofv3 run counts its steps from that kernel's launches
 * (tools/pmc_summary.py) instead of guessing them from a kernel whose launches per step vary. */
int gcc_step_mark(void* hip_stream);
/* diagnostics (tune key inc_check = 1): totals over this forest's checked incremental compresses: how many ran,
 * labels that differed from the roots of the forest the compress started from, bloom words whose LDS copy lacked a
 * mark that memory held. Checked compresses synchronise; never on in a timed region. */
int gcc_forest_inc_check_stats(gcc_forest* h, uint64_t* checks, uint64_t* bad_labels, uint64_t* lost_marks);
/* diagnostics (tune key post_check = 1 or 2): a kernel after every incremental compress (nothing added before or
 * inside it, no synchronisation) checks labels[labels[v]] == labels[v] for every seen v. Returns the checks run and
 * the offenders; `records` (n_records x 8 u32, may be null) receives the first ones: check number, v, label, the
 * label's own label, the true root, whether the label is marked in the compress's bloom (memory-side read), and with
 * post_check 2 the previous compress's labels of v and of the label (UNSEEN otherwise). Synchronises. */
int gcc_forest_post_check_stats(gcc_forest* h, uint64_t* checks, uint64_t* offenders, uint32_t* records,
                                uint32_t n_records);
/* ---- id dictionary: Java Long vertex ids at the boundary (host-only, gelly_idmap.cpp) ----
 * DisjointSet<Long> (…/summaries/DisjointSet.java:30-34) is keyed by any Long; the device forest by dense u32
 * ids. The dictionary assigns dense ids in first-seen order and maps a forest's labels over dense ids back to
 * the reference's canonical form: the minimum ORIGINAL id of the component (signed Long order). */
typedef struct gcc_idmap gcc_idmap;
int gcc_idmap_create(uint32_t capacity, gcc_idmap** out); /* at most `capacity` distinct ids */
int gcc_idmap_destroy(gcc_idmap* m);
int gcc_idmap_size(gcc_idmap* m, uint64_t* n_ids);
/* dense_out[i] = dense id of ids[i] (a new id takes the next one); GCC_E_INVALID past the capacity. All or nothing:
 * on an error the dictionary is left exactly as before the call (no id of the batch is mapped) */
int gcc_idmap_map(gcc_idmap* m, const int64_t* ids, uint64_t n, uint32_t* dense_out);
int gcc_idmap_lookup(gcc_idmap* m, int64_t id, uint32_t* dense); /* GCC_UNSEEN if never mapped */
int gcc_idmap_ids(gcc_idmap* m, int64_t* out, uint64_t n);        /* out[d] = original id of dense id d */
/* out[d] = min original id over d's component, for the first n dense ids; dense_labels = the forest's labels
 * (gcc_forest_labels over the dense range); `unseen` is written for ids the forest has not seen */
int gcc_idmap_canonical(gcc_idmap* m, const uint32_t* dense_labels, uint64_t n, int64_t* out, int64_t unseen);

/* fold-pipeline tuning knobs; results never depend on them, only speed does. Keys: filter, filter_min_batch,
 * filter_min_share, sample_first, sample_growth, sample_div, sample_min, refresh_min_batch, refresh1..refresh3, depth, hook, share_async,
 * drain_at, seed, seed_nt, seed_global, seed_fuse, seed_passes, seed_div, seed_div1, seed_refresh, incremental,
 * inc_min_ids, inc_div, inc_inplace, inc_check, post_check, inc_split, fold_release, experimental, refresh_labels, bucket,
 * bucket_min_batch, bucket_min_ids, bucket_levels, bucket_sample, bucket_sample_sparse, bucket_hub_sample, bucket_p1, bucket_p2_per, bucket_p2_vw,
 * bucket_chunk, scratch_realloc, bucket_windows, bucket_items, bucket_items_p3,
 * bucket_slow2, bucket_defer, bucket_defer_c, compress_split, fold_split, inc_pipe, emit_div, emit_rec, emit_filtered,
 * pin_chunk, lds_edges_per_word. Unknown keys return GCC_E_INVALID.
 * emit_div (round 6): the lazy emission — in the plain regime (no tracked giant) gcc_forest_compress compresses only
 * once the edges folded since the last compress reach id_capacity / emit_div (default 1; 0: every emission compresses);
 * the forest it leaves is the emitted summary (exact for find: every root is its component's minimum id), and every
 * read (labels, find, size, digest, serialize, a merge message) compresses first. emit_rec: the folds between lazy
 * emissions record for an incremental compress (1) or split paths (0). emit_filtered: in the giant-filtered regime the
 * emission refreshes only the tracked component's bitmap (1) or compresses (0). share_async (round 6, default 1): a fresh forest's
 * vote-share check is read back behind an event instead of a host sync, the batch's rest folds plain meanwhile, and a
 * later fold turns the giant filter on once the share has landed (0: wait for it mid-batch). scratch_realloc
 * (diagnostics, tools/placement_probe.py): the next bucketed fold takes freshly allocated scratch lists. One more key is a test hook, not a speed knob: fail_absorb = n makes the n-th next absorb fail with
 * GCC_E_INTERNAL before it launches anything (a rank's failure inside the cross-GPU group merge).
 * One setting is known to give wrong results and is refused (GCC_E_INVALID) unless `experimental` is set to 1 first:
 * inc_split = 1 (path splitting in the recording fold before an in-place incremental compress: round 3's stale label,
 * kept only to reproduce it). */
int gcc_forest_tune(gcc_forest* h, const char* key, double value);

#ifdef __cplusplus
}
#endif

#endif /* GELLY_CC_H */
