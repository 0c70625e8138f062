// signed_bucket_api.h — internal (not part of the C ABI): the bucketed signed fold, implemented in gelly_cc.hip next
// to the CC forest's bucketed fold whose P1 it reuses (kernels: signed_bucket.h), called by gelly_bip.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

struct gcc_forest;

struct GccSignedBucketArgs {
    hipStream_t stream;
    uint32_t* word;         // the signed forest
    uint32_t* out;          // the closing compress's output (the caller swaps it in)
    uint32_t* gbits;        // the snapshot: 2 bits per id (member, parity to r), grown by the fold
    uint32_t* n2;           // scratch: 2 bits per id (reached with parity 0 / 1), zero before and after
    const uint32_t* vote;   // vote[0] = r, C's root at the snapshot
    uint32_t* fail;         // the forest's fail word
    const uint64_t* edges;  // the batch (u64 pairs, 16-B aligned)
    uint64_t n;
    uint32_t cap;
    uint64_t* emit;         // scratch lists of at least n entries each
    uint64_t* slow0;
    uint64_t* slow1;
    uint32_t* ctr;          // scratch: 8 device words
    uint32_t* hist;         // scratch: 6 x 512 device words (per level, the emit and slow lists' per-slice counts)
    int levels;             // filter levels (1 to 3) before the rest
    int items_per_cu;       // work items (slice parts) of the filter and check kernels per CU
    int want_counts;        // 1: fill counts (synchronises)
    uint64_t counts[6];     // out: emitted and slow entries of levels 1-3 (diagnostics)
};

// gcc status; `scratch` = a CC forest of the same id range, used for its bucket storage only (gcc_forest_create).
// Runs on a->stream; the scratch forest's own stream is restored before it returns.
int gcc_internal_signed_bucket(gcc_forest* scratch, GccSignedBucketArgs* a);
// The device error word the bucketed fold's kernels set (an id >= id_capacity skipped, or an internal list entry out
// of range), read on `stream` (synchronises it) and cleared: GCC_OK, or the error the signed handle reports.
int gcc_internal_take_err(gcc_forest* scratch, hipStream_t stream);
