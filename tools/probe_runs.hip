// probe_runs.hip — experiment: what P1's WRITE PATTERN costs, without its LDS sort. P1 reads
// 8 B per edge and writes every 16K-edge tile as 128 runs of 128 entries, one per bucket, each run into the block's
// current 1K-entry chunk of that bucket. Here each block streams its tiles like P1 (16-B loads, the next tile in
// flight) and writes synthetic entries in that run pattern, in three layouts:
//   SPLIT   — P1's: lo (u32) and hi (u16) in two arrays (a 16-B and an 8-B store per 4 entries)
//   CHUNKED — lo and hi of one chunk side by side (a chunk = 4 KiB of lo then 2 KiB of hi): the same stores, but
//             a run's two writes land 4 KiB apart instead of in two distant arrays
//   U64     — 8-B entries (round 2's layout): two 16-B stores per 4 entries, one stream
//   SPLIT_DYN — SPLIT with a write-out loop whose trip count is a kernel argument (as P1's is a run-time count):
//             the compiler cannot count the stores after the next tile's loads, so the loop top waits vmcnt(0) —
//             for every store of the write-out to COMPLETE, not only for the loads
// and, for reference, the same bytes written contiguously (CONTIG: probe_copy's read 8 + write 6 mix).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_runs.hip -o tools/probe_runs
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32;
typedef uint64_t u64;
typedef uint16_t u16;
typedef u32 u4 __attribute__((ext_vector_type(4)));
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int kBlock = 1024;
constexpr int kPer = 16;                      // edges per thread per tile
constexpr u32 kTile = kBlock * kPer;          // 16K edges
constexpr u32 kBuckets = 128;
constexpr u32 kRun = kTile / kBuckets;        // 128 entries per (tile, bucket)
constexpr u32 kChunk = 1024;                  // entries
constexpr u32 kRunsPerChunk = kChunk / kRun;  // 8

enum { SPLIT = 0, CHUNKED = 1, U64 = 2, CONTIG = 3, SPLIT_DYN = 4 };

// entry position (within its bucket) of entry e of the run of bucket s in tile number `it` of block b
__device__ __forceinline__ u64 run_pos(u32 b, u32 nblocks, u32 it, u32 e) {
    const u64 chunk_id = (u64)(it / kRunsPerChunk) * nblocks + b;  // chunks of the blocks interleave
    return chunk_id * kChunk + (u64)(it % kRunsPerChunk) * kRun + e;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_runs(const u4* __restrict__ in, u64 ntiles, u64 bucket_entries,
                                                 u32* __restrict__ lo, u16* __restrict__ hi, u64* __restrict__ out64,
                                                 unsigned char* __restrict__ chunked, u32* sink, u32 nwo) {
    constexpr int kQ = kPer / 2;
    u4 q[kQ];
    u32 acc = 0;
    u32 it = 0;
    auto load = [&](u64 t) {
#pragma unroll
        for (int k = 0; k < kQ; ++k) q[k] = __builtin_nontemporal_load(in + t * (kTile / 2) + (u64)k * kBlock + threadIdx.x);
    };
    u64 t = blockIdx.x;
    if (t < ntiles) load(t);
    for (; t < ntiles; t += gridDim.x, ++it) {
        u32 v[kQ * 4];
#pragma unroll
        for (int k = 0; k < kQ; ++k) {
            v[4 * k] = q[k].x;
            v[4 * k + 1] = q[k].y;
            v[4 * k + 2] = q[k].z;
            v[4 * k + 3] = q[k].w;
        }
        if (t + gridDim.x < ntiles) load(t + gridDim.x);
        // the write-out: 4 entries per lane-step, 4096 steps per tile (the sorted tile's order: bucket-major)
#pragma unroll
        for (int r = 0; r < (MODE == SPLIT_DYN ? 1 : kPer / 4); ++r) {
          for (u32 r2 = 0; r2 < (MODE == SPLIT_DYN ? nwo : 1); ++r2) {
            const u32 rr = MODE == SPLIT_DYN ? r2 : (u32)r;
            const u32 xw = rr * kBlock + threadIdx.x;  // 4-entry group of the tile
            const u32 s = xw / (kRun / 4), e = (xw % (kRun / 4)) * 4;
            // (SPLIT_DYN: v[0..3] with rr mixed in — a run-time index into v[] would move it to scratch)
            const u32 a = (MODE == SPLIT_DYN ? v[0] ^ rr : v[(4 * rr) & 15]) ^ it;
            const u32 c = MODE == SPLIT_DYN ? v[1] + v[5] + v[9] + v[13] : v[(4 * rr + 1) & 15];
            const u32 d = MODE == SPLIT_DYN ? v[2] + v[6] + v[10] + v[14] : v[(4 * rr + 2) & 15];
            const u32 f = MODE == SPLIT_DYN ? v[3] + v[7] + v[11] + v[15] + v[4] + v[8] + v[12] : v[(4 * rr + 3) & 15];
            if constexpr (MODE == CONTIG) {
                const u64 p = t * kTile + 4ull * xw;
                *reinterpret_cast<u4*>(lo + p) = u4{a, c, d, f};
                *reinterpret_cast<u16x4*>(hi + p) = u16x4{(u16)a, (u16)c, (u16)d, (u16)f};
            } else {
                const u64 p = (u64)s * bucket_entries + run_pos(blockIdx.x, gridDim.x, it, e);
                if constexpr (MODE == SPLIT || MODE == SPLIT_DYN) {
                    *reinterpret_cast<u4*>(lo + p) = u4{a, c, d, f};
                    *reinterpret_cast<u16x4*>(hi + p) = u16x4{(u16)a, (u16)c, (u16)d, (u16)f};
                } else if constexpr (MODE == CHUNKED) {
                    unsigned char* region = chunked + (p / kChunk) * (6ull * kChunk);
                    const u32 o = (u32)(p % kChunk);
                    *reinterpret_cast<u4*>(region + 4 * o) = u4{a, c, d, f};
                    *reinterpret_cast<u16x4*>(region + 4 * kChunk + 2 * o) = u16x4{(u16)a, (u16)c, (u16)d, (u16)f};
                } else {
                    typedef u64 u64x2 __attribute__((ext_vector_type(2)));
                    *reinterpret_cast<u64x2*>(out64 + p) = u64x2{(u64)a << 32 | c, (u64)d << 32 | f};
                    *reinterpret_cast<u64x2*>(out64 + p + 2) = u64x2{(u64)c << 32 | a, (u64)f << 32 | d};
                }
            }
            acc += a;
          }
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    const u64 n = 1ull << 30;  // edges (C4)
    const u64 ntiles = n / kTile;
    const u32 grid = 256;
    // per bucket: every block's chunks; ntiles / grid tiles per block, one run per bucket per tile
    const u64 tiles_per_block = (ntiles + grid - 1) / grid;
    const u64 chunks_per_block = (tiles_per_block + kRunsPerChunk - 1) / kRunsPerChunk;
    const u64 bucket_entries = chunks_per_block * grid * kChunk;
    const u64 storage = bucket_entries * kBuckets;  // entries
    printf("probe_runs: %llu edges, tiles of %u, %u buckets, runs of %u, chunks of %u; storage %llu entries\n",
           (unsigned long long)n, kTile, kBuckets, kRun, kChunk, (unsigned long long)storage);
    u4* in;
    u32* lo;
    u16* hi;
    u64* out64;
    unsigned char* chunked;
    u32* sink;
    CK(hipMalloc(&in, n * 8));
    CK(hipMemset(in, 3, n * 8));
    CK(hipMalloc(&sink, grid * sizeof(u32)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[5] = {"SPLIT (P1's)", "CHUNKED", "U64 (8-B entries)", "CONTIG (read 8 + write 6)",
                            "SPLIT_DYN (run-time store count)"};
    const double wbytes[5] = {6, 6, 8, 6, 6};
    for (int mode = 0; mode < 5; ++mode) {
        // allocate per mode (8 GiB of edges + at most 8 GiB of output)
        lo = nullptr; hi = nullptr; out64 = nullptr; chunked = nullptr;
        if (mode == SPLIT || mode == CONTIG || mode == SPLIT_DYN) {
            CK(hipMalloc(&lo, storage * 4));
            CK(hipMalloc(&hi, storage * 2));
        } else if (mode == CHUNKED) {
            CK(hipMalloc(&chunked, storage * 6));
        } else {
            CK(hipMalloc(&out64, storage * 8));
        }
        float best = 1e9f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            if (mode == SPLIT) hipLaunchKernelGGL(k_runs<SPLIT>, dim3(grid), dim3(kBlock), 0, 0, in, ntiles, bucket_entries, lo, hi, out64, chunked, sink, 4u);
            if (mode == CHUNKED) hipLaunchKernelGGL(k_runs<CHUNKED>, dim3(grid), dim3(kBlock), 0, 0, in, ntiles, bucket_entries, lo, hi, out64, chunked, sink, 4u);
            if (mode == U64) hipLaunchKernelGGL(k_runs<U64>, dim3(grid), dim3(kBlock), 0, 0, in, ntiles, bucket_entries, lo, hi, out64, chunked, sink, 4u);
            if (mode == CONTIG) hipLaunchKernelGGL(k_runs<CONTIG>, dim3(grid), dim3(kBlock), 0, 0, in, ntiles, bucket_entries, lo, hi, out64, chunked, sink, 4u);
            if (mode == SPLIT_DYN) hipLaunchKernelGGL(k_runs<SPLIT_DYN>, dim3(grid), dim3(kBlock), 0, 0, in, ntiles, bucket_entries, lo, hi, out64, chunked, sink, 4u);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        printf("%-28s %.3f ms  %.0f GB/s (read 8 + write %.0f B/edge)\n", names[mode], best,
               (8.0 + wbytes[mode]) * n / best / 1e6, wbytes[mode]);
        fflush(stdout);
        if (lo) CK(hipFree(lo));
        if (hi) CK(hipFree(hi));
        if (chunked) CK(hipFree(chunked));
        if (out64) CK(hipFree(out64));
    }
    return 0;
}
