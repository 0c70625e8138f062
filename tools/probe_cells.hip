// probe_cells.hip — the ceiling of a candidate C4 layout (not product code; VERDICT r5 next-2, DESIGN.md §4 "traffic
// floor per layout"): after ONE bucketing pass into 64 cells by (source's eighth of the ids, target's eighth), a second
// pass could test BOTH ends of every edge against the tracked component's 8 MiB bitmap with every lookup served by the
// XCD's own 4 MiB L2 — XCD x streams the cells (x, 0..7) in order, so its working set is two 1 MiB eighths of the
// bitmap. This probe measures that second pass's rate against (a) the bare stream and (b) the same lookups over the
// edges in stream order (both ends random over the whole 8 MiB bitmap: the round-2 measurement, 63.5 G edges/s), on
// 2^30 uniformly random edges over 2^26 ids (uniform: the worst case for the caches; kron hubs only help).
//   k_stream       8 B per edge, no lookups
//   k_random       8 B per edge, two lookups per edge in the global bitmap, stream order
//   k_cells        8 B per edge, two lookups per edge, the edges in cell order, block b on XCD b % 8 takes its XCD's
//                  cells (x, y), y = 0..7, each in a slice of the blocks of that XCD
// Build: hipcc -O3 --offload-arch=gfx950 probe_cells.hip -o probe_cells
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

constexpr u32 kIdBits = 26;
constexpr u64 kEdges = 1ull << 30;
constexpr u32 kCells = 64;

__device__ __forceinline__ u64 mix(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// edges of cell c = (x, y): u in eighth x, v in eighth y; cell c holds edges [c * per, (c + 1) * per) — the bucketing
// pass's output, generated directly in that order
__global__ void k_gen(uint2* e, u64 n, int cells) {
    const u64 per = n / kCells;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        const u64 h = mix(i);
        u32 u = (u32)h & ((1u << kIdBits) - 1), v = (u32)(h >> 32) & ((1u << kIdBits) - 1);
        if (cells) {
            const u32 c = (u32)(i / per);
            u = (u & ((1u << (kIdBits - 3)) - 1)) | ((c >> 3) << (kIdBits - 3));
            v = (v & ((1u << (kIdBits - 3)) - 1)) | ((c & 7) << (kIdBits - 3));
        }
        e[i] = make_uint2(u, v);
    }
}

__device__ __forceinline__ u32 bit(const u32* bm, u32 x) { return (bm[x >> 5] >> (x & 31)) & 1u; }

template <bool LOOKUP>
__global__ __launch_bounds__(256) void k_stream(const u4* __restrict__ e, u64 n2, const u32* __restrict__ bm, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n2; i += (u64)gridDim.x * 256) {
        const u4 a = __builtin_nontemporal_load(e + i);  // two edges
        if (LOOKUP) acc += (bit(bm, a.x) & bit(bm, a.y)) + (bit(bm, a.z) & bit(bm, a.w));
        else acc += a.x ^ a.w;
    }
    if (acc == 0x12345u) sink[0] = acc;
}

// block b: XCD x = b % 8 (the hardware's round-robin of workgroups over XCDs), k = b / 8 its index among x's blocks
__global__ __launch_bounds__(256) void k_cells(const u4* __restrict__ e, u64 n2, const u32* __restrict__ bm, u32* sink) {
    const u32 x = blockIdx.x & 7, k = blockIdx.x >> 3, nk = gridDim.x >> 3;
    const u64 per2 = n2 / kCells;  // 16-B pairs per cell
    u32 acc = 0;
    for (u32 y = 0; y < 8; ++y) {
        const u4* c = e + (u64)(x * 8 + y) * per2;
        for (u64 i = (u64)k * 256 + threadIdx.x; i < per2; i += (u64)nk * 256) {
            const u4 a = __builtin_nontemporal_load(c + i);
            acc += (bit(bm, a.x) & bit(bm, a.y)) + (bit(bm, a.z) & bit(bm, a.w));
        }
    }
    if (acc == 0x12345u) sink[0] = acc;
}

int main() {
    uint2 *e_rand, *e_cells;
    u32 *bm, *sink;
    CK(hipMalloc(&e_rand, kEdges * 8));
    CK(hipMalloc(&e_cells, kEdges * 8));
    CK(hipMalloc(&bm, (1u << kIdBits) / 8));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(bm, 0x5A, (1u << kIdBits) / 8));
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, e_rand, kEdges, 0);
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, 0, e_cells, kEdges, 1);
    CK(hipDeviceSynchronize());
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    const u64 n2 = kEdges / 2;
    for (unsigned grid : {2048u, 4096u, 8192u}) {
        float best[3] = {1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 4; ++rep)
            for (int k = 0; k < 3; ++k) {
                CK(hipEventRecord(t0));
                if (k == 0) hipLaunchKernelGGL(k_stream<false>, dim3(grid), dim3(256), 0, 0, (const u4*)e_rand, n2, bm, sink);
                if (k == 1) hipLaunchKernelGGL(k_stream<true>, dim3(grid), dim3(256), 0, 0, (const u4*)e_rand, n2, bm, sink);
                if (k == 2) hipLaunchKernelGGL(k_cells, dim3(grid), dim3(256), 0, 0, (const u4*)e_cells, n2, bm, sink);
                CK(hipGetLastError());
                CK(hipEventRecord(t1));
                CK(hipEventSynchronize(t1));
                float ms;
                CK(hipEventElapsedTime(&ms, t0, t1));
                if (ms < best[k]) best[k] = ms;
            }
        printf("grid %5u  stream %.3f ms (%.0f G edges/s, %.2f TB/s)  random lookups %.3f ms (%.0f G edges/s)  "
               "cell-ordered lookups %.3f ms (%.0f G edges/s, %.2f TB/s)\n",
               grid, best[0], kEdges / best[0] / 1e6, 8.0 * kEdges / best[0] / 1e9, best[1], kEdges / best[1] / 1e6,
               best[2], kEdges / best[2] / 1e6, 8.0 * kEdges / best[2] / 1e9);
    }
    return 0;
}
