// probe_mall.hip — experiment (DESIGN.md §8, next steps for C4): does data one kernel writes stay in the 256 MiB
// Infinity Cache (MALL) for the next kernel to read? If it does, the bucketed fold could run C4 in chunks whose
// buckets (6 B per edge) never reach HBM: P1 writes a chunk's buckets into a reused buffer, P2 reads them back.
// Per buffer size S: k_write stores S bytes (16-B stores), then k_read reads them back (16-B loads, reduced); times
// from events; optionally a k_stream of T bytes of unrelated non-temporal loads between write and read (the edges P1
// streams meanwhile). Reported: write and read rates in TB/s (HBM streaming ceiling ~6.3 TB/s).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mall.hip -o tools/probe_mall
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int kBlock = 256;
constexpr int kGrid = 2048;

__global__ void k_write(u4* buf, u64 n, u32 v) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        const u4 q = {v, (u32)i, v ^ 1u, (u32)(i >> 7)};
        buf[i] = q;
    }
}

__global__ void k_read(const u4* buf, u64 n, u32* sink) {
    u32 acc = 0;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        const u4 q = buf[i];
        acc += q.x ^ q.y ^ q.z ^ q.w;
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

__global__ void k_stream(const u4* src, u64 n, u32* sink) {
    u32 acc = 0;
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) {
        const u4 q = __builtin_nontemporal_load(src + i);
        acc += q.x ^ q.w;
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const u64 sizes_mb[] = {64, 128, 192, 256, 384, 2048};
    u4* buf;
    const u64 maxb = 2048ull << 20;
    CK(hipMalloc(&buf, maxb));
    u4* other;
    const u64 other_b = 1024ull << 20;
    CK(hipMalloc(&other, other_b));
    CK(hipMemset(other, 1, other_b));
    u32* sink;
    CK(hipMalloc(&sink, kGrid * sizeof(u32)));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    printf("probe_mall: write S bytes, then read them back (16-B accesses, %d x %d threads), best of %d\n", kGrid, kBlock,
           iters);
    for (int withstream = 0; withstream < 2; ++withstream) {
        for (u64 mb : sizes_mb) {
            const u64 n = (mb << 20) / 16;
            // as many unrelated streamed bytes as the buffer, at most the `other` allocation (round 4: the 2 GiB case read
            // past the 1 GiB buffer and faulted the GPU; the figures before it were recorded)
            const u64 ns = withstream ? std::min<u64>((mb << 20) / 16, other_b / 16) : 0;
            float best_w = 1e9f, best_r = 1e9f;
            for (int it = 0; it < iters; ++it) {
                hipLaunchKernelGGL(k_stream, dim3(kGrid), dim3(kBlock), 0, 0, (const u4*)other, other_b / 16, sink);  // cold start
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(k_write, dim3(kGrid), dim3(kBlock), 0, 0, buf, n, (u32)it);
                CK(hipEventRecord(e1, 0));
                if (ns) hipLaunchKernelGGL(k_stream, dim3(kGrid), dim3(kBlock), 0, 0, (const u4*)other, ns, sink);
                hipEvent_t er;
                CK(hipEventCreate(&er));
                CK(hipEventRecord(er, 0));
                hipLaunchKernelGGL(k_read, dim3(kGrid), dim3(kBlock), 0, 0, (const u4*)buf, n, sink);
                CK(hipEventRecord(e2, 0));
                CK(hipEventSynchronize(e2));
                float tw, tr;
                CK(hipEventElapsedTime(&tw, e0, e1));
                CK(hipEventElapsedTime(&tr, er, e2));
                CK(hipEventDestroy(er));
                if (tw < best_w) best_w = tw;
                if (tr < best_r) best_r = tr;
            }
            const double by = (double)(mb << 20);
            printf("%5llu MiB%s: write %.2f TB/s (%.3f ms), read back %.2f TB/s (%.3f ms)\n", (unsigned long long)mb,
                   withstream ? " + as many NT-streamed bytes between" : "", by / best_w / 1e9, best_w,
                   by / best_r / 1e9, best_r);
            fflush(stdout);
        }
    }
    return 0;
}
