// probe_copy.hip — the mixed read/write streaming ceiling of P1's byte mix (not product code): read 8 B per edge,
// write 4 B + 2 B per edge into two contiguous arrays (P1's 6-byte bucket entries without the multi-split), and the
// pure read and pure write ceilings for comparison. 2^30 edges, 16-B loads, 16-B + 8-B stores.
// Build: hipcc -O3 --offload-arch=gfx950 probe_copy.hip -o probe_copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16;
typedef u16 u16x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// each lane: 4 edges per step (two 16-B loads) -> one 16-B store of lo + one 8-B store of hi
template <int MODE>
__global__ __launch_bounds__(1024) void k(const u4* __restrict__ in, u64 n4, u4* __restrict__ lo, u16x4* __restrict__ hi,
                                          u32* sink) {
    u32 acc = 0;
    const u64 stride = (u64)gridDim.x * 1024;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < n4; i += stride) {
        u4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
        if (MODE != 2) {
            a = __builtin_nontemporal_load(in + 2 * i);
            b = __builtin_nontemporal_load(in + 2 * i + 1);
        }
        if (MODE == 1) {
            acc += a.x ^ a.y ^ b.z ^ b.w;
            continue;
        }
        const u4 l = {a.y ^ (a.x << 27), a.w ^ (a.z << 27), b.y ^ (b.x << 27), b.w ^ (b.z << 27)};
        const u16x4 h = {(u16)(a.x >> 5), (u16)(a.z >> 5), (u16)(b.x >> 5), (u16)(b.z >> 5)};
        lo[i] = MODE == 2 ? u4{(u32)i, 1, 2, 3} : l;
        hi[i] = MODE == 2 ? u16x4{(u16)i, 1, 2, 3} : h;
    }
    if (acc == 0x12345u) sink[0] = acc;
}

int main() {
    const u64 n = 1ull << 30, n4 = n / 4;
    u4 *in, *lo;
    u16x4* hi;
    u32* sink;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&lo, n * 4));
    CK(hipMalloc(&hi, n * 2));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 1, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"read 8 + write 6 B/edge", "read 8 B/edge", "write 6 B/edge"};
    const double bytes[3] = {14.0, 8.0, 6.0};
    for (unsigned grid : {256u, 512u, 1024u}) {
        for (int mode = 0; mode < 3; ++mode) {
            float best = 1e9;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(grid), dim3(1024), 0, 0, in, n4, lo, hi, sink);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(grid), dim3(1024), 0, 0, in, n4, lo, hi, sink);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(grid), dim3(1024), 0, 0, in, n4, lo, hi, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float t;
                CK(hipEventElapsedTime(&t, e0, e1));
                if (t < best) best = t;
            }
            printf("grid %4u  %-24s %.3f ms  %.0f GB/s\n", grid, names[mode], best, bytes[mode] * n / best / 1e6);
        }
    }
    return 0;
}
