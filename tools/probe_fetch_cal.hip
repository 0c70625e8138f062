// probe_fetch_cal.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE per access class on gfx950 (not product
// code; VERDICT r5 next-1c, MI355X_MICROARCH.md "HBM": the 2x correction is established for wide streaming reads only,
// "other access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Every kernel touches a KNOWN set of 128-B lines exactly once (a multiplicative permutation of the lines, so the
// order is scattered but no line is touched twice and nothing is re-read from the L2 or the Infinity Cache), in a
// 4 GiB table (16x the 256 MiB Infinity Cache), plus one class with C3's own shape (random 4-B reads of a 64 MiB
// array, the fold's parent[] lookups, which the Infinity Cache holds):
//   k_stream       16-B loads per lane, the whole table          known: 4 GiB read
//   k_line4        one 4-B load per 128-B line                   known: L lines touched (4 B useful each)
//   k_half4        two 4-B loads per line, one in each 64-B half  known: L lines, both halves
//   k_store4       one 4-B plain store per line                   known: L lines written (4 B each)
//   k_cas4         one 4-B atomicCAS per line (result used)       known: L lines, one memory-side atomic each
//   k_c3reads      2^24 x 2 random 4-B loads in a 64 MiB array    C3's fold lookups (Infinity-Cache resident)
// The summary (tools/fetch_cal_summary.py) divides each kernel's counter by its known line count: FETCH_SIZE per
// 128-B line touched says which correction a random 4-B access class needs.
// Build: hipcc -O3 --offload-arch=gfx950 probe_fetch_cal.hip -o probe_fetch_cal
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

constexpr u64 kTableBytes = 4ull << 30;
constexpr u64 kLines = kTableBytes / 128;    // 2^25 lines of 128 B
constexpr u64 kPerm = 0x9E3779B1ull | 1;     // odd: i -> i * kPerm mod 2^25 is a permutation of the lines
__device__ __forceinline__ u64 line_of(u64 i) { return (i * kPerm) & (kLines - 1); }

__global__ __launch_bounds__(1024) void k_stream(const u4* __restrict__ t, u64 n4, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < n4; i += (u64)gridDim.x * 1024) {
        const u4 a = __builtin_nontemporal_load(t + i);
        acc ^= a.x ^ a.w;
    }
    if (acc == 0x9u) sink[0] = acc;
}

__global__ __launch_bounds__(1024) void k_line4(const u32* __restrict__ t, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < kLines; i += (u64)gridDim.x * 1024) acc ^= t[line_of(i) * 32];
    if (acc == 0x9u) sink[0] = acc;
}

__global__ __launch_bounds__(1024) void k_half4(const u32* __restrict__ t, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < kLines; i += (u64)gridDim.x * 1024) {
        const u64 b = line_of(i) * 32;
        acc ^= t[b] ^ t[b + 16];
    }
    if (acc == 0x9u) sink[0] = acc;
}

__global__ __launch_bounds__(1024) void k_store4(u32* __restrict__ t) {
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < kLines; i += (u64)gridDim.x * 1024) t[line_of(i) * 32] = (u32)i;
}

__global__ __launch_bounds__(1024) void k_cas4(u32* __restrict__ t, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < kLines; i += (u64)gridDim.x * 1024)
        acc ^= atomicCAS(t + line_of(i) * 32, (u32)i, (u32)i + 1);
    if (acc == 0x9u) sink[0] = acc;
}

// C3's shape: 2^24 ids (64 MiB), 2 x 9.2M random 4-B loads (splitmix-hashed indices)
__device__ __forceinline__ u32 hidx(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return (u32)((x ^ (x >> 31)) & ((1u << 24) - 1));
}
__global__ __launch_bounds__(1024) void k_c3reads(const u32* __restrict__ t, u64 n, u32* sink) {
    u32 acc = 0;
    for (u64 i = blockIdx.x * 1024ull + threadIdx.x; i < n; i += (u64)gridDim.x * 1024)
        acc ^= t[hidx(2 * i)] ^ t[hidx(2 * i + 1)];
    if (acc == 0x9u) sink[0] = acc;
}

int main() {
    u32 *t, *sink;
    CK(hipMalloc(&t, kTableBytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(t, 1, kTableBytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const u64 c3_edges = 9227469;
    printf("table %llu B, lines %llu (128 B), C3 reads %llu\n", (unsigned long long)kTableBytes, (unsigned long long)kLines,
           (unsigned long long)(2 * c3_edges));
    for (int rep = 0; rep < 3; ++rep) {
        float ms[6];
        for (int k = 0; k < 6; ++k) {
            CK(hipEventRecord(e0));
            switch (k) {
            case 0: hipLaunchKernelGGL(k_stream, dim3(1024), dim3(1024), 0, 0, (const u4*)t, kTableBytes / 16, sink); break;
            case 1: hipLaunchKernelGGL(k_line4, dim3(1024), dim3(1024), 0, 0, t, sink); break;
            case 2: hipLaunchKernelGGL(k_half4, dim3(1024), dim3(1024), 0, 0, t, sink); break;
            case 3: hipLaunchKernelGGL(k_store4, dim3(1024), dim3(1024), 0, 0, t); break;
            case 4: hipLaunchKernelGGL(k_cas4, dim3(1024), dim3(1024), 0, 0, t, sink); break;
            case 5: hipLaunchKernelGGL(k_c3reads, dim3(1024), dim3(1024), 0, 0, t, c3_edges, sink); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[k], e0, e1));
        }
        printf("rep %d ms: stream %.3f (%.0f GB/s)  line4 %.3f (%.1f G lines/s)  half4 %.3f  store4 %.3f  cas4 %.3f  "
               "c3reads %.3f\n",
               rep, ms[0], kTableBytes / ms[0] / 1e6, ms[1], kLines / ms[1] / 1e6, ms[2], ms[3], ms[4], ms[5]);
    }
    return 0;
}
