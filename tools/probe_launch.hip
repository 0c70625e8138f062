// probe_launch.hip — fixed costs of the small kernels in the seeded fold (not product code).
// For each kernel shape: the average duration of one launch inside a chain of 50 back-to-back launches
// (chain total / 50: what a pipeline stage costs) and the dispatch-event duration of a single launch.
//   empty 256x1024 / 1024x256 (+128 KiB dynamic LDS), LDS zero / fill from HBM (128 KiB per block),
//   a 1M-id flag pack, small edge streams (1M / 2M / 8M edges, 1024x256, D=8).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 probe_launch.hip -o probe_launch
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)
typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

template <int B>
__global__ __launch_bounds__(B) void empty_k(u32* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) out[0] = 1;
}

template <int MODE>  // 0 zero LDS, 1 fill LDS from global
__global__ __launch_bounds__(1024) void lds_k(const u32x4* __restrict__ src, u32 n4, u32* out) {
    extern __shared__ __attribute__((aligned(16))) u32 s[];
    u32x4* d = reinterpret_cast<u32x4*>(s);
    const u32x4 z = {0, 0, 0, 0};
    for (u32 w = threadIdx.x; w < n4; w += 1024) d[w] = MODE ? src[w] : z;
    __syncthreads();
    if (s[threadIdx.x * 7 % (n4 * 4)] == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(256) void pack_k(const u32* __restrict__ f, u32 nq, u32* __restrict__ bits) {
    const u32 lane = threadIdx.x & 63;
    for (u64 q0 = (u64)blockIdx.x * 256 + (threadIdx.x - lane); q0 < nq; q0 += (u64)gridDim.x * 256) {
        const u64 q = q0 + lane;
        u32 nib = 0;
        if (q < nq) {
            const u32 x = f[q];
            nib = (x & 1u) | ((x >> 7) & 2u) | ((x >> 14) & 4u) | ((x >> 21) & 8u);
        }
        u32 w = nib << ((lane & 7) * 4);
        w |= __shfl_xor(w, 1, 64);
        w |= __shfl_xor(w, 2, 64);
        w |= __shfl_xor(w, 4, 64);
        if ((lane & 7) == 0 && q < nq) bits[q >> 3] = w;
    }
}

__global__ __launch_bounds__(1024) void stream_k(const u32x4* __restrict__ body, u64 n2, u32* out) {
    constexpr int D = 8;
    const u64 stride = (u64)gridDim.x * 1024;
    const u64 i = (u64)blockIdx.x * 1024 + threadIdx.x;
    const u64 cnt = i < n2 ? (n2 - 1 - i) / stride + 1 : 0;
    u32 acc = 0;
    for (u64 r = 0; r < cnt; r += D) {
        u32x4 q[D];
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (r + k < cnt) q[k] = __builtin_nontemporal_load(body + i + (r + k) * stride);
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (r + k < cnt) acc ^= q[k].x + q[k].y + q[k].z + q[k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <typename F, typename... A>
static void measure(const char* name, F k, dim3 g, dim3 b, size_t sh, A... a) {
    hipEvent_t e0, e1, k0, k1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&k0));
    CK(hipEventCreate(&k1));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, g, b, (unsigned)sh, 0, a...);
    CK(hipDeviceSynchronize());
    const int N = 50;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k, g, b, (unsigned)sh, 0, a...);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float chain = 0;
    CK(hipEventElapsedTime(&chain, e0, e1));
    float single = 0, best = 1e9;
    for (int i = 0; i < 10; ++i) {
        hipExtLaunchKernelGGL(k, g, b, (uint32_t)sh, 0, k0, k1, 0, a...);
        CK(hipEventSynchronize(k1));
        CK(hipEventElapsedTime(&single, k0, k1));
        if (single < best) best = single;
    }
    CK(hipGetLastError());
    printf("%-34s chain %7.2f us/launch   dispatch-events min %7.2f us\n", name, chain * 1e3 / N, best * 1e3);
}

int main() {
    u32* out;
    u32x4* buf;
    const u64 E = 1ull << 24;  // 16M edges = 128 MiB
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&buf, E * 8));
    CK(hipMemset(buf, 1, E * 8));
    const int lds = 128 * 1024;
    CK(hipFuncSetAttribute((const void*)empty_k<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)lds_k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CK(hipFuncSetAttribute((const void*)lds_k<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d\n", ncu);
    measure("empty 256 x 1024 blocks", empty_k<256>, dim3(1024), dim3(256), 0, out);
    measure("empty 1024 x ncu", empty_k<1024>, dim3(ncu), dim3(1024), 0, out);
    measure("empty 1024 x ncu, 128K LDS", empty_k<1024>, dim3(ncu), dim3(1024), lds, out);
    measure("empty 1024 x 16, 128K LDS", empty_k<1024>, dim3(16), dim3(1024), lds, out);
    measure("lds zero 128K, 1024 x ncu", lds_k<0>, dim3(ncu), dim3(1024), lds, (const u32x4*)buf, (u32)(lds / 16), out);
    measure("lds fill 128K, 1024 x ncu", lds_k<1>, dim3(ncu), dim3(1024), lds, (const u32x4*)buf, (u32)(lds / 16), out);
    measure("lds fill 64K, 1024 x ncu", lds_k<1>, dim3(ncu), dim3(1024), lds, (const u32x4*)buf, (u32)(lds / 32), out);
    measure("pack 1M ids, 256 x 1024", pack_k, dim3(1024), dim3(256), 0, (const u32*)buf, (u32)(1 << 18), out + 8);
    for (u64 ne : {1ull << 20, 1ull << 21, 1ull << 23, 1ull << 24}) {
        char nm[64];
        snprintf(nm, sizeof nm, "stream %llu M edges, 1024 x ncu", (unsigned long long)(ne >> 20));
        measure(nm, stream_k, dim3(ncu), dim3(1024), 0, (const u32x4*)buf, ne / 2, out);
    }
    return 0;
}
