// probe_bloom_vis.hip — VERDICT r2 item 1: do bits set by memory-side atomicOr reach a later kernel's plain loads
// when the same 128 KiB buffer was cleared with plain stores (and read into every CU's L2) by earlier kernels?
// This is the incremental compress's bloom hand-off, kernel for kernel:
//   warm    every CU reads the buffer into LDS with plain loads (the previous compress_inc that read it)
//   clear   plain stores of zero from every XCD: compress_bits_kernel's 4-B loop (style 0) or compress_inc_kernel's
//           per-block 16-B share (style 1)
//   stream  an unrelated 64 MiB stream (the fold's edges / parent[] traffic between clear and marks; optional)
//   mark    M memory-side atomicOr marks from 2048 blocks on every XCD (fold_kernel<true>'s BloomRec)
//   check   every CU copies the buffer into LDS with plain loads (compress_inc_kernel's lds_fill), then compares
//           each word with a memory-side read (atomic fetch_or 0) and that with the host's expected bitmap
// Counts, per style: LDS words lacking a bit that memory holds (stale plain loads), memory words lacking an
// expected bit (lost atomics), over `iters` iterations with fresh marks each.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_bloom_vis tools/probe_bloom_vis.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));
#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

constexpr u32 kBits = 1u << 20;
constexpr u32 kWords = kBits / 32;  // 32768
constexpr u32 kW4 = kWords / 4;     // 8192 16-B words

__host__ __device__ inline u32 mix(u32 x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__host__ __device__ inline u32 mark_slot(u32 it, u32 i) { return mix(i * 0x9E3779B1u + it * 0x85EBCA77u + 1u) >> 12; }

__global__ __launch_bounds__(1024) void warm_kernel(const u32* buf, u32* sink) {
    __shared__ u32x4 s[kW4];
    const u32x4* src = reinterpret_cast<const u32x4*>(buf);
    for (u32 w = threadIdx.x; w < kW4; w += 1024) s[w] = src[w];
    __syncthreads();
    if (threadIdx.x == 0 && s[blockIdx.x % kW4].x == 0xDEADBEEFu) sink[0] = 1;
}

__global__ __launch_bounds__(256) void clear4_kernel(u32* buf) {
    for (u32 w = blockIdx.x * 256 + threadIdx.x; w < kWords; w += gridDim.x * 256) buf[w] = 0;
}

__global__ __launch_bounds__(1024) void clear16_kernel(u32* buf) {
    const u32 per = (kW4 + gridDim.x - 1) / gridDim.x, a = blockIdx.x * per, b = min(kW4, a + per);
    const u32x4 z = {0, 0, 0, 0};
    for (u32 w = a + threadIdx.x; w < b; w += 1024) reinterpret_cast<u32x4*>(buf)[w] = z;
}

__global__ __launch_bounds__(256) void stream_kernel(const u32x4* a, u32x4* b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i] + 1u;
}

__global__ __launch_bounds__(256) void mark_kernel(u32* buf, u32 it, u32 m) {
    for (u32 i = blockIdx.x * 256 + threadIdx.x; i < m; i += gridDim.x * 256) {
        const u32 s = mark_slot(it, i);
        atomicOr(&buf[s >> 5], 1u << (s & 31));
    }
}

// cnt[0]: LDS words lacking a bit memory holds; cnt[1]: LDS words with a bit memory lacks; cnt[2]: memory words
// lacking an expected bit; cnt[3]: memory words with an unexpected bit (all summed over blocks)
__global__ __launch_bounds__(1024) void check_kernel(u32* buf, const u32* expect, u32* cnt) {
    extern __shared__ __attribute__((aligned(16))) u32 s_b[];
    {
        constexpr int U = 8;
        const u32x4* src = reinterpret_cast<const u32x4*>(buf);
        u32x4* dst = reinterpret_cast<u32x4*>(s_b);
        for (u32 base = 0; base < kW4; base += U * 1024) {
            u32x4 r[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const u32 w = base + k * 1024 + threadIdx.x;
                r[k] = src[w < kW4 ? w : kW4 - 1];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const u32 w = base + k * 1024 + threadIdx.x;
                if (w < kW4) dst[w] = r[k];
            }
        }
    }
    __syncthreads();
    u32 c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (u32 w = threadIdx.x; w < kWords; w += 1024) {
        const u32 mem = __hip_atomic_fetch_or(buf + w, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const u32 lds = s_b[w];
        c0 += (mem & ~lds) != 0;
        c1 += (lds & ~mem) != 0;
        if (blockIdx.x == 0) {
            const u32 e = expect[w];
            c2 += (e & ~mem) != 0;
            c3 += (mem & ~e) != 0;
        }
    }
    if (c0) atomicAdd(&cnt[0], c0);
    if (c1) atomicAdd(&cnt[1], c1);
    if (c2) atomicAdd(&cnt[2], c2);
    if (c3) atomicAdd(&cnt[3], c3);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 200;
    const u32 m = argc > 2 ? (u32)atoll(argv[2]) : 1000000u;  // marks per iteration (C3's last window: ~1M)
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    u32 *buf, *expect, *cnt, *sink;
    u32x4 *sa, *sb;
    const size_t sn = (64u << 20) / 16;
    CK(hipMalloc(&buf, kWords * 4));
    CK(hipMalloc(&expect, kWords * 4));
    CK(hipMalloc(&cnt, 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMalloc(&sa, sn * 16));
    CK(hipMalloc(&sb, sn * 16));
    CK(hipMemset(buf, 0, kWords * 4));
    CK(hipMemset(sa, 0, sn * 16));
    u32* h_exp;
    CK(hipHostMalloc((void**)&h_exp, kWords * 4, hipHostMallocDefault));
    CK(hipFuncSetAttribute((const void*)check_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kWords * 4));
    printf("probe_bloom_vis: %d CUs, %d iterations per variant, %u marks per iteration\n", ncu, iters, m);
    const char* names[] = {"clear4 (compress_bits style)", "clear16 (compress_inc style)"};
    for (int stream = 0; stream < 2; ++stream)
        for (int style = 0; style < 2; ++style) {
            unsigned long long tot[4] = {0, 0, 0, 0};
            int bad_iters = 0;
            for (int it = 0; it < iters; ++it) {
                const u32 tag = (u32)(it + 1000 * (style + 2 * stream));
                for (u32 w = 0; w < kWords; ++w) h_exp[w] = 0;
                for (u32 i = 0; i < m; ++i) {
                    const u32 s = mark_slot(tag, i);
                    h_exp[s >> 5] |= 1u << (s & 31);
                }
                CK(hipMemcpy(expect, h_exp, kWords * 4, hipMemcpyHostToDevice));
                CK(hipMemset(cnt, 0, 16));
                CK(hipDeviceSynchronize());
                // the chain, asynchronous, one stream
                hipLaunchKernelGGL(warm_kernel, dim3(ncu), dim3(1024), 0, 0, buf, sink);
                if (style == 0) hipLaunchKernelGGL(clear4_kernel, dim3(2048), dim3(256), 0, 0, buf);
                else hipLaunchKernelGGL(clear16_kernel, dim3(ncu), dim3(1024), 0, 0, buf);
                if (stream) hipLaunchKernelGGL(stream_kernel, dim3(2048), dim3(256), 0, 0, sa, sb, sn);
                hipLaunchKernelGGL(mark_kernel, dim3(2048), dim3(256), 0, 0, buf, tag, m);
                hipLaunchKernelGGL(check_kernel, dim3(ncu), dim3(1024), kWords * 4, 0, buf, expect, cnt);
                CK(hipGetLastError());
                u32 h[4];
                CK(hipMemcpy(h, cnt, 16, hipMemcpyDeviceToHost));
                bool bad = false;
                for (int k = 0; k < 4; ++k) {
                    tot[k] += h[k];
                    bad |= h[k] != 0;
                }
                bad_iters += bad;
            }
            printf("%s, %s: iterations with a difference %d / %d; LDS words lacking a memory bit %llu, LDS extra %llu; "
                   "memory words lacking an expected bit %llu, memory extra %llu\n",
                   names[style], stream ? "64 MiB stream between clear and marks" : "no stream", bad_iters, iters, tot[0],
                   tot[1], tot[2], tot[3]);
        }
    return 0;
}
