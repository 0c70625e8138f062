// probe_sparse_vis.hip — experiment (the stale label): do plain loads in a kernel see memory-side
// atomics that OTHER XCDs issued in the previous kernel, on lines this XCD read before and never touched with an
// atomic itself? probe_bloom_vis.hip could not tell: its 1M marks reached every line from every XCD, and an atomic
// drops the issuing XCD's L2 copy. Here the marks are SPARSE and come from the blocks of one XCD only (blockIdx %
// 8 == 0 under the round-robin dispatch of workgroups to XCDs), so every other XCD keeps whatever copy it has.
//
// Per iteration, on a buffer of W u32 words (the bloom: 32K words; also a 16 MiB buffer):
//   k_clear: plain-store zeros (every block a share), then k_warm: every block reads the WHOLE buffer with plain
//   loads (a copy of every line in every XCD's L2);  k_mark: blocks with blockIdx % 8 == 0 OR M random bits with
//   device-scope atomicOr (memory-side);  [optional k_stream: 64 MiB of unrelated streaming];  k_check: every block
//   reads its share of the buffer with plain loads AND with memory-side reads (atomic fetch_or 0) and counts the words
//   whose plain value lacks a bit memory has ("stale"), by the reading block's blockIdx % 8.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_sparse_vis.hip -o tools/probe_sparse_vis
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32;
typedef uint64_t u64;
#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

constexpr int kBlock = 256;
constexpr int kGrid = 2048;  // 8 per CU

__global__ void k_clear(u32* buf, u32 w) {
    for (u32 i = blockIdx.x * kBlock + threadIdx.x; i < w; i += gridDim.x * kBlock) buf[i] = 0u;
}

__global__ void k_warm(const u32* buf, u32 w, u32* sink) {  // every block reads the whole buffer
    u32 acc = 0;
    for (u32 i = threadIdx.x; i < w; i += kBlock) acc += buf[i];
    if (acc == 0x12345678u) sink[(blockIdx.x * kBlock + threadIdx.x) % kGrid] = acc;  // never true: keeps the loads
}

__device__ __forceinline__ u32 mix(u32 x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

// marks: the blocks of "XCD 0" (blockIdx % 8 == 0) set bit (h >> 27) of word h % w for M hashes of (iter, k)
__global__ void k_mark(u32* buf, u32 w, u32 m, u32 iter) {
    if (blockIdx.x % 8 != 0) return;
    const u32 nb = gridDim.x / 8, b = blockIdx.x / 8;
    for (u32 k = b * kBlock + threadIdx.x; k < m; k += nb * kBlock) {
        const u32 h = mix(iter * 0x9E3779B9u + k);
        atomicOr(&buf[h % w], 1u << (h >> 27));
    }
}

__global__ void k_stream(const uint4* src, uint4* dst, u64 n) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) dst[i] = src[i];
}

// every block checks a share of the buffer: plain load vs memory-side read; stale[xcd] += words lacking a bit
__global__ void k_check(u32* buf, u32 w, unsigned long long* stale, unsigned long long* extra) {
    const u32 per = (w + gridDim.x - 1) / gridDim.x, a = blockIdx.x * per, e = a + per < w ? a + per : w;
    for (u32 i = a + threadIdx.x; i < e; i += kBlock) {
        const u32 plain = buf[i];
        const u32 mem = __hip_atomic_fetch_or(buf + i, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mem & ~plain) atomicAdd(&stale[blockIdx.x % 8], 1ull);
        if (plain & ~mem) atomicAdd(&extra[blockIdx.x % 8], 1ull);
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100;
    u32* sink;
    CK(hipMalloc(&sink, kGrid * sizeof(u32)));
    unsigned long long *stale, *extra;
    CK(hipMalloc(&stale, 8 * sizeof(unsigned long long)));
    CK(hipMalloc(&extra, 8 * sizeof(unsigned long long)));
    const u64 stream_n = (64ull << 20) / 16;
    uint4 *s_src, *s_dst;
    CK(hipMalloc(&s_src, stream_n * 16));
    CK(hipMalloc(&s_dst, stream_n * 16));
    CK(hipMemset(s_src, 1, stream_n * 16));
    printf("probe_sparse_vis: grid %d x %d, marks from blocks %% 8 == 0 only, %d iterations per variant\n", kGrid, kBlock,
           iters);
    struct V {
        u32 w, m;
        bool stream;
        const char* name;
    } vs[] = {{32768, 2000, false, "128 KiB buffer, 2000 marks"},
              {32768, 2000, true, "128 KiB buffer, 2000 marks, 64 MiB stream before the check"},
              {32768, 200000, false, "128 KiB buffer, 200K marks"},
              {4u << 20, 20000, false, "16 MiB buffer, 20K marks"}};
    for (const V& v : vs) {
        u32* buf;
        CK(hipMalloc(&buf, (size_t)v.w * 4));
        unsigned long long tot_stale[8] = {}, tot_extra[8] = {};
        int bad_iters = 0;
        for (int it = 0; it < iters; ++it) {
            CK(hipMemset(stale, 0, 8 * sizeof(unsigned long long)));
            CK(hipMemset(extra, 0, 8 * sizeof(unsigned long long)));
            hipLaunchKernelGGL(k_clear, dim3(kGrid), dim3(kBlock), 0, 0, buf, v.w);
            hipLaunchKernelGGL(k_warm, dim3(kGrid), dim3(kBlock), 0, 0, (const u32*)buf, v.w < 65536 ? v.w : 65536, sink);
            hipLaunchKernelGGL(k_mark, dim3(kGrid), dim3(kBlock), 0, 0, buf, v.w, v.m, (u32)it);
            if (v.stream) hipLaunchKernelGGL(k_stream, dim3(kGrid), dim3(kBlock), 0, 0, (const uint4*)s_src, s_dst, stream_n);
            hipLaunchKernelGGL(k_check, dim3(kGrid), dim3(kBlock), 0, 0, buf, v.w, stale, extra);
            CK(hipGetLastError());
            unsigned long long hs[8], he[8];
            CK(hipMemcpy(hs, stale, sizeof(hs), hipMemcpyDeviceToHost));
            CK(hipMemcpy(he, extra, sizeof(he), hipMemcpyDeviceToHost));
            bool bad = false;
            for (int x = 0; x < 8; ++x) {
                tot_stale[x] += hs[x];
                tot_extra[x] += he[x];
                bad |= hs[x] != 0 || he[x] != 0;
            }
            bad_iters += bad;
        }
        printf("%-60s iterations with a difference %d / %d; stale words by reading XCD:", v.name, bad_iters, iters);
        for (int x = 0; x < 8; ++x) printf(" %llu", tot_stale[x]);
        printf("; extra:");
        for (int x = 0; x < 8; ++x) printf(" %llu", tot_extra[x]);
        printf("\n");
        fflush(stdout);
        CK(hipFree(buf));
    }
    return 0;
}
