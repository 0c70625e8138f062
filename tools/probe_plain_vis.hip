// probe_plain_vis.hip — experiment (the stale label; VERDICT r3 "next" 1): the hand-off of the
// in-place incremental compress. That compress rewrites a few parent[] slots with PLAIN 4-B stores while find walks
// of other waves, on every XCD, read the same lines; the next fold then reads those slots with plain loads. If any
// XCD could still read a pre-compress value there after the kernel boundary, the fold could copy a root that was
// hooked in an EARLIER window into a slot (path splitting, or a hang of a new id), unmarked in the current window's
// bloom: exactly the recorded symptom. probe_sparse_vis.hip covered memory-side atomics only.
//
// Per iteration, on a buffer of W u32 words:
//   k_clear: every block plain-stores 0 over its share;  k_warm: every block reads a 2 MiB window of the buffer (a
//   copy of those lines in every XCD's L2);  k_write: blocks with blockIdx % 8 == 0 (one XCD under the round-robin
//   dispatch) store `val` into M sparse words; with READERS the other blocks meanwhile read those same words again
//   and again (their XCDs pull the lines during the write, the compress's pattern);  [k_stream: 64 MiB of unrelated
//   streaming];  k_check: EVERY block reads all M words with plain loads and counts those != val, by blockIdx % 8.
// Writer styles: 0 plain stores, 1 plain stores + fence(release, agent) at the end of each block, 2 sc1 stores
// (agent-scope relaxed atomic store). Build: hipcc --offload-arch=gfx950 -O3 tools/probe_plain_vis.hip -o tools/probe_plain_vis
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

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

__device__ __forceinline__ u32 mix(u32 x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ u32 word_of(u32 iter, u32 k, u32 w) { return mix(iter * 0x9E3779B9u + k) % w; }

__global__ void k_clear(u32* buf, u32 w) {
    for (u32 i = blockIdx.x * kBlock + threadIdx.x; i < w; i += gridDim.x * kBlock) buf[i] = 0u;
}

__global__ void k_warm(const u32* buf, u32 w, u32* sink) {  // every block reads the first min(w, 512K) words
    u32 acc = 0;
    for (u32 i = threadIdx.x; i < w; i += kBlock) acc += buf[i];
    if (acc == 0x12345678u) sink[(blockIdx.x * kBlock + threadIdx.x) % kGrid] = acc;
}

template <int STYLE, bool READERS>
__global__ void k_write(u32* buf, u32 w, u32 m, u32 iter, u32 val, u32* sink) {
    if (blockIdx.x % 8 != 0) {
        if (!READERS) return;
        u32 acc = 0;  // readers: the written words, several passes, while the writers run
        for (int pass = 0; pass < 4; ++pass)
            for (u32 k = threadIdx.x + (blockIdx.x % 7) * 37; k < m; k += kBlock) acc += buf[word_of(iter, k, w)];
        if (acc == 0x12345678u) sink[(blockIdx.x * kBlock + threadIdx.x) % kGrid] = acc;
        return;
    }
    const u32 nb = gridDim.x / 8, b = blockIdx.x / 8;
    for (u32 k = b * kBlock + threadIdx.x; k < m; k += nb * kBlock) {
        u32* p = &buf[word_of(iter, k, w)];
        if (STYLE == 2) __hip_atomic_store(p, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *p = val;
    }
    if (STYLE == 1) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
}

__global__ void k_stream(const uint4* src, uint4* dst, u64 n) {
    for (u64 i = (u64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (u64)gridDim.x * kBlock) dst[i] = src[i];
}

// every block reads every written word with plain loads; stale[xcd] += words != val
__global__ void k_check(const u32* buf, u32 w, u32 m, u32 iter, u32 val, unsigned long long* stale) {
    u32 bad = 0;
    for (u32 k = threadIdx.x; k < m; k += kBlock) bad += buf[word_of(iter, k, w)] != val;
    if (bad) atomicAdd(&stale[blockIdx.x % 8], (unsigned long long)bad);
}

template <int STYLE, bool READERS>
static void run(const char* name, u32 w, u32 m, bool stream, int iters, u32* sink, unsigned long long* stale,
                const uint4* s_src, uint4* s_dst, u64 stream_n) {
    u32* buf;
    CK(hipMalloc(&buf, (size_t)w * 4));
    unsigned long long tot[8] = {};
    int bad_iters = 0;
    for (int it = 0; it < iters; ++it) {
        const u32 val = 0x10000u + (u32)it;
        CK(hipMemset(stale, 0, 8 * sizeof(unsigned long long)));
        hipLaunchKernelGGL(k_clear, dim3(kGrid), dim3(kBlock), 0, 0, buf, w);
        hipLaunchKernelGGL(k_warm, dim3(kGrid), dim3(kBlock), 0, 0, (const u32*)buf, w < (1u << 19) ? w : (1u << 19), sink);
        hipLaunchKernelGGL((k_write<STYLE, READERS>), dim3(kGrid), dim3(kBlock), 0, 0, buf, w, m, (u32)it, val, sink);
        if (stream) hipLaunchKernelGGL(k_stream, dim3(kGrid), dim3(kBlock), 0, 0, s_src, s_dst, stream_n);
        hipLaunchKernelGGL(k_check, dim3(kGrid), dim3(kBlock), 0, 0, (const u32*)buf, w, m, (u32)it, val, stale);
        CK(hipGetLastError());
        unsigned long long hs[8];
        CK(hipMemcpy(hs, stale, sizeof(hs), hipMemcpyDeviceToHost));
        bool bad = false;
        for (int x = 0; x < 8; ++x) {
            tot[x] += hs[x];
            bad |= hs[x] != 0;
        }
        bad_iters += bad;
    }
    printf("%-72s iterations with a stale read %d / %d; stale reads by reading XCD:", name, bad_iters, iters);
    for (int x = 0; x < 8; ++x) printf(" %llu", tot[x]);
    printf("\n");
    fflush(stdout);
    CK(hipFree(buf));
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100;
    u32* sink;
    CK(hipMalloc(&sink, kGrid * sizeof(u32)));
    unsigned long long* stale;
    CK(hipMalloc(&stale, 8 * sizeof(unsigned long long)));
    const u64 stream_n = (64ull << 20) / 16;
    uint4 *s_src, *s_dst;
    CK(hipMalloc(&s_src, stream_n * 16));
    CK(hipMalloc(&s_dst, stream_n * 16));
    CK(hipMemset(s_src, 1, stream_n * 16));
    printf("probe_plain_vis: grid %d x %d, writes from blocks %% 8 == 0 only, every block checks every written word, "
           "%d iterations per variant\n", kGrid, kBlock, iters);
    run<0, false>("plain stores, 128 KiB buffer, 2000 words", 32768, 2000, false, iters, sink, stale, s_src, s_dst, stream_n);
    run<0, true>("plain stores + concurrent readers, 128 KiB, 2000 words", 32768, 2000, false, iters, sink, stale, s_src, s_dst,
                 stream_n);
    run<0, true>("plain stores + concurrent readers, 2 MiB, 20000 words", 1u << 19, 20000, false, iters, sink, stale, s_src,
                 s_dst, stream_n);
    run<0, true>("plain stores + concurrent readers, 64 MiB, 20000 words", 1u << 24, 20000, false, iters, sink, stale, s_src,
                 s_dst, stream_n);
    run<0, true>("plain stores + concurrent readers, 2 MiB, 20000 words, 64 MiB stream", 1u << 19, 20000, true, iters, sink,
                 stale, s_src, s_dst, stream_n);
    run<1, true>("plain stores + release fence + readers, 2 MiB, 20000 words", 1u << 19, 20000, false, iters, sink, stale,
                 s_src, s_dst, stream_n);
    run<2, true>("sc1 stores + readers, 2 MiB, 20000 words", 1u << 19, 20000, false, iters, sink, stale, s_src, s_dst,
                 stream_n);
    return 0;
}
