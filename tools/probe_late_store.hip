// probe_late_store.hip — experiment: can a PLAIN store of one kernel reach memory only after
// the next kernel in the same stream has run? tools/stress_inc.py found the stale label's signature in exactly that
// hand-off (a path-splitting store of the recording fold over a root the in-place compress wrote after it): gone with
// an agent-scope release at the end of every fold block, NOT gone with an s_waitcnt vmcnt(0) at the end of every
// wave. This measures the hand-off directly, with memory-side atomics as the observer (they act on memory, not on
// any XCD's L2):
//   k_write  (A): every block plain-stores `a` into its share of M words (style: sparse 4-B stores at hashed
//                 positions over a 64 MiB buffer, like path splitting; or whole 128-B lines with 16-B stores, like a
//                 compress writing labels; optionally an agent-scope release at the end of every block)
//   k_cas    (B): right after A in the same stream, every word: atomicCAS(word, a, b); "invisible" counts the CASes
//                 that did not find `a` (A's store had not reached memory when B's atomic ran)
//   k_check  (C): after B, every word read back with a memory-side atomic; "clobbered" counts words that hold `a`
//                 again (A's store landed after B's CAS had replaced it)
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_late_store.hip -o tools/probe_late_store
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
constexpr int kGrid = 2048;

__device__ __forceinline__ u32 mix(u32 x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
// word k of the M written words: hashed over the buffer (SPARSE; bit 4 clear, so that word | 16 — 64 B away in the
// same 128-B line — is never a written word) or the first M words (LINES)
template <bool SPARSE>
__device__ __forceinline__ u32 word_of(u32 k, u32 w, u32 salt) {
    return SPARSE ? (mix(k * 0x9E3779B9u + salt) % w) & ~16u : k;
}

__global__ void k_fill(u32* buf, u32 w, u32 v) {
    for (u32 i = blockIdx.x * kBlock + threadIdx.x; i < w; i += gridDim.x * kBlock) buf[i] = v;
}

// ATOMIC_AFTER: after its plain store, the thread issues a memory-side atomic on ANOTHER word of the same 128-B line
// (an atomic drops the issuing XCD's L2 copy of the line: what becomes of the dirty bytes of the plain store?). The
// fold does exactly this: path-splitting stores and hook CASes on neighbouring slots. The other word (x | 16: 64 B
// away, same line) is never one of the M written words (word_of).
template <bool SPARSE, bool RELEASE, bool ATOMIC_AFTER = false>
__global__ void k_write(u32* buf, u32 w, u32 m, u32 salt, u32 a) {
    if (SPARSE) {
        for (u32 k = blockIdx.x * kBlock + threadIdx.x; k < m; k += gridDim.x * kBlock) {
            const u32 x = word_of<true>(k, w, salt);
            buf[x] = a;
            if (ATOMIC_AFTER) atomicAdd(&buf[x | 16u], 0x100000u);
        }
    } else {
        typedef u32 u4 __attribute__((ext_vector_type(4)));
        const u4 q = {a, a, a, a};
        for (u32 k = blockIdx.x * kBlock + threadIdx.x; k < m / 4; k += gridDim.x * kBlock) reinterpret_cast<u4*>(buf)[k] = q;
    }
    if (RELEASE) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
}

// B runs over the words in another order than A (rotated by a block offset), so a word is CASed from another XCD
// than the one that stored it
template <bool SPARSE>
__global__ void k_cas(u32* buf, u32 w, u32 m, u32 salt, u32 a, u32 b, unsigned long long* invisible) {
    u32 bad = 0;
    const u32 nthreads = gridDim.x * kBlock;
    const u32 rot = 97 * kBlock;
    for (u32 t = blockIdx.x * kBlock + threadIdx.x; t < m; t += nthreads) {
        const u32 k = (t + rot) % m;
        u32* p = &buf[word_of<SPARSE>(k, w, salt)];
        const u32 old = atomicCAS(p, a, b);
        bad += old != a && old != b;  // b: a duplicate hashed word already swapped
    }
    if (bad) atomicAdd(invisible, (unsigned long long)bad);
}

template <bool SPARSE>
__global__ void k_check(u32* buf, u32 w, u32 m, u32 salt, u32 a, unsigned long long* clobbered) {
    u32 bad = 0;
    for (u32 k = blockIdx.x * kBlock + threadIdx.x; k < m; k += gridDim.x * kBlock) {
        const u32 v = __hip_atomic_fetch_or(&buf[word_of<SPARSE>(k, w, salt)], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad += v == a;
    }
    if (bad) atomicAdd(clobbered, (unsigned long long)bad);
}

template <bool SPARSE, bool RELEASE, bool ATOMIC_AFTER = false>
static void run(const char* name, u32* buf, u32 w, u32 m, int iters, unsigned long long* d_cnt) {
    unsigned long long inv = 0, clob = 0;
    int bad_iters = 0;
    for (int it = 0; it < iters; ++it) {
        const u32 a = 2u * (u32)it + 1u, b = 2u * (u32)it + 2u, salt = 0x5151u * (u32)it;
        CK(hipMemset(d_cnt, 0, 2 * sizeof(unsigned long long)));
        hipLaunchKernelGGL(k_fill, dim3(kGrid), dim3(kBlock), 0, 0, buf, w, 0u);
        CK(hipDeviceSynchronize());  // the fill is in memory before A starts
        hipLaunchKernelGGL((k_write<SPARSE, RELEASE, ATOMIC_AFTER>), dim3(kGrid), dim3(kBlock), 0, 0, buf, w, m, salt, a);
        hipLaunchKernelGGL((k_cas<SPARSE>), dim3(kGrid), dim3(kBlock), 0, 0, buf, w, m, salt, a, b, d_cnt);
        hipLaunchKernelGGL((k_check<SPARSE>), dim3(kGrid), dim3(kBlock), 0, 0, buf, w, m, salt, a, d_cnt + 1);
        CK(hipGetLastError());
        unsigned long long h[2];
        CK(hipMemcpy(h, d_cnt, sizeof(h), hipMemcpyDeviceToHost));
        inv += h[0];
        clob += h[1];
        bad_iters += (h[0] || h[1]);
    }
    printf("%-64s iterations with a late store %3d / %d; CASes that missed A's store %llu; words A's store clobbered "
           "after B %llu (of %u x %d)\n", name, bad_iters, iters, inv, clob, m, iters);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 50;
    const u32 W = 1u << 24;  // 64 MiB: C3 / C5's parent[]
    u32* buf;
    CK(hipMalloc(&buf, (size_t)W * 4));
    unsigned long long* d_cnt;
    CK(hipMalloc(&d_cnt, 2 * sizeof(unsigned long long)));
    printf("probe_late_store: grid %d x %d, buffer %u words, %d iterations per variant\n", kGrid, kBlock, W, iters);
    run<true, false>("sparse 4-B plain stores, 1M words", buf, W, 1u << 20, iters, d_cnt);
    run<true, false>("sparse 4-B plain stores, 64K words", buf, W, 1u << 16, iters, d_cnt);
    run<true, true>("sparse 4-B plain stores + release per block, 1M words", buf, W, 1u << 20, iters, d_cnt);
    run<false, false>("whole lines, 16-B plain stores, 16M words", buf, W, 1u << 24, iters, d_cnt);
    run<false, false>("whole lines, 16-B plain stores, 1M words", buf, W, 1u << 20, iters, d_cnt);
    run<true, false, true>("sparse 4-B plain stores + an atomic on the same line, 64K", buf, W, 1u << 16, iters, d_cnt);
    run<true, false, true>("sparse 4-B plain stores + an atomic on the same line, 1M", buf, W, 1u << 20, iters, d_cnt);
    run<true, true, true>("... + release per block, 1M", buf, W, 1u << 20, iters, d_cnt);
    return 0;
}
