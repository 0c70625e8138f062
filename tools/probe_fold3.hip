// probe_fold3.hip — prototype of the sampled + giant-filtered fold on C2 (R-MAT s20, 16M edges), with a
// per-phase time breakdown and a check against a sequential host union-find. Not product code.
//   phase S: geometric chunked fold of a prefix (small first launches avoid the hub CAS storm)
//   phase G: compress + majority-vote "giant" label over sampled vertices + giant bitmap
//   phase F: persistent filtered fold of the rest: giant bitmap in LDS, edges with both ends in the giant skip
//            parent[] entirely; the rest take the CAS union-find path
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc probe_fold3.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "edge_gen.h"
#include "gelly_cc.h"
#include "uf_device.h"

using namespace gcc;
#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)
typedef UnionFind<LoadPlain, true> UF;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__global__ void gen(gcc_gen_params p, u64 n, uint2* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u32 a, b;
        gcc_gen_edge(&p, i, &a, &b);
        out[i] = make_uint2(a, b);
    }
}

__global__ __launch_bounds__(256) void fold_base(u32* parent, const uint2* e, u64 n) {
    NoCount c;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 x = __builtin_nontemporal_load(reinterpret_cast<const u64*>(e) + i);
        UF::unite(parent, (u32)x, (u32)(x >> 32), c);
    }
}

__global__ __launch_bounds__(256) void compress(u32* parent, u32* labels, u32 n) {
    NoCount c;
    for (u64 v = blockIdx.x * (u64)blockDim.x + threadIdx.x; v < n; v += (u64)gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        labels[v] = (p >= v) ? p : UF::find_from(parent, (u32)v, p, c);
    }
}

// majority vote (Boyer-Moore, associative pair form) over labels of 16384 sampled seen vertices; one block
__device__ __forceinline__ void bm_merge(u32& c1, u32& n1, u32 c2, u32 n2) {
    if (c1 == c2) n1 += n2;
    else if (n1 >= n2) n1 -= n2;
    else { c1 = c2; n1 = n2 - n1; }
}
__global__ __launch_bounds__(256) void giant_vote(const u32* labels, u32 n, u32* giant) {
    u32 cand = 0xFFFFFFFFu, cnt = 0;
    for (int k = 0; k < 64; ++k) {
        const u32 v = (u32)(gcc_splitmix64((u64)threadIdx.x * 64 + k) % n);
        const u32 l = labels[v];
        if (l != 0xFFFFFFFFu) bm_merge(cand, cnt, l, 1);
    }
    for (int off = 32; off > 0; off >>= 1) {
        const u32 c2 = __shfl_down(cand, off, 64), n2 = __shfl_down(cnt, off, 64);
        bm_merge(cand, cnt, c2, n2);
    }
    __shared__ u32 sc[4], sn[4];
    if ((threadIdx.x & 63) == 0) { sc[threadIdx.x >> 6] = cand; sn[threadIdx.x >> 6] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) bm_merge(sc[0], sn[0], sc[w], sn[w]);
        *giant = sc[0];
    }
}

// bitmap of the giant component: one u64 word per 64 ids, built with a wave ballot
__global__ __launch_bounds__(256) void giant_bits(const u32* labels, u32 n, const u32* giant, unsigned long long* bits) {
    const u32 g = *giant;
    for (u64 v = blockIdx.x * (u64)blockDim.x + threadIdx.x; v < ((u64)n + 63) / 64 * 64; v += (u64)gridDim.x * blockDim.x) {
        const bool in = v < n && labels[v] == g && g != 0xFFFFFFFFu;
        const unsigned long long m = __ballot(in);
        if ((threadIdx.x & 63) == 0) bits[v >> 6] = m;
    }
}

// filtered fold: persistent, LDS bitmap, 8 edges per lane per iteration (4 x 16 B loads in flight)
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void fold_filtered(u32* parent, const u32x4* e2, u64 n2 /* pairs of edges */,
                                                        const unsigned long long* bits, u32 nwords,
                                                        unsigned long long* n_slow) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long s_bits[];
    for (u32 w = threadIdx.x; w < nwords; w += BLOCK) s_bits[w] = bits[w];
    __syncthreads();
    const u32* sb = reinterpret_cast<const u32*>(s_bits);
    auto in_giant = [&](u32 v) { return (sb[v >> 5] >> (v & 31)) & 1u; };
    NoCount c;
    u32 slow = 0;
    const u64 stride = (u64)gridDim.x * BLOCK;
    u64 i = blockIdx.x * (u64)BLOCK + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
        u32x4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = __builtin_nontemporal_load(e2 + i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (!(in_giant(q[k].x) & in_giant(q[k].y))) { UF::unite(parent, q[k].x, q[k].y, c); ++slow; }
            if (!(in_giant(q[k].z) & in_giant(q[k].w))) { UF::unite(parent, q[k].z, q[k].w, c); ++slow; }
        }
    }
    for (; i < n2; i += stride) {
        const u32x4 q = __builtin_nontemporal_load(e2 + i);
        if (!(in_giant(q.x) & in_giant(q.y))) { UF::unite(parent, q.x, q.y, c); ++slow; }
        if (!(in_giant(q.z) & in_giant(q.w))) { UF::unite(parent, q.z, q.w, c); ++slow; }
    }
    if (n_slow) atomicAdd(n_slow, (unsigned long long)slow);
}

static u32 hfind(std::vector<u32>& p, u32 x) {
    u32 r = x;
    while (p[r] != r) r = p[r];
    while (p[x] != r) {
        u32 n = p[x];
        p[x] = r;
        x = n;
    }
    return r;
}

int main(int argc, char** argv) {
    const int scale = argc > 1 ? atoi(argv[1]) : 20;
    const u64 E = 16ull << scale;
    const u32 V = 1u << scale;
    gcc_gen_params prm = {GCC_GEN_RMAT, (uint32_t)scale, 0, E, 0x67656C6C79000002ull, 0, 0, 1, 0};
    uint2* d_e;
    u32 *d_p, *d_l, *d_g;
    unsigned long long *d_bits, *d_slow;
    const u32 nwords = (V + 63) / 64;
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMalloc(&d_p, V * 4));
    CK(hipMalloc(&d_l, V * 4));
    CK(hipMalloc(&d_g, 4));
    CK(hipMalloc(&d_bits, nwords * 8));
    CK(hipMalloc(&d_slow, 8));
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, 0, prm, E, d_e);
    CK(hipDeviceSynchronize());
    std::vector<uint2> h_e(E);
    CK(hipMemcpy(h_e.data(), d_e, E * 8, hipMemcpyDeviceToHost));
    std::vector<u32> hp(V, UINT32_MAX), want(V);
    for (u64 i = 0; i < E; ++i) {
        u32 a = h_e[i].x, b = h_e[i].y;
        if (hp[a] == UINT32_MAX) hp[a] = a;
        if (hp[b] == UINT32_MAX) hp[b] = b;
        u32 ra = hfind(hp, a), rb = hfind(hp, b);
        if (ra < rb) hp[rb] = ra;
        else if (rb < ra) hp[ra] = rb;
    }
    for (u32 v = 0; v < V; ++v) want[v] = hp[v] == UINT32_MAX ? UINT32_MAX : hfind(hp, v);

    const int NEV = 16;
    hipEvent_t ev[NEV];
    for (auto& x : ev) CK(hipEventCreate(&x));
    std::vector<u32> got(V);
    CK(hipFuncSetAttribute((const void*)fold_filtered<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, nwords * 8));
    CK(hipFuncSetAttribute((const void*)fold_filtered<512>, hipFuncAttributeMaxDynamicSharedMemorySize, nwords * 8));
    // sample plans: geometric prefix end points (fraction of E); then filtered rounds (fraction end points)
    struct Plan {
        const char* name;
        std::vector<double> sample;
        std::vector<double> rounds;
        int block;
    };
    std::vector<Plan> plans = {
        {"S[1/1024..1/16]x4 F[1]", {1. / 1024, 1. / 256, 1. / 64, 1. / 16}, {1.}, 1024},
        {"S[1/1024..1/16]x4 F[1/4,1]", {1. / 1024, 1. / 256, 1. / 64, 1. / 16}, {1. / 4, 1.}, 1024},
        {"S[1/4096..1/64]x4 F[1/16,1/4,1]", {1. / 4096, 1. / 1024, 1. / 256, 1. / 64}, {1. / 16, 1. / 4, 1.}, 1024},
        {"S[1/1024..1/64]x4 F[1/8,1]", {1. / 1024, 1. / 256, 1. / 64}, {1. / 8, 1.}, 1024},
        {"S[1/1024..1/64]x4 F[1/8,1] b512", {1. / 1024, 1. / 256, 1. / 64}, {1. / 8, 1.}, 512},
    };
    for (auto& pl : plans) {
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemset(d_p, 0xFF, V * 4));
            CK(hipMemset(d_slow, 0, 8));
            u32 *par = d_p, *lab = d_l;
            int k = 0;
            CK(hipEventRecord(ev[k++]));
            u64 b = 0;
            for (double f : pl.sample) {
                const u64 e = (u64)(E * f);
                hipLaunchKernelGGL(fold_base, dim3((unsigned)std::min<u64>(2048, (e - b + 255) / 256)), dim3(256), 0, 0, par,
                                   d_e + b, e - b);
                b = e;
            }
            CK(hipEventRecord(ev[k++]));  // end of sample
            for (double f : pl.rounds) {
                hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, par, lab, V);
                std::swap(par, lab);
                hipLaunchKernelGGL(giant_vote, dim3(1), dim3(256), 0, 0, par, V, d_g);
                hipLaunchKernelGGL(giant_bits, dim3(1024), dim3(256), 0, 0, par, V, d_g, d_bits);
                CK(hipEventRecord(ev[k++]));
                const u64 e = (u64)(E * f);
                // b is even (all fractions are multiples of 2 edges at these sizes)
                if (pl.block == 1024)
                    hipLaunchKernelGGL(fold_filtered<1024>, dim3(256), dim3(1024), nwords * 8, 0, par,
                                       reinterpret_cast<const u32x4*>(d_e + b), (e - b) / 2, d_bits, nwords, d_slow);
                else
                    hipLaunchKernelGGL(fold_filtered<512>, dim3(256), dim3(512), nwords * 8, 0, par,
                                       reinterpret_cast<const u32x4*>(d_e + b), (e - b) / 2, d_bits, nwords, d_slow);
                CK(hipEventRecord(ev[k++]));
                b = e;
            }
            hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, par, lab, V);
            std::swap(par, lab);
            CK(hipEventRecord(ev[k++]));
            CK(hipEventSynchronize(ev[k - 1]));
            CK(hipMemcpy(got.data(), par, V * 4, hipMemcpyDeviceToHost));
            unsigned long long slow;
            CK(hipMemcpy(&slow, d_slow, 8, hipMemcpyDeviceToHost));
            float tot, ph;
            CK(hipEventElapsedTime(&tot, ev[0], ev[k - 1]));
            printf("%-34s total %.3f ms (%.1f Gedge/s) slow-path edges %.2f%% %s |", pl.name, tot, E / tot / 1e6,
                   100.0 * slow / E, got == want ? "OK" : "BAD");
            for (int j = 1; j < k; ++j) {
                CK(hipEventElapsedTime(&ph, ev[j - 1], ev[j]));
                printf(" %.3f", ph);
            }
            printf("\n");
            fflush(stdout);
        }
    }
    return 0;
}
