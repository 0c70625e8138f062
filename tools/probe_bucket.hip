// probe_bucket.hip — measurement probe (not product code): can 2-D bucketing of an edge batch turn C4's random
// giant-bitmap lookups (8 MiB bitmap, L2/MALL-bound) into LDS / XCD-local L2 lookups, and what does the bucketing
// pass itself cost? Streams the first N edges of C4 (Kronecker s26, V = 2^26) from HBM.
//   stream modes: 0 no lookup, 1 both ends in LDS (masked), 2 both ends in the global 8 MiB bitmap (round 1's
//   filtered kernel), 3 u in LDS + v in the global 8 MiB bitmap, 4 u in LDS + v in a 1 MiB region picked by the
//   block's XCD (HW_REG_XCC_ID), 5 v in a 1 MiB XCD region only.
//   partition: multi-split into NB = 64 (u-slices of 2^20 ids) or 512 (x 8 v-ranges) buckets, tile-local LDS sort.
// Build: hipcc -O3 --offload-arch=gfx950 -I../include -I../gelly-streaming_amd/csrc probe_bucket.hip -o probe_bucket
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "edge_gen.h"

typedef uint32_t u32;
typedef uint64_t u64;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void gen(gcc_gen_params p, u64 n, uint2* out) {
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (u64)gridDim.x * 256) {
        u32 a, b;
        gcc_gen_edge(&p, i, &a, &b);
        out[i] = make_uint2(a, b);
    }
}
__global__ void fill_bits(u32* bits, u64 nw) {
    for (u64 i = blockIdx.x * 256ull + threadIdx.x; i < nw; i += (u64)gridDim.x * 256)
        bits[i] = (u32)gcc_splitmix64(i * 7 + 1);
}

__device__ __forceinline__ u32 xcc_id() {
    u32 x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & 7;
}

constexpr int SB = 1024;
template <int MODE>
__global__ __launch_bounds__(SB) void stream_k(const u32x4* __restrict__ e, u64 n2, const u32* __restrict__ bits,
                                               u32* __restrict__ out) {
    extern __shared__ u32 s[];  // 128 KiB slice
    for (u32 w = threadIdx.x; w < 32768; w += SB) s[w] = bits[w];
    __syncthreads();
    const u32* reg = bits + (MODE >= 4 ? xcc_id() * (1u << 18) : 0);  // 1 MiB = 2^18 u32 words
    u32 acc = 0;
    const u64 stride = (u64)gridDim.x * SB;
    u64 i = blockIdx.x * (u64)SB + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
        u32x4 q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) q[k] = __builtin_nontemporal_load(e + i + k * stride);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u32 a[2] = {q[k].x, q[k].z}, b[2] = {q[k].y, q[k].w};
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                u32 ia = 0, ib = 0;
                if (MODE == 0) { ia = a[j]; ib = b[j]; }
                if (MODE == 1) { ia = s[(a[j] >> 5) & 32767] >> (a[j] & 31); ib = s[(b[j] >> 5) & 32767] >> (b[j] & 31); }
                if (MODE == 2) { ia = bits[a[j] >> 5] >> (a[j] & 31); ib = bits[b[j] >> 5] >> (b[j] & 31); }
                if (MODE == 3) { ia = s[(a[j] >> 5) & 32767] >> (a[j] & 31); ib = bits[b[j] >> 5] >> (b[j] & 31); }
                if (MODE == 4) { ia = s[(a[j] >> 5) & 32767] >> (a[j] & 31); ib = reg[(b[j] >> 5) & ((1u << 18) - 1)] >> (b[j] & 31); }
                if (MODE == 5) { ia = 1; ib = reg[(b[j] >> 5) & ((1u << 18) - 1)] >> (b[j] & 31); }
                acc += ia & ib & 1;
            }
        }
    }
    out[blockIdx.x * SB + threadIdx.x] = acc;
}

// multi-split: NB buckets, b = (u >> 20) * NXV + (v >> VSH) ; tile = BLOCK * PER edges sorted in LDS
template <int BLOCK, int PER>
__global__ __launch_bounds__(BLOCK) void part_k(const u64* __restrict__ e, u64 n, u32 nxv, u32 vsh, u32 nb,
                                                u64* __restrict__ out, u64 cap, u32* __restrict__ cursor,
                                                u32* __restrict__ ovf) {
    constexpr u32 T = BLOCK * PER;
    __shared__ u64 srt[T];
    __shared__ u32 s_cnt[1024], s_start[1024], s_g[1024];
    __shared__ u32 s_wsum[BLOCK / 64];
    const u64 ntiles = (n + T - 1) / T;
    for (u64 t = blockIdx.x; t < ntiles; t += gridDim.x) {
        for (u32 b = threadIdx.x; b < nb; b += BLOCK) s_cnt[b] = 0;
        __syncthreads();
        const u64 base = t * T;
        u64 ev[PER];
        u32 rk[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const u64 i = base + (u64)k * BLOCK + threadIdx.x;
            ev[k] = i < n ? __builtin_nontemporal_load(e + i) : ~0ull;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (ev[k] == ~0ull) continue;
            const u32 u = (u32)ev[k], v = (u32)(ev[k] >> 32);
            const u32 b = (u >> 20) * nxv + (v >> vsh);
            rk[k] = atomicAdd(&s_cnt[b], 1u);
        }
        __syncthreads();
        // exclusive scan of s_cnt (nb <= BLOCK * 2 handled as 2 per thread)
        const u32 per = (nb + BLOCK - 1) / BLOCK;
        u32 loc = 0;
        for (u32 j = 0; j < per; ++j) {
            const u32 b = threadIdx.x * per + j;
            loc += b < nb ? s_cnt[b] : 0;
        }
        u32 inc = loc;
        const u32 lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        for (int o = 1; o < 64; o <<= 1) {
            const u32 y = __shfl_up(inc, o, 64);
            if (lane >= (u32)o) inc += y;
        }
        if (lane == 63) s_wsum[wv] = inc;
        __syncthreads();
        u32 wbase = 0;
        for (u32 w = 0; w < wv; ++w) wbase += s_wsum[w];
        u32 run = wbase + inc - loc;
        for (u32 j = 0; j < per; ++j) {
            const u32 b = threadIdx.x * per + j;
            if (b < nb) {
                const u32 c = s_cnt[b];
                s_start[b] = run;
                run += c;
                s_g[b] = c ? atomicAdd(&cursor[b], c) : 0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            if (ev[k] == ~0ull) continue;
            const u32 u = (u32)ev[k], v = (u32)(ev[k] >> 32);
            const u32 b = (u >> 20) * nxv + (v >> vsh);
            srt[s_start[b] + rk[k]] = ev[k];
        }
        __syncthreads();
        const u32 m = (u32)min<u64>(T, n - base);
        for (u32 x = threadIdx.x; x < m; x += BLOCK) {
            const u64 ed = srt[x];
            const u32 u = (u32)ed, v = (u32)(ed >> 32);
            const u32 b = (u >> 20) * nxv + (v >> vsh);
            const u64 off = (u64)s_g[b] + (x - s_start[b]);
            if (off < cap) out[(u64)b * cap + off] = ed;
            else atomicAdd(ovf, 1u);
        }
        __syncthreads();
    }
}

int main(int argc, char** argv) {
    const u64 n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 28);
    const u32 V = 1u << 26;
    gcc_gen_params p = {GCC_GEN_RMAT, 26, 0, 16ull << 26, 0x67656C6C79000004ull, 0, 0, 1, 0};
    u64* d_e;
    u32 *d_bits, *d_out;
    CK(hipMalloc(&d_e, n * 8));
    CK(hipMalloc(&d_bits, V / 8));
    CK(hipMalloc(&d_out, 4u << 20));
    gen<<<8192, 256>>>(p, n, (uint2*)d_e);
    fill_bits<<<1024, 256>>>(d_bits, V / 32);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto launch, double bytes) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        printf("%-28s %8.3f ms  %7.1f G edges/s  %7.0f GB/s\n", name, best, n / best / 1e6, bytes / best / 1e6);
        fflush(stdout);
    };
    const u64 n2 = n / 2;
    const size_t lds = 128 << 10;
    CK(hipFuncSetAttribute((const void*)stream_k<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)stream_k<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)stream_k<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)stream_k<3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)stream_k<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CK(hipFuncSetAttribute((const void*)stream_k<5>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    const u32x4* e4 = (const u32x4*)d_e;
    timeit("stream, no lookup", [&] { stream_k<0><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    timeit("stream, u+v in LDS", [&] { stream_k<1><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    timeit("stream, u+v global 8MiB", [&] { stream_k<2><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    timeit("stream, u LDS, v global 8MiB", [&] { stream_k<3><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    timeit("stream, u LDS, v XCD 1MiB", [&] { stream_k<4><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    timeit("stream, v XCD 1MiB only", [&] { stream_k<5><<<256, SB, lds>>>(e4, n2, d_bits, d_out); }, n * 8.0);
    // partition
    for (u32 nxv : {1u, 8u}) {
        const u32 nb = 64 * nxv, vsh = nxv == 1 ? 26 : 23;
        const u64 cap = (n / nb) * 5 / 4 + 8192;
        u64* d_o;
        u32 *d_cur, *d_ovf;
        CK(hipMalloc(&d_o, cap * nb * 8));
        CK(hipMalloc(&d_cur, nb * 4));
        CK(hipMalloc(&d_ovf, 4));
        char nm[64];
        snprintf(nm, sizeof nm, "partition NB=%u 512x16", nb);
        timeit(nm, [&] {
            hipMemsetAsync(d_cur, 0, nb * 4);
            hipMemsetAsync(d_ovf, 0, 4);
            part_k<512, 16><<<512, 512>>>(d_e, n, nxv, vsh, nb, d_o, cap, d_cur, d_ovf);
        }, n * 16.0);
        snprintf(nm, sizeof nm, "partition NB=%u 256x32", nb);
        timeit(nm, [&] {
            hipMemsetAsync(d_cur, 0, nb * 4);
            hipMemsetAsync(d_ovf, 0, 4);
            part_k<256, 32><<<512, 256>>>(d_e, n, nxv, vsh, nb, d_o, cap, d_cur, d_ovf);
        }, n * 16.0);
        u32 ovf;
        CK(hipMemcpy(&ovf, d_ovf, 4, hipMemcpyDeviceToHost));
        printf("  overflow edges: %u\n", ovf);
        CK(hipFree(d_o));
        CK(hipFree(d_cur));
        CK(hipFree(d_ovf));
    }
    CK(hipMemcpy(d_out, d_out, 4, hipMemcpyDeviceToDevice));
    return 0;
}
