// probe_stream.hip — where does the time of the LDS-bitmap edge stream go? (seed_bfs / fold_filtered share it)
// Not product code. Times, on C2's 16M R-MAT edges (128 MiB), kernels that add one ingredient at a time:
//   copy     : stream the edges, fold them into a checksum (the HBM floor for this access pattern)
//   fill     : + copy a 128 KiB bitmap into LDS first (1024-thread block per CU)
//   lookup   : + two LDS bitmap lookups per edge (count edges with both ends set)
//   visit    : + the BFS discovery (LDS atomicOr + flag byte store) on a bitmap of density `dens`
// for blocks of 1024 threads x 1 per CU and 512 x 2 per CU (64 KiB bitmaps can't be shared, so the 512 variant
// uses half the bitmap: timing only), and loads in flight per lane D = 4 / 8.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc probe_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "edge_gen.h"
#include "gelly_cc.h"

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
typedef uint8_t u8;
typedef u32 u32x4 __attribute__((ext_vector_type(4)));

__global__ void gen(gcc_gen_params p, u64 n, uint2* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u32 a, b;
        gcc_gen_edge(&p, i, &a, &b);
        out[i] = make_uint2(a, b);
    }
}

enum Mode { COPY = 0, FILL = 1, LOOKUP = 2, VISIT = 3, V_NORTN = 4, V_ATOMIC = 5, V_STORE = 6, V_LDSMARK = 7, V_LOADFIRST = 8 };

template <int BLOCK, int D, int MODE>
__global__ __launch_bounds__(BLOCK) void stream_kernel(const u32x4* __restrict__ body, u64 n2, const u32* __restrict__ bits,
                                                       u32 nwords32, u8* __restrict__ flags, u32* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) u32 s_bm[];
    const u64 stride = (u64)gridDim.x * BLOCK;
    const u64 i = (u64)blockIdx.x * BLOCK + threadIdx.x;
    const u64 cnt = i < n2 ? (n2 - 1 - i) / stride + 1 : 0;
    u32x4 q[D];
#pragma unroll
    for (int k = 0; k < D; ++k)
        if ((u64)k < cnt) q[k] = __builtin_nontemporal_load(body + i + k * stride);
    if (MODE >= FILL) {
        const u32x4* src = reinterpret_cast<const u32x4*>(bits);
        u32x4* dst = reinterpret_cast<u32x4*>(s_bm);
        for (u32 w = threadIdx.x; w < nwords32 / 4; w += BLOCK) dst[w] = src[w];
        __syncthreads();
    }
    const u32 mask = nwords32 * 32 - 1;  // nwords32 is a power of two here
    u32 acc = 0;
    auto visit = [&](u32 a, u32 b) {
        if (MODE <= FILL) {
            acc += a ^ b;
            return;
        }
        a &= mask;
        b &= mask;
        const u32 ia = (s_bm[a >> 5] >> (a & 31)) & 1u, ib = (s_bm[b >> 5] >> (b & 31)) & 1u;
        if (MODE == LOOKUP) {
            acc += ia & ib;
            return;
        }
        if (ia != ib) {
            const u32 x = ia ? b : a, m = 1u << (x & 31);
            if (MODE == VISIT) {  // returning LDS atomic (in-block dedup) + flag byte store
                if (!(atomicOr(&s_bm[x >> 5], m) & m)) {
                    flags[x] = 1;
                    acc += 1;
                }
            } else if (MODE == V_NORTN) {  // non-returning LDS atomic + unconditional flag store
                __hip_atomic_fetch_or(&s_bm[x >> 5], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                flags[x] = 1;
            } else if (MODE == V_ATOMIC) {  // returning LDS atomic only
                acc += (atomicOr(&s_bm[x >> 5], m) & m) ? 0 : 1;
            } else if (MODE == V_STORE) {  // flag store only
                flags[x] = 1;
            } else {  // V_LDSMARK: plain LDS read-modify-write (racy: lost bits only delay discovery) + store
                s_bm[x >> 5] |= m;
                flags[x] = 1;
            }
        }
    };
    for (u64 r = 0; r < cnt; r += D) {
        u32x4 nq[D];
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (r + D + k < cnt) nq[k] = __builtin_nontemporal_load(body + i + (r + D + k) * stride);
        if constexpr (MODE == V_LOADFIRST) {
            // phase A: LDS lookups + block dedup -> up to 2D candidates; B: their flag loads, all in flight;
            // C: store only the ones still 0
            u32 cand[2 * D];
#pragma unroll
            for (int k = 0; k < D; ++k) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    u32 a = (h ? q[k].z : q[k].x) & mask, b = (h ? q[k].w : q[k].y) & mask;
                    u32 c = 0xFFFFFFFFu;
                    if (r + k < cnt) {
                        const u32 ia = (s_bm[a >> 5] >> (a & 31)) & 1u, ib = (s_bm[b >> 5] >> (b & 31)) & 1u;
                        if (ia != ib) {
                            const u32 x = ia ? b : a, m = 1u << (x & 31);
                            if (!(atomicOr(&s_bm[x >> 5], m) & m)) c = x;
                        }
                    }
                    cand[2 * k + h] = c;
                }
            }
            u8 f[2 * D];
#pragma unroll
            for (int j = 0; j < 2 * D; ++j) f[j] = cand[j] != 0xFFFFFFFFu ? flags[cand[j]] : (u8)1;
#pragma unroll
            for (int j = 0; j < 2 * D; ++j)
                if (!f[j]) {
                    flags[cand[j]] = 1;
                    acc += 1;
                }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k)
                if (r + k < cnt) {
                    visit(q[k].x, q[k].y);
                    visit(q[k].z, q[k].w);
                }
        }
#pragma unroll
        for (int k = 0; k < D; ++k) q[k] = nq[k];
    }
    if (acc == 0xFFFFFFFF) out[0] = acc;  // keep the work
}

template <int BLOCK, int D, int MODE>
float run(const u32x4* body, u64 n2, const u32* bits, u32 nw32, u8* flags, u32* out, int blocks_per_cu, int ncu) {
    const size_t lds = (MODE >= FILL) ? (size_t)nw32 * 4 : 0;
    CK(hipFuncSetAttribute((const void*)stream_kernel<BLOCK, D, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                           (int)lds));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e9;
    for (int rep = 0; rep < 7; ++rep) {
        CK(hipMemset(flags, 0, 1 << 20));
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((stream_kernel<BLOCK, D, MODE>), dim3(ncu * blocks_per_cu), dim3(BLOCK), lds, 0, body, n2,
                           bits, nw32, flags, out);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (rep > 0 && ms < best) best = ms;
    }
    return best;
}

int main() {
    gcc_gen_params p{};
    p.kind = GCC_GEN_RMAT;
    p.scale = 20;
    p.n_edges = 1ull << 24;
    p.seed = 0x67656C6C79000002ull;
    p.permute = 1;
    const u64 E = p.n_edges, n2 = E / 2;
    uint2* d_e;
    CK(hipMalloc(&d_e, E * 8));
    hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, p, E, d_e);
    u32 *bits, *out;
    u8* flags;
    const u32 nw32 = (1u << 20) / 32;  // 128 KiB
    CK(hipMalloc(&bits, nw32 * 4));
    CK(hipMalloc(&flags, 1 << 20));
    CK(hipMalloc(&out, 64));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<u32> hb(nw32);
    for (double dens : {0.0, 0.2, 0.6, 0.98}) {
        srand(7);
        for (u32 w = 0; w < nw32; ++w) {
            u32 x = 0;
            for (int b = 0; b < 32; ++b) x |= ((rand() / (double)RAND_MAX) < dens ? 1u : 0u) << b;
            hb[w] = x;
        }
        CK(hipMemcpy(bits, hb.data(), nw32 * 4, hipMemcpyHostToDevice));
        const u32x4* body = reinterpret_cast<const u32x4*>(d_e);
        const double gb = E * 8.0 / 1e9;
        auto rep = [&](const char* name, float ms) {
            printf("dens %.2f %-28s %7.1f us  %6.2f TB/s of edges\n", dens, name, ms * 1e3, gb / (ms * 1e-3) / 1e3);
        };
        if (dens == 0.0) {
            rep("copy  1024x1 D4", run<1024, 4, COPY>(body, n2, bits, nw32, flags, out, 1, ncu));
            rep("copy  1024x1 D8", run<1024, 8, COPY>(body, n2, bits, nw32, flags, out, 1, ncu));
            rep("copy  256x8 D4", run<256, 4, COPY>(body, n2, bits, nw32, flags, out, 8, ncu));
            rep("copy  256x8 D8", run<256, 8, COPY>(body, n2, bits, nw32, flags, out, 8, ncu));
            rep("fill  1024x1 D8", run<1024, 8, FILL>(body, n2, bits, nw32, flags, out, 1, ncu));
        }
        rep("lookup 1024x1 D4", run<1024, 4, LOOKUP>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("lookup 1024x1 D8", run<1024, 8, LOOKUP>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("visit 1024x1 D8", run<1024, 8, VISIT>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("visit 1024x1 D4", run<1024, 4, VISIT>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_nortn 1024x1 D4", run<1024, 4, V_NORTN>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_atomic-only 1024x1 D4", run<1024, 4, V_ATOMIC>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_store-only 1024x1 D4", run<1024, 4, V_STORE>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_ldsmark 1024x1 D4", run<1024, 4, V_LDSMARK>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_loadfirst 1024x1 D4", run<1024, 4, V_LOADFIRST>(body, n2, bits, nw32, flags, out, 1, ncu));
        rep("v_loadfirst 1024x1 D8", run<1024, 8, V_LOADFIRST>(body, n2, bits, nw32, flags, out, 1, ncu));
    }
    return 0;
}
