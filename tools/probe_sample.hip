// probe_sample.hip — what do the sampling launches of the fold pipeline wait on? Replays the C2 sampling
// prefix (launches of 4K, 16K, 64K, 256K, 184K edges on an empty forest) under variants and reports per-launch
// time and per-edge CAS / failed CAS / find steps / stores, plus the worst thread. Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc probe_sample.hip
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

__global__ void gen(gcc_gen_params p, u64 n, uint2* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u32 a, b;
        gcc_gen_edge(&p, i, &a, &b);
        out[i] = make_uint2(a, b);
    }
}

struct Ctr {
    unsigned long long cas, fail, step, store;
    unsigned maxcas, maxstep;
};

template <class L, bool SPLIT, int EPT>
__global__ __launch_bounds__(256) void fold(u32* parent, const u64* e, u64 n, Ctr* ctr) {
    Count c;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 x = __builtin_nontemporal_load(e + i);
        UnionFind<L, SPLIT, Count>::unite(parent, (u32)x, (u32)(x >> 32), c);
    }
    atomicAdd(&ctr->cas, (unsigned long long)c.n_cas);
    atomicAdd(&ctr->fail, (unsigned long long)c.n_fail);
    atomicAdd(&ctr->step, (unsigned long long)c.n_step);
    atomicAdd(&ctr->store, (unsigned long long)c.n_store);
    atomicMax(&ctr->maxcas, c.n_cas);
    atomicMax(&ctr->maxstep, c.n_step);
}

typedef void (*Fn)(u32*, const u64*, u64, Ctr*);

int main() {
    const int scale = 20;
    const u64 E = 16ull << scale;
    const u32 V = 1u << scale;
    gcc_gen_params prm = {GCC_GEN_RMAT, (uint32_t)scale, 0, E, 0x67656C6C79000002ull, 0, 0, 1, 0};
    uint2* d_e;
    u32* d_p;
    Ctr* d_c;
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMalloc(&d_p, V * 4));
    CK(hipMalloc(&d_c, sizeof(Ctr)));
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, 0, prm, E, d_e);
    CK(hipDeviceSynchronize());
    struct V_ {
        const char* name;
        Fn fn;
        unsigned grid_cap;
    } vars[] = {
        {"plain split", fold<LoadPlain, true, 1>, 2048},
        {"plain nosplit", fold<LoadPlain, false, 1>, 2048},
        {"agent split", fold<LoadAgent, true, 1>, 2048},
        {"plain split grid<=256", fold<LoadPlain, true, 1>, 256},
        {"plain split grid<=64", fold<LoadPlain, true, 1>, 64},
    };
    const u64 plan[] = {4096, 16384, 65536, 262144, 176128};
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vars) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipMemset(d_p, 0xFF, V * 4));
            u64 off = 0;
            printf("%-22s", v.name);
            float tot = 0;
            for (u64 n : plan) {
                CK(hipMemset(d_c, 0, sizeof(Ctr)));
                unsigned grid = (unsigned)std::min<u64>(v.grid_cap, (n + 255) / 256);
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(v.fn, dim3(grid), dim3(256), 0, 0, d_p, reinterpret_cast<const u64*>(d_e + off), n, d_c);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                tot += ms;
                Ctr h;
                CK(hipMemcpy(&h, d_c, sizeof h, hipMemcpyDeviceToHost));
                printf(" | %6.1fus cas %.2f fail %.2f step %.2f st %.2f maxcas %u maxstep %u", ms * 1e3, h.cas / (double)n,
                       h.fail / (double)n, h.step / (double)n, h.store / (double)n, h.maxcas, h.maxstep);
                off += n;
            }
            printf(" | total %.1f us\n", tot * 1e3);
            fflush(stdout);
        }
    }
    return 0;
}
