// probe_fold.hip — measurement probe for the fold kernel on the C2 workload (R-MAT scale 20, 16M edges).
// Times fold variants (load scope, path splitting, chunked launches with a compress between chunks,
// block size / edges per lane) with hipEvents, counts CAS / find steps / stores per edge, and checks every
// variant's labels against a sequential host union-find. Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc probe_fold.hip
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

struct Counters {
    unsigned long long cas, fail, step, store;
};

template <class L, bool SPLIT, bool COUNT>
__global__ __launch_bounds__(256) void fold(u32* parent, const uint2* e, u64 n, Counters* ctr) {
    using C = typename std::conditional<COUNT, Count, NoCount>::type;
    C c;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 x = __builtin_nontemporal_load(reinterpret_cast<const u64*>(e) + i);
        UnionFind<L, SPLIT, C>::unite(parent, (u32)x, (u32)(x >> 32), c);
    }
    if constexpr (COUNT) {
        atomicAdd(&ctr->cas, (unsigned long long)c.n_cas);
        atomicAdd(&ctr->fail, (unsigned long long)c.n_fail);
        atomicAdd(&ctr->step, (unsigned long long)c.n_step);
        atomicAdd(&ctr->store, (unsigned long long)c.n_store);
    }
}

__global__ __launch_bounds__(256) void compress(u32* parent, u32* labels, u32 n) {
    NoCount c;
    for (u64 v = blockIdx.x * (u64)blockDim.x + threadIdx.x; v < n; v += (u64)gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        labels[v] = (p >= v) ? p : UnionFind<LoadPlain, true>::find_from(parent, (u32)v, p, c);
    }
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

typedef void (*FoldFn)(u32*, const uint2*, u64, Counters*);

int main(int argc, char** argv) {
    const int scale = argc > 1 ? atoi(argv[1]) : 20;
    const u64 E = 16ull << scale;
    const u32 V = 1u << scale;
    gcc_gen_params prm = {GCC_GEN_RMAT, (uint32_t)scale, 0, E, 0x67656C6C79000002ull, 0, 0, 1, 0};
    uint2* d_e;
    u32 *d_p, *d_l;
    Counters* d_c;
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMalloc(&d_p, V * 4));
    CK(hipMalloc(&d_l, V * 4));
    CK(hipMalloc(&d_c, sizeof(Counters)));
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, 0, prm, E, d_e);
    CK(hipDeviceSynchronize());
    // expected labels on the host
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

    struct Var {
        const char* name;
        FoldFn fn, cnt;
    } vars[] = {
        {"plain  split", fold<LoadPlain, true, false>, fold<LoadPlain, true, true>},
        {"plain  nosplit", fold<LoadPlain, false, false>, fold<LoadPlain, false, true>},
        {"agent  split", fold<LoadAgent, true, false>, fold<LoadAgent, true, true>},
        {"agent  nosplit", fold<LoadAgent, false, false>, fold<LoadAgent, false, true>},
        {"system split", fold<LoadSystem, true, false>, fold<LoadSystem, true, true>},
    };
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    std::vector<u32> got(V);
    const int chunks_list[] = {1, 4, 16, 64};
    const unsigned grids[] = {2048, 8192};
    for (auto& var : vars) {
        for (int chunks : chunks_list) {
            for (unsigned grid : grids) {
                float best = 1e30f, sum = 0.f;
                bool ok = true;
                const int reps = 5;
                for (int r = 0; r < reps; ++r) {
                    CK(hipMemset(d_p, 0xFF, V * 4));
                    CK(hipEventRecord(t0));
                    u32 *par = d_p, *lab = d_l;
                    for (int c = 0; c < chunks; ++c) {
                        const u64 b = E * c / chunks, e = E * (c + 1) / chunks;
                        hipLaunchKernelGGL(var.fn, dim3(grid), dim3(256), 0, 0, par, d_e + b, e - b, d_c);
                        if (c + 1 < chunks) {
                            hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, par, lab, V);
                            std::swap(par, lab);
                        }
                    }
                    CK(hipEventRecord(t1));
                    hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, par, lab, V);
                    CK(hipMemcpy(got.data(), lab, V * 4, hipMemcpyDeviceToHost));
                    float ms;
                    CK(hipEventElapsedTime(&ms, t0, t1));
                    best = std::min(best, ms);
                    sum += ms;
                    ok &= (got == want);
                }
                // counters (single-chunk only)
                Counters hc = {0, 0, 0, 0};
                if (chunks == 1) {
                    CK(hipMemset(d_p, 0xFF, V * 4));
                    CK(hipMemset(d_c, 0, sizeof(Counters)));
                    hipLaunchKernelGGL(var.cnt, dim3(grid), dim3(256), 0, 0, d_p, d_e, E, d_c);
                    CK(hipMemcpy(&hc, d_c, sizeof hc, hipMemcpyDeviceToHost));
                }
                printf("%-16s chunks %3d grid %5u: best %8.3f ms avg %8.3f ms  %7.2f Gedge/s  %s", var.name, chunks, grid,
                       best, sum / reps, E / best / 1e6, ok ? "OK " : "BAD");
                if (chunks == 1)
                    printf("  per-edge cas %.3f fail %.3f steps %.3f stores %.3f", hc.cas / (double)E,
                           hc.fail / (double)E, hc.step / (double)E, hc.store / (double)E);
                printf("\n");
                fflush(stdout);
            }
        }
    }
    return 0;
}
