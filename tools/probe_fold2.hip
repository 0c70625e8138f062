// probe_fold2.hip — second measurement probe for the fold on C2 (R-MAT s20, 16M edges): where does the time go?
//  A baseline single launch; B the same stream folded again into the compressed forest (steady-state cost, no
//  hooks); C identity-initialised parents + a byte seen-map written with plain idempotent stores (no makeSet
//  CAS); D geometric chunking (small first launches, compress between); E max CAS per thread (the tail).
// Not product code. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc
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

__global__ __launch_bounds__(256) void fold_base(u32* parent, const uint2* e, u64 n, unsigned* maxcas) {
    Count c;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 x = __builtin_nontemporal_load(reinterpret_cast<const u64*>(e) + i);
        UnionFind<LoadPlain, true, Count>::unite(parent, (u32)x, (u32)(x >> 32), c);
    }
    if (maxcas) atomicMax(maxcas, c.n_cas);
}

// C: parent initialised to identity; seen[] bytes set with plain stores; hook CAS only
__device__ __forceinline__ void unite_id(u32* parent, unsigned char* seen, u32 u, u32 v) {
    if (!seen[u]) seen[u] = 1;
    if (!seen[v]) seen[v] = 1;
    NoCount c;
    const u32 pu = parent[u], pv = parent[v];
    if (pu == pv) return;
    u32 ru = UnionFind<LoadPlain, true>::find_from(parent, u, pu, c);
    u32 rv = UnionFind<LoadPlain, true>::find_from(parent, v, pv, c);
    while (ru != rv) {
        const u32 lo = min(ru, rv), hi = max(ru, rv);
        const u32 old = atomicCAS(&parent[hi], hi, lo);
        if (old == hi) return;
        ru = UnionFind<LoadPlain, true>::find_from(parent, hi, old, c);
        rv = UnionFind<LoadPlain, true>::find_from(parent, lo, parent[lo], c);
    }
}
__global__ __launch_bounds__(256) void fold_id(u32* parent, unsigned char* seen, const uint2* e, u64 n) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 x = __builtin_nontemporal_load(reinterpret_cast<const u64*>(e) + i);
        unite_id(parent, seen, (u32)x, (u32)(x >> 32));
    }
}
__global__ void init_id(u32* parent, unsigned char* seen, u32 n) {
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        parent[v] = v;
        seen[v] = 0;
    }
}
__global__ void compress_id(u32* parent, const unsigned char* seen, u32* labels, u32 n) {
    NoCount c;
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        const u32 r = (p >= v) ? p : UnionFind<LoadPlain, true>::find_from(parent, v, p, c);
        labels[v] = seen[v] ? r : 0xFFFFFFFFu;
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

int main(int argc, char** argv) {
    const int scale = argc > 1 ? atoi(argv[1]) : 20;
    const u64 E = 16ull << scale;
    const u32 V = 1u << scale;
    gcc_gen_params prm = {GCC_GEN_RMAT, (uint32_t)scale, 0, E, 0x67656C6C79000002ull, 0, 0, 1, 0};
    uint2* d_e;
    u32 *d_p, *d_l;
    unsigned char* d_seen;
    unsigned* d_max;
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMalloc(&d_p, V * 4));
    CK(hipMalloc(&d_l, V * 4));
    CK(hipMalloc(&d_seen, V));
    CK(hipMalloc(&d_max, 4));
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
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    std::vector<u32> got(V);
    auto ms = [&]() {
        float m;
        CK(hipEventSynchronize(t1));
        CK(hipEventElapsedTime(&m, t0, t1));
        return m;
    };
    const int reps = 5;
    // A + B + E
    for (int r = 0; r < reps; ++r) {
        CK(hipMemset(d_p, 0xFF, V * 4));
        CK(hipMemset(d_max, 0, 4));
        CK(hipEventRecord(t0));
        hipLaunchKernelGGL(fold_base, dim3(2048), dim3(256), 0, 0, d_p, d_e, E, d_max);
        CK(hipEventRecord(t1));
        float a = ms();
        unsigned mx;
        CK(hipMemcpy(&mx, d_max, 4, hipMemcpyDeviceToHost));
        hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, d_p, d_l, V);
        CK(hipEventRecord(t0));
        hipLaunchKernelGGL(fold_base, dim3(2048), dim3(256), 0, 0, d_l, d_e, E, (unsigned*)nullptr);
        CK(hipEventRecord(t1));
        float b = ms();
        hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, d_l, d_p, V);
        CK(hipMemcpy(got.data(), d_p, V * 4, hipMemcpyDeviceToHost));
        printf("A single launch %.3f ms (max CAS/thread %u) | B refold compressed %.3f ms (%.1f Gedge/s) %s\n", a, mx, b,
               E / b / 1e6, got == want ? "OK" : "BAD");
    }
    // C
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(init_id, dim3(1024), dim3(256), 0, 0, d_p, d_seen, V);
        CK(hipEventRecord(t0));
        hipLaunchKernelGGL(fold_id, dim3(2048), dim3(256), 0, 0, d_p, d_seen, d_e, E);
        CK(hipEventRecord(t1));
        float c = ms();
        hipLaunchKernelGGL(compress_id, dim3(1024), dim3(256), 0, 0, d_p, d_seen, d_l, V);
        CK(hipMemcpy(got.data(), d_l, V * 4, hipMemcpyDeviceToHost));
        printf("C identity+seen bytes %.3f ms %s\n", c, got == want ? "OK" : "BAD");
    }
    // D geometric chunks
    const double plans[][6] = {{1. / 1024, 1. / 256, 1. / 64, 1. / 16, 1. / 4, 1.}, {1. / 64, 1., 0, 0, 0, 0},
                               {1. / 256, 1. / 16, 1., 0, 0, 0}, {1. / 16, 1., 0, 0, 0, 0}};
    for (auto& plan : plans) {
        for (int r = 0; r < 3; ++r) {
            CK(hipMemset(d_p, 0xFF, V * 4));
            u32 *par = d_p, *lab = d_l;
            CK(hipEventRecord(t0));
            u64 b = 0;
            int nch = 0;
            for (int k = 0; k < 6 && plan[k] > 0; ++k) {
                const u64 e = (u64)(E * plan[k]);
                hipLaunchKernelGGL(fold_base, dim3((unsigned)std::min<u64>(2048, (e - b + 255) / 256)), dim3(256), 0, 0, par,
                                   d_e + b, e - b, (unsigned*)nullptr);
                hipLaunchKernelGGL(compress, dim3(1024), dim3(256), 0, 0, par, lab, V);
                std::swap(par, lab);
                b = e;
                ++nch;
            }
            CK(hipEventRecord(t1));
            float d = ms();
            CK(hipMemcpy(got.data(), par, V * 4, hipMemcpyDeviceToHost));
            printf("D geometric %d launches (incl. compress) %.3f ms %s\n", nch, d, got == want ? "OK" : "BAD");
        }
    }
    return 0;
}
