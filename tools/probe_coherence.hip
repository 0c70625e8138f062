// probe_coherence.hip — experiment: which cross-kernel visibility form does the fold -> compress hand-off need
// on gfx950? Replays the adversarial p10 fixture stream window by window (fold kernel with ONE block, then the
// multi-block compress kernel) under several memory-access variants and counts windows whose labels differ
// from a sequential host union-find. Build: hipcc --offload-arch=gfx950 -O3 -I../include -I../gelly-streaming_amd/csrc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "edge_gen.h"
#include "gelly_cc.h"

typedef uint32_t u32;
#define UNSEEN 0xFFFFFFFFu
#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);       \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

template <int LD>
__device__ __forceinline__ u32 ld(u32* p) {
    if constexpr (LD == 0) return *p;
    else if constexpr (LD == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int LD, int CAS_SYS>
__device__ __forceinline__ u32 cas(u32* p, u32 e, u32 d) {
    if constexpr (CAS_SYS) {
        __hip_atomic_compare_exchange_strong(p, &e, d, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return e;
    } else {
        return atomicCAS(p, e, d);
    }
}

template <int LD>
__device__ __forceinline__ u32 find_from(u32* parent, u32 x, u32 p) {
    if (p >= x) return x;
    u32 prev = x, cur = p;
    while (true) {
        const u32 next = ld<LD>(&parent[cur]);
        if (next >= cur) break;
        parent[prev] = next;
        prev = cur;
        cur = next;
    }
    return cur;
}

template <int LD, int CAS_SYS>
__device__ void unite(u32* parent, u32 u, u32 v) {
    u32 pu = ld<LD>(&parent[u]);
    if (pu == UNSEEN) {
        u32 o = cas<LD, CAS_SYS>(&parent[u], UNSEEN, u);
        pu = o == UNSEEN ? u : o;
    }
    if (u == v) return;
    u32 pv = ld<LD>(&parent[v]);
    if (pv == UNSEEN) {
        u32 o = cas<LD, CAS_SYS>(&parent[v], UNSEEN, v);
        pv = o == UNSEEN ? v : o;
    }
    u32 ru = find_from<LD>(parent, u, pu), rv = find_from<LD>(parent, v, pv);
    while (ru != rv) {
        u32 lo = ru < rv ? ru : rv, hi = ru < rv ? rv : ru;
        u32 old = cas<LD, CAS_SYS>(&parent[hi], hi, lo);
        if (old == hi) return;
        ru = find_from<LD>(parent, hi, old);
        rv = find_from<LD>(parent, lo, ld<LD>(&parent[lo]));
    }
}

template <int LD, int CAS_SYS, int REL>
__global__ void fold(u32* parent, const uint2* e, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) unite<LD, CAS_SYS>(parent, e[i].x, e[i].y);
    if (REL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

template <int LD, int ACQ>
__global__ void compress(u32* parent, u32 n) {
    if (ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        u32 p = ld<LD>(&parent[v]);
        if (p >= v) continue;
        u32 r = find_from<LD>(parent, v, p);
        if (r != p) parent[v] = r;
    }
}

// host sequential union-find (min-id roots)
static u32 hfind(std::vector<u32>& p, u32 x) {
    while (p[x] != x) x = p[x];
    return x;
}

struct Variant {
    const char* name;
    void (*fold)(u32*, const uint2*, int);
    void (*comp)(u32*, u32);
};

int main(int argc, char** argv) {
    int reps = argc > 1 ? atoi(argv[1]) : 30;
    gcc_gen_params prm = {GCC_GEN_ADVERSARIAL, 10, 0, 0, 0x67656C6C79000005ull, 8, 128, 0, 0};
    const int E = (int)gcc_gen_num_edges(&prm);
    const u32 V = (u32)gcc_gen_num_vertices(&prm);
    std::vector<uint2> edges(E);
    for (int i = 0; i < E; ++i) gcc_gen_edge(&prm, i, &edges[i].x, &edges[i].y);
    const int W = 256;
    const int nw = (E + W - 1) / W;
    // expected labels per window
    std::vector<std::vector<u32>> want(nw);
    {
        std::vector<u32> p(V, UNSEEN);
        for (int w = 0; w < nw; ++w) {
            for (int i = w * W; i < std::min(E, (w + 1) * W); ++i) {
                u32 a = edges[i].x, b = edges[i].y;
                if (p[a] == UNSEEN) p[a] = a;
                if (p[b] == UNSEEN) p[b] = b;
                u32 ra = hfind(p, a), rb = hfind(p, b);
                if (ra < rb) p[rb] = ra;
                else if (rb < ra) p[ra] = rb;
            }
            want[w].resize(V);
            for (u32 v = 0; v < V; ++v) want[w][v] = p[v] == UNSEEN ? UNSEEN : hfind(p, v);
        }
    }
    u32* d_par;
    uint2* d_e;
    CK(hipMalloc(&d_par, V * 4));
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMemcpy(d_e, edges.data(), E * 8, hipMemcpyHostToDevice));
    Variant vs[] = {
        {"baseline (plain loads, agent CAS)", fold<0, 0, 0>, compress<0, 0>},
        {"compress: agent acquire fence at start", fold<0, 0, 0>, compress<0, 1>},
        {"compress: agent-scope (sc1) loads", fold<0, 0, 0>, compress<1, 0>},
        {"compress: system-scope loads", fold<0, 0, 0>, compress<2, 0>},
        {"fold: agent release fence at end", fold<0, 0, 1>, compress<0, 0>},
        {"fold: system-scope CAS", fold<0, 1, 0>, compress<0, 0>},
        {"fold: release fence + compress: acquire fence", fold<0, 0, 1>, compress<0, 1>},
        {"fold+compress: agent-scope (sc1) loads", fold<1, 0, 0>, compress<1, 0>},
    };
    std::vector<u32> got(V);
    for (auto& var : vs) {
        int bad = 0, total = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(d_par, 0xFF, V * 4));
            for (int w = 0; w < nw; ++w) {
                int b = w * W, n = std::min(E, (w + 1) * W) - b;
                hipLaunchKernelGGL(var.fold, dim3(1), dim3(256), 0, 0, d_par, d_e + b, n);
                hipLaunchKernelGGL(var.comp, dim3((V + 255) / 256), dim3(256), 0, 0, d_par, V);
                CK(hipMemcpy(got.data(), d_par, V * 4, hipMemcpyDeviceToHost));
                bad += got != want[w];
                ++total;
            }
        }
        printf("%-50s bad windows %d / %d\n", var.name, bad, total);
    }
    // same, without the per-window D2H (only final labels compared)
    for (auto& var : vs) {
        int bad = 0;
        for (int r = 0; r < reps; ++r) {
            CK(hipMemset(d_par, 0xFF, V * 4));
            for (int w = 0; w < nw; ++w) {
                int b = w * W, n = std::min(E, (w + 1) * W) - b;
                hipLaunchKernelGGL(var.fold, dim3(1), dim3(256), 0, 0, d_par, d_e + b, n);
                hipLaunchKernelGGL(var.comp, dim3((V + 255) / 256), dim3(256), 0, 0, d_par, V);
            }
            CK(hipMemcpy(got.data(), d_par, V * 4, hipMemcpyDeviceToHost));
            bad += got != want[nw - 1];
        }
        printf("[no D2H between windows] %-40s bad runs %d / %d\n", var.name, bad, reps);
    }
    return 0;
}
