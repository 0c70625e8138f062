// probe_c3_bounds.hip — what bounds the plain fold of C3 (uniform G(n, m), n = 2^24, m = 9.2M, one fresh window)?
// Not product code. Measures, on the C3 stream resident in HBM:
//   reads2        two random parent[] reads per edge (the floor of any union-find fold)
//   store1        one random plain store per edge
//   reads2store1  both
//   amin1         one non-returning atomicMin per edge (memory-side atomic throughput)
//   cas1          one returning atomicCAS per edge, result used
//   base          the product's plain fold (UF::unite: makeSet CAS + CAS hooks), then the compress
//   plainhook     the candidate: hooks by PLAIN stores (K1, hook record per edge), then a verify kernel (K2) that
//                 re-checks every recorded hook and unites the lost ones with the CAS union; then the compress
// Every fold variant's labels are compared with a host union-find.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc probe_c3_bounds.hip
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
typedef UnionFind<LoadPlain, true> UFS;
typedef UnionFind<LoadPlain, false> UFR;
constexpr u32 UN = 0xFFFFFFFFu;

__global__ void gen(gcc_gen_params p, u64 n, uint2* out) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u32 a, b;
        gcc_gen_edge(&p, i, &a, &b);
        out[i] = make_uint2(a, b);
    }
}

#define EDGE_LOOP                                                                                    \
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) { \
        const u64 x = __builtin_nontemporal_load(reinterpret_cast<const u64*>(e) + i);              \
        const u32 a = (u32)x, b = (u32)(x >> 32);

__global__ __launch_bounds__(256) void k_reads2(const u32* p, const uint2* e, u64 n, u32* sink) {
    u32 acc = 0;
    EDGE_LOOP acc += p[a] ^ p[b]; }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_store1(u32* p, const uint2* e, u64 n) {
    EDGE_LOOP p[a > b ? a : b] = a < b ? a : b; }
}
__global__ __launch_bounds__(256) void k_reads2store1(u32* p, const uint2* e, u64 n) {
    EDGE_LOOP const u32 pa = p[a], pb = p[b];
              if (pa != pb) p[a > b ? a : b] = a < b ? a : b; }
}
__global__ __launch_bounds__(256) void k_amin1(u32* p, const uint2* e, u64 n) {
    EDGE_LOOP atomicMin(&p[a > b ? a : b], a < b ? a : b); }
}
__global__ __launch_bounds__(256) void k_cas1(u32* p, const uint2* e, u64 n, u32* sink) {
    u32 acc = 0;
    EDGE_LOOP const u32 hi = a > b ? a : b; acc += atomicCAS(&p[hi], hi, a < b ? a : b); }
    if (acc == 0x12345678u) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_base(u32* p, const uint2* e, u64 n) {
    NoCount c;
    EDGE_LOOP UFS::unite(p, a, b, c); }
}

// root of x from observed parent word w (UNSEEN or >= x: x is a root); returns the root and its observed word
template <bool SPLIT>
__device__ __forceinline__ u32 root_of(u32* p, u32 x, u32 w, u32& rw) {
    if (w >= x) {
        rw = w;
        return x;
    }
    u32 prev = x, cur = w;
    while (true) {
        const u32 nx = p[cur];
        if (nx >= cur) {
            rw = nx;
            return cur;
        }
        if (SPLIT) p[prev] = nx;
        prev = cur;
        cur = nx;
    }
}

// K1: hooks by plain stores; hook record per edge (hi, lo) or ~0
template <bool SPLIT>
__global__ __launch_bounds__(256) void k_plainhook(u32* p, const uint2* e, u64 n, u64* rec) {
    EDGE_LOOP
        u64 r = ~0ull;
        const u32 pa = p[a], pb = p[b];
        u32 wa, wb;
        const u32 ra = root_of<SPLIT>(p, a, pa, wa);
        const u32 rb = root_of<SPLIT>(p, b, pb, wb);
        if (ra == rb) {
            if (wa == UN) p[ra] = ra;
        } else {
            const u32 lo = ra < rb ? ra : rb, hi = ra < rb ? rb : ra;
            const u32 wlo = ra < rb ? wa : wb;
            p[hi] = lo;
            if (wlo == UN) p[lo] = lo;
            r = ((u64)lo << 32) | hi;
        }
        rec[i] = r;
    }
}
// K2: verify every recorded hook; a lost one is united with the CAS union
__global__ __launch_bounds__(256) void k_verify(u32* p, const u64* rec, u64 n, u32* lost) {
    NoCount c;
    u32 l = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 r = __builtin_nontemporal_load(rec + i);
        if (r == ~0ull) continue;
        const u32 hi = (u32)r, lo = (u32)(r >> 32);
        if (p[hi] != lo) {
            ++l;
            UFS::unite(p, lo, hi, c);
        }
    }
    if (l) atomicAdd(lost, l);
}

__global__ __launch_bounds__(256) void compress(u32* parent, u32* labels, u32 n) {
    NoCount c;
    for (u64 v = blockIdx.x * (u64)blockDim.x + threadIdx.x; v < n; v += (u64)gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        labels[v] = (p >= v) ? p : UFS::find_from(parent, (u32)v, p, c);
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
    const u32 V = 1u << 24;
    const u64 E = 9227469;
    gcc_gen_params prm = {GCC_GEN_GNM, 0, V, E, 0x67656C6C79000003ull, 0, 0, 1, 0};
    uint2* d_e;
    u32 *d_p, *d_l, *d_sink, *d_lost;
    u64* d_rec;
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMalloc(&d_p, V * 4));
    CK(hipMalloc(&d_l, V * 4));
    CK(hipMalloc(&d_rec, E * 8));
    CK(hipMalloc(&d_sink, 4));
    CK(hipMalloc(&d_lost, 4));
    hipLaunchKernelGGL(gen, dim3(8192), dim3(256), 0, 0, prm, E, d_e);
    CK(hipDeviceSynchronize());
    std::vector<uint2> h_e(E);
    CK(hipMemcpy(h_e.data(), d_e, E * 8, hipMemcpyDeviceToHost));
    std::vector<u32> hp(V, UN), want(V);
    for (u64 i = 0; i < E; ++i) {
        u32 a = h_e[i].x, b = h_e[i].y;
        if (hp[a] == UN) hp[a] = a;
        if (hp[b] == UN) hp[b] = b;
        u32 ra = hfind(hp, a), rb = hfind(hp, b);
        if (ra < rb) hp[rb] = ra;
        else if (rb < ra) hp[ra] = rb;
    }
    for (u32 v = 0; v < V; ++v) want[v] = hp[v] == UN ? UN : hfind(hp, v);
    hipEvent_t ev[8];
    for (auto& x : ev) CK(hipEventCreate(&x));
    std::vector<u32> got(V);
    const unsigned grids[3] = {2048, 4096, 8192};
    auto run = [&](const char* name, int init, auto&& body, bool check) {
        for (unsigned gr : grids) {
            float best = 1e9, best2 = 0, best3 = 0;
            bool ok = true;
            u32 lost = 0;
            for (int rep = 0; rep < 5; ++rep) {
                if (init == 0) CK(hipMemset(d_p, 0xFF, V * 4));
                else CK(hipMemcpy(d_p, want.data(), V * 4, hipMemcpyHostToDevice));  // a realistic parent[] (labels)
                CK(hipMemset(d_lost, 0, 4));
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(ev[0]));
                body(gr);  // records ev[1] (and ev[2]) itself when it has phases
                CK(hipEventRecord(ev[3]));
                if (check) hipLaunchKernelGGL(compress, dim3(gr), dim3(256), 0, 0, d_p, d_l, V);
                CK(hipEventRecord(ev[4]));
                CK(hipEventSynchronize(ev[4]));
                float t, tc;
                CK(hipEventElapsedTime(&t, ev[0], ev[3]));
                CK(hipEventElapsedTime(&tc, ev[3], ev[4]));
                if (check) {
                    CK(hipMemcpy(got.data(), d_l, V * 4, hipMemcpyDeviceToHost));
                    ok = ok && got == want;
                    CK(hipMemcpy(&lost, d_lost, 4, hipMemcpyDeviceToHost));
                }
                if (t < best) {
                    best = t;
                    best3 = tc;
                }
            }
            printf("%-16s grid %5u: %.3f ms (%.2f G edges/s)", name, gr, best, E / best / 1e6);
            if (check) printf("  compress %.3f ms  total %.3f ms (%.2f G/s)  lost %u  %s", best3, best + best3,
                              E / (best + best3) / 1e6, lost, ok ? "OK" : "BAD");
            printf("\n");
            fflush(stdout);
            (void)best2;
        }
    };
    run("reads2", 1, [&](unsigned gr) { hipLaunchKernelGGL(k_reads2, dim3(gr), dim3(256), 0, 0, d_p, d_e, E, d_sink); }, false);
    run("store1", 1, [&](unsigned gr) { hipLaunchKernelGGL(k_store1, dim3(gr), dim3(256), 0, 0, d_p, d_e, E); }, false);
    run("reads2store1", 1, [&](unsigned gr) { hipLaunchKernelGGL(k_reads2store1, dim3(gr), dim3(256), 0, 0, d_p, d_e, E); }, false);
    run("amin1", 1, [&](unsigned gr) { hipLaunchKernelGGL(k_amin1, dim3(gr), dim3(256), 0, 0, d_p, d_e, E); }, false);
    run("cas1", 1, [&](unsigned gr) { hipLaunchKernelGGL(k_cas1, dim3(gr), dim3(256), 0, 0, d_p, d_e, E, d_sink); }, false);
    run("base", 0, [&](unsigned gr) { hipLaunchKernelGGL(k_base, dim3(gr), dim3(256), 0, 0, d_p, d_e, E); }, true);
    run("plainhook", 0, [&](unsigned gr) {
        hipLaunchKernelGGL(k_plainhook<false>, dim3(gr), dim3(256), 0, 0, d_p, d_e, E, d_rec);
        hipLaunchKernelGGL(k_verify, dim3(gr), dim3(256), 0, 0, d_p, d_rec, E, d_lost);
    }, true);
    run("plainhook_split", 0, [&](unsigned gr) {
        hipLaunchKernelGGL(k_plainhook<true>, dim3(gr), dim3(256), 0, 0, d_p, d_e, E, d_rec);
        hipLaunchKernelGGL(k_verify, dim3(gr), dim3(256), 0, 0, d_p, d_rec, E, d_lost);
    }, true);
    // phases of plainhook: K1 alone, K2 alone (timed separately)
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(d_p, 0xFF, V * 4));
        CK(hipMemset(d_lost, 0, 4));
        CK(hipEventRecord(ev[0]));
        hipLaunchKernelGGL(k_plainhook<false>, dim3(4096), dim3(256), 0, 0, d_p, d_e, E, d_rec);
        CK(hipEventRecord(ev[1]));
        hipLaunchKernelGGL(k_verify, dim3(4096), dim3(256), 0, 0, d_p, d_rec, E, d_lost);
        CK(hipEventRecord(ev[2]));
        CK(hipEventSynchronize(ev[2]));
        float t1, t2;
        u32 lost;
        CK(hipEventElapsedTime(&t1, ev[0], ev[1]));
        CK(hipEventElapsedTime(&t2, ev[1], ev[2]));
        CK(hipMemcpy(&lost, d_lost, 4, hipMemcpyDeviceToHost));
        printf("plainhook phases: K1 %.3f ms, K2 %.3f ms, lost hooks %u\n", t1, t2, lost);
    }
    return 0;
}
