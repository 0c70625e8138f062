// probe_compress_inplace.hip — the GPU side of the in-place compress question, one run.
// Replays the adversarial p10 fixture stream window by window with the PRODUCT union (uf_device.h UF::unite,
// path splitting, many blocks) and then one of four compresses, and counts windows whose labels differ from a
// sequential host union-find:
//   out       compress_kernel's step (compress_label) into a second buffer, swapped   (the product's full compress)
//   split     in place, finds WITH path splitting                                    (round 1's first compress)
//   nosplit   in place, read-only finds                                             (the round-1 experiment)
//   inc       compress_inc_kernel<true>'s step (inc_label, bloom of the fold's hooks) (the product's inc_inplace)
// tests/cpp/test_uf_replay.cpp replays the same code on host threads; this probe checks the replay's verdicts on the
// hardware. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../gelly-streaming_amd/csrc
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "edge_gen.h"
#include "gelly_cc.h"
#include "uf_device.h"

typedef uint32_t u32;
#define UNSEEN 0xFFFFFFFFu
#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

template <bool REC>
__global__ void fold(u32* parent, const uint2* e, int n, u32* bloom) {
    gcc::NoCount c;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (REC) gcc::UF::unite(parent, e[i].x, e[i].y, c, gcc::BloomRec{bloom});
        else gcc::UF::unite(parent, e[i].x, e[i].y, c);
    }
}

__global__ void comp_out(u32* parent, u32* labels, u32 n) {
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x)
        labels[v] = gcc::compress_label(parent, v);
}

template <bool SPLIT>
__global__ void comp_inplace(u32* parent, u32 n) {
    gcc::NoCount c;
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        if (p >= v) continue;
        const u32 r = gcc::UnionFind<gcc::LoadPlain, SPLIT>::find_from(parent, v, p, c);
        if (r != p) parent[v] = r;
    }
}

// the bloom is read from global memory here (the product copies it into LDS first: same values)
__global__ void comp_inc(u32* parent, u32 n, const u32* bloom, u32* bloom_clear) {
    for (u32 w = blockIdx.x * blockDim.x + threadIdx.x; w < gcc::kBloomBits / 32; w += gridDim.x * blockDim.x)
        bloom_clear[w] = 0;
    for (u32 v = blockIdx.x * blockDim.x + threadIdx.x; v < n; v += gridDim.x * blockDim.x) {
        const u32 p = parent[v];
        const u32 l = gcc::inc_label(parent, bloom, v, p);
        if (l != p) parent[v] = l;
    }
}

static u32 hfind(std::vector<u32>& p, u32 x) {
    while (p[x] != x) x = p[x];
    return x;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 30;
    gcc_gen_params prm = {GCC_GEN_ADVERSARIAL, 10, 0, 0, 0x67656C6C79000005ull, 8, 128, 0, 0};
    const int E = (int)gcc_gen_num_edges(&prm);
    const u32 V = (u32)gcc_gen_num_vertices(&prm);
    std::vector<uint2> edges(E);
    for (int i = 0; i < E; ++i) gcc_gen_edge(&prm, i, &edges[i].x, &edges[i].y);
    const int W = 256;
    const int nw = (E + W - 1) / W;
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
    u32 *d_a, *d_b, *d_bloom;
    uint2* d_e;
    CK(hipMalloc(&d_a, V * 4));
    CK(hipMalloc(&d_b, V * 4));
    CK(hipMalloc(&d_bloom, 2 * gcc::kBloomBits / 8));
    CK(hipMalloc(&d_e, E * 8));
    CK(hipMemcpy(d_e, edges.data(), E * 8, hipMemcpyHostToDevice));
    const char* names[] = {"out (product full compress)", "split (in place, path splitting)",
                           "nosplit (in place, read-only finds)", "inc (compress_inc in place, product)"};
    const unsigned grids[] = {1, 8};  // fold blocks (V is small: a few blocks already race)
    std::vector<u32> got(V);
    printf("adversarial p10: V=%u E=%d windows=%d reps=%d\n", V, E, nw, reps);
    for (unsigned fg : grids)
        for (int var = 0; var < 4; ++var) {
            int bad = 0, total = 0;
            long long bad_ids = 0;
            for (int r = 0; r < reps; ++r) {
                u32 *par = d_a, *spare = d_b;
                CK(hipMemset(par, 0xFF, V * 4));
                CK(hipMemset(d_bloom, 0, 2 * gcc::kBloomBits / 8));
                int cur = 0;
                bool rec_all = false;
                for (int w = 0; w < nw; ++w) {
                    const int b = w * W, n = std::min(E, (w + 1) * W) - b;
                    u32* bl = d_bloom + cur * (gcc::kBloomBits / 32);
                    u32* other = d_bloom + (cur ^ 1) * (gcc::kBloomBits / 32);
                    if (var == 3) hipLaunchKernelGGL(fold<true>, dim3(fg), dim3(256), 0, 0, par, d_e + b, n, bl);
                    else hipLaunchKernelGGL(fold<false>, dim3(fg), dim3(256), 0, 0, par, d_e + b, n, bl);
                    const dim3 cg((V + 255) / 256);
                    if (var == 0 || (var == 3 && !rec_all)) {
                        hipLaunchKernelGGL(comp_out, cg, dim3(256), 0, 0, par, spare, V);
                        std::swap(par, spare);
                        if (var == 3) CK(hipMemset(other, 0, gcc::kBloomBits / 8));
                    } else if (var == 1) {
                        hipLaunchKernelGGL(comp_inplace<true>, cg, dim3(256), 0, 0, par, V);
                    } else if (var == 2) {
                        hipLaunchKernelGGL(comp_inplace<false>, cg, dim3(256), 0, 0, par, V);
                    } else {
                        hipLaunchKernelGGL(comp_inc, cg, dim3(256), 0, 0, par, V, bl, other);
                    }
                    if (var == 3) {
                        cur ^= 1;
                        rec_all = true;
                    }
                    CK(hipMemcpy(got.data(), par, V * 4, hipMemcpyDeviceToHost));
                    int d = 0;
                    for (u32 v = 0; v < V; ++v) d += got[v] != want[w][v];
                    bad += d != 0;
                    bad_ids += d;
                    ++total;
                }
            }
            printf("fold blocks %u  %-40s bad windows %d / %d  (wrong labels %lld)\n", fg, names[var], bad, total,
                   bad_ids);
        }
    return 0;
}
