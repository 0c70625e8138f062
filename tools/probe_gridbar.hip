// probe_gridbar.hip — what does a device-wide barrier cost inside one persistent kernel on MI355X, against the
// kernel boundary it would replace? (the short-window pipeline question)
//   boundary: K back-to-back empty kernels (grid n_cu x 1024)
//   flat:     one kernel, K barriers: thread 0 of each block fences (release), atomicAdd on one counter, spins on
//             a generation word with agent-scope atomic loads, fences (acquire)
//   xcd:      the same, two-level: blocks arrive at their XCD's counter (blockIdx % 8), the last arriver of an XCD
//             arrives at the top counter
//   graph:    the K empty kernels captured once into a hipGraph and replayed (is the per-kernel cost a host-side
//             launch cost that a graph removes, or the GPU's own dispatch + kernel-boundary cost?)
// The kernel is co-resident by construction (one 1024-thread block per CU, occupancy checked on the host).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 probe_gridbar.hip -o probe_gridbar
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                \
    do {                                                                     \
        hipError_t e = (x);                                                  \
        if (e != hipSuccess) {                                               \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

typedef unsigned u32;

__global__ void empty_kernel(u32* p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0xFFFFFFFu) p[0] = 1;
}

__device__ __forceinline__ u32 ld_acq(u32* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// bar[0] = arrive counter, bar[1] = generation (flat); XCD: bar[2 + 16 * x] per-XCD counters (own 64 B line)
template <bool XCD>
__global__ __launch_bounds__(1024) void bar_kernel(u32* bar, int K, u32* sink) {
    u32 gen = 0;
    const u32 nb = gridDim.x;
    u32 acc = 0;
    for (int k = 0; k < K; ++k) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence();  // release this block's writes (agent scope)
            bool last;
            if (XCD) {
                const u32 x = blockIdx.x & 7;
                const u32 nx = (nb - x + 7) / 8;  // blocks of XCD x
                last = false;
                if (atomicAdd(&bar[2 + 16 * x], 1u) == nx - 1) {
                    bar[2 + 16 * x] = 0;  // reset before the release below (no one touches it until the next round)
                    last = atomicAdd(&bar[0], 1u) == ((nb < 8 ? nb : 8) - 1);
                }
            } else {
                last = atomicAdd(&bar[0], 1u) == nb - 1;
            }
            if (last) {
                bar[0] = 0;
                __threadfence();
                atomicAdd(&bar[1], 1u);
            }
            while (ld_acq(&bar[1]) == gen) __builtin_amdgcn_s_sleep(1);
            __threadfence();  // acquire
        }
        ++gen;
        __syncthreads();
        acc += gen;
    }
    if (threadIdx.x == 0 && acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 2000;
    int dev = 0, ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, bar_kernel<false>, 1024, 0));
    printf("CUs %d, co-resident 1024-thread blocks per CU %d\n", ncu, occ);
    if (occ < 1) return 1;
    u32 *bar, *sink;
    CK(hipMalloc(&bar, 4096));
    CK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(empty_kernel, dim3(ncu), dim3(1024), 0, 0, sink);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("boundary: %d empty kernels            %.3f us each\n", K, 1000.0 * ms / K);
        for (int x = 0; x < 2; ++x) {
            CK(hipMemset(bar, 0, 4096));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(a));
            if (x) hipLaunchKernelGGL(bar_kernel<true>, dim3(ncu), dim3(1024), 0, 0, bar, K, sink);
            else hipLaunchKernelGGL(bar_kernel<false>, dim3(ncu), dim3(1024), 0, 0, bar, K, sink);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("%s: %d barriers in one kernel   %.3f us each\n", x ? "xcd " : "flat", K, 1000.0 * ms / K);
        }
    }
    {  // the same K empty kernels as one captured graph
        hipStream_t st;
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        hipGraph_t graph;
        hipGraphExec_t exec;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < K; ++k) hipLaunchKernelGGL(empty_kernel, dim3(ncu), dim3(1024), 0, st, sink);
        CK(hipStreamEndCapture(st, &graph));
        CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(a, st));
            CK(hipGraphLaunch(exec, st));
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("graph: %d empty kernels in one hipGraph  %.3f us each\n", K, 1000.0 * ms / K);
            CK(hipEventRecord(a, st));
            for (int k = 0; k < K; ++k) hipLaunchKernelGGL(empty_kernel, dim3(ncu), dim3(1024), 0, st, sink);
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("stream (non-blocking): %d empty kernels   %.3f us each\n", K, 1000.0 * ms / K);
        }
    }
    return 0;
}
