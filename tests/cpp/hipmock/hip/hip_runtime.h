// hipmock/hip/hip_runtime.h — TEST INFRASTRUCTURE ONLY: the few HIP runtime calls the cross-GPU group merge
// (gelly-streaming_amd/csrc/gelly_group.cpp) and the shared-memory RCCL stand-in (tests/cpp/shm_rccl.cpp) make,
// restated for the host, so that the product's merge protocol compiles with g++ and runs on CPU processes
// (tests/test_group_protocol.py). "Device memory" is host memory, every stream is synchronous, events are no-ops.
// Never on a product path: libgelly_cc.so is built by hipcc against /opt/rocm's real header.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorOutOfMemory = 2 } hipError_t;
typedef enum hipMemcpyKind {
    hipMemcpyHostToHost = 0,
    hipMemcpyHostToDevice = 1,
    hipMemcpyDeviceToHost = 2,
    hipMemcpyDeviceToDevice = 3,
    hipMemcpyDefault = 4
} hipMemcpyKind;
typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;
#define hipHostMallocDefault 0u
#define hipEventDisableTiming 2u

static inline hipError_t hipMalloc(void** p, size_t n) {
    *p = aligned_alloc(256, (n + 255) / 256 * 256 + 256);
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
template <class T>
static inline hipError_t hipMalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), n);
}
static inline hipError_t hipFree(void* p) {
    free(p);
    return hipSuccess;
}
static inline hipError_t hipHostMalloc(void** p, size_t n, unsigned) { return hipMalloc(p, n); }
template <class T>
static inline hipError_t hipHostMalloc(T** p, size_t n, unsigned f) {
    return hipHostMalloc(reinterpret_cast<void**>(p), n, f);
}
static inline hipError_t hipHostFree(void* p) { return hipFree(p); }
static inline hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
    memmove(d, s, n);
    return hipSuccess;
}
static inline hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind k, hipStream_t) {
    return hipMemcpy(d, s, n, k);
}
static inline hipError_t hipMemcpy2DAsync(void* d, size_t dpitch, const void* s, size_t spitch, size_t w, size_t h,
                                          hipMemcpyKind, hipStream_t) {
    for (size_t r = 0; r < h; ++r)
        memmove(static_cast<char*>(d) + r * dpitch, static_cast<const char*>(s) + r * spitch, w);
    return hipSuccess;
}
static inline hipError_t hipMemsetAsync(void* d, int v, size_t n, hipStream_t) {
    memset(d, v, n);
    return hipSuccess;
}
static inline hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
static inline hipError_t hipGetLastError() { return hipSuccess; }
static inline const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "hipmock error"; }
static inline hipError_t hipGetDevice(int* d) {
    *d = 0;
    return hipSuccess;
}
static inline hipError_t hipSetDevice(int) { return hipSuccess; }
static inline hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
    *e = reinterpret_cast<hipEvent_t>(1);
    return hipSuccess;
}
static inline hipError_t hipEventRecord(hipEvent_t, hipStream_t) { return hipSuccess; }
static inline hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned) { return hipSuccess; }
static inline hipError_t hipEventDestroy(hipEvent_t) { return hipSuccess; }
