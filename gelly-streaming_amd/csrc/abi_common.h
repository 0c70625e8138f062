// abi_common.h — error plumbing and host helpers shared by the translation units of libgelly_cc.so
// (gelly_cc.hip: the CC forest; gelly_bip.hip: the signed forest of BipartitenessCheck).
// Conventions (include/gelly_cc.h): every C-ABI function returns 0 or a negative GCC_E_* code and leaves a
// thread-local message for gcc_last_error(); no C++ exception crosses the boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gelly_cc.h"

// records the message of the failing call (defined in gelly_cc.hip, read back by gcc_last_error)
int gcc_set_err(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
// the device exists and is a gfx950 (this library carries gfx950 code only)
int gcc_check_device(int device);
// after an asynchronous kernel fault: " [last kernel started: <name>]" from the kernel-start trace (gelly_cc.hip)
const char* gcc_fault_note(hipError_t e);

#define HIP_TRY(expr)                                                                                      \
    do {                                                                                                   \
        hipError_t e_ = (expr);                                                                            \
        if (e_ != hipSuccess) {                                                                            \
            return gcc_set_err(e_ == hipErrorOutOfMemory ? GCC_E_OOM : GCC_E_HIP, "%s failed: %s (%s:%d)%s", \
                               #expr, hipGetErrorString(e_), __FILE__, __LINE__, gcc_fault_note(e_));       \
        }                                                                                                  \
    } while (0)

#define CHECK_ARG(cond, msg)                                        \
    do {                                                            \
        if (!(cond)) return gcc_set_err(GCC_E_INVALID, "%s", msg); \
    } while (0)

// makes `dev` current for the scope (handles may live on any device of the process)
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

constexpr int kAbiBlock = 256;

static inline unsigned grid_for_n(uint64_t n, unsigned max_blocks, int block = kAbiBlock) {
    uint64_t b = (n + block - 1) / block;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (unsigned)b;
}
