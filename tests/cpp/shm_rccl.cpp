// shm_rccl.cpp — TEST INFRASTRUCTURE ONLY: a stand-in for librccl.so.1 that moves the cross-GPU group merge's
// collectives between processes through host shared memory, so that the production merge loop
// (gelly-streaming_amd/csrc/gelly_group.cpp: gcc_forest_group_merge with nranks > 1 — compact rounds, agree(), the
// failed-status headers, the label fallback) runs with several ranks where only ONE GPU exists: ranks sharing cuda:0
// on the one-GPU test box (tests/test_gpu_group.py), or CPU processes with the host build of the merge
// (tests/test_group_protocol.py, built against tests/cpp/hipmock). It is loaded through the product's dlopen seam
// (GELLY_RCCL_LIB); the product code is the same as under real RCCL. Never used for a measurement.
//
// Exports exactly the symbols gelly_group.cpp resolves. ncclAllGather: wait for the caller's stream, copy this rank's
// bytes into its slot of a shared segment, barrier, copy every slot into the receive buffer, barrier — in 8 MiB
// chunks. The barrier times out (GELLY_SHM_RCCL_TIMEOUT seconds, default 60) and honours an abort flag that
// ncclCommAbort sets, so a failed or dead peer ends in an error on every rank, never a hang.
//
// Fault injection (tests only): GELLY_SHM_RCCL_FAIL="r:k" — rank r's k-th ncclAllGather (1-based) returns
// ncclSystemError without taking part; GELLY_SHM_RCCL_EXIT="r:k" — rank r _exit(3)s inside its k-th ncclAllGather
// (a peer process that dies mid-collective). GELLY_SHM_RCCL_TAG names the segments (/dev/shm/gshm_<tag>_...), so a
// test can remove what a crashed run left.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sched.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

namespace {

constexpr uint64_t kSlot = 8ull << 20;  // bytes per rank per chunk
constexpr uint64_t kHeader = 4096;

struct Shared {
    std::atomic<uint32_t> arrived;
    std::atomic<uint32_t> generation;
    std::atomic<uint32_t> aborted;
};
static_assert(sizeof(Shared) <= kHeader, "header");

struct Comm {
    Shared* sh = nullptr;
    char* slots = nullptr;
    size_t map_bytes = 0;
    int nranks = 1, rank = 0;
    uint64_t calls = 0;
};

double now_s() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

double timeout_s() {
    const char* e = getenv("GELLY_SHM_RCCL_TIMEOUT");
    return e ? atof(e) : 60.0;
}

// "r:k" -> does it name this (rank, call)?
bool fault(const char* var, int rank, uint64_t call) {
    const char* e = getenv(var);
    int r = -1;
    unsigned long long k = 0;
    return e && sscanf(e, "%d:%llu", &r, &k) == 2 && r == rank && k == call;
}

ncclResult_t barrier(Comm* c) {
    Shared* s = c->sh;
    const uint32_t gen = s->generation.load(std::memory_order_acquire);
    if (s->aborted.load(std::memory_order_acquire)) return ncclRemoteError;
    if (s->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)c->nranks) {
        s->arrived.store(0, std::memory_order_relaxed);
        s->generation.fetch_add(1, std::memory_order_acq_rel);
        return ncclSuccess;
    }
    const double t0 = now_s(), limit = timeout_s();
    for (uint64_t spin = 0; s->generation.load(std::memory_order_acquire) == gen; ++spin) {
        if (s->aborted.load(std::memory_order_acquire)) return ncclRemoteError;
        if ((spin & 1023) == 0 && now_s() - t0 > limit) {
            s->aborted.store(1, std::memory_order_release);  // a peer is gone: every rank leaves with an error
            return ncclRemoteError;
        }
        if (spin > 4096) usleep(50);
        else sched_yield();
    }
    return ncclSuccess;
}

void release(Comm* c) {
    if (c->sh) munmap(c->sh, c->map_bytes);
    delete c;
}

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    static std::atomic<unsigned> counter{0};
    const char* tag = getenv("GELLY_SHM_RCCL_TAG");
    memset(id->internal, 0, sizeof(id->internal));
    snprintf(id->internal, sizeof(id->internal), "/gshm_%s_%d_%llx_%u", tag ? tag : "x", (int)getpid(),
             (unsigned long long)(now_s() * 1e9), counter.fetch_add(1));
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks || id.internal[0] != '/') return ncclInvalidArgument;
    char name[NCCL_UNIQUE_ID_BYTES + 1];
    memcpy(name, id.internal, NCCL_UNIQUE_ID_BYTES);
    name[NCCL_UNIQUE_ID_BYTES] = 0;
    Comm* c = new Comm();
    c->nranks = nranks;
    c->rank = rank;
    c->map_bytes = kHeader + (size_t)nranks * kSlot;
    const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
    if (fd < 0) {
        delete c;
        return ncclSystemError;
    }
    void* m = MAP_FAILED;
    if (ftruncate(fd, (off_t)c->map_bytes) == 0) m = mmap(nullptr, c->map_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
        delete c;
        return ncclSystemError;
    }
    c->sh = static_cast<Shared*>(m);
    c->slots = static_cast<char*>(m) + kHeader;
    const ncclResult_t r = barrier(c);  // every rank has mapped the segment
    if (rank == 0) shm_unlink(name);    // nothing is left in /dev/shm once the ranks hold their mappings
    if (r != ncclSuccess) {
        release(c);
        return r;
    }
    *out = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t*, int, const int*) { return ncclInvalidUsage; }

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (comm) release(reinterpret_cast<Comm*>(comm));
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
    if (!comm) return ncclSuccess;
    Comm* c = reinterpret_cast<Comm*>(comm);
    c->sh->aborted.store(1, std::memory_order_release);
    release(c);
    return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* send, void* recv, size_t count, ncclDataType_t dt, ncclComm_t comm,
                           hipStream_t stream) {
    if (!comm || (!send && count) || (!recv && count) || !type_bytes(dt)) return ncclInvalidArgument;
    Comm* c = reinterpret_cast<Comm*>(comm);
    const uint64_t call = ++c->calls;
    if (fault("GELLY_SHM_RCCL_FAIL", c->rank, call)) return ncclSystemError;
    if (fault("GELLY_SHM_RCCL_EXIT", c->rank, call)) _exit(3);
    const uint64_t bytes = (uint64_t)count * type_bytes(dt);
    if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
    char* mine = c->slots + (uint64_t)c->rank * kSlot;
    for (uint64_t off = 0; off < bytes || (bytes == 0 && off == 0); off += kSlot) {
        const uint64_t len = bytes - off < kSlot ? bytes - off : kSlot;
        if (len && hipMemcpy(mine, static_cast<const char*>(send) + off, len, hipMemcpyDeviceToHost) != hipSuccess)
            return ncclUnhandledCudaError;
        ncclResult_t r = barrier(c);
        if (r != ncclSuccess) return r;
        for (int p = 0; p < c->nranks && len; ++p)
            if (hipMemcpy(static_cast<char*>(recv) + (uint64_t)p * bytes + off, c->slots + (uint64_t)p * kSlot, len,
                          hipMemcpyHostToDevice) != hipSuccess)
                return ncclUnhandledCudaError;
        r = barrier(c);  // no rank overwrites a slot before every rank has read it
        if (r != ncclSuccess) return r;
        if (bytes == 0) break;
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error";
        case ncclSystemError: return "shm stand-in: system error (injected or shm failure)";
        case ncclRemoteError: return "shm stand-in: a peer aborted or timed out";
        case ncclInvalidArgument: return "shm stand-in: invalid argument";
        case ncclInvalidUsage: return "shm stand-in: unsupported call";
        default: return "shm stand-in: error";
    }
}

}  // extern "C"
