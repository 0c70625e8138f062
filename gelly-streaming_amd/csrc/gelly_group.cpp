// gelly_group.cpp — the cross-GPU merge of the partial forests behind the C ABI (include/gelly_cc.h, "group").
//
// Reference: SummaryBulkAggregation.run ships every partition's partial DisjointSet, Kryo-serialised, to ONE task —
// timeWindowAll(t).reduce(CombineCC) — and the parallelism-1 Merger folds it into the running summary
// (…/SummaryBulkAggregation.java:81-83, …/library/ConnectedComponents.java:116-125, …/SummaryAggregation.java:107-119).
//
// Here every GPU keeps a full-range forest. A merge compresses each forest and encodes it as the compact message of
// include/gelly_cc.h (header, bitmap of the tracked giant, (v, label) list of the other seen ids), ONE RCCL
// all_gather over xGMI moves every message to every GPU, and each GPU absorbs the P-1 others in one launch
// (gcc_forest_absorb_many) and compresses: every GPU then holds the global partition, with no serial bottleneck.
// The list capacity is speculative (the last merge's need x 1.5); the gathered headers say whether some list did
// not fit, and then the exchange is repeated larger — exact, since union is idempotent. When the compact form is
// not smaller than the label array (no dominant component) the label arrays themselves are all-gathered.
//
// Round 6: the DELTA merge first. After a merge every rank holds the same partition and arms its delta; its next
// plain folds list the ids they change, so the next merge only needs (x, root(x)) for those: at most 2 pairs per edge
// the rank folded in the window, like the reference's per-window partials (…/SummaryBulkAggregation.java:80-83: a
// fresh partial per window, so the all-window reduce moves only that window's unions). One all_gather of the delta
// messages (capacity: twice the largest window any rank reported last time); if any rank's delta is unusable (not
// armed: its window took a fold the lists do not see; or overflowed) or larger than the capacity, the ranks fall back
// to the compact rounds below, which are exact whatever was absorbed before (union is idempotent).
//
// Built only on the public C ABI of the forest (encode / absorb / labels / merge_labels / compress / stream) plus
// HIP and RCCL. RCCL is resolved at run time with dlopen("librccl.so.1"): a process that already mapped one (torch
// does) shares it, so there is exactly one RCCL per process.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "abi_common.h"
#include "gelly_cc.h"

typedef uint32_t u32;
typedef uint64_t u64;

namespace {

struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    std::string error;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        // GELLY_RCCL_LIB: another library with RCCL's ABI in its place — the tests' shared-memory stand-in
        // (tests/cpp/shm_rccl.cpp), which runs this file's merge loop with several ranks on one GPU or on CPU
        const char* alt = getenv("GELLY_RCCL_LIB");
        void* h = nullptr;
        if (alt && *alt) {
            h = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
            if (!h) {
                r.error = std::string("dlopen ") + alt + " (GELLY_RCCL_LIB): " + dlerror();
                return;
            }
        }
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.error = std::string("dlopen librccl.so.1: ") + dlerror();
            return;
        }
        auto sym = [&](const char* n) {
            void* p = dlsym(h, n);
            if (!p && r.error.empty()) r.error = std::string("dlsym ") + n;
            return p;
        };
        r.GetUniqueId = (decltype(r.GetUniqueId))sym("ncclGetUniqueId");
        r.CommInitRank = (decltype(r.CommInitRank))sym("ncclCommInitRank");
        r.CommInitAll = (decltype(r.CommInitAll))sym("ncclCommInitAll");
        r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
        r.CommAbort = (decltype(r.CommAbort))sym("ncclCommAbort");
        r.AllGather = (decltype(r.AllGather))sym("ncclAllGather");
        r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
        r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
        r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
    });
    return r;
}

int rccl_ready() {
    Rccl& r = rccl();
    if (!r.error.empty()) return gcc_set_err(GCC_E_NODEV, "RCCL unavailable: %s", r.error.c_str());
    return GCC_OK;
}

#define NCCL_TRY(expr)                                                                                     \
    do {                                                                                                   \
        ncclResult_t r_ = (expr);                                                                          \
        if (r_ != ncclSuccess)                                                                             \
            return gcc_set_err(GCC_E_HIP, "%s failed: %s", #expr, rccl().GetErrorString(r_));              \
    } while (0)

#define ABI_TRY(expr)          \
    do {                       \
        int rc_ = (expr);      \
        if (rc_) return rc_;   \
    } while (0)

u64 round16(u64 x) { return (x + 15) / 16 * 16; }

}  // namespace

// One rank's communicator (one per GPU) plus the merge's buffers, which it owns.
struct gcc_comm {
    ncclComm_t comm = nullptr;
    int device = 0, nranks = 1, rank = 0;
    void* d_send = nullptr;
    u64 send_bytes = 0;
    void* d_recv = nullptr;
    u64 recv_bytes = 0;
    u32* h_hdr = nullptr;  // pinned: the gathered headers (4 u32 per rank)
    // the status exchange (agree()): 16 B per rank gathered, + this rank's 16 B to send; allocated at init, so a
    // rank can always take part in it
    void* d_status = nullptr;
    u32* h_status = nullptr;
    u64 agreed_msg = 0;  // the message size every rank has buffers for (the same value on every rank)
    u64 cap_others = 0;    // the speculative list capacity (grows on overflow, shrinks slowly)
    bool prefer_labels = false;
    u64 last_bytes = 0;    // bytes each rank contributed to the last merge's all_gather
    int last_rounds = 0;   // all_gathers of the last merge (compact rounds + the label exchange)
    bool last_labels = false;  // the last merge ended with the label exchange
    // the delta merge (round 6): its own buffers, the pair capacity (same on every rank: derived from the gathered
    // headers) and how the last merge ended: 0 compact, 1 labels, 2 delta
    void* d_dsend = nullptr;
    u64 dsend_bytes = 0;
    void* d_drecv = nullptr;
    u64 drecv_bytes = 0;
    u64 agreed_delta = 0;
    u64 cap_delta = 0;
    bool delta_off = false;  // GELLY_GROUP_DELTA=0: compact rounds only (A/B)
    int last_kind = 0;
    u64 last_total_bytes = 0;  // every all_gather of the last merge, bytes per rank summed
    // a merge failed where the ranks could not agree on it (e.g. a buffer allocation before the collective): the
    // communicator was aborted and is unusable; the peers may be left inside the collective, so the job's ranks must
    // all be torn down (as a failed Flink task restarts the job)
    bool broken = false;
    // this rank's forest failed to absorb the peers AFTER the last collective of a merge (the absorb / compress of the
    // final round): the peers' merges succeeded, this rank's returned the error. Sticky: every later merge on this
    // communicator starts from that failure, so the peers learn of it in-band in their next merge (a failed-status
    // header or agree()) and every rank returns an error there — no rank is left waiting in a collective for a rank
    // that stopped calling
    bool poisoned = false;
};

namespace {

// Grow a buffer: the old one is freed first, so the peak is the new size (the label exchange's receive buffer is
// nranks x V x 4 B: 2 GiB at 8 ranks and 2^26 ids). A failed allocation leaves the buffer empty; the caller then
// resets gcc_comm::agreed_msg, so the next merge allocates and agrees again.
int ensure(void*& p, u64& have, u64 need) {
    if (have >= need) return GCC_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    HIP_TRY(hipMalloc(&p, (size_t)need));
    have = need;
    return GCC_OK;
}

int forest_info(gcc_forest* h, int* dev, u32* V, hipStream_t* s) {
    ABI_TRY(gcc_forest_device(h, dev));
    ABI_TRY(gcc_forest_capacity(h, V));
    void* sp = nullptr;
    ABI_TRY(gcc_forest_get_stream(h, &sp));
    *s = (hipStream_t)sp;
    return GCC_OK;
}

// A failure no peer can learn of in-band: abort the communicator (gcc_comm.broken) and return the error.
int fail_comm(gcc_comm* c, int rc) {
    c->broken = true;
    if (c->comm && rccl().CommAbort) (void)rccl().CommAbort(c->comm);
    c->comm = nullptr;
    return rc;
}

int alloc_status(gcc_comm* c) {
    DeviceGuard g(c->device);
    HIP_TRY(hipMalloc(&c->d_status, (size_t)(c->nranks + 1) * 16));
    HIP_TRY(hipHostMalloc((void**)&c->h_status, (size_t)(c->nranks + 1) * 16, hipHostMallocDefault));
    return GCC_OK;
}

// The ranks agree before a collective whose inputs a rank may have failed to produce (a buffer it could not
// allocate, an absorb or compress that failed after its header had gone out): one all_gather of a 16-B status word
// per rank. Every rank reads the same words, so either all of them go on to the collective or all of them return
// (the communicator stays usable). *failed = the first failed rank, or -1. Only a failure of this exchange itself
// aborts the communicator.
int agree(gcc_comm* c, hipStream_t st, int local_rc, int* failed) {
    *failed = -1;
    u32* mine = c->h_status + 4 * c->nranks;
    mine[0] = local_rc ? GCC_MSG_STATUS_FAILED : 0u;
    mine[1] = (u32)local_rc;
    mine[2] = mine[3] = 0;
    char* d_mine = static_cast<char*>(c->d_status) + (u64)16 * c->nranks;
    if (hipMemcpyAsync(d_mine, mine, 16, hipMemcpyHostToDevice, st) != hipSuccess)
        return fail_comm(c, gcc_set_err(GCC_E_HIP, "status word copy: %s", hipGetErrorString(hipGetLastError())));
    const ncclResult_t r = rccl().AllGather(d_mine, c->d_status, 16, ncclUint8, c->comm, st);
    if (r != ncclSuccess)
        return fail_comm(c, gcc_set_err(GCC_E_HIP, "ncclAllGather (status): %s", rccl().GetErrorString(r)));
    if (hipMemcpyAsync(c->h_status, c->d_status, (size_t)16 * c->nranks, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail_comm(c, gcc_set_err(GCC_E_HIP, "status words: %s", hipGetErrorString(hipGetLastError())));
    for (int p = 0; p < c->nranks; ++p)
        if (c->h_status[4 * p] == GCC_MSG_STATUS_FAILED) {
            *failed = p;
            break;
        }
    return GCC_OK;
}

// An error of this rank's own after the merge's last collective (gcc_comm::poisoned)
int own_error(gcc_comm* c, int rc) {
    c->poisoned = true;
    return rc;
}

// local_rc (this rank's own error, or 0) and the peers' statuses -> the error every rank returns, or 0
int agreed_error(int local_rc, int failed) {
    if (local_rc) return local_rc;
    if (failed >= 0) return gcc_set_err(GCC_E_INTERNAL, "group merge: rank %d failed (its error is on that rank)", failed);
    return GCC_OK;
}

// The label-array exchange (no dominant component): all_gather of the canonical labels, absorb the others. The ranks
// agree first (a rank may arrive here with an error from the compact rounds, or fail to get its labels or buffer).
int merge_labels_rccl(gcc_forest* h, gcc_comm* c, u32 V, hipStream_t st, int local_rc) {
    const u32* lab = nullptr;
    int rc = local_rc;
    if (!rc) rc = gcc_forest_labels_device(h, &lab);
    if (!rc) {
        rc = ensure(c->d_recv, c->recv_bytes, (u64)c->nranks * V * sizeof(u32));
        if (rc) c->agreed_msg = 0;  // the receive buffer is gone: a later compact round allocates and agrees again
    }
    int failed = -1;
    ABI_TRY(agree(c, st, rc, &failed));
    if (rc || failed >= 0) return agreed_error(rc, failed);
    const ncclResult_t r = rccl().AllGather(lab, c->d_recv, V, ncclUint32, c->comm, st);
    if (r != ncclSuccess)
        return fail_comm(c, gcc_set_err(GCC_E_HIP, "ncclAllGather (labels): %s", rccl().GetErrorString(r)));
    c->last_bytes = 4ull * V;
    c->last_total_bytes += 4ull * V;
    int rc2 = GCC_OK;
    for (int p = 0; p < c->nranks && !rc2; ++p)
        if (p != c->rank) rc2 = gcc_forest_merge_labels_device(h, static_cast<const u32*>(c->d_recv) + (u64)p * V, V);
    if (!rc2) rc2 = gcc_forest_compress(h);
    if (!rc2) rc2 = gcc_forest_delta_arm(h);
    return rc2 ? own_error(c, rc2) : GCC_OK;
}

// The delta round (round 6). *done = true when the merge is complete (every rank absorbed every delta) or failed in
// agreement (the return code says which); false: the ranks go on to the compact rounds (every rank takes that
// decision from the same gathered headers). Every rank's forest stays valid either way.
int delta_round(gcc_forest* h, gcc_comm* c, u32 V, hipStream_t st, int& local_rc, bool* done) {
    *done = false;
    const u64 cap = c->cap_delta;
    const u64 size = round16(gcc_delta_msg_bytes(cap));
    if (size > c->agreed_delta) {
        int rc = ensure(c->d_dsend, c->dsend_bytes, size);
        if (!rc) rc = ensure(c->d_drecv, c->drecv_bytes, (u64)c->nranks * size);
        if (rc) c->agreed_delta = 0;
        int failed = -1;
        ABI_TRY(agree(c, st, rc ? rc : local_rc, &failed));
        if (rc || failed >= 0) {
            *done = true;
            return agreed_error(rc ? rc : local_rc, failed);
        }
        c->agreed_delta = size;
    }
    if (!local_rc) local_rc = gcc_forest_encode_delta(h, c->d_dsend, cap);
    if (local_rc) {
        const u32 hdr[4] = {0, 0, 0, GCC_MSG_STATUS_FAILED};
        int rc = hipMemcpyAsync(c->d_dsend, hdr, sizeof(hdr), hipMemcpyHostToDevice, st) == hipSuccess ? GCC_OK
                 : gcc_set_err(GCC_E_HIP, "failed-status header copy");
        if (!rc) rc = hipStreamSynchronize(st) == hipSuccess ? GCC_OK : gcc_set_err(GCC_E_HIP, "stream sync");
        if (rc) return fail_comm(c, rc);
    }
    const ncclResult_t r = rccl().AllGather(c->d_dsend, c->d_drecv, (size_t)size, ncclUint8, c->comm, st);
    if (r != ncclSuccess) return fail_comm(c, gcc_set_err(GCC_E_HIP, "ncclAllGather (deltas): %s", rccl().GetErrorString(r)));
    ++c->last_rounds;
    c->last_total_bytes += size;
    if (hipMemcpy2DAsync(c->h_hdr, 16, c->d_drecv, (size_t)size, 16, (size_t)c->nranks, hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail_comm(c, gcc_set_err(GCC_E_HIP, "gathered delta headers: %s", hipGetErrorString(hipGetLastError())));
    u64 nmax = 0, emax = 0;
    bool usable = true;
    for (int p = 0; p < c->nranks; ++p) {
        const u32* hp = c->h_hdr + 4 * p;
        if (hp[3] == GCC_MSG_STATUS_FAILED) {
            *done = true;
            return local_rc ? local_rc : gcc_set_err(GCC_E_INTERNAL, "group merge: rank %d failed (its error is on that rank)", p);
        }
        usable &= hp[3] == 0 && hp[2] == V;
        nmax = std::max<u64>(nmax, hp[1]);
        emax = std::max<u64>(emax, hp[0]);
    }
    // the next capacity: twice the largest window a rank folded (a bound: <= 2 pairs per edge), at least the pairs seen
    c->cap_delta = std::max<u64>({1024, 2 * emax, nmax});
    if (!usable || nmax > cap) return GCC_OK;  // the compact rounds (this one's all_gather is not wasted: see above)
    if (!local_rc) local_rc = gcc_forest_absorb_delta_many(h, c->d_drecv, size, (u32)c->nranks, (u32)c->rank, cap);
    if (!local_rc) local_rc = gcc_forest_delta_arm(h);
    if (!local_rc) local_rc = gcc_forest_compress(h);  // the emission (lazy when the forest's emit_every says so)
    c->last_bytes = size;
    c->last_kind = 2;
    *done = true;
    return local_rc ? own_error(c, local_rc) : GCC_OK;
}

}  // namespace

extern "C" {

int gcc_comm_unique_id(void* id_out) {
    CHECK_ARG(id_out, "id_out is null");
    ABI_TRY(rccl_ready());
    ncclUniqueId id;
    NCCL_TRY(rccl().GetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return GCC_OK;
}

int gcc_comm_init(int device, int nranks, int rank, const void* id, gcc_comm** out) {
    CHECK_ARG(out && id, "null argument");
    *out = nullptr;
    CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "rank out of range");
    ABI_TRY(gcc_check_device(device));
    ABI_TRY(rccl_ready());
    DeviceGuard g(device);
    gcc_comm* c = new gcc_comm();
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = rccl().CommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        return gcc_set_err(GCC_E_HIP, "ncclCommInitRank: %s", rccl().GetErrorString(r));
    }
    const int rc = alloc_status(c);
    if (rc) {
        (void)gcc_comm_destroy(c);
        return rc;
    }
    *out = c;
    return GCC_OK;
}

int gcc_comm_init_all(int ndev, const int* devices, gcc_comm** comms_out) {
    CHECK_ARG(ndev >= 1 && devices && comms_out, "null argument");
    for (int i = 0; i < ndev; ++i) ABI_TRY(gcc_check_device(devices[i]));
    ABI_TRY(rccl_ready());
    std::vector<ncclComm_t> cs(ndev);
    NCCL_TRY(rccl().CommInitAll(cs.data(), ndev, devices));
    for (int i = 0; i < ndev; ++i) {
        gcc_comm* c = new gcc_comm();
        c->comm = cs[i];
        c->device = devices[i];
        c->nranks = ndev;
        c->rank = i;
        comms_out[i] = c;
    }
    for (int i = 0; i < ndev; ++i) ABI_TRY(alloc_status(comms_out[i]));
    return GCC_OK;
}

int gcc_comm_destroy(gcc_comm* c) {
    if (!c) return GCC_OK;
    DeviceGuard g(c->device);
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_recv) (void)hipFree(c->d_recv);
    if (c->d_dsend) (void)hipFree(c->d_dsend);
    if (c->d_drecv) (void)hipFree(c->d_drecv);
    if (c->h_hdr) (void)hipHostFree(c->h_hdr);
    if (c->d_status) (void)hipFree(c->d_status);
    if (c->h_status) (void)hipHostFree(c->h_status);
    if (c->comm) (void)rccl().CommDestroy(c->comm);
    delete c;
    return GCC_OK;
}

int gcc_comm_info(gcc_comm* c, int* nranks, int* rank, uint64_t* last_bytes) {
    CHECK_ARG(c, "null comm");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (last_bytes) *last_bytes = c->last_bytes;
    return GCC_OK;
}

int gcc_comm_last_merge(gcc_comm* c, int* rounds, int* labels, uint64_t* cap_others) {
    CHECK_ARG(c, "null comm");
    if (rounds) *rounds = c->last_rounds;
    if (labels) *labels = c->last_labels ? 1 : 0;
    if (cap_others) *cap_others = c->cap_others;
    return GCC_OK;
}

int gcc_comm_last_merge_kind(gcc_comm* c, int* kind, uint64_t* bytes_per_rank, uint64_t* cap_delta) {
    CHECK_ARG(c, "null comm");
    if (kind) *kind = c->last_kind;
    if (bytes_per_rank) *bytes_per_rank = c->last_total_bytes;
    if (cap_delta) *cap_delta = c->cap_delta;
    return GCC_OK;
}

// Collective: every rank calls it with its forest (same id_capacity everywhere); afterwards every rank's forest is
// the union of all of them, compressed. Synchronises the forest's stream (it reads the gathered headers).
int gcc_forest_group_merge(gcc_forest* h, gcc_comm* c) {
    CHECK_ARG(h && c, "null argument");
    CHECK_ARG(!c->broken, "communicator aborted by an earlier failed merge: destroy it (its peers' too)");
    int dev;
    u32 V;
    hipStream_t st;
    ABI_TRY(forest_info(h, &dev, &V, &st));
    CHECK_ARG(dev == c->device, "forest and communicator are on different devices");
    DeviceGuard g(dev);
    if (c->nranks == 1) return gcc_forest_compress(h);
    if (!c->h_hdr) HIP_TRY(hipHostMalloc((void**)&c->h_hdr, (size_t)c->nranks * 16, hipHostMallocDefault));
    if (c->cap_others == 0) c->cap_others = std::max<u64>(1024, V / 64);
    c->last_rounds = 0;
    c->last_labels = false;
    c->last_kind = 0;
    c->last_total_bytes = 0;
    // Every rank takes the same decisions (sizes, repeats) from the gathered headers. A rank whose own encode, absorb
    // or compress fails keeps following them: in a next compact round it sends a failed-status header
    // (include/gelly_cc.h), before a round that grows the buffers and before the label exchange the ranks agree
    // (agree()), so every rank leaves together with an error instead of one rank leaving its peers in a collective.
    int local_rc = c->poisoned ? gcc_set_err(GCC_E_INTERNAL, "an earlier group merge failed on this rank (its forest is "
                                                              "not the union of the ranks'): destroy the group")
                               : GCC_OK;
    // the delta round first, while a delta message is smaller than the compact one (the same decision on every rank:
    // both sizes come from values every rank holds)
    if (c->cap_delta == 0) {
        const char* e = getenv("GELLY_GROUP_DELTA");
        c->delta_off = e && *e == '0';
        c->cap_delta = 1024;
    }
    if (!c->delta_off && gcc_delta_msg_bytes(c->cap_delta) < std::min<u64>(gcc_msg_bytes(V, c->cap_others), 4ull * V)) {
        bool done = false;
        const int rc = delta_round(h, c, V, st, local_rc, &done);
        if (done || rc) return rc;
    }
    while (!c->prefer_labels) {
        const u64 cap = c->cap_others;
        const u64 size = round16(gcc_msg_bytes(V, cap));
        if (size >= 4ull * V) {  // the compact form does not pay: labels from now on (exact after partial rounds)
            c->prefer_labels = true;
            break;
        }
        // the buffers grow at the same rounds on every rank (sizes follow the gathered headers): the ranks agree on
        // the allocation before the all_gather that needs it
        if (size > c->agreed_msg) {
            int rc = ensure(c->d_send, c->send_bytes, size);
            if (!rc) rc = ensure(c->d_recv, c->recv_bytes, (u64)c->nranks * size);
            if (rc) c->agreed_msg = 0;  // a buffer may be gone: the next merge allocates and agrees again
            int failed = -1;
            ABI_TRY(agree(c, st, rc ? rc : local_rc, &failed));
            if (rc || failed >= 0) return agreed_error(rc ? rc : local_rc, failed);
            c->agreed_msg = size;
        }
        int rc = GCC_OK;
        if (!local_rc) local_rc = gcc_forest_encode(h, c->d_send, cap);
        if (local_rc) {  // a header the absorb skips (id_capacity 0) and every rank reads as "the merge failed"
            const u32 hdr[4] = {0xFFFFFFFFu, 0, 0, GCC_MSG_STATUS_FAILED};
            rc = hipMemcpyAsync(c->d_send, hdr, sizeof(hdr), hipMemcpyHostToDevice, st) == hipSuccess ? GCC_OK
                 : gcc_set_err(GCC_E_HIP, "failed-status header copy");
            if (!rc) rc = hipStreamSynchronize(st) == hipSuccess ? GCC_OK : gcc_set_err(GCC_E_HIP, "stream sync");
            if (rc) return fail_comm(c, rc);
        }
        const ncclResult_t r = rccl().AllGather(c->d_send, c->d_recv, (size_t)size, ncclUint8, c->comm, st);
        if (r != ncclSuccess)
            return fail_comm(c, gcc_set_err(GCC_E_HIP, "ncclAllGather (messages): %s", rccl().GetErrorString(r)));
        if (!local_rc) local_rc = gcc_forest_absorb_many(h, c->d_recv, size, (u32)c->nranks, (u32)c->rank, cap);
        if (hipMemcpy2DAsync(c->h_hdr, 16, c->d_recv, (size_t)size, 16, (size_t)c->nranks, hipMemcpyDeviceToHost, st) !=
                hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail_comm(c, gcc_set_err(GCC_E_HIP, "gathered headers: %s", hipGetErrorString(hipGetLastError())));
        if (!local_rc) local_rc = gcc_forest_compress(h);
        ++c->last_rounds;
        c->last_bytes = size;
        c->last_total_bytes += size;
        u64 nmax = 0;
        int failed = -1;
        for (int p = 0; p < c->nranks; ++p) {
            nmax = std::max<u64>(nmax, c->h_hdr[4 * p + 1]);
            if (c->h_hdr[4 * p + 3] == GCC_MSG_STATUS_FAILED && failed < 0) failed = p;
        }
        if (failed >= 0)
            return local_rc ? local_rc : gcc_set_err(GCC_E_INTERNAL, "group merge: rank %d failed (its error is on that rank)", failed);
        if (nmax <= cap) {
            if (4 * nmax < cap && cap > 1024) c->cap_others = std::max<u64>({1024, 3 * nmax / 2, cap / 2});
            if (!local_rc) local_rc = gcc_forest_delta_arm(h);  // every rank holds the same partition: the next delta's base
            return local_rc ? own_error(c, local_rc) : GCC_OK;  // the peers finish: an error here is this rank's own
        }
        c->cap_others = std::max<u64>(3 * nmax / 2, 2 * cap);  // some list did not fit: again, larger
    }
    ++c->last_rounds;
    c->last_labels = true;
    c->last_kind = 1;
    return merge_labels_rccl(h, c, V, st, local_rc);
}

// Single process, n forests (SummaryTreeReduce's partials, or one forest per GPU of a process that drives several
// GPUs): every forest := the union of all n. Forests on ONE device exchange their messages through one device
// buffer (no RCCL); forests on different devices need comms from gcc_comm_init_all (comms[i] for hs[i]).
int gcc_group_merge(gcc_forest** hs, int n, gcc_comm** comms) {
    CHECK_ARG(hs && n >= 1, "null argument");
    std::vector<int> dev(n);
    std::vector<u32> V(n);
    std::vector<hipStream_t> st(n);
    for (int i = 0; i < n; ++i) {
        CHECK_ARG(hs[i], "null forest");
        ABI_TRY(forest_info(hs[i], &dev[i], &V[i], &st[i]));
        CHECK_ARG(V[i] == V[0], "forests of one group need the same id_capacity");
    }
    if (n == 1) return gcc_forest_compress(hs[0]);
    const bool one_device = std::all_of(dev.begin(), dev.end(), [&](int d) { return d == dev[0]; });
    if (!one_device) {
        CHECK_ARG(comms, "forests on several devices need comms (gcc_comm_init_all)");
        for (int i = 0; i < n; ++i)
            CHECK_ARG(comms[i] && comms[i]->device == dev[i] && comms[i]->rank == i && comms[i]->nranks == n,
                      "comms[i] must be rank i of an n-rank group on forest i's device");
        // one grouped launch of every rank's collective (a single thread drives all of them)
        ABI_TRY(rccl_ready());
        u64 cap = std::max<u64>(1024, V[0] / 64);
        while (true) {
            const u64 size = round16(gcc_msg_bytes(V[0], cap));
            const bool labels = size >= 4ull * V[0];
            for (int i = 0; i < n; ++i) {
                DeviceGuard g(dev[i]);
                gcc_comm* c = comms[i];
                if (!c->h_hdr) HIP_TRY(hipHostMalloc((void**)&c->h_hdr, (size_t)n * 16, hipHostMallocDefault));
                if (labels) {
                    ABI_TRY(ensure(c->d_recv, c->recv_bytes, (u64)n * V[0] * sizeof(u32)));
                } else {
                    ABI_TRY(ensure(c->d_send, c->send_bytes, size));
                    ABI_TRY(ensure(c->d_recv, c->recv_bytes, (u64)n * size));
                    ABI_TRY(gcc_forest_encode(hs[i], c->d_send, cap));
                }
            }
            std::vector<const u32*> lab(n, nullptr);
            if (labels)
                for (int i = 0; i < n; ++i) ABI_TRY(gcc_forest_labels_device(hs[i], &lab[i]));
            NCCL_TRY(rccl().GroupStart());
            for (int i = 0; i < n; ++i) {
                gcc_comm* c = comms[i];
                ncclResult_t r = labels ? rccl().AllGather(lab[i], c->d_recv, V[0], ncclUint32, c->comm, st[i])
                                        : rccl().AllGather(c->d_send, c->d_recv, (size_t)size, ncclUint8, c->comm, st[i]);
                if (r != ncclSuccess) {
                    (void)rccl().GroupEnd();
                    return gcc_set_err(GCC_E_HIP, "ncclAllGather: %s", rccl().GetErrorString(r));
                }
            }
            NCCL_TRY(rccl().GroupEnd());
            u64 nmax = 0;
            for (int i = 0; i < n; ++i) {
                DeviceGuard g(dev[i]);
                gcc_comm* c = comms[i];
                if (labels) {
                    for (int p = 0; p < n; ++p)
                        if (p != i)
                            ABI_TRY(gcc_forest_merge_labels_device(
                                hs[i], static_cast<const u32*>(c->d_recv) + (u64)p * V[0], V[0]));
                } else {
                    ABI_TRY(gcc_forest_absorb_many(hs[i], c->d_recv, size, (u32)n, (u32)i, cap));
                    HIP_TRY(hipMemcpy2DAsync(c->h_hdr, 16, c->d_recv, (size_t)size, 16, (size_t)n,
                                             hipMemcpyDeviceToHost, st[i]));
                }
                ABI_TRY(gcc_forest_compress(hs[i]));
            }
            for (int i = 0; i < n; ++i) {
                DeviceGuard g(dev[i]);
                HIP_TRY(hipStreamSynchronize(st[i]));
                if (!labels)
                    for (int p = 0; p < n; ++p) nmax = std::max<u64>(nmax, comms[i]->h_hdr[4 * p + 1]);
            }
            if (labels || nmax <= cap) return GCC_OK;
            cap = std::max<u64>(3 * nmax / 2, 2 * cap);
        }
    }
    // one device: the messages of all n forests in one buffer, each forest absorbs the others
    DeviceGuard g(dev[0]);
    struct Buf {
        void* d = nullptr;
        u64 bytes = 0;
        u32* hdr = nullptr;
        ~Buf() {
            if (d) (void)hipFree(d);
            if (hdr) (void)hipHostFree(hdr);
        }
    } buf;
    HIP_TRY(hipHostMalloc((void**)&buf.hdr, (size_t)n * 16, hipHostMallocDefault));
    std::vector<hipEvent_t> ev(n, nullptr);
    struct Evs {
        std::vector<hipEvent_t>& e;
        ~Evs() {
            for (auto x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } evs{ev};
    for (int i = 0; i < n; ++i) HIP_TRY(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    // the delta round first (as gcc_forest_group_merge): every forest's delta into one buffer; if all are usable and
    // fit, each forest absorbs the others' and arms again; otherwise the compact rounds, after which every forest arms
    const char* de = getenv("GELLY_GROUP_DELTA");
    for (u64 dcap = 1024; !(de && *de == '0');) {
        const u64 size = round16(gcc_delta_msg_bytes(dcap));
        if (size >= std::min<u64>(gcc_msg_bytes(V[0], std::max<u64>(1024, V[0] / 64)), 4ull * V[0])) break;
        ABI_TRY(ensure(buf.d, buf.bytes, (u64)n * size));
        for (int i = 0; i < n; ++i) {
            ABI_TRY(gcc_forest_encode_delta(hs[i], static_cast<char*>(buf.d) + (u64)i * size, dcap));
            HIP_TRY(hipEventRecord(ev[i], st[i]));
        }
        HIP_TRY(hipStreamWaitEvent(st[0], ev[n - 1], 0));
        for (int j = 0; j < n - 1; ++j) HIP_TRY(hipStreamWaitEvent(st[0], ev[j], 0));
        HIP_TRY(hipMemcpy2DAsync(buf.hdr, 16, buf.d, (size_t)size, 16, (size_t)n, hipMemcpyDeviceToHost, st[0]));
        HIP_TRY(hipStreamSynchronize(st[0]));
        u64 nmax = 0;
        bool usable = true;
        for (int p = 0; p < n; ++p) {
            usable &= buf.hdr[4 * p + 3] == 0 && buf.hdr[4 * p + 2] == V[0];
            nmax = std::max<u64>(nmax, buf.hdr[4 * p + 1]);
        }
        if (!usable) break;
        if (nmax > dcap) {  // again, large enough
            dcap = nmax;
            continue;
        }
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) HIP_TRY(hipStreamWaitEvent(st[i], ev[j], 0));  // every message written
            ABI_TRY(gcc_forest_absorb_delta_many(hs[i], buf.d, size, (u32)n, (u32)i, dcap));
        }
        for (int i = 0; i < n; ++i) HIP_TRY(hipStreamSynchronize(st[i]));  // no later encode overwrites a message early
        for (int i = 0; i < n; ++i) {
            ABI_TRY(gcc_forest_delta_arm(hs[i]));
            ABI_TRY(gcc_forest_compress(hs[i]));
        }
        return GCC_OK;
    }
    u64 cap = std::max<u64>(1024, V[0] / 64);
    while (true) {
        const u64 size = round16(gcc_msg_bytes(V[0], cap));
        if (size >= 4ull * V[0]) {  // labels: CombineCC pairwise into forest 0, then forest 0's partition to all
            for (int i = 1; i < n; ++i) ABI_TRY(gcc_forest_merge(hs[0], hs[i]));
            ABI_TRY(gcc_forest_compress(hs[0]));
            for (int i = 1; i < n; ++i) ABI_TRY(gcc_forest_merge(hs[i], hs[0]));
            for (int i = 0; i < n; ++i) ABI_TRY(gcc_forest_sync(hs[i]));
            for (int i = 0; i < n; ++i) ABI_TRY(gcc_forest_delta_arm(hs[i]));
            return GCC_OK;
        }
        ABI_TRY(ensure(buf.d, buf.bytes, (u64)n * size));
        for (int i = 0; i < n; ++i) {
            ABI_TRY(gcc_forest_encode(hs[i], static_cast<char*>(buf.d) + (u64)i * size, cap));
            HIP_TRY(hipEventRecord(ev[i], st[i]));
        }
        for (int i = 0; i < n; ++i) {
            for (int j = 0; j < n; ++j) HIP_TRY(hipStreamWaitEvent(st[i], ev[j], 0));  // every message written
            ABI_TRY(gcc_forest_absorb_many(hs[i], buf.d, size, (u32)n, (u32)i, cap));
            ABI_TRY(gcc_forest_compress(hs[i]));
        }
        HIP_TRY(hipMemcpy2DAsync(buf.hdr, 16, buf.d, (size_t)size, 16, (size_t)n, hipMemcpyDeviceToHost, st[0]));
        for (int i = 0; i < n; ++i) HIP_TRY(hipStreamSynchronize(st[i]));  // also: no encode overwrites a message early
        u64 nmax = 0;
        for (int p = 0; p < n; ++p) nmax = std::max<u64>(nmax, buf.hdr[4 * p + 1]);
        if (nmax <= cap) {
            for (int i = 0; i < n; ++i) ABI_TRY(gcc_forest_delta_arm(hs[i]));
            return GCC_OK;
        }
        cap = std::max<u64>(3 * nmax / 2, 2 * cap);
    }
}

}  // extern "C"
