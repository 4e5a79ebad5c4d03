// comm.cpp — multi-GPU collectives of the sequence driver over RCCL / xGMI, and plain
// device buffers for callers that keep inputs resident in HBM.
//
// A sequence of Frame360 pairs shards one contiguous run of pairs per GPU (one process per GPU); the only
// data exchange is one all_gather of the per-pair records (pose, information, status: ~220 B per pair, a
// few tens of KB in total, latency-bound) to rank 0, which composes the trajectory
// (Registration/OdometryRGBD360.cpp:257).  The communicator owns a HIP stream and device staging buffers;
// the entry points take host memory and return when the result is back on the host.  The unique id is
// created by rank 0 and handed to the other ranks by the caller (the bench uses torch.distributed's gloo
// group, which never touches the GPU).
#include <cstring>
#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>

#include "../r360_internal.h"

// RCCL is loaded on first use (dlopen), so single-GPU users of the library never load it.
namespace {
struct Rccl {
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclAllReduce) allReduce = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    bool ok = false;
};
const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.getUniqueId = (decltype(r.getUniqueId))dlsym(h, "ncclGetUniqueId");
        r.commInitRank = (decltype(r.commInitRank))dlsym(h, "ncclCommInitRank");
        r.commDestroy = (decltype(r.commDestroy))dlsym(h, "ncclCommDestroy");
        r.allGather = (decltype(r.allGather))dlsym(h, "ncclAllGather");
        r.allReduce = (decltype(r.allReduce))dlsym(h, "ncclAllReduce");
        r.errorString = (decltype(r.errorString))dlsym(h, "ncclGetErrorString");
        r.ok = r.getUniqueId && r.commInitRank && r.commDestroy && r.allGather && r.allReduce && r.errorString;
    });
    return r;
}
}  // namespace


#define R360_NCCL(call)                                                                  \
    do {                                                                                 \
        ncclResult_t _r = (call);                                                        \
        if (_r != ncclSuccess) {                                                         \
            r360_set_error("%s failed: %s (%s:%d)", #call, rccl().errorString(_r), __FILE__, __LINE__); \
            return -1;                                                                   \
        }                                                                                \
    } while (0)

struct r360_comm {
    int device = 0, nranks = 1, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    void* d_buf = nullptr;   // staging: send slice + nranks receive slices
    size_t cap = 0;
};

static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");

#define REQUIRE_RCCL() CHECK_ARG(rccl().ok, "librccl.so.1 could not be loaded")

extern "C" int r360_comm_unique_id(uint8_t id[128]) {
    CHECK_ARG(id, "null id");
    REQUIRE_RCCL();
    ncclUniqueId u;
    R360_NCCL(rccl().getUniqueId(&u));
    memcpy(id, &u, sizeof u);
    return 0;
}

extern "C" int r360_comm_init(int device, int nranks, int rank, const uint8_t id[128], r360_comm** out) {
    CHECK_ARG(id && out, "null arg");
    CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "invalid rank / nranks");
    REQUIRE_RCCL();
    R360_HIP(hipSetDevice(device));
    r360_comm* c = new r360_comm;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId u;
    memcpy(&u, id, sizeof u);
    if (rccl().commInitRank(&c->comm, nranks, u, rank) != ncclSuccess) {
        r360_set_error("ncclCommInitRank failed (rank %d of %d)", rank, nranks);
        delete c;
        return -1;
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        rccl().commDestroy(c->comm);
        delete c;
        r360_set_error("hipStreamCreate failed");
        return -1;
    }
    *out = c;
    return 0;
}

extern "C" void r360_comm_destroy(r360_comm* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    rccl().commDestroy(c->comm);
    hipFree(c->d_buf);
    hipStreamDestroy(c->stream);
    delete c;
}

static int comm_reserve(r360_comm* c, size_t bytes) {
    if (c->cap >= bytes) return 0;
    R360_HIP(hipStreamSynchronize(c->stream));
    if (c->d_buf) R360_HIP(hipFree(c->d_buf));
    c->d_buf = nullptr;
    c->cap = 0;
    R360_HIP(hipMalloc(&c->d_buf, bytes));
    c->cap = bytes;
    return 0;
}

// recv = the nranks send buffers of `bytes` each, in rank order (ncclAllGather over xGMI)
extern "C" int r360_comm_allgather(r360_comm* c, const void* send, void* recv, size_t bytes) {
    CHECK_ARG(c && send && recv, "null arg");
    R360_HIP(hipSetDevice(c->device));
    const size_t slot = (bytes + 255) & ~size_t(255);
    if (int rc = comm_reserve(c, slot * (1 + (size_t)c->nranks))) return rc;
    char* d_send = static_cast<char*>(c->d_buf);
    char* d_recv = d_send + slot;
    R360_HIP(hipMemcpyAsync(d_send, send, bytes, hipMemcpyHostToDevice, c->stream));
    // the receive slices are `bytes` apart (ncclAllGather's layout)
    R360_NCCL(rccl().allGather(d_send, d_recv, bytes, ncclUint8, c->comm, c->stream));
    R360_HIP(hipMemcpyAsync(recv, d_recv, bytes * c->nranks, hipMemcpyDeviceToHost, c->stream));
    R360_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

// v[0..n) = the element-wise maximum over the ranks (ncclAllReduce, ncclMax)
extern "C" int r360_comm_allreduce_max(r360_comm* c, double* v, int n) {
    CHECK_ARG(c && v && n > 0, "null arg");
    R360_HIP(hipSetDevice(c->device));
    const size_t bytes = sizeof(double) * (size_t)n;
    if (int rc = comm_reserve(c, bytes)) return rc;
    R360_HIP(hipMemcpyAsync(c->d_buf, v, bytes, hipMemcpyHostToDevice, c->stream));
    R360_NCCL(rccl().allReduce(c->d_buf, c->d_buf, (size_t)n, ncclFloat64, ncclMax, c->comm, c->stream));
    R360_HIP(hipMemcpyAsync(v, c->d_buf, bytes, hipMemcpyDeviceToHost, c->stream));
    R360_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

// ------------------------------------------------------------------ device buffers
extern "C" int r360_dev_alloc(int device, size_t bytes, void** out) {
    CHECK_ARG(out && bytes, "null arg");
    R360_HIP(hipSetDevice(device));
    R360_HIP(hipMalloc(out, bytes));
    return 0;
}

extern "C" int r360_dev_free(void* p) {
    if (p) R360_HIP(hipFree(p));
    return 0;
}

extern "C" int r360_dev_copy(void* dst, const void* src, size_t bytes, int kind) {
    CHECK_ARG(dst && src, "null arg");
    CHECK_ARG(kind >= 0 && kind <= 2, "kind: 0 host->device, 1 device->host, 2 device->device");
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
    R360_HIP(hipMemcpy(dst, src, bytes, k));
    return 0;
}
