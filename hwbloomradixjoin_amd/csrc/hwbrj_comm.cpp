// hwbrj_comm.cpp -- the native RCCL transport of the multi-GPU joins.
//
// One RCCL communicator per device (one rank per GPU, one process or thread per rank), created from
// a unique id the caller distributes (hwbrj_comm_unique_id on one rank, any side channel to the
// others: torch.distributed, MPI, a file). Two users:
//   * the partitioned join (hwbrj_join_partitioned_rccl): its R-chunk and survivor all-to-alls are
//     grouped ncclSend / ncclRecv and its slice all-gather an in-place ncclAllGather, all enqueued
//     on the join's own stream, so the kernels around them need no host synchronisation; only the
//     per-destination counts cross to the host (they size the variable all-to-alls);
//   * the replicated design's opt-in filter broadcast (hwbrj_set_filter_broadcast): rank 0 builds
//     the slices and ncclBroadcast sends them to every rank over xGMI (the north_star's bitmap
//     broadcast), instead of every rank rebuilding them from its copy of R.
// librccl.so.1 is bound with dlopen at the first communicator, so a single-GPU process never maps
// it (HWBRJ_RCCL_LIB overrides the path).
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include <rccl/rccl.h>

#include "hwbrj_engine.h"

namespace hwbrj {

namespace {

struct Rccl {
    bool        ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*)                                          = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int)                   = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t)                                             = nullptr;
    ncclResult_t (*GroupStart)()                                                        = nullptr;
    ncclResult_t (*GroupEnd)()                                                          = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t)   = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t)                                         = nullptr;
};

const Rccl& rccl() {
    static Rccl      r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* path = getenv("HWBRJ_RCCL_LIB");
        void*       h    = dlopen(path ? path : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h && !path) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            r.err = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                all   = false;
                r.err = std::string("librccl.so.1 lacks ") + name;
            }
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.Send, "ncclSend");
        sym(r.Recv, "ncclRecv");
        sym(r.AllGather, "ncclAllGather");
        sym(r.Broadcast, "ncclBroadcast");
        sym(r.AllReduce, "ncclAllReduce");
        sym(r.GetErrorString, "ncclGetErrorString");
        r.ok = all;
    });
    return r;
}

int fail_rccl(const char* what, ncclResult_t e) {
    set_last_error(std::string(what) + ": " + rccl().GetErrorString(e));
    return 30;
}

int need_rccl() {
    if (rccl().ok) return 0;
    set_last_error(rccl().err);
    return 31;
}

#define RC_CALL(expr, what)                                     \
    do {                                                        \
        const ncclResult_t r_ = (expr);                         \
        if (r_ != ncclSuccess) return fail_rccl(what, r_);      \
    } while (0)

// ------------------------------------------------------------ the native hwbrj_exchange_t
// ctx is the Engine; every collective runs on its stream (the join's).
void* nx_buffer(void* ctx, int slot, uint64_t bytes) {
    Engine* e = (Engine*) ctx;
    if (slot < 0 || slot >= HWBRJ_PJ_NSLOTS) return nullptr;
    DevBuf* b = e->xslot(slot);
    return b->ensure(bytes) ? b->p : nullptr;
}

// The block a rank sends to itself is a copy on the join stream: RCCL's send/recv to self runs
// through its point-to-point protocol at a small fraction of HBM rate (measured at world 1: the
// R and survivor blocks, 0.1-0.5 GB, cost ~1 ms more than a device copy). HWBRJ_RCCL_SELF=1
// (tests) sends it through RCCL like the others, so a one-GPU run exercises ncclSend / ncclRecv.
bool rccl_self() { return getenv("HWBRJ_RCCL_SELF") != nullptr; }

int nx_alltoall_u64(void* ctx, const uint64_t* send, uint64_t* recv, uint64_t n) {
    Engine*        e  = (Engine*) ctx;
    const Rccl&    R  = rccl();
    const int      W  = e->comm_world();
    const int      me = e->comm_rank();
    if (!rccl_self()) {
        memcpy(recv + (uint64_t) me * n, send + (uint64_t) me * n, n * 8);
        if (W == 1) return 0;
    }
    hipStream_t    st = e->stream();
    ncclComm_t     c  = (ncclComm_t) e->comm();
    const uint64_t nb = (uint64_t) W * n * 8;
    if (!e->xcnt()->ensure(2 * nb)) {
        set_last_error("hipMalloc failed (exchange counts)");
        return 4;
    }
    uint64_t* ds = e->xcnt()->as<uint64_t>();
    uint64_t* dr = ds + (uint64_t) W * n;
    if (hipMemcpyAsync(ds, send, nb, hipMemcpyHostToDevice, st) != hipSuccess) return 1;
    RC_CALL(R.GroupStart(), "ncclGroupStart");
    for (int j = 0; j < W; j++) {
        if (j == me && !rccl_self()) continue;
        RC_CALL(R.Send(ds + (uint64_t) j * n, n, ncclUint64, j, c, st), "ncclSend (counts)");
        RC_CALL(R.Recv(dr + (uint64_t) j * n, n, ncclUint64, j, c, st), "ncclRecv (counts)");
    }
    RC_CALL(R.GroupEnd(), "ncclGroupEnd");
    std::vector<uint64_t> own(n);
    memcpy(own.data(), recv + (uint64_t) me * n, n * 8);
    if (hipMemcpyAsync(recv, dr, nb, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    if (!rccl_self()) memcpy(recv + (uint64_t) me * n, own.data(), n * 8);
    return 0;
}

int nx_alltoallv(void* ctx, int sslot, const uint64_t* soff, const uint64_t* sbytes, int rslot,
                 const uint64_t* roff, const uint64_t* rbytes) {
    Engine*       e  = (Engine*) ctx;
    const Rccl&   R  = rccl();
    const int     W  = e->comm_world();
    ncclComm_t    c  = (ncclComm_t) e->comm();
    const uint8_t* s = (const uint8_t*) e->xslot(sslot)->p;
    uint8_t*      d  = (uint8_t*) e->xslot(rslot)->p;
    const int     me = e->comm_rank();
    if (!rccl_self() && sbytes[me]) {  // (rbytes[me] == sbytes[me]: the counts this rank sent itself)
        if (hipMemcpyAsync(d + roff[me], s + soff[me], sbytes[me], hipMemcpyDeviceToDevice, e->stream()) != hipSuccess) {
            set_last_error("device copy of the rank's own block failed");
            return 1;
        }
    }
    if (W == 1 && !rccl_self()) return 0;
    // a block of 0 bytes is neither sent nor received (its peer sees the same 0 in its counts)
    RC_CALL(R.GroupStart(), "ncclGroupStart");
    for (int j = 0; j < W; j++) {
        if (j == me && !rccl_self()) continue;
        if (sbytes[j]) RC_CALL(R.Send(s + soff[j], sbytes[j], ncclUint8, j, c, e->stream()), "ncclSend");
        if (rbytes[j]) RC_CALL(R.Recv(d + roff[j], rbytes[j], ncclUint8, j, c, e->stream()), "ncclRecv");
    }
    RC_CALL(R.GroupEnd(), "ncclGroupEnd");
    return 0;
}

int nx_allgather(void* ctx, int slot, uint64_t bytes) {
    Engine*  e    = (Engine*) ctx;
    uint8_t* base = (uint8_t*) e->xslot(slot)->p;
    // in place: rank r's block already sits at r * bytes
    RC_CALL(rccl().AllGather(base + (uint64_t) e->comm_rank() * bytes, base, bytes, ncclUint8,
                             (ncclComm_t) e->comm(), e->stream()),
            "ncclAllGather (filter slices)");
    return 0;
}

}  // namespace

// All-to-all of n u64 per rank between device buffers, enqueued on the engine's stream (no host
// synchronisation): the partitioned join's counts messages (d_send[j n ..) to rank j).
int rccl_alltoall_u64_dev(Engine* e, const uint64_t* d_send, uint64_t* d_recv, uint64_t n) {
    const int   W  = e->comm_world();
    const int   me = e->comm_rank();
    hipStream_t st = e->stream();
    if (!rccl_self() &&
        hipMemcpyAsync(d_recv + (uint64_t) me * n, d_send + (uint64_t) me * n, n * 8, hipMemcpyDeviceToDevice, st) != hipSuccess) {
        set_last_error("device copy of the rank's own counts failed");
        return 1;
    }
    if (W == 1 && !rccl_self()) return 0;
    if (int rc = need_rccl()) return rc;
    const Rccl& R = rccl();
    ncclComm_t  c = (ncclComm_t) e->comm();
    RC_CALL(R.GroupStart(), "ncclGroupStart");
    for (int j = 0; j < W; j++) {
        if (j == me && !rccl_self()) continue;
        RC_CALL(R.Send(d_send + (uint64_t) j * n, n, ncclUint64, j, c, st), "ncclSend (counts)");
        RC_CALL(R.Recv(d_recv + (uint64_t) j * n, n, ncclUint64, j, c, st), "ncclRecv (counts)");
    }
    RC_CALL(R.GroupEnd(), "ncclGroupEnd");
    return 0;
}

bool rccl_self_blocks() { return rccl_self(); }

// In-place max over the ranks of n u64 in device memory, on the engine's stream (the async
// partitioned join's overflow flag and exchange sizes; a no-op at world 1 but with HWBRJ_RCCL_SELF).
int rccl_allreduce_max_u64(Engine* e, uint64_t* d, uint64_t n) {
    if (e->comm_world() == 1 && !rccl_self()) return 0;
    if (int rc = need_rccl()) return rc;
    RC_CALL(rccl().AllReduce(d, d, n, ncclUint64, ncclMax, (ncclComm_t) e->comm(), e->stream()),
            "ncclAllReduce (max)");
    return 0;
}

int rccl_broadcast(void* comm, void* buf, size_t bytes, int root, hipStream_t stream) {
    if (int rc = need_rccl()) return rc;
    RC_CALL(rccl().Broadcast(buf, buf, bytes, ncclUint8, root, (ncclComm_t) comm, stream),
            "ncclBroadcast (filter slices)");
    return 0;
}

// Status agreement before a collective: every rank contributes its status word to an
// in-place ncclAllGather and reads all of them back (host-synchronous), so a rank that failed
// alone (an allocation, a size check) makes every rank return instead of leaving its peers in the
// collective. Returns rc (this rank's own failure), 22 if another rank failed, 30/31 on RCCL errors.
int rccl_agree_status(void* comm, int world, int rank, int rc, hipStream_t stream, DevBuf* tmp) {
    if (int e = need_rccl()) return rc ? rc : e;
    if (!tmp->ensure((size_t) world * 8)) {  // (allocated by comm_init: this does not allocate)
        set_last_error("hipMalloc failed (status agreement)");
        rc = rc ? rc : 4;
    }
    std::vector<uint64_t> st(world, 0);
    st[rank] = (uint64_t) (uint32_t) rc;
    if (tmp->p == nullptr) return rc;  // no buffer at all: nothing can be exchanged
    uint64_t* d = tmp->as<uint64_t>();
    if (hipMemcpyAsync(d + rank, &st[rank], 8, hipMemcpyHostToDevice, stream) != hipSuccess) return rc ? rc : 1;
    RC_CALL(rccl().AllGather(d + rank, d, 1, ncclUint64, (ncclComm_t) comm, stream), "ncclAllGather (status)");
    if (hipMemcpyAsync(st.data(), d, (size_t) world * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return rc ? rc : 1;
    if (rc) return rc;  // (this rank's own message stays)
    for (int j = 0; j < world; j++)
        if (st[j]) {
            set_last_error("rank " + std::to_string(j) + " failed (code " + std::to_string(st[j]) + ")");
            return 22;
        }
    return 0;
}

int Engine::comm_init(const uint8_t* unique_id, int world, int rank) {
    if (int rc = need_rccl()) return rc;
    if (world < 1 || rank < 0 || rank >= world) {
        set_last_error("rank must lie in [0, world)");
        return 2;
    }
    if (hipSetDevice(device_) != hipSuccess) {
        set_last_error("hipSetDevice failed");
        return 1;
    }
    comm_destroy();  // (drops the async join's plan and joins in flight)
    ncclUniqueId id;
    static_assert(sizeof(id.internal) == NCCL_UNIQUE_ID_BYTES, "unique id size");
    memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    RC_CALL(rccl().CommInitRank(&c, world, id, rank), "ncclCommInitRank");
    comm_       = c;
    comm_world_ = world;
    comm_rank_  = rank;
    // the status agreement's words, allocated here: an agreement never allocates, so a
    // rank whose big allocations just failed still takes part in it
    if (!agree_.ensure(std::max<size_t>(64, (size_t) world * 8))) {
        (void) comm_destroy();
        set_last_error("hipMalloc failed (status agreement words)");
        return 4;
    }
    return 0;
}

int Engine::comm_destroy() {
    if (!comm_) return 0;
    (void) hipSetDevice(device_);
    (void) hipStreamSynchronize(own_stream_);
    pj_plan_ = PjPlan{};  // (the plan and the joins in flight belong to the communicator)
    pj_q_.clear();
    const ncclResult_t e = rccl().CommDestroy((ncclComm_t) comm_);
    comm_       = nullptr;
    comm_world_ = 1;
    comm_rank_  = 0;
    return e == ncclSuccess ? 0 : fail_rccl("ncclCommDestroy", e);
}

int Engine::join_partitioned_rccl(const uint2* dR, uint64_t nR, uint64_t nR_total, const uint2* dS,
                                  uint64_t nS, const bloom_filter_args_t* args, hwbrj_stats_t* st) {
    if (!comm_) {
        set_last_error("no communicator on this device (hwbrj_comm_init)");
        return 32;
    }
    if (const int rc = pj_drain()) return rc;  // (async joins in flight use the buffers it may grow)
    const hwbrj_exchange_t x = native_exchange();
    return join_partitioned(&x, comm_rank_, comm_world_, dR, nR, nR_total, dS, nS, args, st, true);
}

hwbrj_exchange_t Engine::native_exchange() {
    hwbrj_exchange_t x;
    x.ctx          = this;
    x.buffer       = nx_buffer;
    x.alltoall_u64 = nx_alltoall_u64;
    x.alltoallv    = nx_alltoallv;
    x.allgather    = nx_allgather;
    return x;
}

}  // namespace hwbrj

using namespace hwbrj;

extern "C" {

int hwbrj_comm_unique_id(uint8_t* out) {
    if (int rc = need_rccl()) return rc;
    ncclUniqueId id;
    RC_CALL(rccl().GetUniqueId(&id), "ncclGetUniqueId");
    memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int hwbrj_comm_init(const uint8_t* unique_id, int world, int rank) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->comm_init(unique_id, world, rank);
}

int hwbrj_comm_destroy(void) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->comm_destroy();
}

int hwbrj_comm_info(int* world, int* rank) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    if (!e->has_comm()) {
        set_last_error("no communicator on this device (hwbrj_comm_init)");
        return 32;
    }
    if (world) *world = e->comm_world();
    if (rank) *rank = e->comm_rank();
    return 0;
}

int hwbrj_set_filter_broadcast(int on) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    e->set_filter_broadcast(on != 0);
    return 0;
}

int hwbrj_join_partitioned_rccl(const tuple_t* d_R, uint64_t nR, uint64_t nR_total, const tuple_t* d_S,
                                uint64_t nS, const bloom_filter_args_t* args, hwbrj_stats_t* stats) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->join_partitioned_rccl((const uint2*) d_R, nR, nR_total, (const uint2*) d_S, nS, args, stats);
}

}  // extern "C"
