// hwbrj_engine.h -- host-side orchestration of the MI355X join pipeline (internal C++).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <deque>
#include <string>
#include <vector>

#include "../../include/hwbrj.h"
#include "hwbrj_common.h"
#include "hwbrj_kernels.h"

namespace hwbrj {

// Picks mode / partitioning / slice geometry for a filter configuration (DESIGN.md "Modes").
// Returns false (and sets *err) for configurations outside the reference's contract.
// mat: the materializing pipeline's geometry (join jobs sized for its hash
// table, k_join_mat).
bool plan_geometry(const bloom_filter_args_t* args, uint64_t nR, Geometry* g, std::string* err,
                   bool mat = false);

// A materializing join's output: {R.payload, S.payload} pairs into out[0, cap).
struct MatReq {
    uint2*   out;
    uint64_t cap;
};
constexpr int kRcMatGlobal = 11;  // run_mat: global-bitmap mode, use the side pass (materialize)

struct DevBuf {
    void*  p     = nullptr;
    size_t bytes = 0;
    bool   ensure(size_t need);  // grow-only
    void   release();
    template <class T> T* as() const { return (T*) p; }
};

class Engine {
  public:
    explicit Engine(int device);
    ~Engine();
    // Synchronous join of device-resident tuples. Returns 0 on success.
    // jkind: the per-partition join (JoinParams::jkind: 0 PRO, 1 PRH, 2 PRHO).
    int  run(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
             const bloom_filter_args_t* args, hipStream_t stream, hwbrj_stats_t* st, int jkind = 0);
    // Enqueue only (wait = false in run): wait() then waits for the last enqueued join.
    int  run_async(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                   const bloom_filter_args_t* args, hipStream_t stream, int jkind = 0);
    int  wait(hwbrj_stats_t* st);
    // Every join enqueued since the last wait / wait_all, oldest first, each with its own counts
    // (they stay on the device in a ring of kJoinRing result slots, one per join; an enqueue that
    // finds the ring full collects it on the host first). *n = the number of joins; 7 when it
    // exceeds cap (the oldest cap are written).
    static constexpr int kJoinRing = 64;
    int  wait_all(hwbrj_stats_t* st, int cap, int* n);
    // async joins time their S scatter (the dominant kernel) with events on the side stream they
    // run it on: stats ms_s_scatter of every collected join (include/hwbrj.h hwbrj_set_async_timing)
    void set_async_timing(bool on) { async_timing_ = on; }
    // Allocates every buffer a join of these inputs needs, without launching it (the host BPRO
    // stages this before its timed region, like the reference's allocations before its timer).
    int  reserve(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                 const bloom_filter_args_t* args, int jkind = 0);
    int  export_filter(uint8_t* host_out, uint64_t nbytes);
    // The materializing join (the partitioned pipeline carrying payloads): st->matches = pairs
    // (all of them, also beyond cap). kRcMatGlobal: not for the global-bitmap mode.
    int  run_mat(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                 const bloom_filter_args_t* args, hipStream_t stream, const MatReq& mat,
                 hwbrj_stats_t* st);
    // Side pass after a counting join (global-bitmap mode): (R.payload, S.payload) of every match
    // into out[0, cap); *n = number of pairs.
    int  materialize(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS, uint2* out,
                     uint64_t cap, uint64_t* n, hipStream_t stream, double* ms);
    int  generate(uint2* d_out, uint64_t n, uint64_t offset, uint64_t count, uint32_t nthreads,
                  uint64_t maxid, uint64_t threshold, double selectivity, uint64_t seed,
                  hipStream_t stream);
    // The partitioned multi-GPU join of rank `rank` (include/hwbrj.h hwbrj_join_partitioned).
    // native: x is the library's own RCCL exchange, whose collectives are enqueued on this
    // engine's stream (no host synchronisation before them).
    int  join_partitioned(const hwbrj_exchange_t* x, int rank, int world, const uint2* dR,
                          uint64_t nR, uint64_t nR_total, const uint2* dS, uint64_t nS,
                          const bloom_filter_args_t* args, hwbrj_stats_t* st, bool native = false);
    void release();
    int  device() const { return device_; }

    // ---- native RCCL transport (hwbrj_comm.cpp) ----
    int  comm_init(const uint8_t* unique_id, int world, int rank);
    int  comm_destroy();
    bool has_comm() const { return comm_ != nullptr; }
    int  comm_world() const { return comm_world_; }
    int  comm_rank() const { return comm_rank_; }
    // the partitioned join over this engine's communicator
    int  join_partitioned_rccl(const uint2* dR, uint64_t nR, uint64_t nR_total, const uint2* dS,
                               uint64_t nS, const bloom_filter_args_t* args, hwbrj_stats_t* st);
    // replicated design: the filter slices built on rank 0 only and broadcast (ncclBroadcast on the
    // join stream) instead of rebuilt from R on every rank
    void set_filter_broadcast(bool on) { bcast_ = on; }
    hipStream_t stream() const { return own_stream_; }
    DevBuf*     xslot(int s) { return &xslot_[s]; }
    DevBuf*     xcnt() { return &xcnt_; }
    void*       comm() const { return comm_; }
    // the library's own RCCL exchange (hwbrj_comm.cpp): collectives on this engine's stream
    hwbrj_exchange_t native_exchange();

    // ---- the async partitioned join (hwbrj_pjoin_async.cpp; include/hwbrj.h) ----
    static constexpr int kPjDepth = 8;   // joins in flight (result ring slots)
    static constexpr int kPjKey   = 10;  // words of a plan's shape key
    // x == nullptr: over this engine's RCCL communicator (no host wait); else the caller's
    // exchange callbacks (host-synchronous exchanges, the same padded layout and plan)
    int  join_partitioned_async(const hwbrj_exchange_t* x, int rank, int world, const uint2* dR, uint64_t nR,
                                uint64_t nR_total, const uint2* dS, uint64_t nS, const bloom_filter_args_t* args);
    int  join_partitioned_wait(hwbrj_stats_t* st);
    void pj_async_info(uint64_t* out) const;
    // end of a synchronous native join asked for a plan (pj_make_plan()): a collective
    bool pj_make_plan() const { return pj_make_plan_; }
    int  pj_plan_from_sync(int world, int rank, uint64_t nR, uint64_t nR_total, uint64_t nS,
                           const bloom_filter_args_t* args, uint64_t mr, uint64_t mi, uint64_t mw);
    // drains the joins in flight (before a synchronous join grows buffers they use)
    int  pj_drain();

  private:
    struct PjGeom {
        Geometry g{};
        uint32_t F = 0, NSUB = 0, W = 0, QL = 0, q0 = 0, nseg = 1, CH = 0, G = 0, NC = 0, items_max = 0;
        uint64_t BSW = 0, SLOT = 0, capR = 0, capS = 0, LS = 0;
        bool     slice_mode = false;
    };
    struct PjPlan {
        bool     valid = false;
        uint64_t BR = 0, BI = 0, BW = 0;  // block bounds: R chunks, survivor items, survivor words
        uint64_t key[kPjKey] = {};
    };
    struct PjX {  // the transport of an async join
        hwbrj_exchange_t x{};
        bool             native = true;
        int              rank = 0, world = 1;
    };
    struct PjIn {
        PjX                 xc;
        const uint2*        dR = nullptr;
        const uint2*        dS = nullptr;
        uint64_t            nR = 0, nR_total = 0, nS = 0;
        bool                has_args = false;
        bloom_filter_args_t args{};
    };
    struct PjPending {
        PjIn          in;
        PjGeom        G;
        bool          sync = false;  // ran synchronously at enqueue (made the plan): rc, st
        bool          failed_mode = false;
        int           rc   = 0;
        int           slot = 0;
        hwbrj_stats_t st{};
    };
    bool pj_geom(int world, int rank, uint64_t nR, uint64_t nR_total, uint64_t nS,
                 const bloom_filter_args_t* args, PjGeom* G);
    int  pj_async_alloc(const PjGeom& G, const PjPlan& p, bool all, const PjX& c);
    int  pj_a2a_u64(const PjX& c, const uint64_t* d_send, uint64_t* d_recv, uint64_t n);
    int  pj_max_dev(const PjX& c, uint64_t* d, uint64_t n);
    int  pj_max_host(const PjX& c, uint64_t* h, uint64_t n);
    int  pj_establish_plan(const PjGeom& G, uint64_t mr, uint64_t mi, uint64_t mw, const uint64_t* key);
    int  pj_sync_join(const PjIn& in, hwbrj_stats_t* st);
    PjPlan                pj_plan_;
    PjX                   pj_cur_;  // the transport of the synchronous join making a plan
    bloom_filter_args_t   pj_plan_args_{};
    bool                  pj_make_plan_ = false;
    bool                  pj_lost_      = false;  // the plan's buffers were released (this rank)
    std::deque<PjPending> pj_q_;
    uint64_t              pj_seq_ = 0, pj_async_ = 0, pj_sync_ = 0, pj_fallbacks_ = 0, pj_plans_ = 0;
    uint64_t              pj_last_flag_ = 0, pj_last_sizes_[3] = {0, 0, 0};
    DevBuf                pjX, pjRitems, pjRing;  // flag + sizes + counts messages; ritems; result ring
    hipEvent_t            pjEv_[2 * kPjDepth] = {};

  private:
    void*        comm_       = nullptr;  // ncclComm_t of this device's rank (hwbrj_comm_init)
    int          comm_world_ = 1, comm_rank_ = 0;
    bool         bcast_      = false;
    DevBuf       xslot_[HWBRJ_PJ_NSLOTS], xcnt_;  // the native exchange's buffers
    DevBuf       agree_;                           // status words of the broadcast join's agreement
    int          device_;
    int          cus_ = 256;
    hipStream_t  own_stream_ = nullptr;
    hipStream_t  ovl_stream_ = nullptr;             // dev A/B HWBRJ_DEV_OVL: the S pass's stream
    hipEvent_t   ovl_ev_[2]  = {nullptr, nullptr};  // (fork, join of ovl_stream_)
    hipEvent_t   ev_[10];
    bool         have_filter_ = false;
    Geometry     last_g_{};
    // the last enqueued join (collected by wait)
    bool         pending_      = false;
    bool         pending_args_ = false;
    uint64_t     pending_nS_   = 0;
    uint32_t     last_nj_      = 0;  // join jobs of the last enqueue (job_surv layout)
    // phase events: recorded by synchronous joins only (run_async clears phase_ev_); surv_fused_:
    // the pending join's survivor phase is fused into its probe (no ev_[7] of its own)
    bool         phase_ev_     = true;
    bool         pending_ev_   = true;
    // the stream the pending join was enqueued on. Joins on the same stream are ordered by it; a
    // join on another stream waits for ev_[8]. Compared by handle: a stream must outlive the
    // joins enqueued on it (a destroyed stream's handle can be reused by a new one).
    hipStream_t  pending_stream_ = nullptr;
    bool         pending_sfirst_ = false;  // the pending join ran its S pass first (phase boundaries)
    bool         pending_fmt_    = false;  // the pending join counted its unstaged probe items
    bool         pending_slots_  = false;  // the pending join's matches are in k_join's partial sums
    bool         pack3_hint_     = true;   // the last waited join had none: packed join keys pay
    int          pending_rc_     = 0;   // nonzero: the pending join failed after enqueuing kernels
    std::string  pending_err_;
    bool         surv_fused_   = false;
    // per-join results: join i writes its counts and k_join's partial sums into ring slot
    // i mod kJoinRing (jring_), so every join of a back-to-back run can be checked, not only the
    // last (the reference sums every thread's count per run, parallel_radix_join_bloom.c:1696-1707)
    struct JoinRec {
        uint32_t slot = 0;
        bool     args = false, fmt = false, slots = false, timed = false;
        uint32_t kbits = 0;  // packed join-key bits (0: 32-bit codes)
        uint64_t nS   = 0;
        Geometry g{};
    };
    DevBuf                     jring_;
    std::vector<JoinRec>       jr_;     // enqueued since the last wait, oldest first
    std::vector<hwbrj_stats_t> jdone_;  // collected early (the ring was full), oldest first
    uint32_t                   jr_next_ = 0;
    hwbrj_stats_t              last_st_{};  // the last collected join (with its phase times)
    bool                       async_timing_ = false;      // hwbrj_set_async_timing
    hipEvent_t                 tev_[kJoinRing][2] = {};    // per slot: the async S scatter's start, end
    void*        ring_take(uint32_t* slot);            // the next slot's bytes (jring_ grown first)
    void         ring_push(const JoinRec& r) { jr_.push_back(r); }
    int          ring_collect();                       // jr_ (completed) -> jdone_
    void         ring_drop() { jr_.clear(); jdone_.clear(); }
    hipError_t   mark(int i, hipStream_t stream);  // ev_[i] when phase_ev_
    bool         alloc_only_   = false;  // reserve(): enqueue returns after its allocations
    int          enqueue(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                         const bloom_filter_args_t* args, hipStream_t stream, bool dbg, int jkind,
                         const MatReq* mat = nullptr);
    // basic k >= 2 without materialization: the repartitioning pipeline (hwbrj_engine.cpp)
    int          enqueue_basic_kk(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                                  const Geometry& g, hipStream_t stream, int jkind);
    CrcTables*   d_tabs_ = nullptr;
    GenPlan*     d_plan_ = nullptr;
    // R side
    DevBuf poolR, metaR, usedR, wgqcR, wgqeR, wgqoR, lstartR, estartR, istartR, listR;
    // S side
    DevBuf poolS, metaS, usedS, wgqcS, wgqeS, wgqoS, lstartS, estartS, istartS, listS;
    DevBuf slices, bitmap, rjoin, rrun, surv, survcnt, survoff, dense, small, dbgP, dbgJ, dbgS;
    DevBuf bpos;        // basic k >= 2: R bit positions (k_bitpos)
    DevBuf colR, colS;  // per-partition totals from k_plan: u64 elements [F], then u32 chunks [F]
    DevBuf mtab, mcount;  // materialization (side pass): R table, pair counter
    // materializing pipeline: payload pools (chunk layout of poolR / poolS), R payloads of the
    // build sweeps, survivors' chunk positions
    DevBuf ppoolR, ppoolS, rpay, survpos;
    DevBuf dense2, kkcnt;  // basic k >= 2: the second dense candidate buffer, per-pass counts
    DevBuf jtask, jparts;  // join task table; parts per job (+ the task count)
    // partitioned join: owned partitions' lists, tables and received survivor descriptors
    DevBuf pjList, pjLstart, pjSweep, pjTab, pjRegion, pjTot, pjSoff, pjIbase, pjCnt, pjOff, pjIstart, pjJobs;
    DevBuf pjBsum, pjBound, pjWtot, pjWscan, pjTab2;  // device-side item tables (scans, bounds)
};

Engine* engine_for_current_device();
void    set_last_error(const std::string& s);

// RCCL entry points used by the engine (hwbrj_comm.cpp; librccl is bound at first use). Return 0 or
// an error code with the message in set_last_error.
int rccl_broadcast(void* comm, void* buf, size_t bytes, int root, hipStream_t stream);
// The counts a join leaves in the small buffer (`small`: result words, then k_join's partial-sum
// slots), read in one copy: h[0] matches, h[1] dense count, h[2] filtered, h[3] probe ticks,
// h[4] join ticks, h[5] unstaged probe items; with slots, their sums are added to h[0], h[3], h[4].
int read_join_counts(const void* small, bool slots, hipStream_t stream, uint64_t h[6]);
int rccl_agree_status(void* comm, int world, int rank, int rc, hipStream_t stream, DevBuf* tmp);
class Engine;
int rccl_alltoall_u64_dev(Engine* e, const uint64_t* d_send, uint64_t* d_recv, uint64_t n);
int rccl_allreduce_max_u64(Engine* e, uint64_t* d, uint64_t n);
// HWBRJ_RCCL_SELF (tests): a rank's own exchange blocks go through ncclSend / ncclRecv too
bool rccl_self_blocks();
// chunks of a shard's partition pool for n tuples over G scatter workgroups and F partitions
uint64_t pj_region_cap(uint64_t n, uint32_t G, uint32_t F);

// glibc's rand() (stdlib/random_r.c TYPE_3) with private state (hwbrj_gen.cpp).
struct GlibcRand {
    int32_t st[31];
    int     f = 3, r = 0;
    void    seed(uint32_t s);
    int32_t next() {
        st[f]           = (int32_t) ((uint32_t) st[f] + (uint32_t) st[r]);
        const int32_t v = (int32_t) ((uint32_t) st[f] >> 1);
        f               = f == 30 ? 0 : f + 1;
        r               = r == 30 ? 0 : r + 1;
        return v;
    }
};

}  // namespace hwbrj
