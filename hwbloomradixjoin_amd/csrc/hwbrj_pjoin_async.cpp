// hwbrj_pjoin_async.cpp -- the partitioned multi-GPU join without host waits (VERDICT r4 item 7;
// DESIGN.md s6).
//
// The synchronous native join (hwbrj_pjoin.cpp) waits on the host for two counts messages: RCCL
// takes the element counts of a send from the host, so every variable all-to-all is sized by a host
// read. This path sizes them from a plan instead: every (source, destination) block of the R-chunk
// and survivor all-to-alls is padded to a bound all ranks agreed on (the largest block of an earlier
// synchronous join of the same shapes, plus headroom), so the whole join -- counts messages, padded
// exchanges, the owner's tables (k_pjx_rtab / k_pjx_stab build on the device what the host built),
// build, probe and join -- is enqueued on the join stream with no host wait, and K joins run back to
// back. Each join's counts are copied into a ring slot of its own at its end, so up to kPjDepth
// joins can be in flight; hwbrj_join_partitioned_wait collects them in order.
//
// Overflow: a block that does not fit sets a device flag (what is read stays inside the padded
// buffers: the owner's tables clamp every count to its block); the flag is all-reduced (MAX) at the
// end of the join with the join's block sizes, and the wait of a flagged join reruns it
// synchronously on every rank (every rank sees the same all-reduced flag), which makes a new plan.
//
// Collective state: the plan is made by a synchronous join (its block maxima all-reduced; every
// rank allocates the padded buffers and the ranks agree that all could), so it is valid on all
// ranks or on none, and it is dropped on all ranks alike (an all-reduced flag). A rank whose
// shapes do not match the plan (its shard sizes or the filter changed, or its buffers were
// released) cannot tell its peers before the join's first collective: it takes part in every
// collective of the join with empty messages and a failed status (the failed mode), and the flag
// reruns the join on every rank. So all ranks always issue the same collectives in the same order.
#include <string.h>

#include <algorithm>
#include <functional>
#include <vector>

#include "hwbrj_engine.h"

namespace hwbrj {

#define PX_CHECK(expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_last_error(std::string(#expr) + ": " + hipGetErrorString(e_));             \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

// (k_pjx_*'s flag bit for a failed source)
static const uint64_t kFlagPeerFailed = 2;

// The shape key of a plan: a join may use the plan only if every word matches.
static void pj_shape(uint64_t* k, int world, int rank, uint64_t nR, uint64_t nR_total, uint64_t nS,
                     const bloom_filter_args_t* a) {
    const uint64_t v[Engine::kPjKey] = {(uint64_t) world, (uint64_t) rank, nR, nR_total, nS, a ? 1u : 0u,
                                        a ? (uint64_t) a->variant : 0u, a ? a->m : 0u, a ? a->k : 0u,
                                        a ? a->B : 0u};
    memcpy(k, v, sizeof v);
}

// Bytes of one ring slot: the small buffer's result words and k_join's partial-sum slots, then the
// join's flag and the all-reduced {flag, R block, item block, word block}.
static size_t ring_counts_bytes() { return (16 + (size_t) join_sum_slots() * join_sum_stride()) * 8; }
static size_t ring_slot_bytes() { return ring_counts_bytes() + 64; }

bool Engine::pj_geom(int world, int rank, uint64_t nR, uint64_t nR_total, uint64_t nS, const bloom_filter_args_t* args,
                     PjGeom* G) {
    std::string err;
    if (!plan_geometry(args, nR_total, &G->g, &err)) {
        set_last_error(err);
        return false;
    }
    Geometry& g = G->g;
    if (g.mode == MODE_GLOBAL || (g.mode == MODE_SLICE_BASIC && g.k > 1)) {
        set_last_error("the partitioned join needs partition slices (blocked/sectorized, basic k = 1, or no filter)");
        return false;
    }
    g.s_format = g.format;
    G->F       = 1u << g.log2F;
    G->NSUB    = 1u << g.log2NSUB;
    // (the owner's table kernels stage the F = W QL pairs in LDS: F <= 1024)
    if (world < 1 || rank < 0 || rank >= world || G->F % (uint32_t) world != 0 || G->F > 1024) {
        set_last_error("world must divide the partition count F = " + std::to_string(G->F));
        return false;
    }
    G->W          = (uint32_t) world;
    G->QL         = G->F / G->W;
    G->q0         = (uint32_t) rank * G->QL;
    G->slice_mode = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    G->nseg       = G->slice_mode ? g.nseg : 1;
    G->CH         = probe_chunks_per_item();
    G->BSW        = build_chunks_per_sweep();
    G->SLOT       = build_sweep_slot();
    const size_t sc_lds = scatter_lds_bytes(g.log2F);
    G->G         = (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / sc_lds));
    G->capR      = pj_region_cap(nR, G->G, G->F);
    G->capS      = pj_region_cap(nS, G->G, G->F);
    G->LS        = (uint64_t) G->G * G->capS;
    G->items_max = (uint32_t) ((G->LS / G->CH + G->F + 1) * G->nseg);
    G->NC        = G->QL + 4;
    return true;
}

// The exchange buffers and tables of an async join under plan p (grow-only). `all`: also what only
// a join that computes needs (a rank in the failed mode only exchanges).
int Engine::pj_async_alloc(const PjGeom& G, const PjPlan& p, bool all, const PjX& c) {
    const hwbrj_exchange_t& x = c.x;
    const uint64_t   W = G.W, NSUB = G.NSUB, QL = G.QL;
    bool             ok = true;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_R_SEND, W * p.BR * 128 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_R_SEND_ENT, W * p.BR * 4 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_R_RECV, W * p.BR * 128 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_R_RECV_ENT, W * p.BR * 4 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_S_SEND, W * p.BW * 4 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_S_RECV, W * p.BW * 4 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_M_SEND, W * p.BI * NSUB * 4 + 16) != nullptr;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_M_RECV, W * p.BI * NSUB * 4 + 16) != nullptr;
    const uint64_t slice_bytes = G.slice_mode ? (uint64_t) G.F * G.nseg * G.g.seg_words * 4 : 16;
    ok &= x.buffer(x.ctx, HWBRJ_PJ_SLICES, slice_bytes) != nullptr;
    // pjX: [0] flag, [1, 5) the all-reduced flag and block sizes, [8, ...) the two counts messages
    // (send, receive each)
    ok &= pjX.ensure((8 + 4 * W * G.NC) * 8) && pjRing.ensure(kPjDepth * ring_slot_bytes());
    for (int i = 0; i < 2 * kPjDepth && ok; i++)
        if (!pjEv_[i]) ok &= hipEventCreate(&pjEv_[i]) == hipSuccess;
    if (all) {
        const uint64_t sweeps_max = W * p.BR / G.BSW + QL + 1, RI = W * p.BI;
        ok &= pjList.ensure(W * p.BR * 4 + 16) && rjoin.ensure(sweeps_max * G.SLOT * 4) &&
              rrun.ensure(2 * sweeps_max * NSUB * 4);
        ok &= pjTab.ensure(4 * QL * W * 8) && pjLstart.ensure((QL + 1) * 4) && pjSweep.ensure((QL + 1) * 4);
        ok &= pjIbase.ensure(RI * 8 + 16) && pjCnt.ensure(RI * NSUB * 4 + 16) && pjOff.ensure(RI * NSUB * 4 + 16) &&
              pjJobs.ensure(QL * NSUB * 4) && pjWtot.ensure(RI * 4 + 16) && pjWscan.ensure((RI + 1) * 8) &&
              pjBsum.ensure((std::max<uint64_t>(RI, G.items_max) / 1024 + 1) * 8);
        ok &= pjTab2.ensure(3 * QL * W * 4) && pjIstart.ensure((QL + 1) * 4) && pjRitems.ensure(W * 4 + 16);
        ok &= pjRegion.ensure((uint64_t) G.items_max * 8 + 8) && pjTot.ensure((uint64_t) G.items_max * 4 + 4) &&
              pjSoff.ensure((uint64_t) G.items_max * 8 + 8) && pjBound.ensure((uint64_t) (G.F + 1) * 8);
    }
    if (!ok) set_last_error("hipMalloc failed (async partitioned join buffers)");
    return ok ? 0 : 4;
}

// The collectives of an async join on either transport. Native: RCCL on the join stream, no host
// wait. Callbacks: host-synchronous (the join stream drained, the words through the host).
int Engine::pj_a2a_u64(const PjX& c, const uint64_t* d_send, uint64_t* d_recv, uint64_t n) {
    if (c.native) return rccl_alltoall_u64_dev(this, d_send, d_recv, n);
    const uint64_t        W = (uint64_t) c.world;
    std::vector<uint64_t> hs(W * n), hr(W * n);
    PX_CHECK(hipMemcpyAsync(hs.data(), d_send, W * n * 8, hipMemcpyDeviceToHost, own_stream_));
    PX_CHECK(hipStreamSynchronize(own_stream_));
    if (c.x.alltoall_u64(c.x.ctx, hs.data(), hr.data(), n) != 0) {
        set_last_error("exchange failed: counts");
        return 20;
    }
    PX_CHECK(hipMemcpyAsync(d_recv, hr.data(), W * n * 8, hipMemcpyHostToDevice, own_stream_));
    PX_CHECK(hipStreamSynchronize(own_stream_));  // (hr is scoped)
    return 0;
}

int Engine::pj_max_host(const PjX& c, uint64_t* h, uint64_t n) {
    if (c.native) {  // (the agreement words: allocated by comm_init, >= 8 words)
        uint64_t* d = agree_.as<uint64_t>();
        if (!d || agree_.bytes < n * 8) {
            set_last_error("no communicator words for the plan");
            return 32;
        }
        PX_CHECK(hipMemcpyAsync(d, h, n * 8, hipMemcpyHostToDevice, own_stream_));
        if (const int rc = rccl_allreduce_max_u64(this, d, n)) return rc;
        PX_CHECK(hipMemcpyAsync(h, d, n * 8, hipMemcpyDeviceToHost, own_stream_));
        PX_CHECK(hipStreamSynchronize(own_stream_));
        return 0;
    }
    const uint64_t        W = (uint64_t) c.world;
    std::vector<uint64_t> hs(W * n), hr(W * n);
    for (uint64_t j = 0; j < W; j++) memcpy(&hs[j * n], h, n * 8);
    if (c.x.alltoall_u64(c.x.ctx, hs.data(), hr.data(), n) != 0) {
        set_last_error("exchange failed: plan words");
        return 20;
    }
    for (uint64_t j = 0; j < W; j++)
        for (uint64_t i = 0; i < n; i++) h[i] = std::max(h[i], hr[j * n + i]);
    return 0;
}

int Engine::pj_max_dev(const PjX& c, uint64_t* d, uint64_t n) {
    if (c.native) return rccl_allreduce_max_u64(this, d, n);
    std::vector<uint64_t> h(n);
    PX_CHECK(hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, own_stream_));
    PX_CHECK(hipStreamSynchronize(own_stream_));
    if (const int rc = pj_max_host(c, h.data(), n)) return rc;
    PX_CHECK(hipMemcpyAsync(d, h.data(), n * 8, hipMemcpyHostToDevice, own_stream_));
    PX_CHECK(hipStreamSynchronize(own_stream_));  // (h is scoped)
    return 0;
}

// Called by every rank at the end of a synchronous partitioned join asked to make a plan
// (pj_make_plan_): this rank's largest blocks (R chunks, survivor items, survivor words it sent or
// received) are max-reduced over the ranks, the bounds get headroom, every rank allocates the padded
// buffers, and the ranks agree (a second max-reduction) that all could: the plan is valid on all or
// on none. (The transport is pj_cur_, the synchronous join's.)
int Engine::pj_establish_plan(const PjGeom& G, uint64_t mr, uint64_t mi, uint64_t mw, const uint64_t* key) {
    pj_plan_.valid = false;
    const PjX c    = pj_cur_;
    PjPlan    p;
    memcpy(p.key, key, sizeof p.key);
    uint64_t h[3] = {mr, mi, mw};
    if (const int rc = pj_max_host(c, h, 3)) return rc;
    auto     pad  = [](uint64_t v) { return ((v + v / 8 + 64 + 63) / 64) * 64; };  // +12.5 % + 64, in 64s
    uint64_t fail = 0;
    p.BR          = pad(h[0]);
    p.BI          = pad(h[1]);
    p.BW          = pad(h[2]);
    if (const int div = test_hooks().pj_plan_div) {  // (tests: a plan too small, the next join overflows)
        p.BR = std::max<uint64_t>(1, p.BR / (uint64_t) div);
        p.BI = std::max<uint64_t>(1, p.BI / (uint64_t) div);
        p.BW = std::max<uint64_t>(1, p.BW / (uint64_t) div);
    }
    // (27-bit chunk ids in the received entries; 32-bit item and word positions)
    if ((uint64_t) G.W * p.BR >= (1ull << 27) || (uint64_t) G.W * p.BI >= (1ull << 31) ||
        (uint64_t) G.W * p.BW >= (1ull << 32))
        fail = 1;
    else
        fail = pj_async_alloc(G, p, true, c) ? 1u : 0u;
    if (const int rc = pj_max_host(c, &fail, 1)) return rc;
    p.valid  = fail == 0;
    pj_lost_ = false;
    pj_plan_ = p;
    pj_plans_++;
    return 0;
}

int Engine::pj_plan_from_sync(int world, int rank, uint64_t nR, uint64_t nR_total, uint64_t nS,
                              const bloom_filter_args_t* args, uint64_t mr, uint64_t mi, uint64_t mw) {
    PjGeom G;
    if (!pj_geom(world, rank, nR, nR_total, nS, args, &G)) return 2;
    uint64_t key[kPjKey];
    pj_shape(key, world, rank, nR, nR_total, nS, args);
    pj_plan_args_ = args ? *args : bloom_filter_args_t{};
    return pj_establish_plan(G, mr, mi, mw, key);
}

int Engine::pj_drain() {
    if (!pj_q_.empty()) PX_CHECK(hipStreamSynchronize(own_stream_));
    return 0;
}

int Engine::pj_sync_join(const PjIn& in, hwbrj_stats_t* st) {
    if (const int rc = pj_drain()) return rc;  // (the joins in flight finish before buffers grow)
    pj_make_plan_ = true;
    pj_cur_       = in.xc;
    const bloom_filter_args_t* a = in.has_args ? &in.args : nullptr;
    const int rc = in.xc.native ? join_partitioned_rccl(in.dR, in.nR, in.nR_total, in.dS, in.nS, a, st)
                                : join_partitioned(&in.xc.x, in.xc.rank, in.xc.world, in.dR, in.nR, in.nR_total,
                                                   in.dS, in.nS, a, st, false);
    pj_make_plan_ = false;
    return rc;
}

int Engine::join_partitioned_async(const hwbrj_exchange_t* xa, int rank, int world, const uint2* dR, uint64_t nR,
                                   uint64_t nR_total, const uint2* dS, uint64_t nS, const bloom_filter_args_t* args) {
    PX_CHECK(hipSetDevice(device_));
    PjX c;
    if (!xa) {
        if (!comm_) {
            set_last_error("no communicator on this device (hwbrj_comm_init)");
            return 32;
        }
        c.x     = native_exchange();
        c.rank  = comm_rank_;
        c.world = comm_world_;
    } else {
        if (world < 1 || rank < 0 || rank >= world) {
            set_last_error("rank must lie in [0, world)");
            return 2;
        }
        c.x      = *xa;
        c.native = false;
        c.rank   = rank;
        c.world  = world;
    }
    if (pj_q_.size() >= (size_t) kPjDepth) {  // (every rank makes the same calls: fails alike)
        set_last_error("too many partitioned joins in flight (wait for the oldest first)");
        return 6;
    }
    PjPending e{};
    e.in.xc       = c;
    e.in.dR       = dR;
    e.in.nR       = nR;
    e.in.nR_total = nR_total;
    e.in.dS       = dS;
    e.in.nS       = nS;
    e.in.has_args = args != nullptr;
    if (args) e.in.args = *args;
    if (!pj_plan_.valid) {
        // no plan on any rank (the state is collective): this join runs synchronously and makes one
        e.sync = true;
        e.rc   = pj_sync_join(e.in, &e.st);
        pj_sync_++;
        pj_q_.push_back(e);
        return 0;  // (its status is its wait's)
    }
    uint64_t key[kPjKey];
    pj_shape(key, c.world, c.rank, nR, nR_total, nS, args);
    PjGeom     G;
    const bool geom_ok = pj_geom(c.world, c.rank, nR, nR_total, nS, args, &G);
    // the failed mode: this rank's shapes are not the plan's (or its buffers were released); it
    // takes part in the join's collectives with empty messages, under the plan's geometry
    const bool fail = !geom_ok || pj_lost_ || memcmp(key, pj_plan_.key, sizeof key) != 0 || test_hooks().pj_async_fail;
    if (fail) {
        const bloom_filter_args_t* pa = pj_plan_.key[5] ? &pj_plan_args_ : nullptr;
        if (!pj_geom(c.world, c.rank, pj_plan_.key[2], pj_plan_.key[3], pj_plan_.key[4], pa, &G)) return 2;
    }
    const PjPlan& p = pj_plan_;
    if (const int rc = pj_async_alloc(G, p, !fail, c)) return rc;  // (lookups: allocated with the plan)
    const Geometry&  g = G.g;
    const uint32_t   W = G.W, QL = G.QL, F = G.F, NSUB = G.NSUB, NC = G.NC, NJ = QL * NSUB;
    hipStream_t      stream = own_stream_;
    const hwbrj_exchange_t& x = c.x;
    uint8_t*  sendC    = (uint8_t*) x.buffer(x.ctx, HWBRJ_PJ_R_SEND, 0);
    uint32_t* sendE    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_R_SEND_ENT, 0);
    uint8_t*  recvC    = (uint8_t*) x.buffer(x.ctx, HWBRJ_PJ_R_RECV, 0);
    uint32_t* recvE    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_R_RECV_ENT, 0);
    uint32_t* sendS    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_S_SEND, 0);
    uint32_t* recvS    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_S_RECV, 0);
    uint32_t* sendM    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_M_SEND, 0);
    uint32_t* recvM    = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_M_RECV, 0);
    uint32_t* d_slices = (uint32_t*) x.buffer(x.ctx, HWBRJ_PJ_SLICES, 0);
    uint64_t* flag     = pjX.as<uint64_t>();
    uint64_t* stat     = flag + 1;
    uint64_t* rc1s     = flag + 8;
    uint64_t* rc1r     = rc1s + (uint64_t) W * NC;
    uint64_t* rc2s     = rc1r + (uint64_t) W * NC;
    uint64_t* rc2r     = rc2s + (uint64_t) W * NC;
    const int slot     = (int) (pj_seq_ % kPjDepth);
    if (pending_ && pending_stream_ != stream) PX_CHECK(hipStreamWaitEvent(stream, ev_[8], 0));
    // An error return from here on leaves work of this join enqueued (on the join stream and, after
    // the fork below, on the side stream): the side stream is joined back into the join stream and
    // ev_[8] recorded after it, so every later join on this Engine (which shares these buffers)
    // orders after that work. Disarmed where the join completes its enqueue.
    bool forked = false;
    struct Unwind {
        std::function<void()> f;
        ~Unwind() {
            if (f) f();
        }
    } unwind;
    unwind.f = [&] {
        if (forked) (void) hipStreamWaitEvent(stream, ovl_ev_[1], 0);
        (void) hipEventRecord(ev_[8], stream);
        pending_        = true;
        pending_stream_ = stream;
        pending_rc_     = 6;
        pending_err_    = "the last join was a partitioned join that failed: " + std::string(hwbrj_last_error());
        ring_drop();
    };
    PX_CHECK(hipEventRecord(pjEv_[2 * slot], stream));
    PX_CHECK(hipMemsetAsync(flag, 0, 8, stream));
    // this rank's own blocks are written by k_pjx_gather / k_pjx_surv_pack straight into the
    // receive buffers (no copy to itself; HWBRJ_RCCL_SELF: through RCCL like the others)
    // (a callback transport moves every block itself, on its own stream: the join stream is drained
    // before each of its calls)
    const int own = !c.native || rccl_self_blocks() ? -1 : c.rank;
    std::vector<uint64_t> soff(W), sbytes(W), roff(W), rbytes(W);
    auto drain = [&]() -> int {
        if (!c.native) PX_CHECK(hipStreamSynchronize(stream));
        return 0;
    };
    auto xchg = [&](int ss, int rs, uint64_t b, const char* what) -> int {
        for (uint32_t j = 0; j < W; j++) soff[j] = roff[j] = j * b, sbytes[j] = rbytes[j] = (int) j == own ? 0 : b;
        if (const int rc = drain()) return rc;
        if (x.alltoallv(x.ctx, ss, soff.data(), sbytes.data(), rs, roff.data(), rbytes.data())) {
            set_last_error(std::string("exchange failed: ") + what);
            return 20;
        }
        return 0;
    };
    // a failed-mode counts message: zero counts and the failed status to every destination
    std::vector<uint64_t> hmsg;
    auto fail_msg = [&](uint64_t* d) -> int {
        hmsg.assign((size_t) W * NC, 0);
        for (uint32_t j = 0; j < W; j++) hmsg[(size_t) j * NC + QL + 1] = 1;
        PX_CHECK(hipMemcpyAsync(d, hmsg.data(), hmsg.size() * 8, hipMemcpyHostToDevice, stream));
        PX_CHECK(hipStreamSynchronize(stream));  // (hmsg is scoped: the failed mode may wait)
        return 0;
    };
    ScatterParams sp{};
    // The S shard's partitioning (scatter, plan, lists) does not depend on R: it runs on a second
    // stream beside the R side, the R exchange and the slice all-gather, and the probe waits for it,
    // so the collectives' transfer time hides behind the S scatter (HWBRJ_PJ_OVL).
    auto s_pass = [&](hipStream_t st) {
        ScatterParams ss{};
        ss.tabs       = d_tabs_;
        ss.g          = g;
        ss.src        = dS;
        ss.n          = nS;
        ss.pool       = poolS.as<uint32_t>();
        ss.meta       = metaS.as<uint32_t>();
        ss.wg_used    = usedS.as<uint32_t>();
        ss.wgq_chunks = wgqcS.as<uint32_t>();
        ss.wgq_elems  = wgqeS.as<uint32_t>();
        ss.cap        = G.capS;
        launch_scatter(ss, SRC_TUPLES, SIDE_S, G.G, st);
        launch_plan(wgqcS.as<uint32_t>(), wgqeS.as<uint32_t>(), G.G, g.log2F, wgqoS.as<uint32_t>(),
                    colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), st);
        launch_list_fill(metaS.as<uint32_t>(), usedS.as<uint32_t>(), G.capS, g.log2F, wgqoS.as<uint32_t>(),
                         colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), G.CH, G.nseg, lstartS.as<uint32_t>(),
                         estartS.as<uint64_t>(), istartS.as<uint32_t>(), listS.as<uint32_t>(), G.G, st);
    };
    const bool s_side = HWBRJ_PJ_OVL && !fail;
    if (s_side) {
        if (!ovl_stream_) {
            PX_CHECK(hipStreamCreateWithFlags(&ovl_stream_, hipStreamNonBlocking));
            PX_CHECK(hipEventCreateWithFlags(&ovl_ev_[0], hipEventDisableTiming));
            PX_CHECK(hipEventCreateWithFlags(&ovl_ev_[1], hipEventDisableTiming));
        }
        PX_CHECK(hipEventRecord(ovl_ev_[0], stream));
        PX_CHECK(hipStreamWaitEvent(ovl_stream_, ovl_ev_[0], 0));
        s_pass(ovl_stream_);
        PX_CHECK(hipEventRecord(ovl_ev_[1], ovl_stream_));
        forked = true;
    }
    if (!fail) {
        // ---- 1. R shard: partitions and the counts message
        PX_CHECK(hipMemsetAsync(small.p, 0, 64, stream));
        PX_CHECK(hipMemsetAsync(jparts.p, 0, jparts.bytes, stream));  // (the probe adds into job_surv)
        sp.tabs       = d_tabs_;
        sp.g          = g;
        sp.src        = dR;
        sp.n          = nR;
        sp.pool       = poolR.as<uint32_t>();
        sp.meta       = metaR.as<uint32_t>();
        sp.wg_used    = usedR.as<uint32_t>();
        sp.wgq_chunks = wgqcR.as<uint32_t>();
        sp.wgq_elems  = wgqeR.as<uint32_t>();
        sp.cap        = G.capR;
        launch_scatter(sp, SRC_TUPLES, SIDE_R, G.G, stream);
        launch_plan(wgqcR.as<uint32_t>(), wgqeR.as<uint32_t>(), G.G, g.log2F, wgqoR.as<uint32_t>(),
                    colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), stream);
        launch_list_fill(metaR.as<uint32_t>(), usedR.as<uint32_t>(), G.capR, g.log2F, wgqoR.as<uint32_t>(),
                         colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), (uint32_t) G.BSW, 1,
                         lstartR.as<uint32_t>(), estartR.as<uint64_t>(), istartR.as<uint32_t>(),
                         listR.as<uint32_t>(), G.G, stream);
        launch_pj_counts(lstartR.as<uint32_t>(), nullptr, W, QL, NC, 0, nS, nR, rc1s, stream);
    } else {
        PX_CHECK(hipMemcpyAsync(flag, &kFlagPeerFailed, 8, hipMemcpyHostToDevice, stream));
        if (const int rc = fail_msg(rc1s)) return rc;
    }
    // ---- 2. R exchange: blocks of BR chunks
    if (const int rc = pj_a2a_u64(c, rc1s, rc1r, NC)) return rc;
    if (!fail)
        launch_pjx_gather(poolR.as<uint32_t>(), listR.as<uint32_t>(), lstartR.as<uint32_t>(), F, QL, W, p.BR, sendC,
                          sendE, own, recvC, recvE, flag, stream);
    if (const int rc = xchg(HWBRJ_PJ_R_SEND, HWBRJ_PJ_R_RECV, p.BR * 128, "R chunks")) return rc;
    if (const int rc = xchg(HWBRJ_PJ_R_SEND_ENT, HWBRJ_PJ_R_RECV_ENT, p.BR * 4, "R chunk entries")) return rc;
    // ---- 3. owned partitions: tables on the device, lists, build
    const uint64_t sweeps_max = W * p.BR / G.BSW + QL + 1;
    if (!fail) {
        launch_pjx_rtab(rc1r, W, QL, NC, p.BR, (uint32_t) G.BSW, pjTab.as<int64_t>(), pjLstart.as<uint32_t>(),
                        pjSweep.as<uint32_t>(), flag, stream);
        launch_pj_relist(recvE, pjTab.as<int64_t>(), QL * W, pjList.as<uint32_t>(), stream);
        BuildParams bp{};
        bp.g           = g;
        bp.tabs        = d_tabs_;
        bp.pool        = (const uint32_t*) recvC;
        bp.list        = pjList.as<uint32_t>();
        bp.list_start  = pjLstart.as<uint32_t>();
        bp.elem_start  = nullptr;
        bp.slices      = G.slice_mode ? d_slices : nullptr;
        bp.sweep_start = pjSweep.as<uint32_t>();
        bp.out_codes   = rjoin.as<uint32_t>();
        bp.run_cnt     = rrun.as<uint32_t>();
        bp.run_off     = rrun.as<uint32_t>() + sweeps_max * NSUB;
        bp.q_base      = G.q0;
        launch_build(bp, QL, stream);
    }
    // ---- 4. the whole filter on every rank
    if (G.slice_mode && W > 1 && (drain() || x.allgather(x.ctx, HWBRJ_PJ_SLICES, (uint64_t) QL * G.nseg * g.seg_words * 4))) {
        set_last_error("exchange failed: filter slices");
        return 20;
    }
    // ---- 5. S shard: partitions (unless on the side stream), probe, item tables, the counts message
    if (!fail) {
        if (s_side) {
            PX_CHECK(hipStreamWaitEvent(stream, ovl_ev_[1], 0));
            forked = false;
        } else
            s_pass(stream);
        ProbeParams pp{};
        pp.g               = g;
        pp.tabs            = d_tabs_;
        pp.pool            = poolS.as<uint32_t>();
        pp.list            = listS.as<uint32_t>();
        pp.list_start      = lstartS.as<uint32_t>();
        pp.item_start      = istartS.as<uint32_t>();
        pp.slices          = G.slice_mode ? d_slices : nullptr;
        pp.surv            = surv.as<uint32_t>();
        pp.surv_seg_stride = G.LS * 32;
        pp.surv_cnt        = survcnt.as<uint32_t>();
        pp.surv_off        = survoff.as<uint32_t>();
        pp.filtered        = small.as<uint64_t>() + 2;
        pp.job_surv        = jparts.as<uint32_t>() + F * NSUB;
        const size_t   pl_lds = probe_lds_bytes(g, nullptr);
        const uint32_t PG     = (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / pl_lds));
        launch_probe(pp, PG, stream);
        launch_pj_items(istartS.as<uint32_t>(), lstartS.as<uint32_t>(), survcnt.as<uint32_t>(), G.items_max, F,
                        G.nseg, G.CH, G.LS * 32, NSUB, pjRegion.as<uint64_t>(), pjTot.as<uint32_t>(),
                        pjBsum.as<uint64_t>(), pjSoff.as<uint64_t>(), pjBound.as<uint64_t>(), stream);
        launch_pj_counts(istartS.as<uint32_t>(), pjBound.as<uint64_t>(), W, QL, NC, 0, 0, nR, rc2s, stream);
    } else if (const int rc = fail_msg(rc2s)) {
        return rc;
    }
    // ---- 6. survivor exchange: blocks of BW words and BI items
    if (const int rc = pj_a2a_u64(c, rc2s, rc2r, NC)) return rc;
    if (!fail)
        launch_pjx_surv_pack(surv.as<uint32_t>(), pjRegion.as<uint64_t>(), pjTot.as<uint32_t>(),
                             pjSoff.as<uint64_t>(), istartS.as<uint32_t>(), pjBound.as<uint64_t>(),
                             survcnt.as<uint32_t>(), F, QL, NSUB, p.BI, p.BW, sendS, sendM, own, recvS, recvM, flag,
                             stream);
    if (const int rc = xchg(HWBRJ_PJ_S_SEND, HWBRJ_PJ_S_RECV, p.BW * 4, "survivors")) return rc;
    if (const int rc = xchg(HWBRJ_PJ_M_SEND, HWBRJ_PJ_M_RECV, p.BI * NSUB * 4, "survivor run counts")) return rc;
    // ---- 7. the owner's survivor tables on the device, join
    if (!fail) {
        launch_pjx_stab(rc2r, W, QL, NC, p.BI, p.BW, pjTab2.as<uint32_t>(), pjIstart.as<uint32_t>(),
                        pjRitems.as<uint32_t>(), flag, stream);
        PX_CHECK(hipMemsetAsync(pjJobs.p, 0, (size_t) NJ * 4, stream));
        launch_pj_recv_scan(recvM, (uint32_t) (W * p.BI), NSUB, pjWtot.as<uint32_t>(), pjBsum.as<uint64_t>(),
                            pjWscan.as<uint64_t>(), stream, (uint32_t) p.BI, pjRitems.as<uint32_t>());
        launch_pj_item_tables(pjTab2.as<uint32_t>(), QL * W, W, recvM, pjWscan.as<uint64_t>(), NSUB,
                              pjIbase.as<uint64_t>(), pjCnt.as<uint32_t>(), pjOff.as<uint32_t>(),
                              pjJobs.as<uint32_t>(), stream, (uint32_t) p.BI, p.BW);
        PX_CHECK(hipMemsetAsync(jparts.as<uint32_t>() + 2 * F * NSUB, 0, 4, stream));  // nextra
        JoinParams jp{};
        jp.r_codes         = rjoin.as<uint32_t>();
        jp.r_sweep_start   = pjSweep.as<uint32_t>();
        jp.r_cnt           = rrun.as<uint32_t>();
        jp.r_off           = rrun.as<uint32_t>() + sweeps_max * NSUB;
        jp.slot            = (uint32_t) G.SLOT;
        jp.surv            = recvS;
        jp.surv_cnt        = pjCnt.as<uint32_t>();
        jp.surv_off        = pjOff.as<uint32_t>();
        jp.item_start      = pjIstart.as<uint32_t>();
        jp.list_start      = pjIstart.as<uint32_t>();  // (unused: item_base)
        jp.surv_seg_stride = 0;
        jp.nseg            = 1;
        jp.CH              = G.CH;
        jp.log2NSUB        = g.log2NSUB;
        jp.hash_shift      = g.hash_shift;
        jp.bitmap          = (g.sub_shift > 0 && 32 - g.hash_shift <= join_bitmap_log2()) ? 1u : 0u;
        jp.jsum            = (uint64_t*) ((char*) small.p + 128);
        jp.nparts          = jparts.as<uint32_t>();
        jp.extra           = jtask.as<uint2>();
        jp.nextra          = jparts.as<uint32_t>() + 2 * F * NSUB;
        jp.item_base       = pjIbase.as<uint64_t>();
        jp.split_surv      = test_hooks().join_split;
        jp.timing          = 0;
        launch_join(jp, NJ, pjJobs.as<uint32_t>(), stream);
        launch_pjx_stat(rc1r, rc2r, lstartR.as<uint32_t>(), istartS.as<uint32_t>(), pjBound.as<uint64_t>(), W, QL,
                        NC, flag, stat, stream);
    } else {
        const uint64_t h[4] = {kFlagPeerFailed, 0, 0, 0};
        PX_CHECK(hipMemcpyAsync(stat, h, 32, hipMemcpyHostToDevice, stream));
        PX_CHECK(hipStreamSynchronize(stream));  // (h is scoped)
    }
    // ---- 8. the flag and the block sizes, max over the ranks; the counts into this join's ring slot
    if (const int rc = pj_max_dev(c, stat, 4)) return rc;
    uint8_t* ring = pjRing.as<uint8_t>() + (size_t) slot * ring_slot_bytes();
    if (!fail)  // (the failed mode's counts are never read: its flag reruns the join; and after
                // hwbrj_release the counts buffer may not exist)
        PX_CHECK(hipMemcpyAsync(ring, small.p, ring_counts_bytes(), hipMemcpyDeviceToDevice, stream));
    PX_CHECK(hipMemcpyAsync(ring + ring_counts_bytes(), flag, 40, hipMemcpyDeviceToDevice, stream));
    PX_CHECK(hipEventRecord(pjEv_[2 * slot + 1], stream));
    PX_CHECK(hipEventRecord(ev_[8], stream));
    PX_CHECK(hipGetLastError());
    unwind.f = nullptr;  // (enqueued: the state below replaces the unwinding)
    // single-GPU joins on this Engine order after it (ev_[8]); hwbrj_wait does not collect it
    pending_        = true;
    pending_stream_ = stream;
    pending_rc_     = 6;
    ring_drop();
    pending_err_    = "the last join is a partitioned one: collect it with hwbrj_join_partitioned_wait";
    have_filter_    = false;
    last_nj_        = 0;
    e.slot          = slot;
    e.G             = G;
    e.failed_mode   = fail;
    pj_q_.push_back(e);
    pj_seq_++;
    pj_async_++;
    return 0;
}

int Engine::join_partitioned_wait(hwbrj_stats_t* st) {
    PX_CHECK(hipSetDevice(device_));
    if (pj_q_.empty()) {
        set_last_error("no partitioned join has been enqueued");
        return 6;
    }
    const PjPending e = pj_q_.front();
    pj_q_.pop_front();
    if (e.sync) {  // (it ran at enqueue and made the plan)
        if (st) *st = e.st;
        return e.rc;
    }
    PX_CHECK(hipEventSynchronize(pjEv_[2 * e.slot + 1]));
    std::vector<uint64_t> buf(ring_slot_bytes() / 8);
    PX_CHECK(hipMemcpy(buf.data(), pjRing.as<uint8_t>() + (size_t) e.slot * ring_slot_bytes(), buf.size() * 8,
                       hipMemcpyDeviceToHost));
    const uint64_t* stat = buf.data() + ring_counts_bytes() / 8;  // this rank's flag, then the maxima
    if (stat[1]) {
        // a block overflowed (or a rank ran in the failed mode) somewhere: every rank sees the same
        // all-reduced flag, drops the plan and reruns this join synchronously (a new plan)
        pj_fallbacks_++;
        pj_last_flag_  = stat[1];
        pj_plan_.valid = false;
        return pj_sync_join(e.in, st);
    }
    uint64_t h[6];
    for (int i = 0; i < 6; i++) h[i] = buf[i];
    for (size_t j = 0; j < join_sum_slots(); j++) {
        h[0] += buf[16 + j * join_sum_stride()];
        h[3] += buf[16 + j * join_sum_stride() + 1];
        h[4] += buf[16 + j * join_sum_stride() + 2];
    }
    pj_last_sizes_[0] = stat[2];
    pj_last_sizes_[1] = stat[3];
    pj_last_sizes_[2] = stat[4];
    if (st) {
        const PjGeom& G = e.G;
        memset(st, 0, sizeof(*st));
        st->filtered       = e.in.has_args ? h[2] : e.in.nS;
        st->matches        = (int64_t) h[0];
        st->mode           = G.g.mode;
        st->format         = G.g.s_format;
        st->partitions     = G.F;
        st->subparts       = G.NSUB;
        st->slice_segments = G.nseg;
        st->join_keys      = HWBRJ_JOIN_KEYS_32;
        st->join_key_bits  = 32;
        float ms           = 0;  // the join's device time: its first to its last operation on the stream
        PX_CHECK(hipEventElapsedTime(&ms, pjEv_[2 * e.slot], pjEv_[2 * e.slot + 1]));
        st->ms_total = ms;
    }
    return 0;
}

void Engine::pj_async_info(uint64_t* out) const {
    const uint64_t v[16] = {pj_plan_.valid ? 1u : 0u, pj_plan_.BR, pj_plan_.BI, pj_plan_.BW,
                            pj_async_, pj_sync_, pj_fallbacks_, pj_plans_, (uint64_t) pj_q_.size(),
                            pj_last_flag_, pj_last_sizes_[0], pj_last_sizes_[1], pj_last_sizes_[2], 0, 0, 0};
    memcpy(out, v, sizeof v);
}

}  // namespace hwbrj

using namespace hwbrj;

extern "C" {

int hwbrj_join_partitioned_rccl_async(const tuple_t* d_R, uint64_t nR, uint64_t nR_total, const tuple_t* d_S,
                                      uint64_t nS, const bloom_filter_args_t* args) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->join_partitioned_async(nullptr, 0, 1, (const uint2*) d_R, nR, nR_total, (const uint2*) d_S, nS, args);
}

int hwbrj_join_partitioned_async(const hwbrj_exchange_t* x, int rank, int world, const tuple_t* d_R, uint64_t nR,
                                 uint64_t nR_total, const tuple_t* d_S, uint64_t nS, const bloom_filter_args_t* args) {
    if (!x) {
        set_last_error("no exchange (hwbrj_join_partitioned_rccl_async runs over the library's communicator)");
        return 2;
    }
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->join_partitioned_async(x, rank, world, (const uint2*) d_R, nR, nR_total, (const uint2*) d_S, nS, args);
}

int hwbrj_join_partitioned_wait(hwbrj_stats_t* stats) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->join_partitioned_wait(stats);
}

int hwbrj_pj_async_info(uint64_t* out) {
    if (!out) {
        set_last_error("out must hold 16 words");
        return 2;
    }
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    e->pj_async_info(out);
    return 0;
}

}  // extern "C"
