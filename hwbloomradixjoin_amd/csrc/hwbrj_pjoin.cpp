// hwbrj_pjoin.cpp -- the partitioned multi-GPU join.
//
// The reference spreads one join over threads that share every partition (the shared-histogram
// partitioning of src/parallel_radix_join_bloom.c:792-849 and :820-837, one task queue). Here
// ranks (one per GPU) own radix partitions: rank r of G owns [r F / G, (r + 1) F / G). Per join:
//   1. the local R shard is scattered (k_scatter_r, k_plan, k_list_fill);
//   2. R exchange: every partition's chunks go to its owner (k_pj_gather, all-to-all);
//   3. the owner rebuilds its partitions' chunk lists (k_pj_relist) and builds their filter
//      slices and join runs (k_build with q_base);
//   4. the slices are all-gathered: every rank holds the whole filter (the bitmap "broadcast");
//   5. the local S shard is scattered and probed against the whole filter (k_scatter_s, k_probe);
//   6. survivor exchange: every item's survivor runs go to its partition's owner (k_pj_surv_pack,
//      all-to-all), with their per-sub counts;
//   7. the owner joins its partitions (k_join over the received runs, item_base).
// The exchanges are the caller's (hwbrj_exchange_t: RCCL through torch.distributed, gloo, peer
// copies; each synchronous) or the library's own RCCL transport (hwbrj_comm.cpp: collectives on the
// join stream). Host tables between them are built from counts the host has waited for. Before
// every collective the ranks agree on their statuses, so a rank that fails alone (an oversized
// shard, an allocation) makes every rank return instead of leaving its peers in the collective.
// The native transport waits on the host three times per join (the R counts, the survivor counts,
// the result): each counts message is packed on the device and exchanged on the join stream, and
// every receive buffer is allocated at its worst case before the counts step that could size it,
// so its status rides in that step's message and no separate agreement is needed (the callback
// path: a starts read and a counts all-to-all per step, plus three agreements).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "hwbrj_engine.h"

namespace hwbrj {

#define PJ_CHECK(expr)                                                                     \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            set_last_error(std::string(#expr) + ": " + hipGetErrorString(e_));             \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

#define PJ_XCHG(expr, what)                                                                \
    do {                                                                                   \
        if ((expr) != 0) {                                                                 \
            set_last_error(std::string("exchange failed: ") + what);                       \
            return 20;                                                                     \
        }                                                                                  \
    } while (0)

uint64_t pj_region_cap(uint64_t n, uint32_t G, uint32_t F) {
    const uint64_t units = (n + 3) / 4;
    const uint64_t per   = ((units + G - 1) / G) * 4;
    return (per + 31) / 32 + F + 1;
}

template <class T>
static int to_dev(DevBuf& b, const std::vector<T>& v, hipStream_t st) {
    if (!b.ensure(std::max<size_t>(16, v.size() * sizeof(T)))) return 4;
    if (!v.empty() && hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st) != hipSuccess)
        return 1;
    return 0;
}

// HWBRJ_PJ_CHECK=1 (tests): every host table is checked against the buffers it indexes before the
// kernel that reads it is launched, and every stage is synchronised with its name in the error.
static bool pj_check_on() {
    static const bool on = getenv("HWBRJ_PJ_CHECK") != nullptr;
    return on;
}

#define PJ_FAIL(msg)                                                                       \
    do {                                                                                   \
        set_last_error(std::string("partitioned join check: ") + (msg));                   \
        return 21;                                                                         \
    } while (0)

#define PJ_STAGE(name)                                                                     \
    do {                                                                                   \
        if (pj_check_on()) {                                                               \
            hipError_t e_ = hipStreamSynchronize(stream);                                  \
            if (e_ == hipSuccess) e_ = hipGetLastError();                                  \
            if (e_ != hipSuccess) {                                                        \
                set_last_error(std::string("after ") + name + ": " + hipGetErrorString(e_)); \
                return 1;                                                                  \
            }                                                                              \
        }                                                                                  \
    } while (0)

int Engine::join_partitioned(const hwbrj_exchange_t* x, int rank, int world, const uint2* dR,
                             uint64_t nR, uint64_t nR_total, const uint2* dS, uint64_t nS,
                             const bloom_filter_args_t* args, hwbrj_stats_t* st, bool native) {
    PJ_CHECK(hipSetDevice(device_));
    const auto t_start = std::chrono::steady_clock::now();
    // Errors every rank sees alike (arguments, geometry): returned at once, on every rank.
    Geometry    g;
    std::string err;
    if (!plan_geometry(args, nR_total, &g, &err)) {
        set_last_error(err);
        return 2;
    }
    if (g.mode == MODE_GLOBAL || (g.mode == MODE_SLICE_BASIC && g.k > 1)) {
        set_last_error("the partitioned join needs partition slices (blocked/sectorized, basic k = 1, or no filter)");
        return 9;
    }
    g.s_format = g.format;
    const uint32_t F = 1u << g.log2F, NSUB = 1u << g.log2NSUB;
    if (world < 1 || rank < 0 || rank >= world || F % (uint32_t) world != 0) {
        set_last_error("world must divide the partition count F = " + std::to_string(F));
        return 9;
    }
    const uint32_t QL = F / (uint32_t) world, q0 = (uint32_t) rank * QL;
    const uint32_t W  = (uint32_t) world;
    const bool     slice_mode = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    const uint32_t nseg       = slice_mode ? g.nseg : 1;
    const uint32_t CH         = probe_chunks_per_item();
    const uint64_t BSW = build_chunks_per_sweep(), SLOT = build_sweep_slot();
    const size_t   sc_lds = scatter_lds_bytes(g.log2F);
    const uint32_t G      = (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / sc_lds));
    hipStream_t    stream = own_stream_;
    // A callback transport runs its collectives on its own stream: the join stream is drained
    // before each (the native RCCL transport enqueues them on the join stream itself).
    auto drain = [&]() -> int {
        if (!native) PJ_CHECK(hipStreamSynchronize(stream));
        return 0;
    };
    // Errors of one rank only (its shard's capacity, an allocation, a launch, a table check) must
    // not leave the others blocked in a collective it never enters: before every collective the
    // ranks agree on their statuses (carried by the counts exchanges, else one u64 all-to-all),
    // and all of them return together.
    auto peers = [&](const uint64_t* status, uint64_t stride, int rc) -> int {
        if (rc) return rc;  // (this rank's own message stays)
        for (uint32_t j = 0; j < W; j++)
            if (status[(uint64_t) j * stride]) {
                set_last_error("partitioned join: rank " + std::to_string(j) + " failed (code " +
                               std::to_string(status[(uint64_t) j * stride]) + ")");
                return 22;
            }
        return 0;
    };
    auto agree = [&](int rc) -> int {
        std::vector<uint64_t> s(W, (uint64_t) (uint32_t) rc), r(W, 0);
        if (x->alltoall_u64(x->ctx, s.data(), r.data(), 1) != 0) {
            set_last_error("exchange failed: status");
            return 20;
        }
        return peers(r.data(), 1, rc);
    };
    // counts exchanges: QL partition counts, a total, the status, this rank's |S| and |R| shards
    const uint32_t NC = QL + 4;
    // native: a rank's own R-chunk and survivor blocks are written by the gather / pack kernels
    // straight into its receive buffers, and the exchanges skip the copy to itself (HWBRJ_RCCL_SELF:
    // through RCCL like the others)
    const bool self_direct = native && !rccl_self_blocks();
    std::vector<double> ms(8, 0.0);
    auto lap = [&, t = std::chrono::steady_clock::now()](int k) mutable {
        const auto n = std::chrono::steady_clock::now();
        ms[k] += std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    };
    uint64_t capR = 0, capS = 0, LS = 0;
    uint32_t* d_slices = nullptr;
    void *sendC = nullptr, *recvC = nullptr;
    uint32_t *sendE = nullptr, *recvE = nullptr, *sendS = nullptr, *sendM = nullptr, *recvS = nullptr,
             *recvM = nullptr;
    uint64_t* d_result   = nullptr;
    uint64_t* d_filtered = nullptr;
    std::vector<uint32_t> ls(F + 1, 0), isS(F + 1, 0);
    std::vector<uint64_t> scnt((size_t) W * NC, 0), rcnt((size_t) W * NC, 0), bnd(F + 1, 0);
    std::vector<uint64_t> soff(W), sbytes(W), roff(W), rbytes(W);
    uint64_t              RC = 0, sweeps = 0, RI = 0, RW = 0;
    uint64_t              RCmax = 0, RImax = 0, RWmax = 0;  // native: receive capacities (worst case)
    uint64_t              plan_mr = 0, plan_mi = 0, plan_mw = 0;  // native: largest blocks (async plan)
    std::vector<uint64_t> ritems(W), rwords(W), sofs;
    ScatterParams sp{};
    // The native transport's counts step: the message to every destination is packed on the device
    // (k_pj_counts; or, after a local failure, just the status from the host), exchanged by RCCL on
    // the join stream and read back together with the partition starts: ONE host wait per exchange
    // step, where the callback path needs a read of the starts, then a counts all-to-all. Every
    // receive buffer of the native path is allocated before the exchange at its worst-case size
    // (memory is plentiful, 288 GB per GPU), so no allocation can fail alone after a counts step
    // and the status agreements before the data all-to-alls are not needed.
    std::vector<uint64_t> hstat;
    auto native_counts = [&](const uint32_t* d_starts, const uint64_t* d_bound, int rc_local, uint64_t extra,
                             uint32_t* h_starts, uint64_t* h_bound) -> int {
        const uint64_t n  = (uint64_t) W * NC;
        uint64_t*      ds = xcnt()->as<uint64_t>();
        uint64_t*      dr = ds + n;
        if (rc_local == 0) {
            launch_pj_counts(d_starts, d_bound, W, QL, NC, 0, extra, nR, ds, stream);
        } else {
            hstat.assign(n, 0);
            for (uint32_t j = 0; j < W; j++) hstat[(uint64_t) j * NC + QL + 1] = (uint64_t) (uint32_t) rc_local;
            PJ_CHECK(hipMemcpyAsync(ds, hstat.data(), n * 8, hipMemcpyHostToDevice, stream));
        }
        if (rccl_alltoall_u64_dev(this, ds, dr, NC) != 0) {
            set_last_error("exchange failed: counts");
            return 20;
        }
        PJ_CHECK(hipMemcpyAsync(rcnt.data(), dr, n * 8, hipMemcpyDeviceToHost, stream));
        if (rc_local == 0) {
            PJ_CHECK(hipMemcpyAsync(h_starts, d_starts, (F + 1) * 4, hipMemcpyDeviceToHost, stream));
            if (h_bound) PJ_CHECK(hipMemcpyAsync(h_bound, d_bound, (F + 1) * 8, hipMemcpyDeviceToHost, stream));
        }
        PJ_CHECK(hipStreamSynchronize(stream));
        return 0;
    };
    if (native && !xcnt()->ensure((size_t) 2 * W * NC * 8)) {  // (tiny; before any collective)
        set_last_error("hipMalloc failed (exchange counts)");
        return 4;
    }

    // ------------------------------------------------------------- 1. R shard: local partitions
    const int rc1 = [&]() -> int {
        if (pending_) PJ_CHECK(hipStreamWaitEvent(stream, ev_[8], 0));
        capR = pj_region_cap(nR, G, F), capS = pj_region_cap(nS, G, F);
        const uint64_t LR = (uint64_t) G * capR;
        LS = (uint64_t) G * capS;
        // (HWBRJ_HOOK_PJ_FAIL_RANK = r, tests: rank r fails this check, as an oversized shard would)
        if (G > 512 || LS > (1ull << 27) || LR > (1ull << 27) || capS >= (1u << 22) || capR >= (1u << 22) ||
            test_hooks().pj_fail_rank == rank) {
            set_last_error("shard too large for 27-bit chunk ids");
            return 3;
        }
        const uint64_t GF = (uint64_t) G * F;
        bool ok = true;
        ok &= poolR.ensure(LR * 128) && metaR.ensure(LR * 2) && listR.ensure(LR * 4);
        ok &= usedR.ensure(G * 4) && wgqcR.ensure(GF * 4) && wgqeR.ensure(GF * 4) && wgqoR.ensure(GF * 4);
        ok &= lstartR.ensure((F + 1) * 4) && estartR.ensure((F + 1) * 8) && istartR.ensure((F + 1) * 4);
        ok &= poolS.ensure(LS * 128) && metaS.ensure(LS * 2) && listS.ensure(LS * 4);
        ok &= usedS.ensure(G * 4) && wgqcS.ensure(GF * 4) && wgqeS.ensure(GF * 4) && wgqoS.ensure(GF * 4);
        ok &= lstartS.ensure((F + 1) * 4) && estartS.ensure((F + 1) * 8) && istartS.ensure((F + 1) * 4);
        const uint64_t items_max = (LS / CH + F + 1) * nseg;
        ok &= surv.ensure(nseg * LS * 128) && survcnt.ensure(items_max * NSUB * 4) && survoff.ensure(items_max * NSUB * 4);
        ok &= small.ensure(128 + 64 * 128) && colR.ensure(F * 12) && colS.ensure(F * 12);
        ok &= jtask.ensure((size_t) join_extra_tasks() * 8) && jparts.ensure((size_t) (2 * F * NSUB + 1) * 4);
        if (native) {
            // R received by this rank: its QL partitions' chunks from every source, each source
            // region holding at most one partial chunk per partition
            RCmax = nR_total / 32 + (uint64_t) W * G * QL + QL + 1;
            const uint64_t sw_max = RCmax / BSW + QL + 1;
            ok &= pjList.ensure(RCmax * 4) && rjoin.ensure(sw_max * SLOT * 4) && rrun.ensure(2 * sw_max * NSUB * 4);
            ok &= pjTab.ensure((size_t) 4 * QL * W * 8) && pjLstart.ensure((QL + 1) * 4) && pjSweep.ensure((QL + 1) * 4);
            recvC = x->buffer(x->ctx, HWBRJ_PJ_R_RECV, RCmax * 128 + 16);
            recvE = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_R_RECV_ENT, RCmax * 4);
            sendC = x->buffer(x->ctx, HWBRJ_PJ_R_SEND, std::max<uint64_t>(16, LR * 128));
            sendE = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_R_SEND_ENT, std::max<uint64_t>(16, LR * 4));
            ok &= recvC && recvE && sendC && sendE;
        }
        if (!ok) {
            set_last_error("hipMalloc failed (device memory)");
            return 4;
        }
        const uint64_t slice_bytes = slice_mode ? (uint64_t) F * nseg * g.seg_words * 4 : 16;
        d_slices = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_SLICES, slice_bytes);
        if (!d_slices) {
            set_last_error("exchange buffer (slices) unavailable");
            return 20;
        }
        d_result   = small.as<uint64_t>();
        d_filtered = small.as<uint64_t>() + 2;
        PJ_CHECK(hipMemsetAsync(small.p, 0, 64, stream));
        PJ_CHECK(hipMemsetAsync(jparts.p, 0, jparts.bytes, stream));  // the probe adds into job_surv
        sp.tabs       = d_tabs_;
        sp.g          = g;
        sp.src        = dR;
        sp.n          = nR;
        sp.pool       = poolR.as<uint32_t>();
        sp.meta       = metaR.as<uint32_t>();
        sp.wg_used    = usedR.as<uint32_t>();
        sp.wgq_chunks = wgqcR.as<uint32_t>();
        sp.wgq_elems  = wgqeR.as<uint32_t>();
        sp.cap        = capR;
        launch_scatter(sp, SRC_TUPLES, SIDE_R, G, stream);
        launch_plan(wgqcR.as<uint32_t>(), wgqeR.as<uint32_t>(), G, g.log2F, wgqoR.as<uint32_t>(),
                    colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), stream);
        launch_list_fill(metaR.as<uint32_t>(), usedR.as<uint32_t>(), capR, g.log2F, wgqoR.as<uint32_t>(),
                         colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), (uint32_t) BSW, 1, lstartR.as<uint32_t>(),
                         estartR.as<uint64_t>(), istartR.as<uint32_t>(), listR.as<uint32_t>(), G, stream);
        if (native) return 0;  // (the counts message is built on the device)
        PJ_CHECK(hipMemcpyAsync(ls.data(), lstartR.p, (F + 1) * 4, hipMemcpyDeviceToHost, stream));
        PJ_CHECK(hipStreamSynchronize(stream));
        const uint32_t nch = ls[F];
        sendC = x->buffer(x->ctx, HWBRJ_PJ_R_SEND, std::max<uint64_t>(16, (uint64_t) nch * 128));
        sendE = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_R_SEND_ENT, std::max<uint64_t>(16, (uint64_t) nch * 4));
        if (!sendC || !sendE) {
            set_last_error("exchange buffer (R send) unavailable");
            return 20;
        }
        PJ_STAGE("R scatter");
        launch_pj_gather(poolR.as<uint32_t>(), listR.as<uint32_t>(), nch, sendC, sendE, stream);
        PJ_STAGE("k_pj_gather");
        // per destination j: chunks of its QL partitions, then the position of its block's first chunk
        for (uint32_t j = 0; j < W; j++) {
            for (uint32_t i = 0; i < QL; i++) scnt[j * NC + i] = ls[j * QL + i + 1] - ls[j * QL + i];
            scnt[j * NC + QL]     = ls[j * QL];
            scnt[j * NC + QL + 2] = nS;
            scnt[j * NC + QL + 3] = nR;
        }
        return drain();
    }();
    lap(0);
    // ------------------------------------------------------------- 2. R exchange
    // Every rank learns every R shard's size with the R counts: the receive bounds come from the
    // caller's nR_total, so shards that sum to more fail on every rank alike, before any
    // rank enters the R all-to-all.
    auto check_r_total = [&]() -> int {
        uint64_t sum = 0;
        for (uint32_t j = 0; j < W; j++) sum += rcnt[(uint64_t) j * NC + QL + 3];
        if (sum > nR_total) {
            set_last_error("partitioned join: the R shards hold " + std::to_string(sum) + " tuples, nR_total is " +
                           std::to_string(nR_total));
            return 2;
        }
        return 0;
    };
    if (native) {
        if (const int rc = native_counts(lstartR.as<uint32_t>(), nullptr, rc1, nS, ls.data(), nullptr)) return rc;
        if (const int rc = peers(rcnt.data() + QL + 1, NC, rc1)) return rc;
        if (const int rc = check_r_total()) return rc;
        for (uint32_t j = 0; j < W; j++) {  // (the async join's plan: the largest R block)
            uint64_t c = 0;
            for (uint32_t i = 0; i < QL; i++) c += rcnt[(uint64_t) j * NC + i];
            plan_mr = std::max<uint64_t>(plan_mr, std::max<uint64_t>(c, ls[(j + 1) * QL] - ls[j * QL]));
        }
        PJ_STAGE("R scatter");
        PjOwn own;  // (this rank's block to itself: straight into the receive buffers)
        if (self_direct) {
            uint64_t base = 0;  // its first receive chunk: every lower source's chunks come first
            for (uint32_t j = 0; j < (uint32_t) rank; j++)
                for (uint32_t i = 0; i < QL; i++) base += rcnt[(uint64_t) j * NC + i];
            own.lo    = ls[rank * QL];
            own.hi    = ls[(rank + 1) * QL];
            own.delta = (int64_t) base - (int64_t) own.lo;
            own.out   = recvC;
            own.ent   = recvE;
        }
        launch_pj_gather(poolR.as<uint32_t>(), listR.as<uint32_t>(), ls[F], sendC, sendE, stream, own);
        PJ_STAGE("k_pj_gather");
    } else {
        for (uint32_t j = 0; j < W; j++) scnt[j * NC + QL + 1] = (uint64_t) (uint32_t) rc1;
        PJ_XCHG(x->alltoall_u64(x->ctx, scnt.data(), rcnt.data(), NC), "R chunk counts");
        if (const int rc = peers(rcnt.data() + QL + 1, NC, rc1)) return rc;
        if (const int rc = check_r_total()) return rc;
        for (uint32_t j = 0; j < W; j++) {  // (the async join's plan: the largest R block)
            uint64_t c = 0;
            for (uint32_t i = 0; i < QL; i++) c += rcnt[(uint64_t) j * NC + i];
            plan_mr = std::max<uint64_t>(plan_mr, std::max<uint64_t>(c, ls[(j + 1) * QL] - ls[j * QL]));
        }
    }
    const int rc2 = [&]() -> int {
        for (uint32_t j = 0; j < W; j++) {
            soff[j]   = (uint64_t) ls[j * QL] * 128;
            sbytes[j] = (uint64_t) (ls[(j + 1) * QL] - ls[j * QL]) * 128;
            uint64_t c = 0;
            for (uint32_t i = 0; i < QL; i++) c += rcnt[j * NC + i];
            roff[j]   = RC * 128;
            rbytes[j] = c * 128;
            RC += c;
        }
        if (self_direct) sbytes[rank] = rbytes[rank] = 0;  // (written by k_pj_gather)
        if (native) {  // (allocated at RCmax before the counts step; with the R shards summing to at
                       // most nR_total, RC cannot exceed it: a bug guard)
            if (RC > RCmax) {
                set_last_error("partitioned join: received R chunks above their bound");
                return 21;
            }
            return 0;
        }
        recvC = x->buffer(x->ctx, HWBRJ_PJ_R_RECV, std::max<uint64_t>(16, RC * 128 + 16));
        recvE = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_R_RECV_ENT, std::max<uint64_t>(16, RC * 4));
        if (!recvC || !recvE) {
            set_last_error("exchange buffer (R receive) unavailable");
            return 20;
        }
        return 0;
    }();
    if (native) {
        if (rc2) return rc2;  // (a broken bound: no rank can get here but by a bug)
    } else if (const int rc = agree(rc2)) {
        return rc;
    }
    PJ_XCHG(x->alltoallv(x->ctx, HWBRJ_PJ_R_SEND, soff.data(), sbytes.data(), HWBRJ_PJ_R_RECV, roff.data(), rbytes.data()),
            "R chunks");
    for (uint32_t j = 0; j < W; j++) soff[j] /= 32, sbytes[j] /= 32, roff[j] /= 32, rbytes[j] /= 32;
    PJ_XCHG(x->alltoallv(x->ctx, HWBRJ_PJ_R_SEND_ENT, soff.data(), sbytes.data(), HWBRJ_PJ_R_RECV_ENT, roff.data(), rbytes.data()),
            "R chunk entries");
    lap(1);
    // ------------------------------------------------------------- 3. owned partitions: lists, build
    const int rc3 = [&]() -> int {
        // list of owned partition i = its chunks from source 0, 1, ...; sweeps of BSW chunks
        std::vector<uint32_t> lsO(QL + 1, 0), swO(QL + 1, 0);
        std::vector<int64_t>  tab((size_t) 4 * QL * W);
        {
            std::vector<uint64_t> inblk(W, 0);  // entries of source j already assigned (partition order)
            uint64_t              pos = 0;
            for (uint32_t i = 0; i < QL; i++) {
                lsO[i] = (uint32_t) pos;
                for (uint32_t j = 0; j < W; j++) {
                    const uint64_t c  = rcnt[j * NC + i];
                    int64_t*       t  = &tab[4 * ((size_t) i * W + j)];
                    const uint64_t rb = roff[j] / 4;  // source j's first chunk / entry (roff: entry bytes)
                    t[0]               = (int64_t) (rb + inblk[j]);                // first received entry
                    t[1]               = (int64_t) c;
                    t[2]               = (int64_t) pos;                            // list position
                    t[3]               = (int64_t) rb - (int64_t) rcnt[j * NC + QL];  // id adjustment
                    inblk[j] += c;
                    pos += c;
                }
                swO[i + 1] = swO[i] + (uint32_t) ((pos - lsO[i] + BSW - 1) / BSW);
            }
            lsO[QL] = (uint32_t) pos;
        }
        sweeps = swO[QL];
        const bool ok = pjList.ensure(std::max<uint64_t>(16, RC * 4)) &&
                        rjoin.ensure(std::max<uint64_t>(16, sweeps * SLOT * 4)) &&
                        rrun.ensure(std::max<uint64_t>(16, 2 * sweeps * NSUB * 4));
        if (!ok) {
            set_last_error("hipMalloc failed (device memory)");
            return 4;
        }
        if (to_dev(pjTab, tab, stream) || to_dev(pjLstart, lsO, stream) || to_dev(pjSweep, swO, stream)) {
            set_last_error("host tables to the device failed");
            return 4;
        }
        if (pj_check_on()) {
            for (size_t k = 0; k < (size_t) QL * W; k++) {
                const int64_t* t = &tab[4 * k];
                if (t[0] < 0 || t[1] < 0 || (uint64_t) (t[0] + t[1]) > RC || (uint64_t) (t[2] + t[1]) > RC)
                    PJ_FAIL("relist pair " + std::to_string(k) + " outside the received entries");
            }
            if (lsO[QL] != RC) PJ_FAIL("owned lists do not cover the received chunks");
            std::vector<uint32_t> re(RC);
            PJ_CHECK(hipStreamSynchronize(stream));
            if (RC) PJ_CHECK(hipMemcpy(re.data(), recvE, RC * 4, hipMemcpyDeviceToHost));
            for (size_t k = 0; k < (size_t) QL * W; k++) {
                const int64_t* t = &tab[4 * k];
                for (int64_t i = 0; i < t[1]; i++) {
                    const int64_t id = (int64_t) (re[t[0] + i] & ((1u << 27) - 1u)) + t[3];
                    if (id < 0 || (uint64_t) id >= RC)
                        PJ_FAIL("received entry " + std::to_string(t[0] + i) + " maps to chunk " +
                                std::to_string(id) + " of " + std::to_string(RC));
                }
            }
        }
        launch_pj_relist(recvE, pjTab.as<int64_t>(), QL * W, pjList.as<uint32_t>(), stream);
        PJ_STAGE("k_pj_relist");
        BuildParams bp{};
        bp.g           = g;
        bp.tabs        = d_tabs_;
        bp.pool        = (const uint32_t*) recvC;
        bp.list        = pjList.as<uint32_t>();
        bp.list_start  = pjLstart.as<uint32_t>();
        bp.elem_start  = nullptr;
        bp.slices      = slice_mode ? d_slices : nullptr;
        bp.sweep_start = pjSweep.as<uint32_t>();
        bp.out_codes   = rjoin.as<uint32_t>();
        bp.run_cnt     = rrun.as<uint32_t>();
        bp.run_off     = rrun.as<uint32_t>() + sweeps * NSUB;
        bp.q_base      = q0;
        launch_build(bp, QL, stream);
        PJ_STAGE("k_build");
        PJ_CHECK(hipGetLastError());
        return drain();
    }();
    lap(2);
    // (native: every buffer of this step was allocated before the counts step, so it fails alike
    // or not at all, except under HWBRJ_PJ_CHECK's host checks, which then agree as the callback
    // path does)
    if (!native || pj_check_on()) {
        if (const int rc = agree(rc3)) return rc;
    } else if (rc3) {
        return rc3;
    }
    // ------------------------------------------------------------- 4. the whole filter on every rank
    if (slice_mode && W > 1)
        PJ_XCHG(x->allgather(x->ctx, HWBRJ_PJ_SLICES, (uint64_t) QL * nseg * g.seg_words * 4), "filter slices");
    lap(3);
    // ------------------------------------------------------------- 5. S shard: partition, probe
    uint32_t I = 0;
    const uint32_t items_max = (uint32_t) ((LS / CH + F + 1) * nseg);
    const int rc5 = [&]() -> int {
        sp.src        = dS;
        sp.n          = nS;
        sp.pool       = poolS.as<uint32_t>();
        sp.meta       = metaS.as<uint32_t>();
        sp.wg_used    = usedS.as<uint32_t>();
        sp.wgq_chunks = wgqcS.as<uint32_t>();
        sp.wgq_elems  = wgqeS.as<uint32_t>();
        sp.cap        = capS;
        launch_scatter(sp, SRC_TUPLES, SIDE_S, G, stream);
        launch_plan(wgqcS.as<uint32_t>(), wgqeS.as<uint32_t>(), G, g.log2F, wgqoS.as<uint32_t>(),
                    colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), stream);
        launch_list_fill(metaS.as<uint32_t>(), usedS.as<uint32_t>(), capS, g.log2F, wgqoS.as<uint32_t>(),
                         colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), CH, nseg, lstartS.as<uint32_t>(),
                         estartS.as<uint64_t>(), istartS.as<uint32_t>(), listS.as<uint32_t>(), G, stream);
        ProbeParams pp{};
        pp.g               = g;
        pp.tabs            = d_tabs_;
        pp.pool            = poolS.as<uint32_t>();
        pp.list            = listS.as<uint32_t>();
        pp.list_start      = lstartS.as<uint32_t>();
        pp.item_start      = istartS.as<uint32_t>();
        pp.slices          = slice_mode ? d_slices : nullptr;
        pp.surv            = surv.as<uint32_t>();
        pp.surv_seg_stride = LS * 32;
        pp.surv_cnt        = survcnt.as<uint32_t>();
        pp.surv_off        = survoff.as<uint32_t>();
        pp.filtered        = d_filtered;
        pp.job_surv        = jparts.as<uint32_t>() + F * NSUB;
        const size_t   pl_lds = probe_lds_bytes(g, nullptr);
        const uint32_t PG     = (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / pl_lds));
        launch_probe(pp, PG, stream);
        PJ_STAGE("S scatter + probe");
        // ------------------------------------------------------------- 6. survivor exchange
        // item tables on the device (k_pj_items: regions, survivor totals, their scan); the host
        // reads only the item starts and the scan at every partition's first item
        const uint32_t nbk = items_max / 1024 + 1;
        if (!pjRegion.ensure((uint64_t) items_max * 8 + 8) || !pjTot.ensure((uint64_t) items_max * 4 + 4) ||
            !pjSoff.ensure((uint64_t) items_max * 8 + 8) || !pjBsum.ensure((uint64_t) nbk * 8) ||
            !pjBound.ensure((uint64_t) (F + 1) * 8)) {
            set_last_error("hipMalloc failed (device memory)");
            return 4;
        }
        launch_pj_items(istartS.as<uint32_t>(), lstartS.as<uint32_t>(), survcnt.as<uint32_t>(), items_max, F, nseg,
                        CH, LS * 32, NSUB, pjRegion.as<uint64_t>(), pjTot.as<uint32_t>(), pjBsum.as<uint64_t>(),
                        pjSoff.as<uint64_t>(), pjBound.as<uint64_t>(), stream);
        if (native) {
            // every buffer the survivor exchange and the owner's join need, at its worst case:
            // survivors sent <= this shard's S tuples; received <= every shard's (their |S| came
            // with the R counts); items and their run tables likewise
            uint64_t nS_all = 0;
            RImax = 0;
            for (uint32_t j = 0; j < W; j++) {
                const uint64_t nSj = rcnt[(uint64_t) j * NC + QL + 2];
                nS_all += nSj;
                RImax += ((uint64_t) G * pj_region_cap(nSj, G, F) / CH + F + 1) * nseg;
            }
            RWmax = nS_all;
            const uint32_t NJ  = QL * NSUB;
            bool ok = true;
            sendS = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_S_SEND, std::max<uint64_t>(16, nS * 4));
            sendM = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_M_SEND, std::max<uint64_t>(16, (uint64_t) items_max * NSUB * 4));
            recvS = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_S_RECV, std::max<uint64_t>(16, RWmax * 4));
            recvM = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_M_RECV, std::max<uint64_t>(16, RImax * NSUB * 4));
            ok &= sendS && sendM && recvS && recvM;
            ok &= pjIbase.ensure(std::max<uint64_t>(16, RImax * 8)) && pjCnt.ensure(std::max<uint64_t>(16, RImax * NSUB * 4)) &&
                  pjOff.ensure(std::max<uint64_t>(16, RImax * NSUB * 4)) && pjJobs.ensure((uint64_t) NJ * 4) &&
                  pjWtot.ensure(std::max<uint64_t>(16, RImax * 4)) && pjWscan.ensure((RImax + 1) * 8) &&
                  pjBsum.ensure((uint64_t) std::max<uint64_t>(nbk, RImax / 1024 + 1) * 8) &&
                  pjTab2.ensure((size_t) 3 * QL * W * 4) && pjIstart.ensure((QL + 1) * 4);
            if (!ok) {
                set_last_error("hipMalloc failed (device memory)");
                return 4;
            }
            return 0;  // (the counts message is built on the device)
        }
        PJ_CHECK(hipMemcpyAsync(isS.data(), istartS.p, (F + 1) * 4, hipMemcpyDeviceToHost, stream));
        PJ_CHECK(hipMemcpyAsync(bnd.data(), pjBound.p, (F + 1) * 8, hipMemcpyDeviceToHost, stream));
        PJ_CHECK(hipStreamSynchronize(stream));
        return 0;
    }();
    // survivors of this shard packed per destination (after the starts have reached the host)
    auto pack_survivors = [&]() -> int {
        I = isS[F];
        sofs = bnd;  // (sofs at partition starts: all the host needs)
        sendS = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_S_SEND, std::max<uint64_t>(16, bnd[F] * 4));
        sendM = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_M_SEND, std::max<uint64_t>(16, (uint64_t) I * NSUB * 4));
        if (!sendS || !sendM) {
            set_last_error("exchange buffer (survivor send) unavailable");
            return 20;
        }
        if (pj_check_on()) {
            std::vector<uint64_t> region(I), so(I + 1);
            std::vector<uint32_t> tot(I);
            if (I) {
                PJ_CHECK(hipMemcpy(region.data(), pjRegion.p, (size_t) I * 8, hipMemcpyDeviceToHost));
                PJ_CHECK(hipMemcpy(tot.data(), pjTot.p, (size_t) I * 4, hipMemcpyDeviceToHost));
            }
            PJ_CHECK(hipMemcpy(so.data(), pjSoff.p, (size_t) (I + 1) * 8, hipMemcpyDeviceToHost));
            for (uint32_t it = 0; it < I; it++)
                if (region[it] + tot[it] > nseg * LS * 32 || so[it + 1] != so[it] + tot[it])
                    PJ_FAIL("item " + std::to_string(it) + " region or survivor scan inconsistent");
            if (so[I] != bnd[F]) PJ_FAIL("survivor scan total");
        }
        PjOwn own;
        uint64_t own_items = 0;  // (self_direct: this rank's items to itself, at receive item own_ri)
        uint64_t own_ri = 0;
        if (self_direct) {
            uint64_t rw = 0;  // its first receive word / item: every lower source's come first
            for (uint32_t j = 0; j < (uint32_t) rank; j++) {
                rw += rcnt[(uint64_t) j * NC + QL];
                for (uint32_t i = 0; i < QL; i++) own_ri += rcnt[(uint64_t) j * NC + i];
            }
            own.lo    = isS[rank * QL];
            own.hi    = isS[(rank + 1) * QL];
            own.delta = (int64_t) rw - (int64_t) bnd[rank * QL];
            own.out   = recvS;
            own_items = own.hi - own.lo;
        }
        launch_pj_surv_pack(surv.as<uint32_t>(), pjRegion.as<uint64_t>(), pjTot.as<uint32_t>(), pjSoff.as<uint64_t>(),
                            I, sendS, stream, own);
        PJ_STAGE("k_pj_surv_pack");
        if (I) PJ_CHECK(hipMemcpyAsync(sendM, survcnt.p, (size_t) I * NSUB * 4, hipMemcpyDeviceToDevice, stream));
        if (own_items)
            PJ_CHECK(hipMemcpyAsync(recvM + own_ri * NSUB, survcnt.as<uint32_t>() + (uint64_t) own.lo * NSUB,
                                    own_items * NSUB * 4, hipMemcpyDeviceToDevice, stream));
        return 0;
    };
    lap(4);
    if (native) {
        if (const int rc = native_counts(istartS.as<uint32_t>(), pjBound.as<uint64_t>(), rc5, 0, isS.data(), bnd.data()))
            return rc;
        if (const int rc = peers(rcnt.data() + QL + 1, NC, rc5)) return rc;
        // (what follows allocates nothing: a failure here is a bug or a broken device, and returns)
        if (const int rc = pack_survivors()) return rc;
    } else {
        int rc5b = rc5 ? rc5 : pack_survivors();
        if (!rc5b) {
            // per destination j: items of each of its partitions, then its survivor words
            for (uint32_t j = 0; j < W; j++) {
                for (uint32_t i = 0; i < QL; i++) scnt[j * NC + i] = isS[j * QL + i + 1] - isS[j * QL + i];
                scnt[j * NC + QL] = bnd[(j + 1) * QL] - bnd[j * QL];
            }
            rc5b = drain();
        }
        for (uint32_t j = 0; j < W; j++) scnt[j * NC + QL + 1] = (uint64_t) (uint32_t) rc5b;
        PJ_XCHG(x->alltoall_u64(x->ctx, scnt.data(), rcnt.data(), NC), "survivor counts");
        if (const int rc = peers(rcnt.data() + QL + 1, NC, rc5b)) return rc;
    }
    lap(4);
    const int rc6 = [&]() -> int {
        for (uint32_t j = 0; j < W; j++) {
            uint64_t c = 0;
            for (uint32_t i = 0; i < QL; i++) c += rcnt[j * NC + i];
            ritems[j] = c;
            rwords[j] = rcnt[j * NC + QL];
            RI += c;
            RW += rwords[j];
            plan_mi = std::max<uint64_t>(plan_mi, std::max<uint64_t>(c, isS[(j + 1) * QL] - isS[j * QL]));
            plan_mw = std::max<uint64_t>(plan_mw, std::max<uint64_t>(rwords[j], bnd[(j + 1) * QL] - bnd[j * QL]));
        }
        if (native) {  // (allocated at RImax / RWmax before the counts step, from every shard's exact
                       // |S|, so no input can exceed them: a bug guard)
            if (RI > RImax || RW > RWmax) {
                set_last_error("partitioned join: received survivors above their bound");
                return 21;
            }
            return 0;
        }
        recvS = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_S_RECV, std::max<uint64_t>(16, RW * 4));
        recvM = (uint32_t*) x->buffer(x->ctx, HWBRJ_PJ_M_RECV, std::max<uint64_t>(16, RI * NSUB * 4));
        if (!recvS || !recvM) {
            set_last_error("exchange buffer (survivor receive) unavailable");
            return 20;
        }
        return 0;
    }();
    if (native) {
        if (rc6) return rc6;
    } else if (const int rc = agree(rc6)) {
        return rc;
    }
    {
        uint64_t ro = 0;
        for (uint32_t j = 0; j < W; j++) {
            soff[j]   = sofs[j * QL] * 4;  // (sofs: the survivor scan at every partition's first item)
            sbytes[j] = (sofs[(j + 1) * QL] - sofs[j * QL]) * 4;
            roff[j]   = ro * 4;
            rbytes[j] = rwords[j] * 4;
            ro += rwords[j];
        }
        if (self_direct) sbytes[rank] = rbytes[rank] = 0;  // (written by k_pj_surv_pack)
    }
    PJ_XCHG(x->alltoallv(x->ctx, HWBRJ_PJ_S_SEND, soff.data(), sbytes.data(), HWBRJ_PJ_S_RECV, roff.data(), rbytes.data()),
            "survivors");
    {
        uint64_t ri = 0;
        for (uint32_t j = 0; j < W; j++) {
            soff[j]   = (uint64_t) isS[j * QL] * NSUB * 4;
            sbytes[j] = (uint64_t) (isS[(j + 1) * QL] - isS[j * QL]) * NSUB * 4;
            roff[j]   = ri * NSUB * 4;
            rbytes[j] = ritems[j] * NSUB * 4;
            ri += ritems[j];
        }
        if (self_direct) sbytes[rank] = rbytes[rank] = 0;  // (copied from survcnt)
    }
    PJ_XCHG(x->alltoallv(x->ctx, HWBRJ_PJ_M_SEND, soff.data(), sbytes.data(), HWBRJ_PJ_M_RECV, roff.data(), rbytes.data()),
            "survivor run counts");
    lap(5);
    // ------------------------------------------------------------- 7. join of the owned partitions
    // (no collective of the join follows: a failure here is this rank's alone; the async join's
    // plan step, when asked for, comes after it on every rank whatever this returns)
    // The owner's item tables on the device (k_pj_item_tables) from the received per-item counts;
    // the host lays out only the (owned partition, source) pairs: items of owned partition i are
    // those of source 0, 1, ... (each source's block is in partition order).
    uint64_t small_h[6] = {0, 0, 0, 0, 0, 0};
    const int rc7 = [&]() -> int {
    const uint32_t NJ = QL * NSUB;
    std::vector<uint32_t> tab2((size_t) 3 * QL * W), istart(QL + 1, 0);
    {
        std::vector<uint64_t> jitem(W), jpos(W, 0);  // per source: first received item, cursor
        uint64_t              ai = 0;
        for (uint32_t j = 0; j < W; j++) {
            jitem[j] = ai;
            ai += ritems[j];
        }
        uint32_t out = 0;
        for (uint32_t i = 0; i < QL; i++) {
            istart[i] = out;
            for (uint32_t j = 0; j < W; j++) {
                const uint32_t c = (uint32_t) rcnt[j * NC + i];
                uint32_t*      t = &tab2[3 * ((size_t) i * W + j)];
                t[0]             = (uint32_t) (jitem[j] + jpos[j]);
                t[1]             = c;
                t[2]             = out;
                jpos[j] += c;
                out += c;
            }
        }
        istart[QL] = out;
    }
    const uint32_t nbr = (uint32_t) (RI / 1024 + 1);
    if (!pjIbase.ensure(std::max<uint64_t>(16, RI * 8)) || !pjCnt.ensure(std::max<uint64_t>(16, RI * NSUB * 4)) ||
        !pjOff.ensure(std::max<uint64_t>(16, RI * NSUB * 4)) || !pjJobs.ensure((uint64_t) NJ * 4) ||
        !pjWtot.ensure(std::max<uint64_t>(16, RI * 4)) || !pjWscan.ensure((RI + 1) * 8) ||
        !pjBsum.ensure((uint64_t) nbr * 8)) {
        set_last_error("hipMalloc failed (device memory)");
        return 4;
    }
    if (to_dev(pjTab2, tab2, stream) || to_dev(pjIstart, istart, stream)) {
        set_last_error("host tables to the device failed");
        return 4;
    }
    PJ_CHECK(hipMemsetAsync(pjJobs.p, 0, (size_t) NJ * 4, stream));
    launch_pj_recv_scan(recvM, (uint32_t) RI, NSUB, pjWtot.as<uint32_t>(), pjBsum.as<uint64_t>(),
                        pjWscan.as<uint64_t>(), stream);
    launch_pj_item_tables(pjTab2.as<uint32_t>(), QL * W, W, recvM, pjWscan.as<uint64_t>(), NSUB,
                          pjIbase.as<uint64_t>(), pjCnt.as<uint32_t>(), pjOff.as<uint32_t>(), pjJobs.as<uint32_t>(),
                          stream);
    if (pj_check_on()) {
        PJ_CHECK(hipStreamSynchronize(stream));
        std::vector<uint64_t> ibase(RI), ws(RI + 1);
        std::vector<uint32_t> icnt((size_t) RI * NSUB);
        if (RI) {
            PJ_CHECK(hipMemcpy(ibase.data(), pjIbase.p, RI * 8, hipMemcpyDeviceToHost));
            PJ_CHECK(hipMemcpy(icnt.data(), pjCnt.p, RI * NSUB * 4, hipMemcpyDeviceToHost));
        }
        PJ_CHECK(hipMemcpy(ws.data(), pjWscan.p, (RI + 1) * 8, hipMemcpyDeviceToHost));
        if (ws[RI] != RW) PJ_FAIL("received survivor scan total " + std::to_string(ws[RI]) + " != " + std::to_string(RW));
        for (uint64_t it = 0; it < RI; it++) {
            uint64_t t = 0;
            for (uint32_t s2 = 0; s2 < NSUB; s2++) t += icnt[it * NSUB + s2];
            if (ibase[it] + t > RW) PJ_FAIL("item " + std::to_string(it) + " runs outside the received survivors");
        }
        if (istart[QL] != RI) PJ_FAIL("owned items do not cover the received items");
    }
    PJ_CHECK(hipMemsetAsync(jparts.as<uint32_t>() + 2 * F * NSUB, 0, 4, stream));  // nextra
    JoinParams jp{};
    jp.r_codes         = rjoin.as<uint32_t>();
    jp.r_sweep_start   = pjSweep.as<uint32_t>();
    jp.r_cnt           = rrun.as<uint32_t>();
    jp.r_off           = rrun.as<uint32_t>() + sweeps * NSUB;
    jp.slot            = (uint32_t) SLOT;
    jp.surv            = recvS;
    jp.surv_cnt        = pjCnt.as<uint32_t>();
    jp.surv_off        = pjOff.as<uint32_t>();
    jp.item_start      = pjIstart.as<uint32_t>();
    jp.list_start      = pjIstart.as<uint32_t>();  // (unused: item_base)
    jp.surv_seg_stride = 0;
    jp.nseg            = 1;
    jp.CH              = CH;
    jp.log2NSUB        = g.log2NSUB;
    jp.hash_shift      = g.hash_shift;
    jp.bitmap          = (g.sub_shift > 0 && 32 - g.hash_shift <= join_bitmap_log2()) ? 1u : 0u;
    jp.jsum            = (uint64_t*) ((char*) small.p + 128);
    jp.nparts          = jparts.as<uint32_t>();
    jp.extra           = jtask.as<uint2>();
    jp.nextra          = jparts.as<uint32_t>() + 2 * F * NSUB;
    jp.item_base       = pjIbase.as<uint64_t>();
    jp.split_surv      = test_hooks().join_split;
    jp.timing          = 1;
    launch_join(jp, NJ, pjJobs.as<uint32_t>(), stream);
    PJ_STAGE("k_join");
    PJ_CHECK(hipGetLastError());
    return read_join_counts(d_result, true, stream, small_h);
    }();
    lap(6);
    if (pj_make_plan()) {  // (every rank: a collective, on the join's transport)
        PJ_CHECK(hipStreamSynchronize(stream));
        if (const int rc = pj_plan_from_sync(world, rank, nR, nR_total, nS, args, plan_mr, plan_mi, plan_mw))
            return rc7 ? rc7 : rc;
    }
    if (rc7) return rc7;
    pending_ = false;
    ring_drop();  // (single-GPU joins enqueued before it are no longer collected)
    have_filter_ = false;  // (the slices live in the caller's exchange buffer)
    last_nj_     = 0;      // job_surv holds this join's counts: the next enqueue clears the table
    if (st) {
        memset(st, 0, sizeof(*st));
        st->join_key_bits  = 32;  // (survivor words travel as codes)
        st->filtered       = args ? small_h[2] : nS;
        st->matches        = (int64_t) small_h[0];
        st->mode           = g.mode;
        st->format         = g.s_format;
        st->partitions     = F;
        st->subparts       = NSUB;
        st->slice_segments = nseg;
        // host wall time per stage: R pass, R exchange, build, slice all-gather, S pass (scatter +
        // probe), survivor exchange, join. With the native transport a stage's kernels may finish
        // inside the next stage's host wait (the stream is only drained where counts are read).
        st->ms_r_scatter = ms[0];
        st->ms_r_index   = ms[1];  // R exchange
        st->ms_build     = ms[2];
        st->ms_surv      = ms[3] + ms[5];  // slice all-gather + survivor exchange
        st->ms_s_scatter = ms[4];
        st->ms_join      = ms[6];
        st->ms_join_probe = small_h[4] ? ms[6] * (double) small_h[3] / (double) small_h[4] : 0.0;
        st->ms_total =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    return 0;
}

}  // namespace hwbrj
