// hwbrj_engine.cpp -- host orchestration of the MI355X bloom radix join (DESIGN.md "Pipeline").
//
// The reference runs R pass-1 (+ bloom add), S pass-1 (+ bloom contains), pass-2 and the
// bucket-chaining join inside pthreads with barriers (src/parallel_radix_join_bloom.c:1059-1506).
// Here every barrier is a kernel boundary on one HIP stream, and the task queues are replaced by
// device-built chunk lists and item tables (no host round trips inside the join).
#include "hwbrj_engine.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

namespace hwbrj {

#define HWBRJ_CHECK(expr)                                                                 \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            set_last_error(std::string(#expr) + ": " + hipGetErrorString(e_));            \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

// ---------------------------------------------------------------------------- tables
bool build_crc_tables(CrcTables* t) {
    uint32_t col[32];  // f(e_i)
    for (int i = 0; i < 32; i++) col[i] = crc_f_bitwise(1u << i);
    for (int j = 0; j < 8; j++)
        for (int v = 0; v < 16; v++) t->fwd[j][v] = crc_f_bitwise((uint32_t) v << (4 * j));
    // Invert the 32x32 GF(2) matrix whose column i is col[i]: solve f(x) = e_r for every r.
    // Gauss-Jordan on rows of [M | I] packed as 64-bit rows (row r: bit c of M, bit 32+c of I).
    uint64_t rows[32];
    for (int r = 0; r < 32; r++) {
        uint64_t row = 0;
        for (int c = 0; c < 32; c++)
            if ((col[c] >> r) & 1u) row |= 1ull << c;
        rows[r] = row | (1ull << (32 + r));
    }
    for (int c = 0; c < 32; c++) {
        int piv = -1;
        for (int r = c; r < 32; r++)
            if ((rows[r] >> c) & 1ull) {
                piv = r;
                break;
            }
        if (piv < 0) return false;
        std::swap(rows[c], rows[piv]);
        for (int r = 0; r < 32; r++)
            if (r != c && ((rows[r] >> c) & 1ull)) rows[r] ^= rows[c];
    }
    // rows now = [I | M^-1]; column j of M^-1 = finv(e_j)
    uint32_t icol[32];
    for (int j = 0; j < 32; j++) {
        uint32_t v = 0;
        for (int r = 0; r < 32; r++)
            if ((rows[r] >> (32 + j)) & 1ull) v |= 1u << r;
        icol[j] = v;
    }
    for (int j = 0; j < 8; j++)
        for (int v = 0; v < 16; v++) {
            uint32_t x = (uint32_t) v << (4 * j), r = 0;
            for (int b = 0; b < 32; b++)
                if ((x >> b) & 1u) r ^= icol[b];
            t->inv[j][v] = r;
        }
    // self-check on a few values
    for (uint32_t x : {0u, 1u, 42u, 0xDEADBEEFu, 0x7FFFFFFFu}) {
        if (nibble_map(&t->inv[0][0], nibble_map(&t->fwd[0][0], x)) != x) return false;
        if (nibble_map(&t->fwd[0][0], x) != crc_f_bitwise(x)) return false;
    }
    return true;
}

// ------------------------------------------------------------------------- generator plan
int make_gen_plan(GenPlan* plan, uint64_t num_tuples, uint32_t nthreads, uint64_t maxid,
                  uint64_t threshold, double selectivity) {
    // src/generator.c:331-395, integer widths as in the reference
    if (nthreads == 0 || nthreads > (uint32_t) kMaxGenChunks || threshold == 0) return 1;
    const unsigned int pagesize      = 4096;
    unsigned int       npages        = (unsigned int) ((num_tuples * 8u) / pagesize + 1u);
    unsigned int       npages_perthr = npages / nthreads;
    uint64_t ntuples_perthr = (uint64_t) npages_perthr * (uint64_t) (pagesize / 8u);
    uint64_t ntuples_above  = (uint64_t) ((double) num_tuples * (1 - selectivity));
    if (npages_perthr == 0) ntuples_perthr = num_tuples / nthreads;
    uint64_t ntuples_above_perthr  = (uint64_t) ((double) ntuples_perthr * (1 - selectivity));
    uint64_t ntuples_lastthr       = num_tuples - ntuples_perthr * (nthreads - 1);
    uint64_t ntuples_above_lastthr = ntuples_above - (uint64_t) (nthreads - 1) * ntuples_above_perthr;
    uint64_t offset = 0, offset_above = 0;
    plan->nchunks    = nthreads;
    plan->num_tuples = num_tuples;
    plan->threshold  = threshold;
    const uint64_t span = maxid > threshold ? maxid - threshold : 0;
    for (uint32_t t = 0; t < nthreads; t++) {
        GenChunk& c  = plan->chunk[t];
        c.firstkey   = (int64_t) ((offset + 1) % threshold);
        c.firstabove = (int64_t) (threshold + (offset_above + 1) % (span > 1 ? span : 1));
        uint64_t na  = (t == nthreads - 1) ? ntuples_above_lastthr : ntuples_above_perthr;
        c.n          = (t == nthreads - 1) ? ntuples_lastthr : ntuples_perthr;
        c.start      = offset + offset_above;
        if (na > c.n || c.start + c.n > num_tuples) return 2;  // the reference would overrun
        c.n_below = c.n - na;
        offset += ntuples_perthr - ntuples_above_perthr;
        offset_above += ntuples_above_perthr;
    }
    return 0;
}

// ------------------------------------------------------------------------------ geometry
bool plan_geometry(const bloom_filter_args_t* a, uint64_t nR, Geometry* g, std::string* err, bool mat) {
    memset(g, 0, sizeof(*g));
    g->variant = -1;
    if (!a) {
        g->mode  = MODE_NOBLOOM;
        g->log2F = kMaxLog2F;
    } else {
        const uint64_t m = a->m, B = a->B, k = a->k;
        if (m == 0 || (m & (m - 1)) != 0) {
            *err = "m must be a power of 2";  // src/bloom_filter.c:27
            return false;
        }
        if (m > (1ull << 32)) {
            *err = "m > 2^32 bits is outside the 32-bit hash contract of src/bloom_filter.c";
            return false;
        }
        if (k > 4096) {
            *err = "k > 4096 is not supported";
            return false;
        }
        if (a->variant != BASIC && a->variant != BLOCKED && a->variant != SECTORIZED) {
            *err = "unknown filter variant";
            return false;
        }
        g->variant = (int) a->variant;
        g->k       = (uint32_t) k;
        g->m       = m;
        if (a->variant != BASIC) {
            if (B == 0 || (B & (B - 1)) != 0) {
                *err = "B must be a power 2";  // src/bloom_filter.c:30
                return false;
            }
            if (m % B != 0) {
                *err = "m must be a multiple of B";  // :31
                return false;
            }
            if (B > (1ull << 31)) {
                *err = "B too large";
                return false;
            }
            g->B          = (uint32_t) B;
            g->nblocks    = (uint32_t) std::min<uint64_t>(m / B, 0xFFFFFFFFull);
            g->block_span = (uint32_t) ((B / 8) * 8);
        }
        uint64_t F = 0;
        if (a->variant == BASIC) {
            // k >= 2: KIND_BASIC_KK, whose slice build partitions k * |R| bit positions (bounded by
            // the scatter's chunk ids; beyond that the global fallback)
            if (k >= 1 && m >= 32 && k * nR <= (1ull << 31)) {
                g->mode = MODE_SLICE_BASIC;
                F       = std::min<uint64_t>(1024, m / 32);
            } else {
                g->mode = MODE_GLOBAL;
            }
        } else {
            if (B >= 8 && m >= 32 && (m / B) <= 0xFFFFFFFFull) {
                g->mode = MODE_SLICE_BLOCK;
                F       = std::min<uint64_t>(std::min<uint64_t>(1024, m / B), m / 32);
                if (dev_knobs().maxf) F = std::min<uint64_t>(F, dev_knobs().maxf);  // dev A/B
            } else {
                g->mode = MODE_GLOBAL;
            }
        }
        g->log2F = (g->mode == MODE_GLOBAL) ? kMaxLog2F : ilog2u(F);
        if (g->mode == MODE_SLICE_BLOCK || g->mode == MODE_SLICE_BASIC) {
            g->slice_bits = (uint32_t) (m >> g->log2F);
            g->seg_bits   = std::min(g->slice_bits, kSliceMaxBits);
            g->nseg       = g->slice_bits / g->seg_bits;
            g->seg_words  = std::max<uint32_t>(4, g->seg_bits / 32);
        }
        if (g->mode == MODE_SLICE_BLOCK && ilog2u(B) <= g->log2F) g->format = FMT_PACKED;
        // S partitions use R's word format (the 22-bit S words of round 2, FMT_C22, cut 2.6 GB of
        // S traffic but cost more in the probe's key recovery: removed in round 6)
        g->s_format = g->format;
        if (g->mode == MODE_SLICE_BLOCK || g->mode == MODE_SLICE_BASIC) g->log2seg = ilog2u(g->seg_bits);
        if (a->variant != BASIC) {
            g->log2B    = ilog2u(B);
            g->log2secw = std::min<uint32_t>(g->log2B, 6);
            g->nsecmask = (uint32_t) (B >> g->log2secw) - 1u;
            if (g->mode == MODE_SLICE_BLOCK) g->lbmask = (g->nblocks >> g->log2F) - 1u;
        }
    }
    // Join sub-partitions (k_join): codes of a job share their low hash_shift bits. Where the
    // partition digit is a code digit (sub_shift = log2F), 2^(14 - log2F) subs make the job keys
    // v = code >> hash_shift fit the 2^18-bit LDS bitmap; otherwise (or when that needs > 64 subs)
    // the hash table path needs <= ~4096 R keys per job.
    const uint64_t F    = 1ull << g->log2F;
    const uint64_t rper = (nR + F - 1) / F;
    uint32_t       l2s  = 0;
    g->sub_shift  = (g->mode == MODE_SLICE_BASIC) ? 0 : g->log2F;
    if (mat && g->sub_shift > 0) {  // k_join_mat's bitmap path: keys v < 2^17, <= 4096 R tuples per job
        l2s = g->log2F >= 15 ? 0 : std::min<uint32_t>(6, 15 - g->log2F);
        while (l2s < 6 && (rper >> l2s) > 4000) l2s++;
    } else if (mat) {  // its hash table: <= 2048 R tuples per piece, so ~1536 per job on average
        while (l2s < 6 && (rper >> l2s) > 1536) l2s++;
    } else if (g->sub_shift > 0 && g->log2F + 6 >= 14) {
        l2s = g->log2F >= 14 ? 0 : 14 - g->log2F;
        if (dev_knobs().l2sub && g->log2F + dev_knobs().l2sub >= 14)  // dev A/B: more, smaller jobs
            l2s = std::min<uint32_t>(6, dev_knobs().l2sub);
    } else {
        while (l2s < 6 && (rper >> l2s) > 4096) l2s++;
    }
    if (g->sub_shift + l2s == 0) l2s = 1;  // k_join stores code >> hash_shift with an empty sentinel
    g->log2NSUB   = l2s;
    g->hash_shift = g->sub_shift + g->log2NSUB;
    return true;
}

// ---------------------------------------------------------------------------- buffers
bool DevBuf::ensure(size_t need) {
    if (need == 0) need = 16;
    if (need <= bytes) return true;
    release();
    if (hipMalloc(&p, need) != hipSuccess) {
        p     = nullptr;
        bytes = 0;
        return false;
    }
    bytes = need;
    return true;
}

void DevBuf::release() {
    if (p) (void) hipFree(p);
    p     = nullptr;
    bytes = 0;
}

// ------------------------------------------------------------- dev knobs and test hooks
const DevKnobs& dev_knobs() {
    static const DevKnobs k = [] {
        DevKnobs d;
#ifdef HWBRJ_DEV_BUILD
        auto u = [](const char* n) -> uint32_t {
            const char* e = getenv(n);
            return e ? (uint32_t) strtoul(e, nullptr, 0) : 0u;
        };
        d.kk1       = getenv("HWBRJ_DEV_KK1") != nullptr;
        d.kk_gather = getenv("HWBRJ_DEV_KK_GATHER") != nullptr;
        d.noxcd     = getenv("HWBRJ_DEV_NOXCD") != nullptr;
        d.dbg       = getenv("HWBRJ_DBG") != nullptr;
        d.maxf      = u("HWBRJ_DEV_MAXF");
        d.scwpc     = u("HWBRJ_DEV_SCWPC");
        if (getenv("HWBRJ_DEV_EVFLAGS")) d.evflags = (int) u("HWBRJ_DEV_EVFLAGS");
        d.l2sub     = u("HWBRJ_DEV_L2SUB");
        d.ovl       = getenv("HWBRJ_DEV_OVL") != nullptr;
        d.rfirst    = getenv("HWBRJ_DEV_RFIRST") != nullptr;
#endif
        return d;
    }();
    return k;
}

std::string dev_knobs_string() {
    const DevKnobs& d = dev_knobs();
    std::string     r;
    auto add = [&](const std::string& w) { r += (r.empty() ? "" : " ") + w; };
    if (d.kk1) add("HWBRJ_DEV_KK1");
    if (d.kk_gather) add("HWBRJ_DEV_KK_GATHER");
    if (d.noxcd) add("HWBRJ_DEV_NOXCD");
    if (d.dbg) add("HWBRJ_DBG");
    if (d.maxf) add("HWBRJ_DEV_MAXF=" + std::to_string(d.maxf));
    if (d.scwpc) add("HWBRJ_DEV_SCWPC=" + std::to_string(d.scwpc));
    if (d.evflags >= 0) add("HWBRJ_DEV_EVFLAGS=" + std::to_string(d.evflags));
    if (d.l2sub) add("HWBRJ_DEV_L2SUB=" + std::to_string(d.l2sub));
    if (d.ovl) add("HWBRJ_DEV_OVL");
    if (d.rfirst) add("HWBRJ_DEV_RFIRST");
    return r;
}

TestHooks& test_hooks() {
    static TestHooks h;
    return h;
}

Engine::Engine(int device) : device_(device) {
    (void) dev_knobs();  // the dev environment is read once, here (dev builds only)
    (void) hipSetDevice(device);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) cus_ = prop.multiProcessorCount;
    (void) hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking);
    // ev_[0..7] only time phases (elapsed-time reads after ev_[8] has completed): no system-scope
    // fence on record, whose cache writeback idled the GPU ~6 us per marker. ev_[8] (waited on,
    // and ordering later joins) and ev_[9] keep the default release.
    const unsigned evf = dev_knobs().evflags >= 0 ? (unsigned) dev_knobs().evflags : hipEventDisableSystemFence;
    for (int i = 0; i < 10; i++)
        (void) (i < 8 ? hipEventCreateWithFlags(&ev_[i], evf) : hipEventCreate(&ev_[i]));
    CrcTables t;
    if (!build_crc_tables(&t)) set_last_error("CRC table inversion failed");
    (void) hipMalloc((void**) &d_tabs_, sizeof(CrcTables));
    (void) hipMemcpy(d_tabs_, &t, sizeof(CrcTables), hipMemcpyHostToDevice);
    (void) hipMalloc((void**) &d_plan_, sizeof(GenPlan));
}

Engine::~Engine() { release(); }

void Engine::release() {
    (void) pj_drain();
    pj_q_.clear();                       // (joins in flight are dropped)
    if (pj_plan_.valid) pj_lost_ = true;  // (the next async join runs in the failed mode: a new plan)
    for (DevBuf* b : {&pjX, &pjRitems, &pjRing}) b->release();
    for (DevBuf* b : {&poolR, &metaR, &usedR, &wgqcR, &wgqeR, &wgqoR, &lstartR, &estartR, &istartR,
                      &listR, &poolS, &metaS, &usedS, &wgqcS, &wgqeS, &wgqoS, &lstartS, &estartS,
                      &istartS, &listS, &slices, &bitmap, &rjoin, &rrun, &surv, &survcnt, &survoff,
                      &dense, &small, &bpos, &colR, &colS, &mtab, &mcount, &jtask, &jparts, &pjList,
                      &pjLstart, &pjSweep, &pjTab, &pjRegion, &pjTot, &pjSoff, &pjIbase, &pjCnt, &pjOff,
                      &pjIstart, &pjJobs, &ppoolR, &ppoolS, &rpay, &survpos, &dense2, &kkcnt, &xcnt_, &pjBsum, &pjBound, &pjWtot, &pjWscan, &pjTab2})
        b->release();
    for (DevBuf& b : xslot_) b.release();
    if (pending_) (void) hipEventSynchronize(ev_[8]);  // (the ring's joins end before it is freed)
    ring_drop();
    jring_.release();
    have_filter_ = false;
}

// One join's result slot: 128 bytes of result words (read_join_counts), then k_join's partial sums
static size_t ring_slot_bytes() { return 128 + join_sum_slots() * join_sum_stride() * 8; }

static uint64_t region_cap(uint64_t n, uint32_t G, uint32_t F) {
    const uint64_t units = (n + 3) / 4;
    const uint64_t per   = ((units + G - 1) / G) * 4;
    return (per + 31) / 32 + F + 1;
}

int Engine::run(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                const bloom_filter_args_t* args, hipStream_t stream, hwbrj_stats_t* st, int jkind) {
    const int rc = enqueue(dR, nR, dS, nS, args, stream, dev_knobs().dbg, jkind);
    return rc ? rc : wait(st);
}

int Engine::run_async(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                      const bloom_filter_args_t* args, hipStream_t stream, int jkind) {
    // back-to-back joins: no phase events (each marker idles the GPU ~6 us between the kernels
    // around it, profiles/r03/gaps_*), so hwbrj_join_wait reports counts only
    phase_ev_    = false;
    const int rc = enqueue(dR, nR, dS, nS, args, stream, false, jkind);
    phase_ev_    = true;
    return rc;
}

// Phase boundary i (synchronous joins only). A marker idles the GPU ~6 us between the kernels
// around it; attaching the boundary to the next kernel's dispatch instead (hipExtLaunchKernel's
// start event) measured slower still (~10 us gaps, profiles/r03/async_no_events_ab.log).
hipError_t Engine::mark(int i, hipStream_t stream) {
    return phase_ev_ ? hipEventRecord(ev_[i], stream) : hipSuccess;
}

int Engine::reserve(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                    const bloom_filter_args_t* args, int jkind) {
    alloc_only_  = true;
    const int rc = enqueue(dR, nR, dS, nS, args, nullptr, false, jkind);
    alloc_only_  = false;
    last_nj_     = 0;  // buffers may be new: the next join clears its job table
    return rc;
}

int Engine::run_mat(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                    const bloom_filter_args_t* args, hipStream_t stream, const MatReq& mat,
                    hwbrj_stats_t* st) {
    const int rc = enqueue(dR, nR, dS, nS, args, stream, false, 0, &mat);
    return rc ? rc : wait(st);
}

int Engine::enqueue(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                    const bloom_filter_args_t* args, hipStream_t stream, bool dbg, int jkind,
                    const MatReq* mat) {
    if (jkind < 0 || jkind > 2) {
        set_last_error("unknown per-partition join algorithm");
        return 2;
    }
    HWBRJ_CHECK(hipSetDevice(device_));
    Geometry    g;
    std::string err;
    if (!plan_geometry(args, nR, &g, &err, mat != nullptr)) {
        set_last_error(err);
        return 2;
    }
    if (mat && g.mode == MODE_GLOBAL) {
        set_last_error("global-bitmap mode: materialized by the side pass");
        return kRcMatGlobal;
    }
    const bool kk1 = dev_knobs().kk1;  // dev A/B: basic k = 1 on the bit-pass path
    if (!mat && g.mode == MODE_SLICE_BASIC && (g.k > 1 || kk1) && (uint64_t) g.k * nR <= (1ull << 31) &&
        !dev_knobs().kk_gather) {
        if (!stream) stream = own_stream_;
        if (pending_ && stream != pending_stream_) HWBRJ_CHECK(hipStreamWaitEvent(stream, ev_[8], 0));
        return enqueue_basic_kk(dR, nR, dS, nS, g, stream, jkind);
    }
    if (!stream) stream = own_stream_;
    // Every join on this device shares this Engine's scratch (pools, lists, slices, counters):
    // a join enqueued on another stream than a still-pending one must run after it (on the same
    // stream, stream order does it: no wait packet between back-to-back joins).
    if (pending_ && stream != pending_stream_) HWBRJ_CHECK(hipStreamWaitEvent(stream, ev_[8], 0));
    const uint32_t F = 1u << g.log2F, NSUB = 1u << g.log2NSUB, NJ = F * NSUB;
    const bool     slice_mode = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    const uint32_t nseg       = slice_mode ? g.nseg : 1;
    const uint32_t CH         = probe_chunks_per_item();  // chunks per probe item
    const size_t   sc_lds     = mat ? scatter_pay_lds_bytes(g.log2F) : scatter_lds_bytes(g.log2F);
    uint32_t       sc_wpc     = (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / sc_lds));
    if (dev_knobs().scwpc)  // dev A/B: scatter workgroups per CU
        sc_wpc = std::max(1u, std::min(sc_wpc, dev_knobs().scwpc));
    const uint32_t G          = (uint32_t) cus_ * sc_wpc;
    // basic k >= 2: the S-side buffers first partition the R keys' k * |R| bit positions
    const bool     basic_kk = g.mode == MODE_SLICE_BASIC && g.k > 1;
    const uint64_t nRk      = basic_kk ? (uint64_t) g.k * nR : 0;
    // the north_star's bitmap broadcast (opt-in, hwbrj_set_filter_broadcast) makes this join a
    // collective: from here on a failure of this rank alone must not leave its peers waiting in
    // ncclBroadcast, so every return before the first kernel goes through one status agreement
    // (argument errors above fail alike on every rank)
    const bool bcast = bcast_ && comm_ && slice_mode && !basic_kk;
    auto pre = [&](int rc) -> int {
        if (!bcast || alloc_only_) return rc;
        return rccl_agree_status(comm_, comm_world_, comm_rank_, rc, stream, &agree_);
    };
    const uint64_t capR = region_cap(nR, G, F), capS = region_cap(std::max(nS, nRk), G, F);
    const uint64_t LR = (uint64_t) G * capR, LS = (uint64_t) G * capS;  // max chunks
    const uint64_t items_max = (LS / CH + F + 1) * nseg;
    // list entries hold a 27-bit chunk id (hwbrj_kernels.hip, K4); metas a 22-bit region offset
    if (G > 512) {
        set_last_error("more than 512 scatter workgroups (k_plan row groups)");
        return pre(3);
    }
    if (LS > (1ull << 27) || LR > (1ull << 27) || capS >= (1u << 22) || capR >= (1u << 22)) {
        set_last_error("relation too large for 27-bit chunk ids (|S| or |R| > ~4.2e9 tuples per GPU)");
        return pre(3);
    }
    if (mat && (capS >= (1u << 21) || capR >= (1u << 21))) {  // half indices (scatter_body_pay) < 2^22
        set_last_error("relation too large for the materializing scatter's 22-bit half indices");
        return pre(3);
    }
    const uint64_t GF = (uint64_t) G * F;
    bool ok = true;
    ok &= poolR.ensure(LR * 128) && metaR.ensure(LR * 2) && listR.ensure(LR * 4);
    ok &= usedR.ensure(G * 4) && wgqcR.ensure(GF * 4) && wgqeR.ensure(GF * 4) && wgqoR.ensure(GF * 4);
    ok &= lstartR.ensure((F + 1) * 4) && estartR.ensure((F + 1) * 8) && istartR.ensure((F + 1) * 4);
    ok &= poolS.ensure(LS * 128) && metaS.ensure(LS * 2) && listS.ensure(LS * 4);
    ok &= usedS.ensure(G * 4) && wgqcS.ensure(GF * 4) && wgqeS.ensure(GF * 4) && wgqoS.ensure(GF * 4);
    ok &= lstartS.ensure((F + 1) * 4) && estartS.ensure((F + 1) * 8) && istartS.ensure((F + 1) * 4);
    const uint64_t BSW = build_chunks_per_sweep(), SLOT = build_sweep_slot();
    const uint64_t sweeps_max = LR / BSW + F + 1;  // build sweeps over all R partitions
    ok &= rjoin.ensure(sweeps_max * SLOT * 4) && rrun.ensure(2 * sweeps_max * NSUB * 4);
    ok &= surv.ensure(nseg * LS * 128) && survcnt.ensure(items_max * NSUB * 4) &&
          survoff.ensure(items_max * NSUB * 4);
    ok &= jring_.ensure(kJoinRing * ring_slot_bytes()) && colR.ensure(F * 12) && colS.ensure(F * 12);  // u64 elems | u32 chunks
    // jparts: nparts [NJ] | job_surv [NJ] | nextra; jtask: extra parts {job, part}
    // (job_surv is left zero by k_join_split for the NJ jobs it saw: a join with another NJ
    // clears the whole buffer, so no stale count of an earlier job layout is read)
    const bool jnew = jparts.bytes < (size_t) (2 * NJ + 1) * 4 || NJ != last_nj_;
    last_nj_ = NJ;
    ok &= jtask.ensure((size_t) join_extra_tasks() * 8) && jparts.ensure((size_t) (2 * NJ + 1) * 4);
    if (slice_mode) ok &= slices.ensure((uint64_t) F * nseg * g.seg_words * 4);
    if (g.mode == MODE_GLOBAL) ok &= bitmap.ensure(((g.m + 31) / 32) * 4) && dense.ensure(nS * 4);
    if (basic_kk) ok &= bpos.ensure(nRk * 4);
    if (mat) {
        ok &= ppoolR.ensure(LR * 128) && ppoolS.ensure(LS * 128) && rpay.ensure(sweeps_max * SLOT * 4) &&
              survpos.ensure(nseg * LS * 128);
    }
    if (!ok) {
        set_last_error("hipMalloc failed (device memory)");
        return pre(4);
    }
    if (alloc_only_) return 0;
    if (const int rc = pre(0)) return rc;
    // this join's result slot (ring_take collects a full ring first)
    uint32_t  rslot      = 0;
    bool      rtimed     = false;  // (the S scatter's timing events, below)
    char*     sm         = (char*) ring_take(&rslot);
    if (!sm) return 1;
    uint64_t* d_result   = (uint64_t*) sm;      // [0] matches
    uint64_t* d_dcount   = (uint64_t*) sm + 1;  // [1] dense survivor count (global mode)
    uint64_t* d_filtered = (uint64_t*) sm + 2;  // [2] S-tuples after filter

    // zeroing (the reference callocs before its timer, :1583, :1601): the counts and the join's
    // extra-task count are zeroed by the R scatter's workgroup 0 (two memset dispatches less per
    // join); job_surv is left zero by every join's k_join_split, so it is cleared only when new
    if (jnew) HWBRJ_CHECK(hipMemsetAsync(jparts.p, 0, jparts.bytes, stream));
    if (g.mode == MODE_GLOBAL) HWBRJ_CHECK(hipMemsetAsync(bitmap.p, 0, bitmap.bytes, stream));

    ScatterParams sp{};
    sp.tabs = d_tabs_;
    sp.g    = g;
    sp.zero_small = (uint32_t*) sm;  // (the R scatter only: cleared below)
    sp.zero_word  = jparts.as<uint32_t>() + 2 * NJ;

    // S pass-1 and its lists (below; dev A/B HWBRJ_DEV_OVL: on a second stream, concurrent with
    // the R side)
    auto s_pass = [&](hipStream_t st, bool marks, hipEvent_t* tev = nullptr) -> int {
        ScatterParams ss = sp;
        ss.zero_small    = nullptr;
        ss.zero_word     = nullptr;
        if (g.mode == MODE_GLOBAL) {
            launch_probe_global(dS, nS, g, d_tabs_, bitmap.as<uint32_t>(), dense.as<uint32_t>(),
                                d_dcount, st);
            ss.src   = dense.p;
            ss.n     = nS;
            ss.n_dev = d_dcount;
        } else {
            ss.src   = dS;
            ss.n     = nS;
            ss.n_dev = nullptr;
        }
        ss.pool       = poolS.as<uint32_t>();
        ss.meta       = metaS.as<uint32_t>();
        ss.wg_used    = usedS.as<uint32_t>();
        ss.wgq_chunks = wgqcS.as<uint32_t>();
        ss.wgq_elems  = wgqeS.as<uint32_t>();
        ss.cap        = capS;
        if (dbg) {  // dev-only phase stamps (HWBRJ_DBG)
            if (!dbgS.ensure((size_t) G * 64)) {
                set_last_error("hipMalloc failed (device memory)");
                return 4;
            }
            HWBRJ_CHECK(hipMemsetAsync(dbgS.p, 0, dbgS.bytes, st));
            ss.dbg = dbgS.as<uint64_t>();
        }
        ss.ppool = mat ? ppoolS.as<uint32_t>() : nullptr;
        if (tev) HWBRJ_CHECK(hipEventRecord(tev[0], st));
        launch_scatter(ss, g.mode == MODE_GLOBAL ? SRC_CODES : SRC_TUPLES, SIDE_S, G, st);
        if (tev) HWBRJ_CHECK(hipEventRecord(tev[1], st));
        if (marks) HWBRJ_CHECK(mark(4, st));
        launch_plan(wgqcS.as<uint32_t>(), wgqeS.as<uint32_t>(), G, g.log2F, wgqoS.as<uint32_t>(),
                    colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), st);
        launch_list_fill(metaS.as<uint32_t>(), usedS.as<uint32_t>(), capS, g.log2F, wgqoS.as<uint32_t>(),
                         colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), CH, nseg, lstartS.as<uint32_t>(),
                         estartS.as<uint64_t>(), istartS.as<uint32_t>(), listS.as<uint32_t>(), G, st);
        if (marks) HWBRJ_CHECK(mark(5, st));
        return 0;
    };
    HWBRJ_CHECK(mark(0, stream));
    const bool ovl = (dev_knobs().ovl || (HWBRJ_OVL_ASYNC && !phase_ev_)) && g.mode != MODE_GLOBAL && !basic_kk &&
                     !mat && !bcast;
    if (ovl) {  // S pass on the side stream (with phase events, its phases would show inside the R side's)
        if (!ovl_stream_) {
            HWBRJ_CHECK(hipStreamCreateWithFlags(&ovl_stream_, hipStreamNonBlocking));
            HWBRJ_CHECK(hipEventCreateWithFlags(&ovl_ev_[0], hipEventDisableTiming));
            HWBRJ_CHECK(hipEventCreateWithFlags(&ovl_ev_[1], hipEventDisableTiming));
        }
        HWBRJ_CHECK(hipEventRecord(ovl_ev_[0], stream));
        HWBRJ_CHECK(hipStreamWaitEvent(ovl_stream_, ovl_ev_[0], 0));
        // (opt-in, hwbrj_set_async_timing: the S scatter bracketed by timing events on the side
        // stream, so the dominant kernel is timed in the schedule the back-to-back joins run)
        hipEvent_t* tev = nullptr;
        if (async_timing_) {
            for (int i = 0; i < 2; i++)
                if (!tev_[rslot][i]) HWBRJ_CHECK(hipEventCreateWithFlags(&tev_[rslot][i], hipEventDisableSystemFence));
            tev = tev_[rslot];
        }
        rtimed = tev != nullptr;
        if (const int rc = s_pass(ovl_stream_, false, tev)) return rc;
        HWBRJ_CHECK(hipEventRecord(ovl_ev_[1], ovl_stream_));
    }
    // The S pass runs first: then the filter slices (written by k_build) and the R pool (written by
    // k_scatter_r) are the most recent writes when k_probe and k_build read them, so the Infinity
    // Cache still holds much of them. Not in the global mode (the R scatter's workgroup 0 zeroes the
    // dense count the S pass's global probe adds to) nor for basic k >= 2 (the R side borrows the
    // S-side buffers).
    const bool s_first = !ovl && !dev_knobs().rfirst && g.mode != MODE_GLOBAL && !basic_kk;
    if (s_first)
        if (const int rc = s_pass(stream, true)) return rc;
    // ---------------------------------------------------------------- R: pass-1 (+ filter)
    if (g.mode == MODE_GLOBAL)
        launch_build_global(dR, nR, g, d_tabs_, bitmap.as<uint32_t>(), stream);
    sp.src        = dR;
    sp.n          = nR;
    sp.n_dev      = nullptr;
    sp.pool       = poolR.as<uint32_t>();
    sp.ppool      = mat ? ppoolR.as<uint32_t>() : nullptr;
    sp.meta       = metaR.as<uint32_t>();
    sp.wg_used    = usedR.as<uint32_t>();
    sp.wgq_chunks = wgqcR.as<uint32_t>();
    sp.wgq_elems  = wgqeR.as<uint32_t>();
    sp.cap        = capR;
    launch_scatter(sp, SRC_TUPLES, SIDE_R, G, stream);
    HWBRJ_CHECK(mark(1, stream));
    launch_plan(wgqcR.as<uint32_t>(), wgqeR.as<uint32_t>(), G, g.log2F, wgqoR.as<uint32_t>(),
                colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), stream);
    launch_list_fill(metaR.as<uint32_t>(), usedR.as<uint32_t>(), capR, g.log2F, wgqoR.as<uint32_t>(),
                     colR.as<uint32_t>() + 2 * F, colR.as<uint64_t>(), (uint32_t) BSW, 1, lstartR.as<uint32_t>(),
                     estartR.as<uint64_t>(), istartR.as<uint32_t>(), listR.as<uint32_t>(), G, stream);
    HWBRJ_CHECK(mark(2, stream));
    sp.ppool      = nullptr;
    sp.zero_small = nullptr;
    sp.zero_word  = nullptr;
    BuildParams bp{};
    bp.g          = g;
    bp.tabs       = d_tabs_;
    bp.pool       = poolR.as<uint32_t>();
    bp.list       = listR.as<uint32_t>();
    bp.list_start = lstartR.as<uint32_t>();
    bp.elem_start = estartR.as<uint64_t>();
    bp.slices     = slice_mode ? slices.as<uint32_t>() : nullptr;
    bp.sweep_start = istartR.as<uint32_t>();  // (R items = build sweeps)
    bp.out_codes   = rjoin.as<uint32_t>();
    bp.run_cnt     = rrun.as<uint32_t>();
    bp.run_off     = rrun.as<uint32_t>() + sweeps_max * NSUB;
    bp.ppool       = mat ? ppoolR.as<uint32_t>() : nullptr;
    bp.out_pay     = mat ? rpay.as<uint32_t>() : nullptr;
    // 3-byte join keys from build / probe to k_join, unless the last join this Engine waited for had
    // probe items too large for the stage (their 32-bit survivor runs make the join read two formats,
    // k_join_mixed): a performance hint only, both paths give the same counts
    const bool     pack3 = !mat && join_pack3(g) && pack3_hint_;
    const uint32_t kbits = pack3 ? join_key_bits(g) : 0u;  // 18 at the north star
    bp.kbits       = kbits;
    // the broadcast: rank 0 builds the slices, the other ranks only sub-partition R for the join
    // and receive them over RCCL (HWBRJ_HOOK_BCAST_NONROOT: this rank takes the non-root side, for
    // tests at world 1; value 2 zeroes the slices first, so the counts show whether k_build wrote any)
    const int nonroot_hook = bcast && comm_world_ == 1 ? test_hooks().bcast_nonroot : 0;  // (tests only: world 1)
    bp.no_slices = bcast && (comm_rank_ != 0 || nonroot_hook) ? 1u : 0u;
    if (nonroot_hook == 2) HWBRJ_CHECK(hipMemsetAsync(slices.p, 0, slices.bytes, stream));
    launch_build(bp, F, stream);
    if (bcast) {
        const int rc = rccl_broadcast(comm_, slices.p, (size_t) F * nseg * g.seg_words * 4, 0, stream);
        if (rc) {  // kernels of this join are enqueued: later joins must still order after them
            (void) hipEventRecord(ev_[8], stream);
            pending_        = true;
            pending_stream_ = stream;
            pending_rc_     = rc;
            pending_err_    = hwbrj_last_error();
            return rc;
        }
    }
    if (basic_kk) {
        // basic k >= 2: the k bit positions of every R key, partitioned by slice with the S-side
        // scatter buffers (free until the S pass), then one LDS slice build per partition
        launch_bitpos(dR, nR, g, bpos.as<uint32_t>(), stream);
        sp.src        = bpos.p;
        sp.n          = nRk;
        sp.n_dev      = nullptr;
        sp.pool       = poolS.as<uint32_t>();
        sp.meta       = metaS.as<uint32_t>();
        sp.wg_used    = usedS.as<uint32_t>();
        sp.wgq_chunks = wgqcS.as<uint32_t>();
        sp.wgq_elems  = wgqeS.as<uint32_t>();
        sp.cap        = capS;
        launch_scatter(sp, SRC_CODES, SIDE_R, G, stream);
        launch_plan(wgqcS.as<uint32_t>(), wgqeS.as<uint32_t>(), G, g.log2F, wgqoS.as<uint32_t>(),
                    colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), stream);
        launch_list_fill(metaS.as<uint32_t>(), usedS.as<uint32_t>(), capS, g.log2F, wgqoS.as<uint32_t>(),
                         colS.as<uint32_t>() + 2 * F, colS.as<uint64_t>(), (uint32_t) BSW, 1,
                         lstartS.as<uint32_t>(), estartS.as<uint64_t>(), istartS.as<uint32_t>(),
                         listS.as<uint32_t>(), G, stream);
        launch_slice_fill(poolS.as<uint32_t>(), listS.as<uint32_t>(), lstartS.as<uint32_t>(), g,
                          slices.as<uint32_t>(), stream);
    }
    HWBRJ_CHECK(mark(3, stream));
    // ---------------------------------------------------------------- S: pass-1 (+ probe)
    if (ovl) {
        HWBRJ_CHECK(hipStreamWaitEvent(stream, ovl_ev_[1], 0));
        HWBRJ_CHECK(mark(4, stream));
        HWBRJ_CHECK(mark(5, stream));
    } else if (!s_first) {
        if (const int rc = s_pass(stream, true)) return rc;
    }
    ProbeParams pp{};
    pp.g               = g;
    pp.tabs            = d_tabs_;
    pp.pool            = poolS.as<uint32_t>();
    pp.list            = listS.as<uint32_t>();
    pp.list_start      = lstartS.as<uint32_t>();
    pp.item_start      = istartS.as<uint32_t>();
    pp.slices          = slice_mode ? slices.as<uint32_t>() : nullptr;
    pp.surv            = surv.as<uint32_t>();
    pp.surv_seg_stride = LS * 32;
    pp.surv_cnt        = survcnt.as<uint32_t>();
    pp.surv_off        = survoff.as<uint32_t>();
    pp.filtered        = d_filtered;
    pp.job_surv        = jparts.as<uint32_t>() + NJ;
    pp.surv_pos        = mat ? survpos.as<uint32_t>() : nullptr;
    pp.kbits           = kbits;
    pp.fmt_cnt         = mat ? nullptr : (uint32_t*) sm + 10;  // (u64 word 5 of the slot: zeroed by the R scatter)
    const size_t   pl_lds = probe_lds_bytes(g, nullptr, mat != nullptr);
    const uint32_t PG = (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / pl_lds));
    const bool dbg_on = dbg;  // dev-only phase stamps (HWBRJ_DBG)
    if (dbg_on) {
        ok &= dbgP.ensure((size_t) std::max<uint32_t>(PG, F) * 64) && dbgJ.ensure((size_t) std::max<uint64_t>(F, 1024) * 64);
        HWBRJ_CHECK(hipMemsetAsync(dbgP.p, 0, dbgP.bytes, stream));
        HWBRJ_CHECK(hipMemsetAsync(dbgJ.p, 0, dbgJ.bytes, stream));
        pp.dbg = dbgP.as<uint64_t>();
    }
    launch_probe(pp, PG, stream);
    HWBRJ_CHECK(mark(6, stream));  // (survivor sub-partitioning is fused into k_probe: no ev_[7])
    surv_fused_ = true;
    // -------------------------------------------------------------------------- join
    JoinParams jp{};
    jp.r_codes         = rjoin.as<uint32_t>();
    jp.r_sweep_start   = istartR.as<uint32_t>();
    jp.r_cnt           = rrun.as<uint32_t>();
    jp.r_off           = rrun.as<uint32_t>() + sweeps_max * NSUB;
    jp.slot            = (uint32_t) SLOT;
    jp.surv            = surv.as<uint32_t>();
    jp.surv_cnt        = survcnt.as<uint32_t>();
    jp.surv_off        = survoff.as<uint32_t>();
    jp.item_start      = istartS.as<uint32_t>();
    jp.list_start      = lstartS.as<uint32_t>();
    jp.surv_seg_stride = LS * 32;
    jp.nseg            = nseg;
    jp.CH              = CH;
    jp.log2NSUB        = g.log2NSUB;
    jp.hash_shift      = g.hash_shift;
    jp.bitmap          = (g.sub_shift > 0 && 32 - g.hash_shift <= join_bitmap_log2()) ? 1u : 0u;
    jp.jsum            = (uint64_t*) (sm + 128);  // 64 partial sums, one per 128-B line
    jp.dbg             = dbg_on ? dbgJ.as<uint64_t>() : nullptr;
    jp.nparts          = jparts.as<uint32_t>();
    jp.extra           = jtask.as<uint2>();
    jp.nextra          = jparts.as<uint32_t>() + 2 * NJ;
    jp.jkind           = (uint32_t) jkind;
    jp.split_surv      = test_hooks().join_split;  // (tests: force the skew split)
    jp.r_kbits         = kbits;
    jp.fmt_cnt         = pp.fmt_cnt;
    jp.timing          = phase_ev_ ? 1u : 0u;  // (back-to-back joins: counts only)
    if (mat) {
        // (k_join_split, which leaves job_surv zero for the next join, does not run here)
        HWBRJ_CHECK(hipMemsetAsync(jparts.as<uint32_t>() + NJ, 0, (size_t) NJ * 4, stream));
        MatJoinParams mp{};
        mp.r_codes         = jp.r_codes;
        mp.r_pay           = rpay.as<uint32_t>();
        mp.r_sweep_start   = jp.r_sweep_start;
        mp.r_cnt           = jp.r_cnt;
        mp.r_off           = jp.r_off;
        mp.slot            = jp.slot;
        mp.surv            = jp.surv;
        mp.surv_pos        = survpos.as<uint32_t>();
        mp.surv_cnt        = jp.surv_cnt;
        mp.surv_off        = jp.surv_off;
        mp.item_start      = jp.item_start;
        mp.list_start      = jp.list_start;
        mp.surv_seg_stride = jp.surv_seg_stride;
        mp.nseg            = nseg;
        mp.CH              = CH;
        mp.log2NSUB        = g.log2NSUB;
        mp.hash_shift      = g.hash_shift;
        mp.bm              = (g.sub_shift > 0 && 32 - g.hash_shift <= 17) ? 1u : 0u;
        mp.s_pay           = ppoolS.as<uint32_t>();
        mp.out             = mat->out;
        mp.cap             = mat->cap;
        mp.count           = (unsigned long long*) d_result;
        launch_join_mat(mp, NJ, stream);
    } else {
        launch_join(jp, NJ, jparts.as<uint32_t>() + NJ, stream);
    }
    HWBRJ_CHECK(hipEventRecord(ev_[8], stream));
    HWBRJ_CHECK(hipGetLastError());
    pending_      = true;
    pending_rc_   = 0;
    pending_args_ = args != nullptr;
    pending_nS_   = nS;
    pending_ev_   = phase_ev_;
    pending_sfirst_ = s_first;
    pending_fmt_    = pp.fmt_cnt != nullptr;
    pending_slots_  = !mat;
    pending_stream_ = stream;
    have_filter_  = args != nullptr;
    last_g_       = g;
    {
        JoinRec r;
        r.slot  = rslot;
        r.args  = args != nullptr;
        r.fmt   = pending_fmt_;
        r.kbits = kbits;
        r.slots = !mat;
        r.timed = rtimed;
        r.nS    = nS;
        r.g     = g;
        ring_push(r);
    }

    if (dbg_on) {
        HWBRJ_CHECK(hipEventSynchronize(ev_[8]));
        std::vector<uint64_t> hp(PG * 8);
        HWBRJ_CHECK(hipMemcpy(hp.data(), dbgP.p, hp.size() * 8, hipMemcpyDeviceToHost));
        double sp_[6] = {0};
        for (uint32_t b = 0; b < PG; b++)
            for (int k = 0; k < 6; k++) sp_[k] += (double) hp[b * 8 + k] / PG;
        std::vector<uint64_t> hs(G * 8);
        HWBRJ_CHECK(hipMemcpy(hs.data(), dbgS.p, hs.size() * 8, hipMemcpyDeviceToHost));
        double ss[6] = {0};
        for (uint32_t b = 0; b < G; b++)
            for (int k = 0; k < 6; k++) ss[k] += (double) hs[b * 8 + k] / G;
        fprintf(stderr, "[dbg] S scatter cyc/WG: hash %.0f load+flush %.0f rank %.0f b1 %.0f write+plan %.0f b2 %.0f\n",
                ss[0], ss[1], ss[2], ss[3], ss[4], ss[5]);
        {  // workgroup start/end spread (100 MHz real-time clock): the kernel's tail
            uint64_t t0 = ~0ull;
            std::vector<double> st(G), en(G);
            for (uint32_t b = 0; b < G; b++) t0 = std::min<uint64_t>(t0, hs[b * 8 + 6]);
            for (uint32_t b = 0; b < G; b++) {
                st[b] = (hs[b * 8 + 6] - t0) / 100.0;
                en[b] = (hs[b * 8 + 7] - t0) / 100.0;
            }
            std::sort(st.begin(), st.end());
            std::sort(en.begin(), en.end());
            fprintf(stderr, "[dbg] S scatter WG start us: max %.1f | end us: min %.1f p10 %.1f p50 %.1f p90 %.1f max %.1f\n",
                    st[G - 1], en[0], en[G / 10], en[G / 2], en[G * 9 / 10], en[G - 1]);
        }
        fprintf(stderr, "[dbg] probe cyc/WG: top %.0f test %.0f b1 %.0f scan+b2 %.0f write %.0f b3+copy %.0f\n",
                sp_[0], sp_[1], sp_[2], sp_[3], sp_[4], sp_[5]);
        {  // k_join: workgroups summed into 1024 slots
            std::vector<uint64_t> hj2(1024 * 8);
            HWBRJ_CHECK(hipMemcpy(hj2.data(), dbgJ.p, hj2.size() * 8, hipMemcpyDeviceToHost));
            double sj2[6] = {0};
            const double nwg = (double) F * (1u << g.log2NSUB);
            for (uint32_t b = 0; b < 1024; b++)
                for (int k = 0; k < 6; k++) sj2[k] += (double) hj2[b * 8 + k] / nwg;
            fprintf(stderr, "[dbg] join cyc/WG (wave 0): desc %.0f R+sets %.0f popcnt %.0f surv1 %.0f surv2 %.0f end %.0f\n",
                    sj2[0], sj2[1], sj2[2], sj2[3], sj2[4], sj2[5]);
        }
    }
    return 0;
}

// Basic k >= 2. A key's k bits lie in k unrelated slices, so the S words are
// tested one bit per pass: pass j partitions the candidates by the slice of their bit j and tests
// it in LDS (k_probe_bitj), the passing words (dense) feed pass j + 1's scatter. The survivors of
// the last pass are re-partitioned by code (MODE_CODE_OF_KEY), the join's layout, so the join
// takes its bitmap path like the blocked filter's: R is partitioned by code for the join, and the
// slices are built from R's partitioned bit positions (k_bitpos, k_slice_fill).
int Engine::enqueue_basic_kk(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS,
                             const Geometry& g, hipStream_t stream, int jkind) {
    Geometry    gj;  // the join layout: R and the survivors partitioned by code
    std::string err;
    if (!plan_geometry(nullptr, nR, &gj, &err)) {
        set_last_error(err);
        return 2;
    }
    const uint32_t F = 1u << g.log2F, Fj = 1u << gj.log2F, Fm = std::max(F, Fj);
    const uint32_t NSUB = 1u << gj.log2NSUB, NJ = Fj * NSUB;
    const uint32_t nseg = g.nseg, CH = probe_chunks_per_item();
    // one workgroup per CU for every scatter and bit pass: pass j's workgroup w writes region w
    // (rw words) and pass j + 1's scatter workgroup w partitions it
    const uint32_t G    = (uint32_t) cus_;
    const uint64_t nRk  = (uint64_t) g.k * nR;
    const uint64_t Ib   = ((nS / 32 + (uint64_t) G * (Fm + 1)) / CH + Fm + 1) * nseg;  // items of a pass
    const uint64_t rw   = ((Ib + G - 1) / G) * CH * 32;  // words a pass workgroup may append
    const uint64_t capR = region_cap(nR, G, Fm);
    const uint64_t capS = std::max(region_cap(std::max(nS, nRk), G, Fm), rw / 32 + Fm + 1);
    const uint64_t LR = (uint64_t) G * capR, LS = (uint64_t) G * capS;
    const uint64_t items_max = (LS / CH + Fm + 1) * nseg;
    if (G > 512 || LS > (1ull << 27) || LR > (1ull << 27) || capS >= (1u << 22) || capR >= (1u << 22)) {
        set_last_error("relation too large for 27-bit chunk ids (|S| or |R| > ~4.2e9 tuples per GPU)");
        return 3;
    }
    const uint64_t GF = (uint64_t) G * Fm;
    bool ok = true;
    ok &= poolR.ensure(LR * 128) && metaR.ensure(LR * 2) && listR.ensure(LR * 4);
    ok &= usedR.ensure(G * 4) && wgqcR.ensure(GF * 4) && wgqeR.ensure(GF * 4) && wgqoR.ensure(GF * 4);
    ok &= lstartR.ensure((Fm + 1) * 4) && estartR.ensure((Fm + 1) * 8) && istartR.ensure((Fm + 1) * 4);
    ok &= poolS.ensure(LS * 128) && metaS.ensure(LS * 2) && listS.ensure(LS * 4);
    ok &= usedS.ensure(G * 4) && wgqcS.ensure(GF * 4) && wgqeS.ensure(GF * 4) && wgqoS.ensure(GF * 4);
    ok &= lstartS.ensure((Fm + 1) * 4) && estartS.ensure((Fm + 1) * 8) && istartS.ensure((Fm + 1) * 4);
    const uint64_t BSW = build_chunks_per_sweep(), SLOT = build_sweep_slot();
    const uint64_t sweeps_max = LR / BSW + Fm + 1;
    ok &= rjoin.ensure(sweeps_max * SLOT * 4) && rrun.ensure(2 * sweeps_max * NSUB * 4);
    ok &= surv.ensure(LS * 128) && survcnt.ensure(items_max * NSUB * 4) && survoff.ensure(items_max * NSUB * 4);
    ok &= jring_.ensure(kJoinRing * ring_slot_bytes()) && colR.ensure(Fm * 12) && colS.ensure(Fm * 12);
    const bool jnew = jparts.bytes < (size_t) (2 * NJ + 1) * 4 || NJ != last_nj_;
    last_nj_ = NJ;
    ok &= jtask.ensure((size_t) join_extra_tasks() * 8) && jparts.ensure((size_t) (2 * NJ + 1) * 4);
    ok &= slices.ensure((uint64_t) F * nseg * g.seg_words * 4) && (g.k <= G || bpos.ensure(nRk * 4));
    const uint32_t NC = (g.k + 64) & ~63u;  // pass counters [0, k - 1) + the dummy [NC - 1]
    ok &= dense.ensure(G * rw * 4) && dense2.ensure(G * rw * 4) && kkcnt.ensure(NC * 8 + 2 * G * 4);
    if (!ok) {
        set_last_error("hipMalloc failed (device memory)");
        return 4;
    }
    if (alloc_only_) return 0;
    uint32_t  rslot      = 0;
    char*     sm         = (char*) ring_take(&rslot);
    if (!sm) return 1;
    uint64_t* d_filtered = (uint64_t*) sm + 2;
    uint64_t* cnt        = kkcnt.as<uint64_t>();  // [j]: candidates after pass j (j < k - 1); [NC - 1]: dummy
    uint32_t* wgc[2]     = {(uint32_t*) (cnt + NC), (uint32_t*) (cnt + NC) + G};  // per-workgroup counts
    HWBRJ_CHECK(hipMemsetAsync(sm, 0, 64, stream));
    HWBRJ_CHECK(hipMemsetAsync(kkcnt.p, 0, kkcnt.bytes, stream));
    if (jnew) HWBRJ_CHECK(hipMemsetAsync(jparts.p, 0, jparts.bytes, stream));
    HWBRJ_CHECK(hipMemsetAsync(jparts.as<uint32_t>() + 2 * NJ, 0, 4, stream));

    auto side = [&](bool r) {
        ScatterParams sp{};
        sp.tabs       = d_tabs_;
        sp.pool       = (r ? poolR : poolS).as<uint32_t>();
        sp.meta       = (r ? metaR : metaS).as<uint32_t>();
        sp.wg_used    = (r ? usedR : usedS).as<uint32_t>();
        sp.wgq_chunks = (r ? wgqcR : wgqcS).as<uint32_t>();
        sp.wgq_elems  = (r ? wgqeR : wgqeS).as<uint32_t>();
        sp.cap        = r ? capR : capS;
        return sp;
    };
    auto index = [&](bool r, uint32_t log2F, uint32_t ch, uint32_t ns) {
        const uint32_t Fx = 1u << log2F;
        DevBuf& col = r ? colR : colS;
        launch_plan((r ? wgqcR : wgqcS).as<uint32_t>(), (r ? wgqeR : wgqeS).as<uint32_t>(), G, log2F,
                    (r ? wgqoR : wgqoS).as<uint32_t>(), col.as<uint32_t>() + 2 * Fx, col.as<uint64_t>(), stream);
        launch_list_fill((r ? metaR : metaS).as<uint32_t>(), (r ? usedR : usedS).as<uint32_t>(), r ? capR : capS,
                         log2F, (r ? wgqoR : wgqoS).as<uint32_t>(), col.as<uint32_t>() + 2 * Fx, col.as<uint64_t>(),
                         ch, ns, (r ? lstartR : lstartS).as<uint32_t>(), (r ? estartR : estartS).as<uint64_t>(),
                         (r ? istartR : istartS).as<uint32_t>(), (r ? listR : listS).as<uint32_t>(), G, stream);
    };

    HWBRJ_CHECK(mark(0, stream));
    // ---------------------------------------------------------------- R: the join layout
    ScatterParams sp = side(true);
    sp.g   = gj;
    sp.src = dR;
    sp.n   = nR;
    launch_scatter(sp, SRC_TUPLES, SIDE_R, G, stream);
    HWBRJ_CHECK(mark(1, stream));
    index(true, gj.log2F, (uint32_t) BSW, 1);
    HWBRJ_CHECK(mark(2, stream));
    BuildParams bp{};
    bp.g           = gj;
    bp.tabs        = d_tabs_;
    bp.pool        = poolR.as<uint32_t>();
    bp.list        = listR.as<uint32_t>();
    bp.list_start  = lstartR.as<uint32_t>();
    bp.elem_start  = estartR.as<uint64_t>();
    bp.sweep_start = istartR.as<uint32_t>();
    bp.out_codes   = rjoin.as<uint32_t>();
    bp.run_cnt     = rrun.as<uint32_t>();
    bp.run_off     = rrun.as<uint32_t>() + sweeps_max * NSUB;
    launch_build(bp, Fj, stream);
    // ---------------------------------------------------------------- the filter slices
    sp = side(false);
    if (g.k <= G) {  // R's k bit positions partitioned by slice straight from the tuples
        Geometry gp = g;
        gp.mode     = MODE_BASIC_POS;
        sp.g        = gp;
        sp.src      = dR;
        sp.n        = nRk;
        sp.vn       = nR;
        launch_scatter(sp, SRC_TUPLES, SIDE_R, G, stream);
    } else {
        launch_bitpos(dR, nR, g, bpos.as<uint32_t>(), stream);
        sp.g   = g;
        sp.src = bpos.p;
        sp.n   = nRk;
        launch_scatter(sp, SRC_CODES, SIDE_R, G, stream);
    }
    index(false, g.log2F, (uint32_t) BSW, 1);
    launch_slice_fill(poolS.as<uint32_t>(), listS.as<uint32_t>(), lstartS.as<uint32_t>(), g,
                      slices.as<uint32_t>(), stream);
    HWBRJ_CHECK(mark(3, stream));
    // ---------------------------------------------------------------- S: by the slice of bit 0
    sp     = side(false);
    sp.g   = g;
    sp.src = dS;
    sp.n   = nS;
    launch_scatter(sp, SRC_TUPLES, SIDE_S, G, stream);
    HWBRJ_CHECK(mark(4, stream));
    index(false, g.log2F, CH, nseg);
    HWBRJ_CHECK(mark(5, stream));
    // ---------------------------------------------------------------- one bit per pass
    const uint32_t PG = G;
    ProbeParams    pb{};
    pb.pool       = poolS.as<uint32_t>();
    pb.list       = listS.as<uint32_t>();
    pb.list_start = lstartS.as<uint32_t>();
    pb.item_start = istartS.as<uint32_t>();
    pb.slices     = slices.as<uint32_t>();
    uint32_t* dz[2] = {dense.as<uint32_t>(), dense2.as<uint32_t>()};
    for (uint32_t j = 0; j < g.k; j++) {
        Geometry gb = g;
        gb.bitj     = j;
        if (j > 0) {  // the candidates of pass j - 1, by the slice of bit j
            gb.mode       = MODE_BASIC_BITJ;
            sp            = side(false);
            sp.g          = gb;
            sp.src        = dz[(j - 1) & 1];
            sp.seg_cnt    = wgc[(j - 1) & 1];
            sp.seg_stride = rw;
            launch_scatter(sp, SRC_CODES, SIDE_S, G, stream);
            index(false, g.log2F, CH, nseg);
        }
        pb.g               = gb;
        pb.surv            = dz[j & 1];
        pb.surv_seg_stride = rw;
        pb.wg_cnt          = wgc[j & 1];
        pb.filtered        = j + 1 < g.k ? cnt + j : d_filtered;
        launch_probe_bitj(pb, PG, stream);
    }
    HWBRJ_CHECK(mark(6, stream));
    // ---------------------------------------------------------------- survivors: the join layout
    {
        Geometry gc = gj;
        gc.mode     = MODE_CODE_OF_KEY;
        sp          = side(false);
        sp.g        = gc;
        sp.src        = dz[(g.k - 1) & 1];
        sp.seg_cnt    = wgc[(g.k - 1) & 1];
        sp.seg_stride = rw;
        launch_scatter(sp, SRC_CODES, SIDE_S, G, stream);
        index(false, gj.log2F, CH, 1);
    }
    ProbeParams pp{};
    pp.g               = gj;
    pp.tabs            = d_tabs_;
    pp.pool            = poolS.as<uint32_t>();
    pp.list            = listS.as<uint32_t>();
    pp.list_start      = lstartS.as<uint32_t>();
    pp.item_start      = istartS.as<uint32_t>();
    pp.surv            = surv.as<uint32_t>();
    pp.surv_seg_stride = LS * 32;
    pp.surv_cnt        = survcnt.as<uint32_t>();
    pp.surv_off        = survoff.as<uint32_t>();
    pp.filtered        = cnt + NC - 1;  // (counted by the last bit pass)
    pp.job_surv        = jparts.as<uint32_t>() + NJ;
    const size_t   pl_lds = probe_lds_bytes(gj, nullptr);
    launch_probe(pp, (uint32_t) cus_ * (uint32_t) std::max<size_t>(1, std::min<size_t>(2, 163840 / pl_lds)), stream);
    HWBRJ_CHECK(mark(7, stream));
    surv_fused_ = false;
    // -------------------------------------------------------------------------- join
    JoinParams jp{};
    jp.r_codes         = rjoin.as<uint32_t>();
    jp.r_sweep_start   = istartR.as<uint32_t>();
    jp.r_cnt           = rrun.as<uint32_t>();
    jp.r_off           = rrun.as<uint32_t>() + sweeps_max * NSUB;
    jp.slot            = (uint32_t) SLOT;
    jp.surv            = surv.as<uint32_t>();
    jp.surv_cnt        = survcnt.as<uint32_t>();
    jp.surv_off        = survoff.as<uint32_t>();
    jp.item_start      = istartS.as<uint32_t>();
    jp.list_start      = lstartS.as<uint32_t>();
    jp.surv_seg_stride = LS * 32;
    jp.nseg            = 1;
    jp.CH              = CH;
    jp.log2NSUB        = gj.log2NSUB;
    jp.hash_shift      = gj.hash_shift;
    jp.bitmap          = (gj.sub_shift > 0 && 32 - gj.hash_shift <= join_bitmap_log2()) ? 1u : 0u;
    jp.jsum            = (uint64_t*) (sm + 128);
    jp.nparts          = jparts.as<uint32_t>();
    jp.extra           = jtask.as<uint2>();
    jp.nextra          = jparts.as<uint32_t>() + 2 * NJ;
    jp.jkind           = (uint32_t) jkind;
    jp.split_surv      = test_hooks().join_split;
    jp.timing          = phase_ev_ ? 1u : 0u;
    launch_join(jp, NJ, jparts.as<uint32_t>() + NJ, stream);
    HWBRJ_CHECK(hipEventRecord(ev_[8], stream));
    HWBRJ_CHECK(hipGetLastError());
    pending_      = true;
    pending_rc_   = 0;
    pending_args_ = true;
    pending_nS_   = nS;
    pending_ev_   = phase_ev_;
    pending_sfirst_ = false;
    pending_fmt_    = false;
    pending_slots_  = true;
    pending_stream_ = stream;
    have_filter_  = true;
    last_g_       = g;
    {
        JoinRec r;
        r.slot  = rslot;
        r.args  = true;
        r.slots = true;
        r.nS    = nS;
        r.g     = g;
        ring_push(r);
    }
    return 0;
}

int read_join_counts(const void* small, bool slots, hipStream_t stream, uint64_t h[6]) {
    const size_t          S = join_sum_slots(), W = join_sum_stride();
    std::vector<uint64_t> buf(16 + (slots ? S * W : 0));  // 128 bytes of result words, then the slots
    if (hipMemcpyAsync(buf.data(), small, buf.size() * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess) {
        set_last_error("reading the join's counts failed");
        return 1;
    }
    for (int i = 0; i < 6; i++) h[i] = buf[i];
    if (slots)
        for (size_t j = 0; j < S; j++) {
            h[0] += buf[16 + j * W];
            h[3] += buf[16 + j * W + 1];
            h[4] += buf[16 + j * W + 2];
        }
    return 0;
}

void* Engine::ring_take(uint32_t* slot) {
    if (jr_.size() >= (size_t) kJoinRing && ring_collect()) return nullptr;
    *slot    = jr_next_;
    jr_next_ = (jr_next_ + 1) % kJoinRing;
    return (char*) jring_.p + (size_t) *slot * ring_slot_bytes();
}

// The counts of every join in jr_ (all completed once ev_[8] has: they share the device's scratch,
// so each ran after the one before), read in one copy of the ring, appended to jdone_.
int Engine::ring_collect() {
    if (jr_.empty()) return 0;
    HWBRJ_CHECK(hipEventSynchronize(ev_[8]));
    const size_t          SB = ring_slot_bytes();
    std::vector<uint64_t> buf(kJoinRing * SB / 8);
    // the slots in use are consecutive mod kJoinRing: one copy of [first, last], or of the ring
    const uint32_t a = jr_.front().slot, z = jr_.back().slot;
    const size_t   off = a <= z ? (size_t) a * SB : 0, len = a <= z ? (size_t) (z - a + 1) * SB : kJoinRing * SB;
    HWBRJ_CHECK(hipMemcpy((char*) buf.data() + off, (char*) jring_.p + off, len, hipMemcpyDeviceToHost));
    const size_t S = join_sum_slots(), W = join_sum_stride();
    for (const JoinRec& r : jr_) {
        const uint64_t* b = buf.data() + (size_t) r.slot * (SB / 8);
        uint64_t        h[6];
        for (int i = 0; i < 6; i++) h[i] = b[i];
        if (r.slots)
            for (size_t j = 0; j < S; j++) {
                h[0] += b[16 + j * W];
                h[3] += b[16 + j * W + 1];
                h[4] += b[16 + j * W + 2];
            }
        if (r.fmt) pack3_hint_ = (uint32_t) h[5] == 0;  // (k_probe's count, ProbeParams::fmt_cnt)
        const Geometry& g = r.g;
        hwbrj_stats_t   st;
        memset(&st, 0, sizeof(st));
        st.filtered       = r.args ? h[2] : r.nS;
        st.matches        = (int64_t) h[0];
        st.mode           = g.mode;
        st.format         = g.s_format;
        st.partitions     = 1u << g.log2F;
        st.subparts       = 1u << g.log2NSUB;
        st.slice_segments = (g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC) ? g.nseg : 1;
        st.unstaged_items = r.fmt ? (uint32_t) h[5] : 0u;
        st.join_keys      = !r.kbits ? HWBRJ_JOIN_KEYS_32
                            : st.unstaged_items ? HWBRJ_JOIN_KEYS_MIXED : HWBRJ_JOIN_KEYS_PACKED;
        st.join_key_bits  = r.kbits ? r.kbits : 32u;
        // (probe / join ticks: the synchronous joins' phase split, added by wait())
        st.ms_join_probe  = (double) h[3];
        st.ms_join        = (double) h[4];
        if (r.timed) {  // the S scatter as the async schedule ran it (hwbrj_set_async_timing)
            float f = 0;
            HWBRJ_CHECK(hipEventElapsedTime(&f, tev_[r.slot][0], tev_[r.slot][1]));
            st.ms_s_scatter = f;
        }
        jdone_.push_back(st);
    }
    jr_.clear();
    return 0;
}

// Waits for the last join and collects every join since the last wait; the last one's phase times
// (synchronous joins) are read from its events.
static int wait_common(hwbrj_stats_t* last, bool phases, const hipEvent_t* ev, bool sfirst, bool surv_fused) {
    float ms[9] = {0, 0, 0, 0, (float) last->ms_s_scatter, 0, 0, 0, 0};  // (async: the timed S scatter only)
    if (phases) {  // (async joins: counts only)
        hipEvent_t e[9];
        for (int i = 0; i <= 8; i++) e[i] = ev[i];
        if (surv_fused) e[7] = ev[6];
        // phase i ends at boundary i and starts at boundary from[i] (S pass first: it starts the
        // join, the R scatter starts after the S lists, the probe after the build)
        static const int kFrom[2][9] = {{0, 0, 1, 2, 3, 4, 5, 6, 7}, {0, 5, 1, 2, 0, 4, 3, 6, 7}};
        const int* from = kFrom[sfirst ? 1 : 0];
        for (int i = 1; i <= 8; i++) HWBRJ_CHECK(hipEventElapsedTime(&ms[i], e[from[i]], e[i]));
        HWBRJ_CHECK(hipEventElapsedTime(&ms[0], e[0], e[8]));
    }
    const double pt = last->ms_join_probe, jt = last->ms_join;  // (ticks, ring_collect)
    last->ms_total      = ms[0];
    last->ms_r_scatter  = ms[1];
    last->ms_r_index    = ms[2];
    last->ms_build      = ms[3];
    last->ms_s_scatter  = ms[4];
    last->ms_s_index    = ms[5];
    last->ms_probe      = ms[6];
    last->ms_surv       = ms[7];
    last->ms_join       = ms[8];
    // the probe share of the join's workgroup time (k_join's wall_clock64 sections)
    last->ms_join_probe = jt > 0 ? ms[8] * pt / jt : 0.0;
    return 0;
}

int Engine::wait_all(hwbrj_stats_t* st, int cap, int* n) {
    HWBRJ_CHECK(hipSetDevice(device_));
    if (n) *n = 0;
    if (!pending_) {
        ring_drop();
        set_last_error("no join has been enqueued");
        return 6;
    }
    HWBRJ_CHECK(hipEventSynchronize(ev_[8]));
    if (pending_rc_) {  // the last join stopped after some of its kernels (a failed broadcast)
        ring_drop();
        set_last_error(pending_err_);
        return pending_rc_;
    }
    if (const int rc = ring_collect()) return rc;
    for (size_t i = 0; i < jdone_.size(); i++) {  // ticks -> ms (only the last has phase times)
        if (i + 1 == jdone_.size()) {
            if (const int rc = wait_common(&jdone_[i], pending_ev_, ev_, pending_sfirst_, surv_fused_)) return rc;
        } else {
            jdone_[i].ms_join_probe = jdone_[i].ms_join = 0;  // (the ticks: not phase times)
        }
    }
    const size_t tot = jdone_.size();
    if (tot) last_st_ = jdone_.back();
    if (n) *n = (int) tot;
    if (st)
        for (size_t i = 0; i < tot && (int) i < cap; i++) st[i] = jdone_[i];
    jdone_.clear();
    if (st && (size_t) cap < tot) {
        set_last_error("more joins than the stats array holds (the oldest were written)");
        return 7;
    }
    return 0;
}

int Engine::wait(hwbrj_stats_t* st) {
    HWBRJ_CHECK(hipSetDevice(device_));
    if (!pending_) {
        ring_drop();
        set_last_error("no join has been enqueued");
        return 6;
    }
    HWBRJ_CHECK(hipEventSynchronize(ev_[8]));
    if (pending_rc_) {  // the last join stopped after some of its kernels (a failed broadcast)
        ring_drop();
        set_last_error(pending_err_);
        return pending_rc_;
    }
    if (const int rc = ring_collect()) return rc;
    if (!jdone_.empty()) {  // (else: the last join was collected before; its stats again)
        last_st_ = jdone_.back();
        jdone_.clear();
        if (const int rc = wait_common(&last_st_, pending_ev_, ev_, pending_sfirst_, surv_fused_)) return rc;
    }
    if (st) *st = last_st_;
    return 0;
}

int Engine::export_filter(uint8_t* host_out, uint64_t nbytes) {
    HWBRJ_CHECK(hipSetDevice(device_));
    if (!have_filter_) {
        set_last_error("no filter has been built");
        return 5;
    }
    const Geometry& g = last_g_;
    if (nbytes != g.m / 8) {
        set_last_error("nbytes must equal m/8");
        return 6;
    }
    if (g.mode == MODE_GLOBAL) {
        HWBRJ_CHECK(hipMemcpy(host_out, bitmap.p, nbytes, hipMemcpyDeviceToHost));
        return 0;
    }
    const uint64_t nwords = (g.m + 31) / 32;
    DevBuf tmp;
    if (!tmp.ensure(nwords * 4)) {
        set_last_error("hipMalloc failed");
        return 4;
    }
    launch_export(slices.as<uint32_t>(), g, tmp.as<uint32_t>(), nwords, own_stream_);
    HWBRJ_CHECK(hipStreamSynchronize(own_stream_));
    HWBRJ_CHECK(hipMemcpy(host_out, tmp.p, nbytes, hipMemcpyDeviceToHost));
    tmp.release();
    return 0;
}

int Engine::materialize(const uint2* dR, uint64_t nR, const uint2* dS, uint64_t nS, uint2* out,
                        uint64_t cap, uint64_t* n, hipStream_t stream, double* ms) {
    HWBRJ_CHECK(hipSetDevice(device_));
    if (!stream) stream = own_stream_;
    uint64_t T = 2;
    while (T < 2 * nR) T <<= 1;
    if (!mtab.ensure(T * 8) || !mcount.ensure(8)) {
        set_last_error("hipMalloc failed (materialization table)");
        return 4;
    }
    HWBRJ_CHECK(hipMemsetAsync(mtab.p, 0, T * 8, stream));
    HWBRJ_CHECK(hipMemsetAsync(mcount.p, 0, 8, stream));
    HWBRJ_CHECK(hipEventRecord(ev_[0], stream));
    if (nR) launch_mat_build(dR, nR, mtab.as<unsigned long long>(), T - 1, stream);
    if (nR && nS) {
        Geometry g = last_g_;  // the counting join's filter (materialize follows it)
        if (!have_filter_) g.mode = MODE_NOBLOOM;
        launch_mat_probe(dS, nS, dR, mtab.as<unsigned long long>(), T - 1, out, cap,
                         mcount.as<unsigned long long>(), g, slices.as<uint32_t>(),
                         bitmap.as<uint32_t>(), d_tabs_, stream);
    }
    HWBRJ_CHECK(hipEventRecord(ev_[8], stream));
    HWBRJ_CHECK(hipGetLastError());
    HWBRJ_CHECK(hipEventSynchronize(ev_[8]));
    HWBRJ_CHECK(hipMemcpy(n, mcount.p, 8, hipMemcpyDeviceToHost));
    if (ms) {
        float f = 0;
        HWBRJ_CHECK(hipEventElapsedTime(&f, ev_[0], ev_[8]));
        *ms = f;
    }
    return 0;
}

int Engine::generate(uint2* d_out, uint64_t n, uint64_t offset, uint64_t count, uint32_t nthreads,
                     uint64_t maxid, uint64_t threshold, double selectivity, uint64_t seed,
                     hipStream_t stream) {
    HWBRJ_CHECK(hipSetDevice(device_));
    std::vector<GenPlan> plan(1);
    if (make_gen_plan(&plan[0], n, nthreads, maxid, threshold, selectivity)) {
        set_last_error("invalid generator parameters");
        return 2;
    }
    if (!stream) stream = own_stream_;
    HWBRJ_CHECK(hipMemcpyAsync(d_plan_, plan.data(), sizeof(GenPlan), hipMemcpyHostToDevice, stream));
    if (offset > n || count > n - offset) {
        set_last_error("generator range outside the relation");
        return 2;
    }
    launch_gen(d_out, offset, count, d_plan_, make_perm(n, seed), stream);
    HWBRJ_CHECK(hipGetLastError());
    HWBRJ_CHECK(hipStreamSynchronize(stream));
    return 0;
}

// ----------------------------------------------------------------- per-device singletons
static std::mutex g_mu;
static Engine*    g_engines[64] = {};

Engine* engine_for_current_device() {
    int        dev = 0;
    hipError_t e   = hipGetDevice(&dev);
    if (e != hipSuccess) {  // a runtime not yet initialised in this library's HIP instance
        (void) hipInit(0);
        e = hipGetDevice(&dev);
    }
    if (e != hipSuccess || dev < 0 || dev >= 64) {
        set_last_error(std::string("no HIP device (hipGetDevice: ") + hipGetErrorString(e) + ")");
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_engines[dev]) g_engines[dev] = new Engine(dev);
    return g_engines[dev];
}

}  // namespace hwbrj
