// hwbrj_kernels.h -- kernel parameter blocks and launch wrappers (internal C++ interface between
// the HIP kernels and the host engine in hwbrj_engine.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <stddef.h>
#include <stdint.h>

#include "hwbrj_common.h"

namespace hwbrj {

enum Source : int { SRC_TUPLES = 0, SRC_CODES = 1 };

struct ScatterParams {
    const void*      src;          // uint2 tuples {key, payload} or uint32 codes
    uint64_t         n;            // element count (ignored when n_dev != nullptr)
    const uint64_t*  n_dev;        // optional device-resident element count
    uint32_t*        pool;         // [G * cap][32] chunk words
    uint32_t*        ppool;        // [G * cap][32] the words' payloads (materialization), or nullptr
    uint32_t*        meta;         // [G * cap] 16-bit entries (meta16): partition | (count - 1) << 10
    uint32_t*        wg_used;      // [G] chunks used by each workgroup
    uint32_t*        wgq_chunks;   // [G][F] chunks of partition q in workgroup wg's region
    uint32_t*        wgq_elems;    // [G][F] elements of partition q in workgroup wg's region
    uint64_t*        dbg;          // dev-only: per-workgroup phase cycles (HWBRJ_DBG), or nullptr
    uint64_t         cap;          // chunk capacity of one workgroup region
    const uint32_t*  seg_cnt;      // SRC_CODES from per-workgroup segments: workgroup w partitions
    uint64_t         seg_stride;   // src + w * seg_stride (elements), seg_cnt[w] of them; or nullptr
    uint64_t         vn;           // MODE_BASIC_POS: tuples of src (n = k * vn elements, k <= grid)
    // the join's per-call zeroing, done by workgroup 0 instead of memset dispatches: zero_small[0, 16)
    // (counts) and *zero_word (the join's extra-task count), each when not nullptr
    uint32_t*        zero_small;
    uint32_t*        zero_word;
    Geometry         g;
    const CrcTables* tabs;
};

// Packed join keys between the build / probe and the join (BuildParams::kbits): on when the join
// key v = code >> hash_shift fits 24 bits and the run formats are private to k_join (not the
// materializing join, which reads codes, nor the partitioned join, which ships survivor words).
// Keys are a bit stream of kbits-bit fields: 18 bits when hash_shift = 14 (the bitmap path's keys,
// every north-star job: 16 keys per 9 dwords), else 24 (4 keys per 12 bytes); 0 = 32-bit codes.
#ifndef HWBRJ_PACK3
#define HWBRJ_PACK3 1
#endif
#ifndef HWBRJ_PACK18
#define HWBRJ_PACK18 1  // 0: 24-bit keys for the hash_shift = 14 launches too (A/B)
#endif
inline bool join_pack3(const Geometry& g) { return HWBRJ_PACK3 != 0 && g.sub_shift > 0 && g.hash_shift >= 8; }
inline uint32_t join_key_bits(const Geometry& g) {
    return !join_pack3(g) ? 0u : (HWBRJ_PACK18 && g.hash_shift == 14) ? 18u : 24u;
}

// Joins enqueued without phase events (hwbrj_join_device_async: the timed back-to-back joins) run
// their S pass on a second stream beside the R side, joined before the probe (A/B: 0 = one stream,
// S pass first). Synchronous joins keep one stream, so their phase times stay separate.
#ifndef HWBRJ_OVL_ASYNC
#define HWBRJ_OVL_ASYNC 1
#endif
#ifndef HWBRJ_PJ_OVL
#define HWBRJ_PJ_OVL 1  // async partitioned joins: the S shard's partitioning on a second stream
#endif

struct BuildParams {
    Geometry         g;
    const CrcTables* tabs;
    const uint32_t*  pool;
    const uint32_t*  list;        // chunk lists (entry = chunk id | count << 27)
    const uint32_t*  list_start;  // [F + 1]
    const uint64_t*  elem_start;  // [F + 1]
    uint32_t*        slices;      // [F][nseg][seg_words]
    const uint32_t*  sweep_start; // [F + 1] first build sweep of each partition
    uint32_t*        out_codes;   // [sweeps][kBSlot]: each sweep's R codes sorted by sub
    uint32_t*        run_cnt;     // [sweeps][NSUB] codes of each (sweep, sub) run
    uint32_t*        run_off;     // [sweeps][NSUB] run offset inside the sweep's slot
    uint32_t         q_base;      // partition of workgroup 0 (list/sweep tables indexed from it)
    const uint32_t*  ppool;       // payloads of pool's words (materialization), or nullptr
    uint32_t*        out_pay;     // [sweeps][kBSlot]: the payloads of out_codes (ppool set)
    uint32_t         no_slices;   // 1: join runs only (the slices arrive by broadcast from rank 0)
    uint32_t         kbits;       // 18 / 24: out_codes hold the slot's keys (code >> hash_shift) as a
                                  // stream of kbits-bit fields from its byte 0 (join_key_bits; not
                                  // PAY); 0: 32-bit codes
};

struct ProbeParams {
    Geometry         g;
    const CrcTables* tabs;
    const uint32_t*  pool;
    const uint32_t*  list;        // chunk lists (entry = chunk id | count << 27)
    const uint32_t*  list_start;  // [F + 1]
    const uint32_t*  item_start;  // [F + 1]
    const uint32_t*  slices;
    uint32_t*        surv;        // item region at (seg * surv_seg_stride + list_pos * 32), by sub
    uint64_t         surv_seg_stride;
    uint32_t*        surv_cnt;    // [items][NSUB] survivors of each (item, sub) run
    uint32_t*        surv_off;    // [items][NSUB] run offset inside the item region
    uint64_t*        filtered;    // += survivors ("S-tuples after filter")
    uint32_t*        job_surv;    // [F * NSUB] += survivors of each join job (zero on entry)
    uint32_t         stage_cap;   // survivor stage words (set by launch_probe)
    uint32_t*        surv_pos;    // materialization: each survivor's chunk position (its payload's
                                  // index in the S payload pool), parallel to surv; or nullptr
    uint32_t*        wg_cnt;      // k_probe_bitj: words appended to workgroup w's region
                                  // (surv + w * surv_seg_stride)
    uint64_t*        dbg;         // dev-only: per-workgroup phase cycles (HWBRJ_DBG), or nullptr
    uint32_t         kbits;       // 18 / 24: staged items store their join keys (code >> hash_shift)
                                  // as a stream of kbits-bit fields from the item region's byte 0,
                                  // flagged by bit 31 of their surv_off entries (unstaged items keep
                                  // 32-bit codes); 0: 32-bit codes
    uint32_t*        fmt_cnt;     // kbits: += the unstaged items (zeroed by the R scatter), or nullptr
};

struct JoinParams {
    const uint32_t* r_codes;      // build sweep slots (BuildParams::out_codes)
    const uint32_t* r_sweep_start;  // [F + 1]
    const uint32_t* r_cnt;        // [sweeps][NSUB]
    const uint32_t* r_off;        // [sweeps][NSUB]
    const uint32_t* surv;         // survivor runs written by k_probe
    const uint32_t* surv_cnt;
    const uint32_t* surv_off;
    const uint32_t* item_start;   // S items [F + 1]
    const uint32_t* list_start;   // S lists [F + 1]
    uint64_t        surv_seg_stride;
    uint32_t        nseg, CH, log2NSUB, hash_shift;
    uint32_t        slot;         // r_codes words per build sweep
    uint32_t        bitmap;       // 1: keys fit the direct-address bitmap (32 - hash_shift <= 18)
    uint64_t*       jsum;         // kJoinSumSlots partial sums, one per 128-byte line (zeroed by
                                  // k_join_split, summed by the host)
    uint32_t        jobs;         // F * NSUB (set by launch_join)
    uint32_t*       nparts;       // [jobs] parts of each job (k_join_split)
    uint2*          extra;        // [join_extra_tasks()] {job, part} of the further parts
    uint32_t*       nextra;       // parts requested beyond part 0 (zeroed before the join)
    uint32_t        split_surv;   // survivors per join part (0: the default, kJoinTaskSurv)
    uint64_t*       dbg;          // dev-only: per-workgroup phase cycles (HWBRJ_DBG), or nullptr
    uint32_t        jkind;        // per-partition join: 0 bucket chaining's role (bitmap / hash
                                  // table, PRO), 1 histogram join (PRH), 2 + 16-byte compares (PRHO)
    const uint64_t* item_base;    // [items] survivor region of each item (partitioned multi-GPU
                                  // join: received runs), or nullptr (k_probe's item regions)
    uint32_t        r_kbits;      // 18 / 24: r_codes hold packed join keys (BuildParams::kbits), and so
                                  // do the survivor runs flagged by bit 31 of surv_off; 0: codes
    const uint32_t* fmt_cnt;      // ProbeParams::fmt_cnt (the launch's survivor-run formats), or nullptr
    uint32_t        timing;       // 1: accumulate the probe / total ticks (result[3], result[4]) for
                                  // ms_join_probe (synchronous joins; 0: one count add per workgroup)
};

// The materializing join (k_join_mat): R codes + payloads of the build sweeps, survivors + their
// chunk positions, {R.payload, S.payload} pairs appended to out (up to cap; count = all pairs).
struct MatJoinParams {
    const uint32_t* r_codes;
    const uint32_t* r_pay;          // BuildParams::out_pay
    const uint32_t* r_sweep_start;  // [F + 1]
    const uint32_t* r_cnt;
    const uint32_t* r_off;
    uint32_t        slot;
    const uint32_t* surv;
    const uint32_t* surv_pos;       // ProbeParams::surv_pos
    const uint32_t* surv_cnt;
    const uint32_t* surv_off;
    const uint32_t* item_start;
    const uint32_t* list_start;
    uint64_t        surv_seg_stride;
    uint32_t        nseg, CH, log2NSUB, hash_shift;
    uint32_t        bm;             // 1: job keys v = code >> hash_shift < 2^17 (the bitmap path)
    uint32_t        xcd8;           // 1: XCD-aware job order (F a multiple of 8; set by launch_join_mat)
    const uint32_t* s_pay;          // S payload pool (ScatterParams::ppool of the S pass)
    uint2*          out;
    uint64_t        cap;
    unsigned long long* count;      // += pairs (zero on entry)
};

void   launch_gen(uint2* out, uint64_t offset, uint64_t count, const GenPlan* d_plan, const Perm& perm,
                  hipStream_t st);
void   launch_zipf(const int32_t* rnd, uint64_t cnt, uint64_t row0, const double* lut,
                   const uint32_t* alphabet, uint32_t size, uint2* out, uint64_t n_above,
                   uint32_t above_base, const Perm& perm, hipStream_t st);
void   launch_build_global(const uint2* R, uint64_t n, const Geometry& g, const CrcTables* tabs,
                           uint32_t* bm, hipStream_t st);
void   launch_probe_global(const uint2* S, uint64_t n, const Geometry& g, const CrcTables* tabs,
                           const uint32_t* bm, uint32_t* out, uint64_t* out_count, hipStream_t st);
// basic k >= 2: every R key's k bit positions (element j * n + i), then the slices from their
// partitioned chunk lists
void   launch_bitpos(const uint2* R, uint64_t n, const Geometry& g, uint32_t* out, hipStream_t st);
void   launch_slice_fill(const uint32_t* pool, const uint32_t* list, const uint32_t* list_start,
                         const Geometry& g, uint32_t* slices, hipStream_t st);
size_t scatter_lds_bytes(uint32_t log2F);
size_t scatter_pay_lds_bytes(uint32_t log2F);  // (ScatterParams::ppool set)
enum { SIDE_R = 0, SIDE_S = 1 };  // which relation a scatter partitions (kernel name; S uses g.s_format)
void   launch_scatter(const ScatterParams& p, int src, int side, uint32_t grid, hipStream_t st);
// k_plan: per-(wg, q) list offsets + per-partition chunk / element totals (colc, cole);
// k_list_fill: scans the totals into list / element / item starts [F + 1] and fills the lists.
void   launch_list_fill(const uint32_t* meta, const uint32_t* wg_used, uint64_t cap,
                        uint32_t log2F, const uint32_t* wgq_off, const uint32_t* colc,
                        const uint64_t* cole, uint32_t CH, uint32_t nseg, uint32_t* list_start,
                        uint64_t* elem_start, uint32_t* item_start, uint32_t* list, uint32_t grid,
                        hipStream_t st);
bool   launch_plan(const uint32_t* wgq_chunks, const uint32_t* wgq_elems, uint32_t G,
                   uint32_t log2F, uint32_t* wgq_off, uint32_t* colc, uint64_t* cole,
                   hipStream_t st);
uint32_t probe_chunks_per_item();
size_t   probe_lds_bytes(const Geometry& g, uint32_t* stage_cap, bool pay = false);
size_t slice_lds_bytes(const Geometry& g);
uint32_t build_chunks_per_sweep();  // R chunks per k_build sweep
uint32_t build_sweep_slot();        // out_codes words per k_build sweep
void   launch_build(const BuildParams& p, uint32_t F, hipStream_t st);
void   launch_probe(const ProbeParams& p, uint32_t grid, hipStream_t st);
// basic k >= 2 (k_probe_bitj): bit g.bitj of the words partitioned by its slice, passing words
// appended densely to p.surv; p.filtered += their count
size_t probe_bitj_lds_bytes(const Geometry& g);
void   launch_probe_bitj(const ProbeParams& p, uint32_t grid, hipStream_t st);
// splits skewed jobs (job_surv: survivors per job from k_probe, cleared here) and runs the join
void   launch_join(const JoinParams& p, uint32_t jobs, uint32_t* job_surv, hipStream_t st);
uint32_t join_extra_tasks();
// k_join's partial sums (JoinParams::jsum): join_sum_slots() slots of join_sum_stride() u64 words,
// word 0 matches, 1 probe ticks, 2 total ticks (P.timing); the host adds them up
uint32_t join_sum_slots();
uint32_t join_sum_stride();
uint32_t join_bitmap_log2();  // k_join's bitmap path: job keys v < 2^join_bitmap_log2()
void   launch_join_mat(const MatJoinParams& p, uint32_t jobs, hipStream_t st);
// result materialization (K12): R table build, S probe writing (R.payload, S.payload) pairs
void   launch_mat_build(const uint2* R, uint64_t n, unsigned long long* tab, uint64_t mask,
                        hipStream_t st);
// g/slices/bm/tabs: the last join's filter, used as a pre-test (g.mode = MODE_NOBLOOM: none)
void   launch_mat_probe(const uint2* S, uint64_t n, const uint2* R, const unsigned long long* tab,
                        uint64_t mask, uint2* out, uint64_t cap, unsigned long long* count,
                        const Geometry& g, const uint32_t* slices, const uint32_t* bm,
                        const CrcTables* tabs, hipStream_t st);
// partitioned multi-GPU join (K13): chunks in list order + rebased entries; receiver lists;
// survivor runs of items packed per destination
// partitioned join, device-side item tables: probe items -> region, survivor totals, their
// exclusive scan sofs [I + 1] and sofs at every partition's first item (bound [F + 1]); received
// items -> exclusive scan of their totals (wscan [n + 1]); the owner's join tables per
// (owned partition, source) pair (tab: first received item, items, first output item)
void   launch_pj_items(const uint32_t* item_start, const uint32_t* list_start, const uint32_t* cnt,
                       uint32_t items_max, uint32_t F, uint32_t nseg, uint32_t CH, uint64_t seg_words, uint32_t NSUB,
                       uint64_t* region, uint32_t* tot, uint64_t* bsum, uint64_t* sofs, uint64_t* bound,
                       hipStream_t st);
// (BI > 0: the async join's padded blocks of BI items / BW words per source, ritems[j] valid items)
void   launch_pj_recv_scan(const uint32_t* cnt, uint32_t n, uint32_t NSUB, uint32_t* tot, uint64_t* bsum,
                           uint64_t* wscan, hipStream_t st, uint32_t BI = 0, const uint32_t* ritems = nullptr);
void   launch_pj_item_tables(const uint32_t* tab, uint32_t pairs, uint32_t W, const uint32_t* rcnt,
                             const uint64_t* wscan, uint32_t NSUB, uint64_t* ibase, uint32_t* icnt, uint32_t* ioff,
                             uint32_t* jobs, hipStream_t st, uint32_t BI = 0, uint64_t BW = 0);
// the async partitioned join's fixed exchange blocks (hwbrj_pjoin_async.cpp; k_pjx_*): R chunks
// gathered into blocks of BR per destination, the owner's R tables from the received counts, the
// survivors packed into blocks of BI items / BW words, the owner's survivor tables, and the exchange
// sizes of the join for the next plan ({flag, R block, item block, word block} maxima)
// (own >= 0: this rank's own block written straight into the receive buffers own_out / own_ent)
void   launch_pjx_gather(const uint32_t* pool, const uint32_t* list, const uint32_t* lstart, uint32_t F, uint32_t QL,
                         uint32_t W, uint64_t BR, void* out, uint32_t* ent, int own, void* own_out, uint32_t* own_ent,
                         uint64_t* flag, hipStream_t st);
void   launch_pjx_rtab(const uint64_t* rc, uint32_t W, uint32_t QL, uint32_t NC, uint64_t BR, uint32_t bsw,
                       int64_t* tab, uint32_t* lsO, uint32_t* swO, uint64_t* flag, hipStream_t st);
void   launch_pjx_surv_pack(const uint32_t* surv, const uint64_t* region, const uint32_t* tot, const uint64_t* sofs,
                            const uint32_t* item_start, const uint64_t* bound, const uint32_t* cnt, uint32_t F,
                            uint32_t QL, uint32_t NSUB, uint64_t BI, uint64_t BW, uint32_t* out, uint32_t* out_cnt,
                            int own, uint32_t* own_out, uint32_t* own_cnt, uint64_t* flag, hipStream_t st);
void   launch_pjx_stab(const uint64_t* rc, uint32_t W, uint32_t QL, uint32_t NC, uint64_t BI, uint64_t BW,
                       uint32_t* tab2, uint32_t* istart, uint32_t* ritems, uint64_t* flag, hipStream_t st);
void   launch_pjx_stat(const uint64_t* rc1, const uint64_t* rc2, const uint32_t* ls, const uint32_t* is,
                       const uint64_t* bd, uint32_t W, uint32_t QL, uint32_t NC, const uint64_t* flag, uint64_t* out,
                       hipStream_t st);
// The synchronous partitioned join's own block (this rank to itself) written straight into the
// receive buffers: elements in [lo, hi) go to out / ent at index + delta (lo = hi: none).
struct PjOwn {
    uint32_t  lo = 0, hi = 0;
    int64_t   delta = 0;
    void*     out = nullptr;
    uint32_t* ent = nullptr;
};
void   launch_pj_gather(const uint32_t* pool, const uint32_t* list, uint32_t n, void* out, uint32_t* ent,
                        hipStream_t st, const PjOwn& own = PjOwn{});
// the native transport's per-destination counts message (k_pj_counts), built on the device
void   launch_pj_counts(const uint32_t* starts, const uint64_t* bound, uint32_t W, uint32_t QL, uint32_t NC,
                        uint64_t status, uint64_t extra, uint64_t extra2, uint64_t* out, hipStream_t st);
void   launch_pj_relist(const uint32_t* rent, const int64_t* tab, uint32_t pairs, uint32_t* list,
                        hipStream_t st);
void   launch_pj_surv_pack(const uint32_t* surv, const uint64_t* region, const uint32_t* tot,
                           const uint64_t* soff, uint32_t n, uint32_t* out, hipStream_t st,
                           const PjOwn& own = PjOwn{});
void   launch_export(const uint32_t* slices, const Geometry& g, uint32_t* out, uint64_t nwords,
                     hipStream_t st);
// a streaming copy of bytes (multiple of 16) from src to dst, grid workgroups of contiguous ranges
// (hwbrj_copy_bandwidth)
void   launch_copy_bw(const void* src, void* dst, uint64_t bytes, int grid, hipStream_t st);

// every compile-time switch of hwbrj_kernels.hip that differs from the product default ("" for the
// product build); hwbrj_version() appends it
const char* kernel_build_knobs();

// Dev-only runtime switches (A/B experiments of measured alternatives), read from the HWBRJ_DEV_*
// environment once, at the first Engine's construction, and only in builds with -DHWBRJ_DEV_BUILD:
// a product build ignores the environment, so no stray variable changes its path.
struct DevKnobs {
    bool     kk1 = false;        // HWBRJ_DEV_KK1: basic k = 1 on the bit-pass pipeline
    bool     kk_gather = false;  // HWBRJ_DEV_KK_GATHER: basic k >= 2 by global-slice gathers
    bool     noxcd = false;      // HWBRJ_DEV_NOXCD: k_join_mat without XCD-aware job order
    bool     dbg = false;        // HWBRJ_DBG: in-kernel phase stamps (a -DHWBRJ_STAMPS build)
    uint32_t maxf = 0;           // HWBRJ_DEV_MAXF: cap on the partition count F
    uint32_t scwpc = 0;          // HWBRJ_DEV_SCWPC: scatter workgroups per CU
    int      evflags = -1;       // HWBRJ_DEV_EVFLAGS: phase-event creation flags
    uint32_t l2sub = 0;          // HWBRJ_DEV_L2SUB: join sub-partition bits (code-digit joins)
    bool     ovl   = false;      // HWBRJ_DEV_OVL: S pass on a second stream beside the R side
    bool     rfirst = false;     // HWBRJ_DEV_RFIRST: R side before the S pass (the round-3 order)
};
const DevKnobs& dev_knobs();
// "name=value" of every dev knob that is set ("" in product builds); hwbrj_version() appends it
std::string dev_knobs_string();

// Test hooks (hwbrj_set_test_hook, include/hwbrj.h): explicit process-wide settings that force
// rarely taken paths (no result changes) or inject a failure; all off by default.
struct TestHooks {
    uint32_t join_split    = 0;   // HWBRJ_HOOK_JOIN_SPLIT: survivors per join part (0: the default)
    int      pj_fail_rank  = -1;  // HWBRJ_HOOK_PJ_FAIL_RANK: this rank fails the shard check
    int      bcast_nonroot = 0;   // HWBRJ_HOOK_BCAST_NONROOT: the broadcast join as a non-root rank
    int      pj_plan_div   = 0;   // HWBRJ_HOOK_PJ_PLAN_DIV: async plans' blocks divided by it (overflow)
    int      pj_async_fail = 0;   // HWBRJ_HOOK_PJ_ASYNC_FAIL: async joins run in the failed mode
};
TestHooks& test_hooks();

}  // namespace hwbrj
