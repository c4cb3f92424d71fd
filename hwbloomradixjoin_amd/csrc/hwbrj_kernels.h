// hwbrj_kernels.h -- kernel parameter blocks and launch wrappers (internal C++ interface between
// the HIP kernels and the host engine in hwbrj_engine.cpp).
#pragma once

#include <hip/hip_runtime.h>
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
    uint32_t*        meta;         // [G * cap]: partition | count << 16
    uint32_t*        wg_used;      // [G] chunks used by each workgroup
    uint32_t*        part_chunks;  // [F] (atomic)
    uint64_t*        part_elems;   // [F] (atomic)
    uint64_t         cap;          // chunk capacity of one workgroup region
    Geometry         g;
    const CrcTables* tabs;
    uint32_t         ablate;       // dev-only timing ablation (HWBRJ_SC_ABLATE); results invalid if != 0
};

struct BuildParams {
    Geometry         g;
    const CrcTables* tabs;
    const uint32_t*  pool;
    const uint32_t*  meta;
    const uint32_t*  list;
    const uint32_t*  list_start;  // [F + 1]
    const uint64_t*  elem_start;  // [F + 1]
    uint32_t*        slices;      // [F][nseg][seg_words]
    uint64_t*        qs_off;      // [F * NSUB + 1] start of each (q, sub) run in out_codes
    uint32_t*        out_codes;   // R codes grouped by (q, sub)
};

struct ProbeParams {
    Geometry         g;
    const CrcTables* tabs;
    const uint32_t*  pool;
    const uint32_t*  meta;
    const uint32_t*  list;
    const uint32_t*  list_start;  // [F + 1]
    const uint32_t*  item_start;  // [F + 1]
    const uint32_t*  slices;
    uint32_t*        surv;        // per item: survivors at (seg * surv_seg_stride + list_pos * 32)
    uint64_t         surv_seg_stride;
    uint32_t*        surv_cnt;    // [items][NSUB]
    uint32_t         CH;          // chunks per item
};

struct SurvParams {
    uint32_t        log2F, log2NSUB, sub_shift, nseg, CH;
    const uint32_t* item_start;
    const uint32_t* list_start;
    const uint32_t* surv;
    uint64_t        surv_seg_stride;
    const uint32_t* surv_cnt;
    const uint32_t* item_off;
    const uint64_t* qs_off;
    uint32_t*       out;
};

struct JoinParams {
    const uint32_t* r_codes;
    const uint64_t* r_off;  // [jobs + 1]
    const uint32_t* s_codes;
    const uint64_t* s_off;  // [jobs + 1]
    uint32_t        hash_shift;
    uint64_t*       result;
};

void   launch_gen(uint2* out, uint64_t offset, uint64_t count, const GenPlan* d_plan, const Perm& perm,
                  hipStream_t st);
void   launch_build_global(const uint2* R, uint64_t n, const Geometry& g, const CrcTables* tabs,
                           uint32_t* bm, hipStream_t st);
void   launch_probe_global(const uint2* S, uint64_t n, const Geometry& g, const CrcTables* tabs,
                           const uint32_t* bm, uint32_t* out, uint64_t* out_count, hipStream_t st);
size_t scatter_lds_bytes(uint32_t log2F);
void   launch_scatter(const ScatterParams& p, int src, uint32_t grid, hipStream_t st);
void   launch_list_fill(const uint32_t* meta, const uint32_t* wg_used, uint64_t cap,
                        uint32_t log2F, uint32_t* list_cursor, uint32_t* list, uint32_t grid,
                        hipStream_t st);
void   launch_plan(const uint32_t* part_chunks, const uint64_t* part_elems, uint32_t log2F,
                   uint32_t CH, uint32_t nseg, uint32_t* list_start, uint32_t* list_cursor,
                   uint64_t* elem_start, uint32_t* item_start, hipStream_t st);
void   launch_scan_u64(const uint64_t* in, uint64_t* out, uint32_t n, hipStream_t st);
size_t slice_lds_bytes(const Geometry& g);
void   launch_build(const BuildParams& p, uint32_t F, hipStream_t st);
void   launch_probe(const ProbeParams& p, uint32_t grid, hipStream_t st);
void   launch_surv_totals(const uint32_t* item_start, const uint32_t* surv_cnt, uint32_t log2F,
                          uint32_t log2NSUB, uint32_t* item_off, uint64_t* qs_tot, hipStream_t st);
void   launch_surv_scatter(const SurvParams& p, uint32_t grid, hipStream_t st);
void   launch_join(const JoinParams& p, uint32_t jobs, hipStream_t st);
void   launch_export(const uint32_t* slices, const Geometry& g, uint32_t* out, uint64_t nwords,
                     hipStream_t st);

}  // namespace hwbrj
