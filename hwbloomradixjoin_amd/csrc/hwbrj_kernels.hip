// hwbrj_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the bloom-filtered radix join.
//
// Pipeline (DESIGN.md "Pipeline"; reference: src/parallel_radix_join_bloom.c:1059-1506):
//   k_scatter    R/S tuples -> F radix partitions of 32-element (128 B) chunks, written through a
//                per-workgroup LDS write-combining stage (the reference's pass-1, :758-852).
//                The digit is taken from the bloom *block index* bits, so every partition only
//                touches a 1/F slice of the filter.
//   k_list_fill  chunk lists per partition (the reference's task creation, :1183-1253).
//   k_build      per partition: set the filter bits of its R keys in an LDS slice, write the slice
//                (bloom add, src/bloom_filter.c:73-132), and sub-partition R codes for the join
//                (pass-2, :703-748).
//   k_probe      per item (partition, chunk range): test S elements against the LDS slice
//                (bloom contains, src/bloom_filter.c:92-141), compact survivors.
//   k_surv_*     sub-partition survivors for the join (pass-2 of S).
//   k_join       per (partition, sub): LDS open-addressing table of R codes, probe S codes, count
//                equal keys (bucket_chaining_join, :259-329).
// Keys travel as 32-bit "codes" = crc32c(42, key): a bijection of the key, so code equality is key
// equality and the code's low bits ARE the bloom block index.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "hwbrj_common.h"
#include "hwbrj_kernels.h"

namespace hwbrj {

// ================================================================== small device helpers
__device__ __forceinline__ void load_tab(uint32_t* dst, const uint32_t* src) {
    for (int i = threadIdx.x; i < 128; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// Where an element's filter bits live inside its partition slice (KIND != KIND_PASS).
struct Loc {
    uint32_t seg;   // slice segment
    uint32_t base;  // bit offset of the block (or the single bit, basic) inside the segment
    uint32_t h, y;  // enhanced double hashing state (block-relative)
};

template <int KIND>
__device__ __forceinline__ Loc locate(uint32_t w, const Geometry& g, const uint32_t* inv) {
    Loc L;
    if (KIND == KIND_BASIC_K1) {
        const uint32_t key = code_key(inv, w);
        const uint32_t b   = mod_m(crapwow(kSeed, key), (uint32_t) g.m);  // add_basic, k = 1
        const uint32_t lb  = b >> g.log2F;
        L.seg  = lb >> g.log2seg;
        L.base = lb & (g.seg_bits - 1u);
        L.h = L.y = 0;
        return L;
    }
    uint32_t lb;
    if (KIND == KIND_BLOCK_PK1) {
        lb  = w & g.lbmask;           // (code >> log2F) & (nblocks/F - 1)
        L.h = w >> (32u - g.log2F);   // crapwow(key) & (B-1), stored by the scatter
        L.y = 0;
    } else {
        const uint32_t key = code_key(inv, w);
        lb  = (w >> g.log2F) & g.lbmask;
        L.h = crapwow(kSeed, key) & (g.B - 1u);
        L.y = (key + kSeed) & (g.B - 1u);
    }
    const uint32_t sbit = lb << g.log2B;
    L.seg  = sbit >> g.log2seg;
    L.base = sbit & (g.seg_bits - 1u);
    return L;
}

// SET: add the key's bits (ds_or); otherwise test them (src/bloom_filter.c:73-111 per variant).
template <int KIND, bool SET>
__device__ __forceinline__ bool apply_bits(const Loc& L, const Geometry& g, uint32_t* slice) {
    if (KIND == KIND_BASIC_K1 || KIND == KIND_BLOCK_PK1) {
        const uint32_t b = L.base + L.h;
        if (SET) {
            atomicOr(slice + (b >> 5), 1u << (b & 31u));
            return true;
        }
        return (slice[b >> 5] >> (b & 31u)) & 1u;
    }
    uint32_t       h    = L.h, y = L.y;
    const uint32_t mask = g.B - 1u;
    const uint32_t s0   = h >> g.log2secw;
    const bool     sect = g.variant == VAR_SECTORIZED;
    for (uint32_t i = 0; i < g.k; i++) {
        // SECTORIZED: bit i lands in 64-bit sector (s0 + i) mod nsec (hwbrj_common.h sectorize)
        const uint32_t pos = sect ? (((s0 + i) & g.nsecmask) << g.log2secw) | (h & ((1u << g.log2secw) - 1u))
                                  : h;
        const uint32_t b   = L.base + pos;
        if (SET) {
            atomicOr(slice + (b >> 5), 1u << (b & 31u));
        } else if (!((slice[b >> 5] >> (b & 31u)) & 1u)) {
            return false;
        }
        h = (h + y) & mask;
        y = (y + i + 1u) & mask;
    }
    return true;
}

template <int KIND>
__device__ __forceinline__ uint32_t decode_k(uint32_t w, uint32_t q, uint32_t log2F) {
    if (KIND == KIND_BLOCK_PK1) return (w << log2F) | q;  // log2F >= 3: (w << log2F) drops the h bits
    return w;
}

// ========================================================================= K0: generator
__global__ void k_gen(uint2* out, uint64_t offset, uint64_t count, const GenPlan* plan, Perm perm) {
    uint64_t       i      = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < count; i += stride) {
        const uint64_t row = offset + i;
        const uint64_t g   = perm_apply(perm, row);
        out[i]             = make_uint2((uint32_t) gen_key_at(*plan, g), (uint32_t) row);
    }
}

// ============================================== K1/K2: global-bitmap fallback (MODE_GLOBAL)
// Reference layout: bit b of the filter = bit (b & 31) of 32-bit word b >> 5 (== byte b >> 3,
// bit b & 7 on little-endian, as bloom_filter.c addresses it).
__device__ __forceinline__ void global_positions_apply_add(uint32_t key, uint32_t code,
                                                           const Geometry& g, uint32_t* bm) {
    uint64_t base;
    uint32_t size;
    if (g.variant == VAR_BASIC) {
        base = 0;
        size = (uint32_t) g.m;
    } else {
        base = (uint64_t) (code & (g.nblocks - 1u)) * g.block_span;
        size = g.B;
    }
    uint32_t       h  = mod_m(crapwow(kSeed, key), size);
    uint32_t       y  = mod_m(key + kSeed, size);
    const uint32_t s0 = (g.variant == VAR_SECTORIZED) ? h / (g.B < 64u ? g.B : 64u) : 0u;
    for (uint32_t i = 0; i < g.k; i++) {
        const uint32_t pos = (g.variant == VAR_SECTORIZED) ? sectorize(h, s0, i, g.B) : h;
        const uint64_t b   = base + pos;
        atomicOr(bm + (b >> 5), 1u << (uint32_t) (b & 31u));
        h = mod_m(h + y, size);
        y = mod_m(y + i + 1u, size);
    }
}

__device__ __forceinline__ bool global_contains(uint32_t key, uint32_t code, const Geometry& g,
                                                const uint32_t* bm) {
    uint64_t base;
    uint32_t size;
    if (g.variant == VAR_BASIC) {
        base = 0;
        size = (uint32_t) g.m;
    } else {
        base = (uint64_t) (code & (g.nblocks - 1u)) * g.block_span;
        size = g.B;
    }
    uint32_t       h  = mod_m(crapwow(kSeed, key), size);
    uint32_t       y  = mod_m(key + kSeed, size);
    const uint32_t s0 = (g.variant == VAR_SECTORIZED) ? h / (g.B < 64u ? g.B : 64u) : 0u;
    for (uint32_t i = 0; i < g.k; i++) {
        const uint32_t pos = (g.variant == VAR_SECTORIZED) ? sectorize(h, s0, i, g.B) : h;
        const uint64_t b   = base + pos;
        if (!((bm[b >> 5] >> (uint32_t) (b & 31u)) & 1u)) return false;
        h = mod_m(h + y, size);
        y = mod_m(y + i + 1u, size);
    }
    return true;
}

__global__ __launch_bounds__(256) void k_build_global(const uint2* R, uint64_t n, Geometry g,
                                                      const CrcTables* tabs, uint32_t* bm) {
    __shared__ uint32_t fwd[128];
    load_tab(fwd, &tabs->fwd[0][0]);
    __syncthreads();
    uint64_t       i      = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        const uint32_t key = R[i].x;
        global_positions_apply_add(key, key_code(fwd, key), g, bm);
    }
}

// Direct probe of the global bitmap; survivors' codes are appended densely (one atomic per block).
__global__ __launch_bounds__(1024) void k_probe_global(const uint2* S, uint64_t n, Geometry g,
                                                       const CrcTables* tabs, const uint32_t* bm,
                                                       uint32_t* out, uint64_t* out_count) {
    __shared__ uint32_t fwd[128];
    __shared__ uint32_t wsum[16];
    __shared__ uint64_t bbase;
    load_tab(fwd, &tabs->fwd[0][0]);
    __syncthreads();
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (uint64_t t0 = (uint64_t) blockIdx.x * 1024; t0 < n; t0 += (uint64_t) gridDim.x * 1024) {
        const uint64_t i    = t0 + threadIdx.x;
        uint32_t       code = 0;
        uint32_t       pass = 0;
        if (i < n) {
            const uint32_t key = S[i].x;
            code               = key_code(fwd, key);
            pass               = global_contains(key, code, g, bm) ? 1u : 0u;
        }
        const uint32_t incl = wave_incl_scan(pass);
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            for (int w = 0; w < 16; w++) {
                uint32_t c = wsum[w];
                wsum[w]    = tot;
                tot += c;
            }
            bbase = tot ? atomicAdd((unsigned long long*) out_count, (unsigned long long) tot) : 0;
        }
        __syncthreads();
        if (pass) out[bbase + wsum[wave] + incl - 1] = code;
        __syncthreads();
    }
}

// ================================================================= K3: SWWC partitioning
// One workgroup per CU (the 128 KiB stage fills the LDS). Each round a workgroup takes 4096
// elements; element e of partition q goes to stage slot fill[q]++. A partition whose stage reaches
// 32 elements is flushed as one 128-byte chunk into the workgroup's private chunk region (no
// cross-workgroup coordination); a round that overfills a partition (skew) writes its extra whole
// chunks directly. Chunk metadata = partition | count << 16.
constexpr int      kScThreads = 1024;
constexpr uint32_t kCbBits    = 22;                       // ncb: chunk base | nchunks << 22
constexpr uint32_t kCbMask    = (1u << kCbBits) - 1u;

template <int SRC, int MODE, int FMT>
__device__ __forceinline__ void sc_word(uint32_t x, const Geometry& g, const uint32_t* fwd,
                                        uint32_t& w, uint32_t& q) {
    const uint32_t F1 = (1u << g.log2F) - 1u;
    if (SRC == SRC_CODES) {  // already a code (fallback survivors)
        w = x;
        q = x & F1;
        return;
    }
    const uint32_t key  = x;
    const uint32_t code = key_code(fwd, key);
    if (MODE == MODE_SLICE_BASIC) {
        q = mod_m(crapwow(kSeed, key), (uint32_t) g.m) & F1;
        w = code;
    } else if (MODE == MODE_SLICE_BLOCK && FMT == FMT_PACKED) {
        q = code & F1;
        w = (code >> g.log2F) | ((crapwow(kSeed, key) & (g.B - 1u)) << (32u - g.log2F));
    } else {
        q = code & F1;
        w = code;
    }
}

template <int SRC, int MODE, int FMT, int kScE>
__global__ __launch_bounds__(kScThreads) void k_scatter(ScatterParams P) {
    constexpr uint32_t kScRound = kScThreads * kScE;  // elements per workgroup round
    constexpr uint32_t kNone    = 0xFFFFFFFFu;        // no pending word
    constexpr uint32_t kDirect  = 0x80000000u;        // pending word goes to the pool, not the stage
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t F     = 1u << P.g.log2F;
    uint32_t*      stage = lds;            // F * 32
    uint32_t*      fill  = stage + F * 32; // F: words in the stage (incl. pending ones)
    uint32_t*      ncb   = fill + F;       // F: chunk base | nchunks << kCbBits (this round)
    uint32_t*      tch   = ncb + F;        // F: chunks of q (this workgroup)
    uint32_t*      tel   = tch + F;        // F: elements of q (this workgroup)
    uint32_t*      flq   = tel + F;        // F: flush queue
    uint32_t*      fwd   = flq + F;        // 128
    uint32_t*      misc  = fwd + 128;      // [0],[1] flush counts by round parity, [2] chunks used

    const int tid = threadIdx.x;
    for (uint32_t i = tid; i < F; i += kScThreads) {
        fill[i] = 0;
        tch[i]  = 0;
        tel[i]  = 0;
    }
    load_tab(fwd, &P.tabs->fwd[0][0]);
    if (tid < 4) misc[tid] = 0;
    __syncthreads();

    const uint64_t n     = P.n_dev ? *P.n_dev : P.n;
    const uint64_t units = (n + 3) >> 2;
    const uint64_t G     = gridDim.x, wg = blockIdx.x;
    const uint64_t e0    = 4 * (wg * units / G);
    const uint64_t e1r   = 4 * ((wg + 1) * units / G);
    const uint64_t e1    = e1r < n ? e1r : n;
    const uint32_t len   = e1 > e0 ? (uint32_t) (e1 - e0) : 0u;  // < 2^32 per workgroup
    uint32_t* __restrict__ pool = P.pool + wg * P.cap * 32;
    uint32_t* __restrict__ meta = P.meta + wg * P.cap;

    // Raw round data is prefetched one round ahead so the loads overlap the LDS phases below.
    constexpr int      NR      = (SRC == SRC_TUPLES) ? kScE / 2 : kScE / 4;  // uint4 per round
    constexpr uint32_t RSTRIDE = (SRC == SRC_TUPLES) ? 2 * kScThreads : 4 * kScThreads;
    const uint2*    tsrc = (const uint2*) P.src + e0;
    const uint32_t* csrc = (const uint32_t*) P.src + e0;
    uint4 pre[NR];
    auto fetch = [&](uint32_t base) {
#pragma unroll
        for (int h = 0; h < NR; h++) {
            if (SRC == SRC_TUPLES) {
                const uint32_t i = base + (uint32_t) h * RSTRIDE + 2 * tid;
                if (i + 1 < len) pre[h] = *(const uint4*) (tsrc + i);
                else if (i < len) pre[h] = make_uint4(tsrc[i].x, 0, 0, 0);
            } else {
                const uint32_t i = base + (uint32_t) h * RSTRIDE + 4 * tid;
                if (i + 3 < len) {
                    pre[h] = *(const uint4*) (csrc + i);
                } else {
                    pre[h].x = i < len ? csrc[i] : 0u;
                    pre[h].y = i + 1 < len ? csrc[i + 1] : 0u;
                    pre[h].z = i + 2 < len ? csrc[i + 2] : 0u;
                    pre[h].w = 0u;
                }
            }
        }
    };
    uint32_t pend[kScE], pendw[kScE];  // overflow words of the previous round
#pragma unroll
    for (int j = 0; j < kScE; j++) pend[j] = kNone;
    uint32_t wv[kScE], q[kScE], e[kScE];
    bool     v[kScE];
#pragma unroll
    for (int j = 0; j < kScE; j++) v[j] = false;
    // Overflow words of the previous round are parked in registers (read ncb before it changes).
    auto capture_pending = [&]() {
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            pend[j] = kNone;
            if (v[j] && e[j] >= 32) {  // whole extra chunks go to the pool, the rest start the stage
                const uint32_t qq = q[j], ch = e[j] >> 5, sl = e[j] & 31u;
                const uint32_t cb = ncb[qq];
                pend[j]  = ch < (cb >> kCbBits) ? (kDirect | (((cb & kCbMask) + ch) * 32 + sl))
                                                : qq * 32 + sl;
                pendw[j] = wv[j];
            }
        }
    };
    // D: flush every full stage of the previous round as one 128-byte line (8 lanes x 16 B).
    // Issued after this round's prefetched words are consumed and before the next prefetch, so the
    // stores are acknowledged during the round's compute (vmcnt also counts stores on CDNA).
    auto flush_prev = [&](uint32_t pp) {
        const uint32_t nfl = misc[pp];
        for (uint32_t i = tid >> 3; i < nfl; i += kScThreads / 8) {
            const uint32_t qq = flq[i];
            const uint32_t l8 = tid & 7;
            const uint32_t cb = ncb[qq];
            const uint4    vv = *(const uint4*) &stage[qq * 32 + l8 * 4];
            if (P.ablate & 2u) {
                asm volatile("" ::"v"(vv.x), "v"(vv.y), "v"(vv.z), "v"(vv.w));
            } else {
                *(uint4*) &pool[(cb & kCbMask) * 32 + l8 * 4] = vv;
                if (!(P.ablate & 1u))  // metas of this flush's chunks
                    for (uint32_t c = l8; c < (cb >> kCbBits); c += 8)
                        meta[(cb & kCbMask) + c] = qq | (32u << 16);
            }
        }
    };
    if (len) fetch(0);
    uint32_t par = 0;  // round parity (selects the flush counter)
    for (uint32_t base = 0; base < len; base += kScRound, par ^= 1u) {
        capture_pending();
        uint32_t x[kScE];
#pragma unroll
        for (int h = 0; h < NR; h++) {
            if (SRC == SRC_TUPLES) {
                const uint32_t i = base + (uint32_t) h * RSTRIDE + 2 * tid;
                x[2 * h]         = pre[h].x;
                x[2 * h + 1]     = pre[h].z;
                v[2 * h]         = i < len;
                v[2 * h + 1]     = i + 1 < len;
            } else {
                const uint32_t i = base + (uint32_t) h * RSTRIDE + 4 * tid;
                x[4 * h]         = pre[h].x;
                x[4 * h + 1]     = pre[h].y;
                x[4 * h + 2]     = pre[h].z;
                x[4 * h + 3]     = pre[h].w;
#pragma unroll
                for (int j = 0; j < 4; j++) v[4 * h + j] = i + j < len;
            }
        }
        // ---- A1: hash this round's words (consumes the prefetched registers)
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            if (P.ablate & 4u) {
                wv[j] = x[j];
                q[j]  = x[j] & (F - 1u);
            } else {
                sc_word<SRC, MODE, FMT>(x[j], P.g, fwd, wv[j], q[j]);
            }
        }
        flush_prev(par ^ 1u);
        if (base + kScRound < len) fetch(base + kScRound);
        // ---- A2: rank every word in its partition's stage
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            if (P.ablate & 8u) {
                e[j] = 0;
                asm volatile("" ::"v"(wv[j]), "v"(q[j]));
                v[j] = false;
            } else {
                e[j] = v[j] ? atomicAdd(&fill[q[j]], 1u) : 0u;
            }
        }
        __syncthreads();
        // ---- B: previous round's overflow words, this round's in-stage words; C: flush plan
        if (tid == 0) misc[par ^ 1u] = 0;
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            if (pend[j] != kNone) {
                if (pend[j] & kDirect) pool[pend[j] & ~kDirect] = pendw[j];
                else stage[pend[j]] = pendw[j];
            }
            if (v[j] && e[j] < 32) stage[q[j] * 32 + e[j]] = wv[j];
        }
        for (uint32_t qq = tid; qq < F; qq += kScThreads) {
            const uint32_t f = fill[qq];
            if (f >= 32) {
                const uint32_t c  = f >> 5;
                const uint32_t cb = atomicAdd(&misc[2], c);
                ncb[qq]           = cb | (c << kCbBits);
                tch[qq] += c;
                tel[qq] += c * 32;
                fill[qq]          = f & 31u;
                flq[atomicAdd(&misc[par], 1u)] = qq;
            }
        }
        __syncthreads();
    }
    capture_pending();
    flush_prev(par ^ 1u);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScE; j++) {
        if (pend[j] != kNone) {
            if (pend[j] & kDirect) pool[pend[j] & ~kDirect] = pendw[j];
            else stage[pend[j]] = pendw[j];
        }
    }
    __syncthreads();
    for (uint32_t qq = tid; qq < F; qq += kScThreads) {
        const uint32_t f = fill[qq];
        if (f > 0) {
            const uint32_t cb = atomicAdd(&misc[2], 1u);
            meta[cb]          = qq | (f << 16);
            for (uint32_t s2 = 0; s2 < f; s2++) pool[cb * 32 + s2] = stage[qq * 32 + s2];
            tch[qq] += 1;
            tel[qq] += f;
        }
    }
    __syncthreads();
    if (tid == 0) P.wg_used[wg] = misc[2];
    for (uint32_t qq = tid; qq < F; qq += kScThreads) {
        if (tch[qq]) {
            atomicAdd(&P.part_chunks[qq], tch[qq]);
            atomicAdd((unsigned long long*) &P.part_elems[qq], (unsigned long long) tel[qq]);
        }
    }
}

// =================================================================== K4: chunk lists
__global__ __launch_bounds__(1024) void k_list_fill(const uint32_t* meta, const uint32_t* wg_used,
                                                    uint64_t cap, uint32_t log2F,
                                                    uint32_t* list_cursor, uint32_t* list) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t F   = 1u << log2F;
    uint32_t*      cnt = lds;
    uint32_t*      cur = lds + F;
    for (uint32_t i = threadIdx.x; i < F; i += blockDim.x) cnt[i] = 0;
    __syncthreads();
    const uint64_t region = blockIdx.x * cap;
    const uint32_t used   = wg_used[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < used; i += blockDim.x)
        atomicAdd(&cnt[meta[region + i] & 0xFFFFu], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < F; i += blockDim.x)
        if (cnt[i]) cur[i] = atomicAdd(&list_cursor[i], cnt[i]);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < used; i += blockDim.x) {
        const uint32_t q   = meta[region + i] & 0xFFFFu;
        const uint32_t pos = atomicAdd(&cur[q], 1u);
        list[pos]          = (uint32_t) (region + i);
    }
}

// ======================================================= K5: single-block scans / planning
// After a scatter: list_start = excl-scan(part_chunks), elem_start = excl-scan(part_elems),
// item_start = excl-scan(ceil(chunks / CH) * nseg). Arrays have F + 1 entries.
__global__ __launch_bounds__(1024) void k_plan(const uint32_t* part_chunks,
                                               const uint64_t* part_elems, uint32_t log2F,
                                               uint32_t CH, uint32_t nseg, uint32_t* list_start,
                                               uint32_t* list_cursor, uint64_t* elem_start,
                                               uint32_t* item_start) {
    __shared__ uint32_t sc[1024];
    __shared__ uint32_t si[1024];
    __shared__ uint64_t se[1024];
    const uint32_t F = 1u << log2F;
    const uint32_t t = threadIdx.x;
    uint32_t c = 0, it = 0;
    uint64_t e = 0;
    if (t < F) {
        c  = part_chunks[t];
        e  = part_elems[t];
        it = ((c + CH - 1) / CH) * nseg;
    }
    sc[t] = c;
    si[t] = it;
    se[t] = e;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
        uint32_t ac = 0, ai = 0;
        uint64_t ae = 0;
        if (t >= off) {
            ac = sc[t - off];
            ai = si[t - off];
            ae = se[t - off];
        }
        __syncthreads();
        sc[t] += ac;
        si[t] += ai;
        se[t] += ae;
        __syncthreads();
    }
    if (t < F) {
        list_start[t + 1] = sc[t];
        item_start[t + 1] = si[t];
        elem_start[t + 1] = se[t];
        list_cursor[t]    = sc[t] - c;
    }
    if (t == 0) {
        list_start[0] = 0;
        item_start[0] = 0;
        elem_start[0] = 0;
    }
}

// Exclusive scan of n (<= 1M) u64 counts by one block: out[i] = sum_{j<i} in[j], out[n] = total.
__global__ __launch_bounds__(1024) void k_scan_u64(const uint64_t* in, uint64_t* out, uint32_t n) {
    __shared__ uint64_t part[1024];
    const uint32_t t   = threadIdx.x;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t b   = t * per, e = min(b + per, n);
    uint64_t       s   = 0;
    for (uint32_t i = b; i < e; i++) s += in[i];
    part[t] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        uint64_t a = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += a;
        __syncthreads();
    }
    uint64_t run = part[t] - s;
    for (uint32_t i = b; i < e; i++) {
        out[i] = run;
        run += in[i];
    }
    if (t == 1023) out[n] = part[1023];
}

// ======================================================== chunk-walking helpers (8 lanes)
// A sweep covers kSweep = 128 * kPQ chunks of a chunk list: 8 threads share a chunk (16 B each) and
// every thread issues kPQ independent list loads, then kPQ independent meta + chunk loads, so a
// workgroup keeps kPQ * 16 KiB in flight per round trip instead of one dependent load chain.
constexpr int      kPQ    = 8;
constexpr uint32_t kSweep = 128u * kPQ;

struct Sweep {
    uint4    v[kPQ];
    uint32_t n[kPQ];  // valid words of this thread's quad (0..4)
};

__device__ __forceinline__ void load_sweep(const uint32_t* __restrict__ list,
                                           const uint32_t* __restrict__ pool,
                                           const uint32_t* __restrict__ meta, uint32_t lb,
                                           uint32_t le, Sweep& S) {
    const uint32_t l8 = threadIdx.x & 7, cslot = threadIdx.x >> 3;
    uint32_t       cid[kPQ];
#pragma unroll
    for (int j = 0; j < kPQ; j++) {
        const uint32_t l = lb + cslot + (uint32_t) j * 128u;
        cid[j]           = l < le ? list[l] : 0xFFFFFFFFu;
    }
    uint32_t cnt[kPQ];
#pragma unroll
    for (int j = 0; j < kPQ; j++) {
        if (cid[j] != 0xFFFFFFFFu) {
            cnt[j]  = meta[cid[j]] >> 16;
            S.v[j]  = *(const uint4*) &pool[(uint64_t) cid[j] * 32 + l8 * 4];
        } else {
            cnt[j] = 0;
            S.v[j] = make_uint4(0, 0, 0, 0);
        }
    }
#pragma unroll
    for (int j = 0; j < kPQ; j++) {
        const uint32_t first = l8 * 4;
        S.n[j]               = cnt[j] > first ? min(cnt[j] - first, 4u) : 0u;
    }
}

__device__ __forceinline__ uint32_t sweep_word(const Sweep& S, int j, int t) {
    return t == 0 ? S.v[j].x : t == 1 ? S.v[j].y : t == 2 ? S.v[j].z : S.v[j].w;
}

// ======================================================================== K6: R build
// One workgroup per partition q. Filter bits of R go into an LDS slice segment (ds_or), the slice
// is written once (coalesced); then R codes are written grouped by sub-partition.
template <int KIND>
__global__ __launch_bounds__(1024) void k_build(BuildParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const Geometry& g      = P.g;
    const uint32_t  NSUB   = 1u << g.log2NSUB;
    constexpr bool  slices = KIND != KIND_PASS;
    const uint32_t  segw   = slices ? g.seg_words : 0;  // multiple of 4
    uint32_t*       slice  = lds;
    uint32_t*       inv    = slice + segw;
    uint32_t*       subh   = inv + 128;   // NSUB
    uint64_t*       subc   = (uint64_t*) (subh + 64);  // NSUB (8-byte aligned: segw, 128, 64 even)
    const uint32_t  q      = blockIdx.x;
    load_tab(inv, &P.tabs->inv[0][0]);
    for (uint32_t i = threadIdx.x; i < NSUB; i += blockDim.x) subh[i] = 0;
    const uint32_t l0 = P.list_start[q], l1 = P.list_start[q + 1];
    const uint32_t nseg = slices ? g.nseg : 1;
    for (uint32_t seg = 0; seg < nseg; seg++) {
        for (uint32_t i = threadIdx.x; i < segw; i += blockDim.x) slice[i] = 0;
        __syncthreads();
        const bool last = seg + 1 == nseg;
        for (uint32_t lb = l0; lb < l1; lb += kSweep) {
            Sweep S;
            load_sweep(P.list, P.pool, P.meta, lb, l1, S);
#pragma unroll
            for (int j = 0; j < kPQ; j++) {
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    if ((uint32_t) t >= S.n[j]) continue;
                    const uint32_t w = sweep_word(S, j, t);
                    if (slices) {
                        const Loc L = locate<KIND>(w, g, inv);
                        if (L.seg == seg) apply_bits<KIND, true>(L, g, slice);
                    }
                    if (last) {
                        const uint32_t c = decode_k<KIND>(w, q, g.log2F);
                        atomicAdd(&subh[(c >> g.sub_shift) & (NSUB - 1u)], 1u);
                    }
                }
            }
        }
        __syncthreads();
        if (slices) {
            uint4*       dst = (uint4*) (P.slices + ((uint64_t) q * g.nseg + seg) * segw);
            const uint4* src = (const uint4*) slice;
            for (uint32_t i = threadIdx.x; i < segw / 4; i += blockDim.x) dst[i] = src[i];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint64_t run = P.elem_start[q];
        for (uint32_t s = 0; s < NSUB; s++) {
            P.qs_off[(uint64_t) q * NSUB + s] = run;
            subc[s] = run;
            run += subh[s];
        }
        if (q == gridDim.x - 1) P.qs_off[(uint64_t) gridDim.x * NSUB] = run;
    }
    __syncthreads();
    for (uint32_t lb = l0; lb < l1; lb += kSweep) {
        Sweep S;
        load_sweep(P.list, P.pool, P.meta, lb, l1, S);
#pragma unroll
        for (int j = 0; j < kPQ; j++) {
#pragma unroll
            for (int t = 0; t < 4; t++) {
                if ((uint32_t) t >= S.n[j]) continue;
                const uint32_t c   = decode_k<KIND>(sweep_word(S, j, t), q, g.log2F);
                const uint32_t s   = (c >> g.sub_shift) & (NSUB - 1u);
                const uint64_t pos = atomicAdd((unsigned long long*) &subc[s], 1ull);
                P.out_codes[pos]   = c;
            }
        }
    }
}

// ======================================================================== K7: S probe
// Items = (partition q, slice segment, range of <= CH chunks of q's list). Workgroups take
// contiguous item ranges, so a slice segment is (re)loaded only when (q, seg) changes.
__device__ __forceinline__ uint32_t find_q(const uint32_t* item_start, uint32_t F, uint32_t it) {
    uint32_t lo = 0, hi = F - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (item_start[mid] <= it) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int KIND>
__global__ __launch_bounds__(1024) void k_probe(ProbeParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const Geometry& g      = P.g;
    const uint32_t  F      = 1u << g.log2F;
    const uint32_t  NSUB   = 1u << g.log2NSUB;
    constexpr bool  slices = KIND != KIND_PASS;
    const uint32_t  segw   = slices ? g.seg_words : 0;  // multiple of 4
    uint32_t*       slice  = lds;
    uint32_t*       inv    = slice + segw;
    uint32_t*       subc   = inv + 128;  // NSUB
    uint32_t*       misc   = subc + 64;  // [0] survivor cursor
    load_tab(inv, &P.tabs->inv[0][0]);
    for (uint32_t i = threadIdx.x; i < NSUB; i += blockDim.x) subc[i] = 0;
    if (threadIdx.x == 0) misc[0] = 0;
    __syncthreads();
    const uint32_t I   = P.item_start[F];
    const uint32_t it0 = (uint32_t) ((uint64_t) blockIdx.x * I / gridDim.x);
    const uint32_t it1 = (uint32_t) ((uint64_t) (blockIdx.x + 1) * I / gridDim.x);
    const uint32_t nseg = slices ? g.nseg : 1;
    const int      lane = threadIdx.x & 63;
    if (it0 >= it1) return;
    // walk partitions sequentially from the first item's (one binary search per workgroup)
    uint32_t q      = find_q(P.item_start, F, it0);
    uint32_t q_it0  = P.item_start[q], q_it1 = P.item_start[q + 1];
    uint32_t lq0    = P.list_start[q], lq1 = P.list_start[q + 1];
    uint32_t loaded = 0xFFFFFFFFu;
    for (uint32_t it = it0; it < it1; it++) {
        while (it >= q_it1) {  // uniform
            q++;
            q_it0 = q_it1;
            q_it1 = P.item_start[q + 1];
            lq0   = lq1;
            lq1   = P.list_start[q + 1];
        }
        const uint32_t local = it - q_it0;
        const uint32_t seg   = local % nseg;
        const uint32_t piece = local / nseg;
        const uint32_t lb    = lq0 + piece * P.CH;
        const uint32_t le    = min(lq1, lb + P.CH);
        if (slices) {
            const uint32_t tag = q * nseg + seg;
            if (loaded != tag) {
                const uint4* src = (const uint4*) (P.slices + (uint64_t) tag * segw);
                uint4*       dst = (uint4*) slice;
                for (uint32_t i = threadIdx.x; i < segw / 4; i += blockDim.x) dst[i] = src[i];
                loaded = tag;
                __syncthreads();
            }
        }
        uint32_t* __restrict__ out = P.surv + (uint64_t) seg * P.surv_seg_stride + (uint64_t) lb * 32;
        for (uint32_t l0 = lb; l0 < le; l0 += kSweep) {
            Sweep S;
            load_sweep(P.list, P.pool, P.meta, l0, le, S);
#pragma unroll
            for (int j = 0; j < kPQ; j++) {
                uint32_t cw[4];
                uint32_t pm = 0;  // pass mask of this thread's (up to) 4 words
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const uint32_t w    = sweep_word(S, j, t);
                    bool           pass = (uint32_t) t < S.n[j];
                    if (slices && pass) {
                        const Loc L = locate<KIND>(w, g, inv);
                        pass        = (nseg == 1 || L.seg == seg) && apply_bits<KIND, false>(L, g, slice);
                    }
                    cw[t] = decode_k<KIND>(w, q, g.log2F);
                    if (pass) {
                        pm |= 1u << t;
                        atomicAdd(&subc[(cw[t] >> g.sub_shift) & (NSUB - 1u)], 1u);
                    }
                }
                const uint32_t ns   = __popc(pm);
                const uint32_t incl = wave_incl_scan(ns);
                uint32_t       wb   = 0;
                if (lane == 63 && incl) wb = atomicAdd(&misc[0], incl);
                wb = __shfl(wb, 63, 64);
                const uint32_t o = wb + incl - ns;
#pragma unroll
                for (int t = 0; t < 4; t++)
                    if (pm & (1u << t)) out[o + __popc(pm & ((1u << t) - 1u))] = cw[t];
            }
        }
        __syncthreads();
        for (uint32_t s = threadIdx.x; s < NSUB; s += blockDim.x) {
            P.surv_cnt[(uint64_t) it * NSUB + s] = subc[s];
            subc[s]                             = 0;
        }
        if (threadIdx.x == 0) misc[0] = 0;
        __syncthreads();
    }
}

// ============================================ K8: survivor offsets per (q, sub) and per item
// One block per partition, one thread per sub: relative offsets of each item inside (q, sub)
// and the (q, sub) totals.
__global__ void k_surv_totals(const uint32_t* item_start, const uint32_t* surv_cnt,
                              uint32_t log2NSUB, uint32_t* item_off, uint64_t* qs_tot) {
    const uint32_t q = blockIdx.x, NSUB = 1u << log2NSUB;
    const uint32_t i0 = item_start[q], i1 = item_start[q + 1];
    for (uint32_t s = threadIdx.x; s < NSUB; s += blockDim.x) {
        uint64_t run = 0;
        for (uint32_t it = i0; it < i1; it++) {
            item_off[(uint64_t) it * NSUB + s] = (uint32_t) run;
            run += surv_cnt[(uint64_t) it * NSUB + s];
        }
        qs_tot[(uint64_t) q * NSUB + s] = run;
    }
}

// K9: move each item's survivors into the (q, sub)-grouped join layout.
__global__ __launch_bounds__(256) void k_surv_scatter(SurvParams P) {
    __shared__ uint64_t cur[64];
    const uint32_t F = 1u << P.log2F, NSUB = 1u << P.log2NSUB;
    const uint32_t I = P.item_start[F];
    for (uint32_t it = blockIdx.x; it < I; it += gridDim.x) {
        const uint32_t q     = find_q(P.item_start, F, it);
        const uint32_t local = it - P.item_start[q];
        const uint32_t seg   = local % P.nseg;
        const uint32_t piece = local / P.nseg;
        const uint32_t lb    = P.list_start[q] + piece * P.CH;
        __syncthreads();
        uint32_t total = 0;
        for (uint32_t s = 0; s < NSUB; s++) total += P.surv_cnt[(uint64_t) it * NSUB + s];
        for (uint32_t s = threadIdx.x; s < NSUB; s += blockDim.x)
            cur[s] = P.qs_off[(uint64_t) q * NSUB + s] + P.item_off[(uint64_t) it * NSUB + s];
        __syncthreads();
        const uint32_t* src = P.surv + (uint64_t) seg * P.surv_seg_stride + (uint64_t) lb * 32;
        for (uint32_t i0 = threadIdx.x; i0 < total; i0 += blockDim.x * 8) {
            uint32_t c[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t i = i0 + j * blockDim.x;
                c[j]             = i < total ? src[i] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                if (i0 + j * blockDim.x >= total) continue;
                const uint32_t s   = (c[j] >> P.sub_shift) & (NSUB - 1u);
                const uint64_t pos = atomicAdd((unsigned long long*) &cur[s], 1ull);
                P.out[pos]         = c[j];
            }
        }
    }
}

// ========================================================================= K10: join
// One workgroup per (q, sub): R codes -> LDS open-addressing table (linear probing, occupancy
// bits claimed with ds_or), then every S code walks its cluster counting equal codes. R runs
// larger than the table are processed in pieces (S is re-streamed per piece).
constexpr uint32_t kJoinLog2T  = 14;
constexpr uint32_t kJoinT      = 1u << kJoinLog2T;
constexpr uint32_t kJoinPiece  = kJoinT / 2;
constexpr int      kJoinB      = 16;           // independent loads per thread per batch
constexpr uint32_t kEmpty      = 0xFFFFFFFFu;  // codes of one job share their low hash_shift >= 1
                                               // bits, so (code >> hash_shift) never equals it

__device__ __forceinline__ uint32_t join_slot(uint32_t v) {
    return (v * 0x9E3779B1u) >> (32 - kJoinLog2T);
}

__global__ __launch_bounds__(512) void k_join(JoinParams P) {
    __shared__ uint32_t keys[kJoinT];
    __shared__ uint64_t wsum[8];
    const uint32_t job = blockIdx.x;
    const uint64_t r0 = P.r_off[job], r1 = P.r_off[job + 1];
    const uint64_t s0 = P.s_off[job], s1 = P.s_off[job + 1];
    if (r1 == r0 || s1 == s0) return;
    const uint32_t sh  = P.hash_shift;
    uint64_t       cnt = 0;
    for (uint64_t rb = r0; rb < r1; rb += kJoinPiece) {
        const uint64_t re = min(r1, rb + kJoinPiece);
        for (uint32_t i = threadIdx.x; i < kJoinT / 4; i += blockDim.x)
            ((uint4*) keys)[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
        __syncthreads();
        for (uint64_t i0 = rb + threadIdx.x; i0 < re; i0 += (uint64_t) blockDim.x * kJoinB) {
            uint32_t c[kJoinB];
#pragma unroll
            for (int j = 0; j < kJoinB; j++) {
                const uint64_t i = i0 + (uint64_t) j * blockDim.x;
                c[j]             = i < re ? P.r_codes[i] : 0u;
            }
#pragma unroll
            for (int j = 0; j < kJoinB; j++) {
                if (i0 + (uint64_t) j * blockDim.x >= re) continue;
                const uint32_t v = c[j] >> sh;
                uint32_t       h = join_slot(v);
                while (atomicCAS(&keys[h], kEmpty, v) != kEmpty) h = (h + 1u) & (kJoinT - 1u);
            }
        }
        __syncthreads();
        for (uint64_t i0 = s0 + threadIdx.x; i0 < s1; i0 += (uint64_t) blockDim.x * kJoinB) {
            uint32_t c[kJoinB];
#pragma unroll
            for (int j = 0; j < kJoinB; j++) {
                const uint64_t i = i0 + (uint64_t) j * blockDim.x;
                c[j]             = i < s1 ? P.s_codes[i] : 0u;
            }
#pragma unroll
            for (int j = 0; j < kJoinB; j++) {
                if (i0 + (uint64_t) j * blockDim.x >= s1) continue;
                const uint32_t v = c[j] >> sh;
                uint32_t       h = join_slot(v);
                for (uint32_t k = keys[h]; k != kEmpty; k = keys[h]) {
                    cnt += k == v;
                    h = (h + 1u) & (kJoinT - 1u);
                }
            }
        }
        __syncthreads();
    }
    cnt = wave_sum_u64(cnt);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (uint32_t w = 0; w < blockDim.x / 64; w++) t += wsum[w];
        if (t) atomicAdd((unsigned long long*) P.result, (unsigned long long) t);
    }
}

// ============================================== K11: export the filter in reference layout
// Output word o holds reference bits 32*o .. 32*o+31 (src/bloom_filter.c byte addressing).
__global__ void k_export(const uint32_t* slices, Geometry g, uint32_t* out, uint64_t nwords) {
    uint64_t       o      = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    const uint32_t log2seg = ilog2u(g.seg_bits), segw = g.seg_words;
    for (; o < nwords; o += stride) {
        uint32_t r = 0;
        for (uint32_t t = 0; t < 32; t++) {
            const uint64_t gb = o * 32 + t;
            uint32_t       q, lb;
            if (g.mode == MODE_SLICE_BASIC) {
                q  = (uint32_t) (gb & ((1u << g.log2F) - 1u));
                lb = (uint32_t) (gb >> g.log2F);
            } else {
                const uint32_t blk = (uint32_t) (gb / g.B), h = (uint32_t) (gb % g.B);
                q  = blk & ((1u << g.log2F) - 1u);
                lb = (blk >> g.log2F) * g.B + h;
            }
            const uint32_t seg = lb >> log2seg, off = lb & (g.seg_bits - 1u);
            const uint32_t* s  = slices + ((uint64_t) q * g.nseg + seg) * segw;
            r |= ((s[off >> 5] >> (off & 31u)) & 1u) << t;
        }
        out[o] = r;
    }
}

// ===================================================================== launch wrappers
void launch_gen(uint2* out, uint64_t offset, uint64_t count, const GenPlan* d_plan, const Perm& perm,
                hipStream_t st) {
    k_gen<<<4096, 256, 0, st>>>(out, offset, count, d_plan, perm);
}

void launch_build_global(const uint2* R, uint64_t n, const Geometry& g, const CrcTables* tabs,
                         uint32_t* bm, hipStream_t st) {
    k_build_global<<<4096, 256, 0, st>>>(R, n, g, tabs, bm);
}

void launch_probe_global(const uint2* S, uint64_t n, const Geometry& g, const CrcTables* tabs,
                         const uint32_t* bm, uint32_t* out, uint64_t* out_count, hipStream_t st) {
    k_probe_global<<<2048, 1024, 0, st>>>(S, n, g, tabs, bm, out, out_count);
}

size_t scatter_lds_bytes(uint32_t log2F) {
    const size_t F = 1u << log2F;
    return (F * 32 + F * 5 + 128 + 4) * sizeof(uint32_t);  // stage, 5 arrays, table, misc
}

static int scatter_elems() {  // dev knob for A/B runs: HWBRJ_SCE=4|8 elements per thread/round
    const char* v = getenv("HWBRJ_SCE");
    return (v && atoi(v) == 8) ? 8 : 4;
}

template <int SRC, int MODE, int FMT>
static void scatter_inst(const ScatterParams& p, uint32_t grid, hipStream_t st) {
    const size_t lds = scatter_lds_bytes(p.g.log2F);
    if (scatter_elems() == 8) {
        (void) hipFuncSetAttribute((const void*) &k_scatter<SRC, MODE, FMT, 8>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
        k_scatter<SRC, MODE, FMT, 8><<<grid, kScThreads, lds, st>>>(p);
    } else {
        (void) hipFuncSetAttribute((const void*) &k_scatter<SRC, MODE, FMT, 4>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
        k_scatter<SRC, MODE, FMT, 4><<<grid, kScThreads, lds, st>>>(p);
    }
}

void launch_scatter(const ScatterParams& p0, int src, uint32_t grid, hipStream_t st) {
    ScatterParams p = p0;
    const char*   ab = getenv("HWBRJ_SC_ABLATE");
    p.ablate         = ab ? (uint32_t) atoi(ab) : 0u;
    const Geometry& g = p.g;
    if (src == SRC_CODES) return scatter_inst<SRC_CODES, MODE_GLOBAL, FMT_CODE>(p, grid, st);
    switch (g.mode) {
        case MODE_SLICE_BLOCK:
            if (g.format == FMT_PACKED)
                return scatter_inst<SRC_TUPLES, MODE_SLICE_BLOCK, FMT_PACKED>(p, grid, st);
            return scatter_inst<SRC_TUPLES, MODE_SLICE_BLOCK, FMT_CODE>(p, grid, st);
        case MODE_SLICE_BASIC:
            return scatter_inst<SRC_TUPLES, MODE_SLICE_BASIC, FMT_CODE>(p, grid, st);
        default: return scatter_inst<SRC_TUPLES, MODE_NOBLOOM, FMT_CODE>(p, grid, st);
    }
}

void launch_list_fill(const uint32_t* meta, const uint32_t* wg_used, uint64_t cap, uint32_t log2F,
                      uint32_t* list_cursor, uint32_t* list, uint32_t grid, hipStream_t st) {
    k_list_fill<<<grid, 1024, (2u << log2F) * sizeof(uint32_t), st>>>(meta, wg_used, cap, log2F,
                                                                      list_cursor, list);
}

void launch_plan(const uint32_t* part_chunks, const uint64_t* part_elems, uint32_t log2F,
                 uint32_t CH, uint32_t nseg, uint32_t* list_start, uint32_t* list_cursor,
                 uint64_t* elem_start, uint32_t* item_start, hipStream_t st) {
    k_plan<<<1, 1024, 0, st>>>(part_chunks, part_elems, log2F, CH, nseg, list_start, list_cursor,
                               elem_start, item_start);
}

void launch_scan_u64(const uint64_t* in, uint64_t* out, uint32_t n, hipStream_t st) {
    k_scan_u64<<<1, 1024, 0, st>>>(in, out, n);
}

size_t slice_lds_bytes(const Geometry& g) {
    const bool slices = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    return ((slices ? g.seg_words : 0) + 128 + 64 + 2 * 64 + 4) * sizeof(uint32_t);
}

int consumer_kind(const Geometry& g) {
    if (g.mode == MODE_SLICE_BASIC) return KIND_BASIC_K1;
    if (g.mode == MODE_SLICE_BLOCK) return g.format == FMT_PACKED ? KIND_BLOCK_PK1 : KIND_BLOCK;
    return KIND_PASS;
}

template <int KIND>
static void build_inst(const BuildParams& p, uint32_t F, size_t lds, hipStream_t st) {
    (void) hipFuncSetAttribute((const void*) &k_build<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_build<KIND><<<F, 1024, lds, st>>>(p);
}

template <int KIND>
static void probe_inst(const ProbeParams& p, uint32_t grid, size_t lds, hipStream_t st) {
    (void) hipFuncSetAttribute((const void*) &k_probe<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_probe<KIND><<<grid, 1024, lds, st>>>(p);
}

void launch_build(const BuildParams& p, uint32_t F, hipStream_t st) {
    const size_t lds = slice_lds_bytes(p.g);
    switch (consumer_kind(p.g)) {
        case KIND_BLOCK_PK1: return build_inst<KIND_BLOCK_PK1>(p, F, lds, st);
        case KIND_BLOCK: return build_inst<KIND_BLOCK>(p, F, lds, st);
        case KIND_BASIC_K1: return build_inst<KIND_BASIC_K1>(p, F, lds, st);
        default: return build_inst<KIND_PASS>(p, F, lds, st);
    }
}

void launch_probe(const ProbeParams& p, uint32_t grid, hipStream_t st) {
    const size_t lds = slice_lds_bytes(p.g);
    switch (consumer_kind(p.g)) {
        case KIND_BLOCK_PK1: return probe_inst<KIND_BLOCK_PK1>(p, grid, lds, st);
        case KIND_BLOCK: return probe_inst<KIND_BLOCK>(p, grid, lds, st);
        case KIND_BASIC_K1: return probe_inst<KIND_BASIC_K1>(p, grid, lds, st);
        default: return probe_inst<KIND_PASS>(p, grid, lds, st);
    }
}

void launch_surv_totals(const uint32_t* item_start, const uint32_t* surv_cnt, uint32_t log2F,
                        uint32_t log2NSUB, uint32_t* item_off, uint64_t* qs_tot, hipStream_t st) {
    k_surv_totals<<<1u << log2F, 64, 0, st>>>(item_start, surv_cnt, log2NSUB, item_off, qs_tot);
}

void launch_surv_scatter(const SurvParams& p, uint32_t grid, hipStream_t st) {
    k_surv_scatter<<<grid, 256, 0, st>>>(p);
}

void launch_join(const JoinParams& p, uint32_t jobs, hipStream_t st) {
    k_join<<<jobs, 512, 0, st>>>(p);
}

void launch_export(const uint32_t* slices, const Geometry& g, uint32_t* out, uint64_t nwords,
                   hipStream_t st) {
    k_export<<<2048, 256, 0, st>>>(slices, g, out, nwords);
}

}  // namespace hwbrj
