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
//                (bloom contains, src/bloom_filter.c:92-141), write the survivors grouped by join
//                sub-partition (pass-2 of S).
//   k_join_split splits (partition, sub) jobs with skewed survivor counts into parts.
//   k_join       per job part: LDS bitmap (or hash table) of the R codes of (partition, sub),
//                survivors count equal keys (bucket_chaining_join, :259-329).
//   k_mat_*      result materialization (JOIN_RESULT_MATERIALIZE): {R.payload, S.payload} pairs.
// Keys travel as 32-bit "codes" = crc32c(42, key): a bijection of the key, so code equality is key
// equality and the code's low bits ARE the bloom block index.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <type_traits>

#include "hwbrj_common.h"
#include "hwbrj_kernels.h"

// Ablations ("results invalid": they skip work to time what is left) and cycle stamps exist for
// measurements only. They build only with -DHWBRJ_DEV_BUILD (tools/build_abl.sh sets it), so no
// product build can carry one by accident; hwbrj_version() names every non-default knob.
#if !defined(HWBRJ_DEV_BUILD) &&                                                                   \
    (defined(HWBRJ_ABL_NOCRC) || defined(HWBRJ_ABL_NOCRAP) || defined(HWBRJ_ABL_NOSTORE) ||        \
     defined(HWBRJ_ABL_SPLITH) || defined(HWBRJ_ABL_PNOPST) || defined(HWBRJ_ABL_BNOBITS) ||       \
     defined(HWBRJ_ABL_BNOSORT) || defined(HWBRJ_ABL_PNOB1) || defined(HWBRJ_ABL_JNOR) ||          \
     defined(HWBRJ_ABL_JNOS) || defined(HWBRJ_ABL_MJ_EMPTY) || defined(HWBRJ_ABL_MJ_NOLOAD) ||     \
     defined(HWBRJ_ABL_MJ_NOINS) || defined(HWBRJ_ABL_MJ_R) || defined(HWBRJ_ABL_PROBE) ||         \
     defined(HWBRJ_STAMPS))
#error "HWBRJ_ABL_* / HWBRJ_STAMPS give invalid results or perturb timing: dev builds only (-DHWBRJ_DEV_BUILD)"
#endif

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

// Inclusive wave64 prefix sum on the VALU (DPP row shifts + row broadcasts; no LDS traffic).
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false);  // row_bcast:15
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}

// Raw buffer access: out-of-range stores are dropped and loads return 0, so a fixed number of
// instructions can be issued unconditionally (static vmcnt bookkeeping in pipelined loops).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int) bytes, 0x00020000);
}

// 24-bit join keys (pack3): the join needs only v = code >> hash_shift, < 2^24 when hash_shift >= 8
// (18 bits at the north star), so the build's R runs and the probe's staged survivor runs store
// 4 keys per 12 bytes -- 25 % fewer bytes written there and read back by the join. Key i of a run
// at byte b is the low 24 bits of the (unaligned) dword at b + 3 i; the last key's dword ends
// inside the run's 4-byte-per-key region, so no read leaves it.
typedef unsigned int v3u __attribute__((ext_vector_type(3)));
__device__ __forceinline__ v3u pack3x4(v4u v, uint32_t sh) {
    const uint32_t a = v.x >> sh, b = v.y >> sh, c = v.z >> sh, d = v.w >> sh;
    return v3u{a | (b << 24), (b >> 8) | (c << 16), (c >> 16) | (d << 8)};
}
// 18-bit join keys (hash_shift = 14, every bitmap-path launch; join_key_bits): key i of a run at
// bit b is bits [b + 18 i, b + 18 i + 18) of the stream, read as the dword at byte (b + 18 i) >> 3
// shifted right by (b + 18 i) & 7 (18 + 7 < 32 bits). 25 % fewer bytes than 24-bit keys (north
// star: 0.19 GB of R keys and as much of survivors, each written by k_build / k_probe and read back
// by k_join). A writer builds dword d of the stream from the three codes that overlap it, read from
// the LDS stage they are sorted in (c[ka + 1], c[ka + 2] may lie past the last key: they only fill
// bits past the stream's end), so no thread holds more than its four output dwords.
__device__ __forceinline__ uint32_t pack18_dword(const uint32_t* c, uint32_t d, uint32_t sh) {
    const uint32_t p = 32u * d, ka = p / 18u, s = p - 18u * ka;
    const uint32_t k0 = (c[ka] >> sh) & 0x3FFFFu, k1 = (c[ka + 1] >> sh) & 0x3FFFFu, k2 = (c[ka + 2] >> sh) & 0x3FFFFu;
    return (k0 >> s) | (k1 << (18u - s)) | (s > 4u ? k2 << (36u - s) : 0u);
}
__device__ __forceinline__ v4u pack18_quad(const uint32_t* c, uint32_t i, uint32_t sh) {  // dwords 4i .. 4i + 3
    return v4u{pack18_dword(c, 4 * i, sh), pack18_dword(c, 4 * i + 1, sh), pack18_dword(c, 4 * i + 2, sh),
               pack18_dword(c, 4 * i + 3, sh)};
}
// The same stream from 16 codes held in registers (4 quads) into 9 dwords: the build's form (its
// copy-out has registers to spare and measured faster this way than with the LDS reads above; the
// probe's has not: 16 live codes spill it)
__device__ __forceinline__ void pack18x16(const v4u* q, uint32_t sh, uint32_t out[9]) {
    uint64_t acc = 0;
    int      nb = 0, d = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const v4u      v = q[k >> 2];
        const uint32_t c = (k & 3) == 0 ? v.x : (k & 3) == 1 ? v.y : (k & 3) == 2 ? v.z : v.w;
        acc |= (uint64_t) ((c >> sh) & 0x3FFFFu) << nb;
        nb += 18;
        if (nb >= 32) {
            out[d++] = (uint32_t) acc;
            acc >>= 32;
            nb -= 32;
        }
    }
}
typedef uint32_t u32_unaligned __attribute__((aligned(1)));

// Copy a slice segment (words, a multiple of 4) from HBM into LDS with global_load_lds (16 bytes
// per lane, no VGPR destination), all loads issued before any wait: one latency per slice instead
// of one per 16 KiB (a register copy loop waits for each load before its ds_write). The caller's
// __syncthreads() after it retires the loads (its fence waits vmcnt(0)). 1024 threads.
__device__ __forceinline__ void slice_to_lds(uint32_t* dst, const uint32_t* src, uint32_t words) {
    const uint4*   s4 = (const uint4*) src;
    uint4*         d4 = (uint4*) dst;
    const uint32_t n  = words / 4, wb = threadIdx.x & ~63u;
    if (n % 64 != 0) {  // (small filters) a plain copy
        for (uint32_t i = threadIdx.x; i < n; i += 1024) d4[i] = s4[i];
        return;
    }
    for (uint32_t i0 = 0; i0 < n; i0 += 1024)
        if (i0 + wb < n)  // (wave-uniform) the wave's 64 lanes fill d4[i0 + wb .. + 64)
            __builtin_amdgcn_global_load_lds((const void*) (s4 + i0 + threadIdx.x),
                                             (__attribute__((address_space(3))) void*) (d4 + i0 + wb), 16, 0, 0);
}

// Where an element's filter bits live inside its partition slice (KIND != KIND_PASS).
struct Loc {
    uint32_t seg;   // slice segment
    uint32_t base;  // bit offset of the block (or the single bit, basic) inside the segment
    uint32_t h, y;  // enhanced double hashing state (block-relative)
};

template <int KIND>
__device__ __forceinline__ uint32_t decode_k(uint32_t w, uint32_t q, const Geometry& g);

// q: the element's partition (packed kinds recover the code from it).
template <int KIND>
__device__ __forceinline__ Loc locate(uint32_t w, const Geometry& g, const uint32_t* inv, uint32_t q) {
    Loc L;
    if (KIND == KIND_BASIC_K1 || KIND == KIND_BASIC_KK) {
        const uint32_t key = bunmix(w);  // MODE_SLICE_BASIC words are bmix(key)
        const uint32_t b   = mod_m(crapwow(kSeed, key), (uint32_t) g.m);  // add_basic, first bit
        const uint32_t lb  = b >> g.log2F;
        L.seg  = lb >> g.log2seg;
        L.base = lb & (g.seg_bits - 1u);
        L.h = L.y = 0;
        return L;
    }
    uint32_t lb;
    if (KIND == KIND_BLOCK_PK1 || KIND == KIND_BLOCK_PKK) {
        lb  = (w >> g.log2B) & g.lbmask;  // (code >> log2F) & (nblocks/F - 1)
        L.h = w & (g.B - 1u);             // crapwow(key) & (B-1), stored by the scatter
        L.y = KIND == KIND_BLOCK_PKK ? (code_key(inv, decode_k<KIND>(w, q, g)) + kSeed) & (g.B - 1u) : 0u;
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
    if (KIND == KIND_BASIC_K1 || KIND == KIND_BASIC_KK || KIND == KIND_BLOCK_PK1) {
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
__device__ __forceinline__ uint32_t decode_k(uint32_t w, uint32_t q, const Geometry& g) {
    if (KIND == KIND_BLOCK_PK1 || KIND == KIND_BLOCK_PKK) return ((w >> g.log2B) << g.log2F) | q;  // drops the h bits
    return w;
}

// Basic filter bit b in the partition-slice layout (MODE_SLICE_BASIC): slice q = b & (F-1) holds
// it at lb = b >> log2F. Returns the word; the bit inside it is lb & 31.
__device__ __forceinline__ const uint32_t* basic_word(const uint32_t* slices, const Geometry& g, uint32_t b) {
    const uint32_t lb = b >> g.log2F;
    return slices + ((uint64_t) (b & ((1u << g.log2F) - 1u)) * g.nseg + (lb >> g.log2seg)) * g.seg_words +
           ((lb & (g.seg_bits - 1u)) >> 5);
}

// KIND_BASIC_KK: bits 2..k of add_basic (src/bloom_filter.c:73-111, the double-hashing sequence of
// global_contains below) read from the slices in HBM; bit 1 was tested from the LDS slice.
__device__ __forceinline__ bool basic_rest(uint32_t key, const Geometry& g, const uint32_t* inv,
                                           const uint32_t* __restrict__ slices) {
    (void) inv;
    const uint32_t msz = (uint32_t) g.m;
    uint32_t       h = mod_m(crapwow(kSeed, key), msz), y = mod_m(key + kSeed, msz);
    h = mod_m(h + y, msz);
    y = mod_m(y + 1u, msz);
    for (uint32_t i = 1; i < g.k; i++) {
        if (!((*basic_word(slices, g, h) >> ((h >> g.log2F) & 31u)) & 1u)) return false;
        h = mod_m(h + y, msz);
        y = mod_m(y + i + 1u, msz);
    }
    return true;
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

// Zipf stream on the device (src/genzipf.c:119-150): rnd holds the rand() draws of rows
// [row0, row0 + cnt), each becomes alphabet[pos] by the reference's binary search over the CDF.
// This build's selectivity extension: rows whose permuted index u < n_above get the unique
// non-matching key above_base + u instead (n_above = 0: the reference's stream).
__global__ void k_zipf(const int32_t* __restrict__ rnd, uint64_t cnt, uint64_t row0,
                       const double* __restrict__ lut, const uint32_t* __restrict__ alphabet,
                       uint32_t size, uint2* __restrict__ out, uint64_t n_above, uint32_t above_base,
                       Perm perm) {
    uint64_t       i      = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < cnt; i += stride) {
        const double r     = ((double) rnd[i]) / 2147483647;
        uint32_t     left  = 0, right = size - 1, pos;
        if (lut[0] >= r) {
            pos = 0;
        } else {
            while (right - left > 1) {
                const uint32_t m = (left + right) / 2;
                if (lut[m] < r) left = m;
                else right = m;
            }
            pos = right;
        }
        const uint64_t row = row0 + i;
        uint32_t       key = alphabet[pos];
        if (n_above) {
            const uint64_t u = perm_apply(perm, row);
            if (u < n_above) key = above_base + (uint32_t) u;
        }
        out[i] = make_uint2(key, (uint32_t) row);
    }
}

void launch_zipf(const int32_t* rnd, uint64_t cnt, uint64_t row0, const double* lut,
                 const uint32_t* alphabet, uint32_t size, uint2* out, uint64_t n_above,
                 uint32_t above_base, const Perm& perm, hipStream_t st) {
    k_zipf<<<8192, 256, 0, st>>>(rnd, cnt, row0, lut, alphabet, size, out, n_above, above_base, perm);
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
// One workgroup per CU (the 128 KiB stage fills the LDS), private contiguous chunk region per
// workgroup (no cross-workgroup coordination). A round takes kScRound elements (8 per thread):
//   A  hash the round's words (loaded two rounds ahead), copy out the stage lines planned in the
//      previous round (a fixed number of buffer stores per thread), rank every word in its
//      partition's stage (ds_add_rtn on fill[q]);
//   B1 (barrier) B  write the previous round's overflow words and this round's in-stage words;
//      one thread per partition plans the flush of every stage that reached 32 words;
//   B2 (barrier).
// A plan turns floor(fill/32) chunks into consecutive chunk ids: the first is the stage
// line, further ones (only when a round overfills a partition by > 32, i.e. skew) are written
// directly by the threads holding those overflow words. Chunk metadata (16 bits, meta16):
// partition | (count - 1) << 10, which is the low 15 bits of k_list_fill's sort entry.
// (Reference pass-1: src/parallel_radix_join_bloom.c:758-852, SWWC variant :611-700.)
__device__ __forceinline__ uint16_t meta16(uint32_t q, uint32_t count) {  // q < 1024, count 1..32
    return (uint16_t) (q | ((count - 1u) << 10));
}
#ifndef HWBRJ_SC_T
#define HWBRJ_SC_T 1024  // threads per scatter workgroup (A/B: 512)
#endif
constexpr int      kScThreads = HWBRJ_SC_T;
constexpr int      kScPlanPer = (1024 + kScThreads - 1) / kScThreads;  // partitions per plan thread (F <= 1024)
constexpr int      kScPayThreads = 1024;  // the materializing scatter (scatter_body_pay)
#ifndef HWBRJ_SC_E
#define HWBRJ_SC_E 8
#define HWBRJ_SC_K 2
#endif
#ifndef HWBRJ_SC_PRE
#define HWBRJ_SC_PRE 1
#endif
#ifndef HWBRJ_SC_KEEPY
#define HWBRJ_SC_KEEPY 1
#endif
#ifndef HWBRJ_SC_LAUX
#define HWBRJ_SC_LAUX 2  // cache policy of the tuple loads: nt (read once; 0 measured 2 % slower)
#endif
#ifndef HWBRJ_SC_SAUX
#define HWBRJ_SC_SAUX 2  // cache policy of the chunk stores: nt (16 = sc1 measured slower)
#endif
#ifndef HWBRJ_SC_SAUX_R
#define HWBRJ_SC_SAUX_R HWBRJ_SC_SAUX  // (the R scatter's, A/B)
#endif
constexpr int      kScPre     = HWBRJ_SC_PRE;             // rounds of loads in flight (1 or 2)
constexpr int      kScE       = HWBRJ_SC_E;                        // elements per thread per round
constexpr uint32_t kScRound   = kScThreads * kScE;        // elements per workgroup round
constexpr int      kScK       = HWBRJ_SC_K;                        // flush tasks per thread per round (fixed)
constexpr uint32_t kCbBits    = 22;                       // ncb: chunk base | nchunks << 22
constexpr uint32_t kCbMask    = (1u << kCbBits) - 1u;
constexpr uint32_t kOob       = 0x7FFFFFF0u;              // buffer offset that is always dropped

// 4 x (byte K of x) or (byte K of x) / 4, in one VALU op (SDWA source select).
template <int K, bool RIGHT>
__device__ __forceinline__ uint32_t byte_sh2(uint32_t x) {
    static_assert(K >= 0 && K < 4, "byte index");
    uint32_t r;
#define HWBRJ_SDWA(op, sel) asm(op "_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" sel : "=v"(r) : "v"(x))
    if (!RIGHT) {
        if (K == 0) HWBRJ_SDWA("v_lshlrev_b32", "BYTE_0");
        if (K == 1) HWBRJ_SDWA("v_lshlrev_b32", "BYTE_1");
        if (K == 2) HWBRJ_SDWA("v_lshlrev_b32", "BYTE_2");
        if (K == 3) HWBRJ_SDWA("v_lshlrev_b32", "BYTE_3");
    } else {
        if (K == 0) HWBRJ_SDWA("v_lshrrev_b32", "BYTE_0");
        if (K == 1) HWBRJ_SDWA("v_lshrrev_b32", "BYTE_1");
        if (K == 2) HWBRJ_SDWA("v_lshrrev_b32", "BYTE_2");
        if (K == 3) HWBRJ_SDWA("v_lshrrev_b32", "BYTE_3");
    }
#undef HWBRJ_SDWA
    return r;
}

// CRC32-C code of a key from the 8 x 16 nibble table in static LDS (at address 0, so row offsets
// are immediates; row 0 has f(kSeed) folded in: code = f(key ^ kSeed) = f(key) ^ f(kSeed)).
// 16 entries per row sit in 16 distinct banks: the reads are conflict-free. Byte offsets of the
// entries: even nibbles from key & 0x0F0F0F0F (<< 2), odd ones from key & 0xF0F0F0F0 (>> 2).
__device__ __forceinline__ uint32_t crc_nib(const uint32_t* tab, uint32_t key) {
    const char*    b = (const char*) tab;
    const uint32_t y = key & 0x0F0F0F0Fu, z = key & 0xF0F0F0F0u;
    auto T = [&](uint32_t off) { return *(const uint32_t*) (b + off); };
    const uint32_t t0 = T(byte_sh2<0, false>(y)), t1 = T(byte_sh2<0, true>(z) + 64);
    const uint32_t t2 = T(byte_sh2<1, false>(y) + 128), t3 = T(byte_sh2<1, true>(z) + 192);
    const uint32_t t4 = T(byte_sh2<2, false>(y) + 256), t5 = T(byte_sh2<2, true>(z) + 320);
    const uint32_t t6 = T(byte_sh2<3, false>(y) + 384), t7 = T(byte_sh2<3, true>(z) + 448);
    const uint32_t a = __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96);  // three-way xor
    const uint32_t c = __builtin_amdgcn_bitop3_b32(t3, t4, t5, 0x96);
    return __builtin_amdgcn_bitop3_b32(a, c, t6 ^ t7, 0x96);
}

template <int SRC, int MODE, int FMT>
__device__ __forceinline__ void sc_word_lds0(uint32_t x, const Geometry& g, const uint32_t* tab,
                                             uint32_t& w, uint32_t& q) {
    const uint32_t F1 = (1u << g.log2F) - 1u;
    if (SRC == SRC_CODES) {
        if (MODE == MODE_BASIC_BITJ) {  // basic k >= 2 candidates: by the slice of their next bit
            q = basic_bit(bunmix(x), g.bitj, (uint32_t) g.m) & F1;
            w = x;
        } else if (MODE == MODE_CODE_OF_KEY) {  // basic k >= 2 survivors: into the join layout
            w = crc_nib(tab, bunmix(x));
            q = w & F1;
        } else {  // already a code (fallback survivors)
            w = x;
            q = x & F1;
        }
        return;
    }
    const uint32_t key  = x;
#ifdef HWBRJ_ABL_NOCRC
    const uint32_t code = key * 0x9E3779B1u;  // dev ablation (results invalid)
#else
    const uint32_t code = crc_nib(tab, key);
#endif
    if (MODE == MODE_SLICE_BASIC) {
        // the partition is the first filter bit's slice, not a code digit, so the word carries
        // the key (mixed, bmix): the join compares words, and nothing downstream needs the CRC
        q = mod_m(crapwow(kSeed, key), (uint32_t) g.m) & F1;
        w = bmix(key);
    } else if (MODE == MODE_SLICE_BLOCK && FMT == FMT_PACKED) {
        q = code & F1;
#ifdef HWBRJ_ABL_NOCRAP
        w = (key & (g.B - 1u)) | ((code >> g.log2F) << g.log2B);  // dev ablation (results invalid)
#else
        w = (crapwow(kSeed, key) & (g.B - 1u)) | ((code >> g.log2F) << g.log2B);
#endif
    } else {
        q = code & F1;
        w = code;
    }
}

template <int SRC>
struct ScRaw {  // one round's raw loads of this thread (tuples: keys only; codes: 4 per uint4)
    uint32_t k[SRC == SRC_TUPLES ? kScE : 1];
    uint4    v[SRC == SRC_TUPLES ? 1 : kScE / 4];
    uint32_t jb[SRC == SRC_TUPLES ? kScE : 1];  // MODE_BASIC_POS: which bit of the key
    // the payloads of a 16-byte tuple-pair load, unused but held until the keys are consumed: a
    // load's destination registers must not be reused while it is in flight, so a dead payload
    // register taken for a temporary costs an s_waitcnt vmcnt(0) right after the loads are issued
    uint32_t y[SRC == SRC_TUPLES && HWBRJ_SC_KEEPY ? kScE : 1];
};

// LDS: static CRC nibble table (512 B, at 0, so its row offsets are immediates); dynamic (words):
// stage F x 32 | 64 dummy slots | fill F + 4 | ncb 2F | flq F | misc 8 (per-partition totals: registers of the plan thread)
template <int SRC, int MODE, int FMT, int SAUX = HWBRJ_SC_SAUX>
__device__ __forceinline__ void scatter_body(const ScatterParams& P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint32_t crc_tab[128];
    constexpr int NL = SRC == SRC_TUPLES ? kScE / 2 : kScE / 4;  // uint4 loads per thread per round
    const uint32_t F     = 1u << P.g.log2F;
    uint32_t*      stage = lds;                  // F * 32, then 64 per-lane dummy slots
    uint32_t*      fill  = stage + F * 32 + 64;  // F + 1 (entry F: invalid elements)
    uint32_t*      ncb   = fill + F + 4;         // 2 x F: plan by round parity (chunk base | nchunks << 22)
    uint32_t*      flq   = ncb + 2 * F;          // F: partitions flushed by the last plan
    uint32_t*      misc  = flq + F;  // [0] chunks used, [1 + parity] flushes of a plan, [3 + parity] skew
    const int      tid   = threadIdx.x, lane = tid & 63;
    const uint32_t dummy = F * 32 + lane;        // stage index of this lane's dummy slot
    for (uint32_t i = tid; i < F + 1; i += kScThreads) fill[i] = 0;
    // chunks / elements of partitions tid + i * kScThreads (their plan thread) here
    uint32_t my_tch[kScPlanPer], my_tel[kScPlanPer];
#pragma unroll
    for (int i = 0; i < kScPlanPer; i++) my_tch[i] = my_tel[i] = 0;
    if (tid < 128) {  // nibble table; f(kSeed) folded into row 0
        const uint32_t* src = &P.tabs->fwd[0][0];
        uint32_t        v   = src[tid];
        if (tid < 16) {
#pragma unroll
            for (int j = 0; j < 8; j++) v ^= src[j * 16 + ((kSeed >> (4 * j)) & 15u)];
        }
        crc_tab[tid] = v;
    }
    if (tid < 8) misc[tid] = 0;
    if (blockIdx.x == 0 && P.zero_small && tid < 16) P.zero_small[tid] = 0;
    if (blockIdx.x == 0 && P.zero_word && tid == 0) *P.zero_word = 0;

    if (P.dbg && tid == 0) P.dbg[blockIdx.x * 8 + 6] = __builtin_amdgcn_s_memrealtime();  // dev-only: start
    const uint64_t n     = P.n_dev ? *P.n_dev : P.n;
    const uint64_t units = (n + 3) >> 2;
    const uint64_t G = gridDim.x, wg = blockIdx.x;
    uint64_t       e0  = 4 * (wg * units / G);
    const uint64_t e1r = 4 * ((wg + 1) * units / G);
    const uint64_t e1  = e1r < n ? e1r : n;
    uint32_t       len = __builtin_amdgcn_readfirstlane(e1 > e0 ? (uint32_t) (e1 - e0) : 0u);
    if (SRC == SRC_CODES && P.seg_cnt) {  // this workgroup's segment of a probe pass's output
        e0  = wg * P.seg_stride;
        len = __builtin_amdgcn_readfirstlane(P.seg_cnt[wg]);
    }
    constexpr uint32_t CW = 32u;  // dwords per chunk
    uint32_t* __restrict__ pool = P.pool + wg * P.cap * CW;
    uint16_t* __restrict__ meta = (uint16_t*) P.meta + wg * P.cap;
    constexpr uint32_t EB = SRC == SRC_TUPLES ? 8u : 4u;  // bytes per element
    const auto rsrc = buf_rsrc((const uint8_t*) P.src + e0 * EB, len * EB);  // OOB loads return 0
    const auto rpool = buf_rsrc(pool, (uint32_t) (P.cap * CW * 4));
    const auto rmeta = buf_rsrc(meta, (uint32_t) (P.cap * 2));
    __syncthreads();

    // MODE_BASIC_POS: element e0 + i is bit jj of tuple e0 + i - jj |R| (a workgroup's range
    // usually crosses at most one multiple of |R|; tiny relations step further)
    const uint64_t vn  = MODE == MODE_BASIC_POS && P.vn ? P.vn : 1;  // (P.vn = 0: no elements)
    const uint32_t jb0 = MODE == MODE_BASIC_POS ? (uint32_t) (e0 / vn) : 0u;
    const uint64_t vb  = (uint64_t) (jb0 + 1) * vn;
    // Loads of the round at `base`: a full round of tuples takes the lane offset in voffset and the
    // round offset in soffset (no per-element VALU); a partial round checks every index.
    auto load_round = [&](uint32_t base, ScRaw<SRC>& R) {
        if (MODE == MODE_BASIC_POS) {
#pragma unroll
            for (int j = 0; j < kScE; j++) {
                const uint32_t i  = base + j * kScThreads + tid;
                const uint64_t ev = e0 + (i < len ? i : 0u);  // (past the range: any valid tuple)
                uint32_t       jj = jb0;
                for (uint64_t b = vb; ev >= b; b += vn) jj++;  // (ev < k vn: at most k steps)
                const uint64_t t = ev - (uint64_t) jj * vn;
                R.k[j]  = len ? ((const uint32_t*) P.src)[2 * t] : 0u;  // (len = 0: R may be empty)
                R.jb[j] = jj;
            }
        } else if (SRC == SRC_TUPLES && base + kScRound <= len) {  // two tuples per 16-byte load
#pragma unroll
            for (int h = 0; h < kScE / 2; h++) {
                const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 2 * tid * EB, (base + h * 2 * kScThreads) * EB, HWBRJ_SC_LAUX);
                R.k[2 * h]     = x.x;
                R.k[2 * h + 1] = x.z;
                if (HWBRJ_SC_KEEPY) {
                    R.y[2 * h]     = x.y;
                    R.y[2 * h + 1] = x.w;
                }
            }
        } else if (SRC == SRC_TUPLES) {
#pragma unroll
            for (int j = 0; j < kScE; j++) {
                const uint32_t i = base + (j >> 1) * 2 * kScThreads + 2 * tid + (j & 1);
                R.k[j] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, i < len ? i * EB : kOob, 0, 0);
                if (HWBRJ_SC_KEEPY) R.y[j] = 0;
            }
        } else {
#pragma unroll
            for (int h = 0; h < NL; h++) {
                const uint32_t i = base + h * (4 * kScThreads) + 4 * tid;
                const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rsrc, i < len ? i * EB : kOob, 0, 0);
                R.v[h]      = make_uint4(x.x, x.y, x.z, x.w);
            }
        }
    };
    // element j of this thread in the round at `base`, and its index inside the workgroup's slice
    auto elem = [&](const ScRaw<SRC>& R, uint32_t base, int j, uint32_t& x, uint32_t& idx) {
        if (SRC == SRC_TUPLES) {
            x   = R.k[j];
            idx = MODE == MODE_BASIC_POS ? base + j * kScThreads + tid : base + (j >> 1) * 2 * kScThreads + 2 * tid + (j & 1);
        } else {
            const int h = j >> 2, t = j & 3;
            x   = t == 0 ? R.v[h].x : t == 1 ? R.v[h].y : t == 2 ? R.v[h].z : R.v[h].w;
            idx = base + h * (4 * kScThreads) + 4 * tid + t;
        }
    };
    // Copy out the stage lines of the last plan: task k = (flush entry k >> 3, 16-byte lane k & 7).
    uint32_t par = 0;  // round parity: misc[1 + par] counts this round's plan
    auto flush_copy = [&]() {
        const uint32_t nf = misc[1 + (par ^ 1u)];  // plan of the previous round
        auto task = [&](uint32_t k) {
            const bool     ok = k < nf * 8;
            const uint32_t qq = flq[ok ? k >> 3 : 0];
            const uint32_t l8 = k & 7;
            const uint32_t cb = ncb[(par ^ 1u) * F + qq] & kCbMask;
            const v4u      v  = *(const v4u*) &stage[qq * 32 + l8 * 4];
#ifdef HWBRJ_ABL_NOSTORE
            if (v.x == 0x12345678u && v.y == 0x9abcdef0u)  // dev ablation: practically never stores
#endif
            __builtin_amdgcn_raw_buffer_store_b128(v, rpool, ok ? (cb * 32 + l8 * 4) * 4 : kOob, 0, SAUX);
            __builtin_amdgcn_raw_buffer_store_b16((short) meta16(qq, 32u), rmeta, ok && l8 == 0 ? cb * 2 : kOob, 0, 0);
        };
#pragma unroll
        for (int i = 0; i < kScK; i++) task(tid + i * kScThreads);
        for (uint32_t k = kScK * kScThreads + tid; k < nf * 8; k += kScThreads) task(k);  // rare
    };

    uint64_t tph[6] = {0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
    (void) tlast;
    auto stamp = [&](int k) {  // dev-only phase stamps (build with -DHWBRJ_STAMPS, run with HWBRJ_DBG)
#ifdef HWBRJ_STAMPS
        if (P.dbg) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tph[k] += t - tlast;
            tlast = t;
        }
#else
        (void) k;
#endif
    };
    ScRaw<SRC> RA, RB;
    load_round(0, RA);
    if (kScPre == 2) load_round(kScRound, RB);
    // Overflow words of the previous round (rank >= 32 in their partition's stage), written after
    // the flush copy-out freed the stage line. Usual form (no partition of that round reached 64):
    // stage index q * 32 + slot (the word goes to index - 32), or kNoPend. Skew form (pskew): the
    // packed q | slot << 11, resolved against the plan (words beyond the stage line go to the
    // directly written chunks).
    constexpr uint32_t kNoPend = 0xFFFFFFFFu;
    uint32_t pq[kScE], pw[kScE];
    bool     pskew = false;
#pragma unroll
    for (int j = 0; j < kScE; j++) pq[j] = kNoPend;
    auto write_pending = [&]() {
        if (!pskew) {
#pragma unroll
            for (int j = 0; j < kScE; j++) stage[pq[j] != kNoPend ? pq[j] - 32u : dummy] = pw[j];
        } else {  // (plan of the previous round: ncb[par ^ 1])
#pragma unroll
            for (int j = 0; j < kScE; j++) {
                const bool     ok = pq[j] != kNoPend;
                const uint32_t qq = ok ? pq[j] & 2047u : 0u, sl = pq[j] >> 11;
                const uint32_t cb = ncb[(par ^ 1u) * F + qq], nch = cb >> kCbBits;
                const bool     st = sl >= nch * 32;
                stage[ok && st ? qq * 32 + sl - nch * 32 : dummy] = pw[j];
                const uint32_t po = ((cb & kCbMask) + (sl >> 5)) * 128 + (sl & 31u) * 4;
                __builtin_amdgcn_raw_buffer_store_b32(pw[j], rpool, ok && !st ? po : kOob, 0, 0);
            }
        }
    };

    // The round's words: hash (consumes R) of the round at `base`; q = F marks elements past len.
    uint32_t q[kScE], w[kScE];
    auto hash = [&](uint32_t base, const ScRaw<SRC>& R) {
        const bool full = base + kScRound <= len;  // uniform
        if (SRC == SRC_TUPLES && MODE != MODE_BASIC_POS && HWBRJ_SC_KEEPY) {
#pragma unroll
            for (int j = 0; j < kScE; j++) asm volatile("" ::"v"(R.y[j]));  // (ScRaw::y)
        }
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            uint32_t x, idx;
            elem(R, base, j, x, idx);
            if (MODE == MODE_BASIC_POS) {
                w[j] = basic_bit(x, R.jb[j], (uint32_t) P.g.m);
                q[j] = w[j] & (F - 1u);
            } else {
                sc_word_lds0<SRC, MODE, FMT>(x, P.g, crc_tab, w[j], q[j]);
            }
            // the word (CrapWow) computed here, among the CRC reads, not after the barrier where the
            // compiler would sink it (phase B is the longer one: 2.66 -> 2.56 ms at the north star)
            asm volatile("" : "+v"(w[j]));
#ifndef HWBRJ_SC_SB
#define HWBRJ_SC_SB 2
#endif
            if ((j % HWBRJ_SC_SB) == HWBRJ_SC_SB - 1) __builtin_amdgcn_sched_barrier(0);  // bound the CRC reads in flight
        }
        if (!full) {
#pragma unroll
            for (int j = 0; j < kScE; j++) {
                uint32_t x, idx;
                elem(R, base, j, x, idx);
                if (idx >= len) q[j] = F;  // invalid: ranked on the dummy counter
            }
        }
    };
    auto round = [&](uint32_t base, ScRaw<SRC>& R) {
        const bool full = base + kScRound <= len;  // uniform
        // ---- A: hash (consumes R), refill R, copy out the last plan, rank
        hash(base, R);
        stamp(0);
        load_round(base + kScPre * kScRound, R);
        uint32_t slot[kScE];  // ranks issued first: their returns overlap the copy-out
#pragma unroll
        for (int j = 0; j < kScE; j++) slot[j] = atomicAdd(&fill[q[j]], 1u);
        flush_copy();
        if (tid == 0) {
            misc[1 + par]        = 0;  // (last read by the previous round's flush_copy)
            misc[3 + (par ^ 1u)] = 0;  // (last read by the previous round's phase B)
        }
        stamp(1);
        bool sk = false;  // a slot >= 63: some partition reaches 64 words this round
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            q[j] |= slot[j] << 11;
            sk |= q[j] >= (63u << 11) && (q[j] & 2047u) < F;
        }
        if (__builtin_amdgcn_ballot_w64(sk) != 0 && lane == 0) misc[3 + par] = 1u;
        stamp(2);
        __syncthreads();  // B1: last plan copied out; every rank of this round taken
        stamp(3);
        // ---- B: overflow words of the previous round, in-stage words of this round, plan
        write_pending();
        const bool skew = __builtin_amdgcn_readfirstlane(misc[3 + par]) != 0;
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            const uint32_t qq = q[j] & 2047u, sl = q[j] >> 11;
            const uint32_t a  = qq * 32 + sl;
            const bool     ok = full || qq < F;
            stage[ok && sl < 32 ? a : dummy] = w[j];
            if (!skew) pq[j] = ok && sl >= 32 ? a : kNoPend;
            else pq[j] = ok && sl >= 32 ? q[j] : kNoPend;
            pw[j] = w[j];
        }
        pskew = skew;
#pragma unroll
        for (int pp = 0; pp < kScPlanPer; pp++) {
            // one thread per partition (F <= 1024): flush plan
            const uint32_t qq  = tid + pp * kScThreads;
            const uint32_t f   = qq < F ? fill[qq] : 0u;
            const uint32_t nch = f >> 5;
            // wave prefix of (chunks, flushes); one LDS atomic per wave for the bases
            const uint32_t v    = nch | (nch ? (1u << 16) : 0u);
            const uint32_t incl = wave_incl_scan_dpp(v);
            const uint32_t tot  = __builtin_amdgcn_readlane(incl, 63);
            uint32_t       wbc = 0, wbf = 0;
            if (lane == 0 && tot) {
                wbc = atomicAdd(&misc[0], tot & 0xFFFFu);
                wbf = atomicAdd(&misc[1 + par], tot >> 16);
            }
            wbc = __builtin_amdgcn_readfirstlane(wbc);
            wbf = __builtin_amdgcn_readfirstlane(wbf);
            if (nch) {
                const uint32_t cb = wbc + (incl & 0xFFFFu) - nch;  // region-local chunk
                ncb[par * F + qq] = cb | (nch << kCbBits);
                flq[wbf + (incl >> 16) - 1] = qq;
                fill[qq]          = f & 31u;
                my_tch[pp] += nch;
                my_tel[pp] += nch * 32;
                for (uint32_t c = 1; c < nch; c++) meta[cb + c] = meta16(qq, 32u);  // direct chunks
            }
        }
        stamp(4);
        __syncthreads();  // B2: plan visible
        stamp(5);
        par ^= 1u;
    };
    uint32_t base = 0;
    if (kScPre == 2) {
        for (; base + kScRound < len; base += 2 * kScRound) {
            round(base, RA);
            round(base + kScRound, RB);
        }
        if (base < len) round(base, RA);
    } else {
        for (; base < len; base += kScRound) round(base, RA);
    }
    // ---- tail: last plan, the last overflow words, then every partial stage as a partial chunk
    {
        flush_copy();
        __syncthreads();
        write_pending();
        __syncthreads();
#pragma unroll
        for (int pp = 0; pp < kScPlanPer; pp++) {  // one thread per partition (F <= 1024): chunk ids of the partial stages (wave scan)
            const uint32_t qq   = tid + pp * kScThreads;
            const uint32_t f    = qq < F ? fill[qq] : 0u;
            const uint32_t has  = f > 0 ? 1u : 0u;
            const uint32_t incl = wave_incl_scan_dpp(has);
            const uint32_t tot  = __builtin_amdgcn_readlane(incl, 63);
            uint32_t       wb   = 0;
            if (lane == 0 && tot) wb = atomicAdd(&misc[0], tot);
            wb = __builtin_amdgcn_readfirstlane(wb);
            if (has) {
                const uint32_t cb = wb + incl - 1u;
                ncb[qq]  = cb;
                meta[cb] = meta16(qq, f);
                my_tch[pp] += 1;
                my_tel[pp] += f;
            }
        }
        __syncthreads();
        // copy-out of the partial stages, 16 bytes per task (words past the count are never read)
        for (uint32_t k = tid; k < F * 8; k += kScThreads) {
            const uint32_t qq = k >> 3, l8 = k & 7;
            const bool     ok = fill[qq] > 0;
            const v4u      v  = *(const v4u*) &stage[qq * 32 + l8 * 4];
            __builtin_amdgcn_raw_buffer_store_b128(v, rpool, ok ? (ncb[qq] * 32 + l8 * 4) * 4 : kOob, 0, 0);
        }
        __syncthreads();
        if (tid == 0) P.wg_used[wg] = misc[0];
        if (P.dbg && tid == 0) {
            for (int k = 0; k < 6; k++) P.dbg[wg * 8 + k] = tph[k];
            P.dbg[wg * 8 + 7] = __builtin_amdgcn_s_memrealtime();  // dev-only: end (100 MHz clock)
        }
        // this workgroup's row of the (workgroup x partition) chunk / element matrices (k_plan
        // scans them column-wise: no global atomics)
#pragma unroll
        for (int pp = 0; pp < kScPlanPer; pp++) {
            const uint32_t qq = tid + pp * kScThreads;
            if (qq < F) {
                P.wgq_chunks[wg * F + qq] = my_tch[pp];
                P.wgq_elems[wg * F + qq]  = my_tel[pp];
            }
        }
    }
}

// ------------------------------------------------- K3p: SWWC partitioning with payloads
// Result materialization (JOIN_RESULT_MATERIALIZE, src/parallel_radix_join_bloom.c:307-312) needs
// every tuple's payload where its word lands: `ppool` shares the chunk layout of `pool`, so a
// survivor names its payload by chunk position. The LDS stage holds words and payloads of
// kPayDepth = 16 {word, payload} slots per partition (128 KiB at F = 1024): a stage line is half a chunk, and
// a partition's chunk is written as two 64-byte halves, rounds apart. Chunk ids are taken when a
// chunk's first half is flushed; per partition cst = current chunk << 1 | 1 while only its first
// half is written (0: none). Halves are numbered chunk * 2 + half: a plan sends the stage line to
// half H0 and, in a skewed round (a partition overfilled by >= 16), its further halves k = 1 ..
// nh - 1 to Bk + k, written directly by the threads holding those words. Pending words (slots past
// the stage line) go to the line after its flush, at slot - 16 * nh; in a skewed round they are
// resolved against the plan before the next round's first barrier. All chunks but a partition's
// last are full, so the per-partition chunk count is ceil(elements / 32).
constexpr uint32_t kPayDepth = 16;
#ifndef HWBRJ_SC_KP
#define HWBRJ_SC_KP 3
#endif
constexpr int      kScKP     = HWBRJ_SC_KP;  // flush tasks per thread per round (4 per half: 16 B of
                                             // words + of payloads); ~512 halves per round on average
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

template <int MODE, int FMT>
__device__ __forceinline__ void scatter_body_pay(const ScatterParams& P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    __shared__ uint32_t crc_tab[128];
    const uint32_t F     = 1u << P.g.log2F;
    const uint32_t SL    = F * kPayDepth + 64;  // stage slots (+ 64 per-lane dummy slots)
    uint2*         stg   = (uint2*) lds;        // {word, payload} per slot
    uint32_t*      fill  = lds + 2 * SL;        // F + 4 (entry F: invalid elements)
    uint32_t*      pl0   = fill + F + 4;        // F: half index of the stage line's flush
    uint32_t*      pl1   = pl0 + F;             // F: Bk | nh << 22
    uint32_t*      cst   = pl1 + F;             // F: current chunk << 1 | 1, or 0
    uint32_t*      tel   = cst + F;             // F: elements of q (this workgroup)
    uint32_t*      flq   = tel + F;             // F: partitions flushed by the last plan
    uint32_t*      misc  = flq + F;             // [0] chunks used, [1 + parity] flushes, [3 + parity] skew
    const int      tid   = threadIdx.x, lane = tid & 63;
    const uint32_t dummy = F * kPayDepth + lane;
    for (uint32_t i = tid; i < F + 1; i += kScPayThreads) fill[i] = 0;
    for (uint32_t i = tid; i < F; i += kScPayThreads) {
        cst[i] = 0;
        tel[i] = 0;
    }
    if (tid < 128) {  // nibble table; f(kSeed) folded into row 0 (as in scatter_body)
        const uint32_t* src = &P.tabs->fwd[0][0];
        uint32_t        v   = src[tid];
        if (tid < 16) {
#pragma unroll
            for (int j = 0; j < 8; j++) v ^= src[j * 16 + ((kSeed >> (4 * j)) & 15u)];
        }
        crc_tab[tid] = v;
    }
    if (tid < 8) misc[tid] = 0;
    if (blockIdx.x == 0 && P.zero_small && tid < 16) P.zero_small[tid] = 0;  // (as scatter_body)
    if (blockIdx.x == 0 && P.zero_word && tid == 0) *P.zero_word = 0;

    const uint64_t n     = P.n;
    const uint64_t units = (n + 3) >> 2;
    const uint64_t G = gridDim.x, wg = blockIdx.x;
    const uint64_t e0  = 4 * (wg * units / G);
    const uint64_t e1r = 4 * ((wg + 1) * units / G);
    const uint64_t e1  = e1r < n ? e1r : n;
    const uint32_t len = __builtin_amdgcn_readfirstlane(e1 > e0 ? (uint32_t) (e1 - e0) : 0u);
    uint16_t* __restrict__ meta = (uint16_t*) P.meta + wg * P.cap;
    const auto rsrc   = buf_rsrc((const uint8_t*) P.src + e0 * 8, len * 8);  // OOB loads return 0
    const auto rpool  = buf_rsrc(P.pool + wg * P.cap * 32, (uint32_t) (P.cap * 128));
    const auto rppool = buf_rsrc(P.ppool + wg * P.cap * 32, (uint32_t) (P.cap * 128));
    const auto rmeta  = buf_rsrc(meta, (uint32_t) (P.cap * 2));
    __syncthreads();

#ifdef HWBRJ_ABL_SPLITH  // dev ablation (results invalid): second halves in a separate array
    auto hword = [&](uint32_t H) { return (H & 1u) * (uint32_t) (P.cap * 16) + (H >> 1) * 16u; };
#else
    auto hword = [&](uint32_t H) { return H * 16u; };  // word offset of half H in the region
#endif
    auto load_round = [&](uint32_t base, v2u (&R)[kScE]) {  // {key, payload} as one 8-byte load
        if (base + kScRound <= len) {
#pragma unroll
            for (int j = 0; j < kScE; j++)
                R[j] = __builtin_amdgcn_raw_buffer_load_b64(rsrc, tid * 8, (base + j * kScPayThreads) * 8, 0);
        } else {
#pragma unroll
            for (int j = 0; j < kScE; j++) {
                const uint32_t i = base + j * kScPayThreads + tid;
                R[j] = __builtin_amdgcn_raw_buffer_load_b64(rsrc, i < len ? i * 8 : kOob, 0, 0);
            }
        }
    };
    uint32_t par = 0;
    // copy-out of the last plan's stage lines: task k = (flush entry k >> 2, 16-byte column k & 3)
    auto flush_copy = [&]() {
        const uint32_t nf = misc[1 + (par ^ 1u)];
        auto task = [&](uint32_t k) {
            const bool     ok = k < nf * 4;
            const uint32_t qq = flq[ok ? k >> 2 : 0];
            const uint32_t l4 = k & 3;
            const uint32_t H  = pl0[qq];
            const v4u      x0 = *(const v4u*) &stg[qq * kPayDepth + l4 * 4];
            const v4u      x1 = *(const v4u*) &stg[qq * kPayDepth + l4 * 4 + 2];
            v4u            vw, vp;  // (de-interleave)
            vw.x = x0.x; vw.y = x0.z; vw.z = x1.x; vw.w = x1.z;
            vp.x = x0.y; vp.y = x0.w; vp.z = x1.y; vp.w = x1.w;
            const uint32_t o  = ok ? (hword(H) + l4 * 4) * 4 : kOob;
            __builtin_amdgcn_raw_buffer_store_b128(vw, rpool, o, 0, 0);
#ifdef HWBRJ_ABL_PNOPST  // dev ablation (results invalid): no payload stores
            if (vp.x == 0x12345678u && vp.y == 0x9abcdef0u)
#endif
            __builtin_amdgcn_raw_buffer_store_b128(vp, rppool, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b16((short) meta16(qq, 32u), rmeta, ok && l4 == 0 && (H & 1u) ? (H >> 1) * 2 : kOob, 0, 0);
        };
#pragma unroll
        for (int i = 0; i < kScKP; i++) task(tid + i * kScPayThreads);
        for (uint32_t k = kScKP * kScPayThreads + tid; k < nf * 4; k += kScPayThreads) task(k);  // rare
    };
    // previous round's pending words: q | slot << 11 (kNoPend: none); resolved into a stage index
    // (ps) or, in a skewed round, written directly into the plan's further halves
    constexpr uint32_t kNoPend = 0xFFFFFFFFu;
    uint32_t pq[kScE], pw[kScE], pp[kScE], ps[kScE];
    bool     pskew = false;
#pragma unroll
    for (int j = 0; j < kScE; j++) pq[j] = kNoPend;
    auto resolve_pending = [&]() {
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            const bool     ok = pq[j] != kNoPend;
            const uint32_t qq = ok ? pq[j] & 2047u : 0u, sl = pq[j] >> 11;
            uint32_t       nh = 1, Bk = 0;
            if (pskew) {
                const uint32_t b = pl1[qq];
                nh = b >> 22;
                Bk = b & ((1u << 22) - 1u);
            }
            const uint32_t k      = sl >> 4;
            const bool     direct = ok && pskew && k < nh;
            if (pskew) {  // (uniform; a skewed round is rare, so the waits it costs are too)
                const uint32_t o = direct ? (hword(Bk + k) + (sl & 15u)) * 4 : kOob;
                __builtin_amdgcn_raw_buffer_store_b32(pw[j], rpool, o, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(pp[j], rppool, o, 0, 0);
            }
            ps[j] = ok && !direct ? qq * kPayDepth + sl - nh * kPayDepth : dummy;
        }
    };
    auto write_pending = [&]() {
#pragma unroll
        for (int j = 0; j < kScE; j++) stg[ps[j]] = make_uint2(pw[j], pp[j]);
    };

    v2u RA[kScE];
    load_round(0, RA);
    auto round = [&](uint32_t base) {
        const bool full = base + kScRound <= len;  // uniform
        uint32_t   q[kScE], w[kScE], p[kScE];
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            sc_word_lds0<SRC_TUPLES, MODE, FMT>(RA[j].x, P.g, crc_tab, w[j], q[j]);
            p[j] = RA[j].y;
            if ((j % HWBRJ_SC_SB) == HWBRJ_SC_SB - 1) __builtin_amdgcn_sched_barrier(0);
        }
        if (!full) {
#pragma unroll
            for (int j = 0; j < kScE; j++)
                if (base + j * kScPayThreads + tid >= len) q[j] = F;  // invalid: ranked on the dummy counter
        }
        load_round(base + kScRound, RA);
        flush_copy();
        resolve_pending();
        if (tid == 0) {
            misc[1 + par]        = 0;
            misc[3 + (par ^ 1u)] = 0;
        }
        bool sk = false;  // a slot >= 31: some partition reaches 32 words this round
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            q[j] |= atomicAdd(&fill[q[j]], 1u) << 11;
            sk |= q[j] >= (31u << 11) && (q[j] & 2047u) < F;
        }
        if (__builtin_amdgcn_ballot_w64(sk) != 0 && lane == 0) misc[3 + par] = 1u;
        __syncthreads();  // B1: last plan copied out, pending resolved; every rank taken
        write_pending();
        const bool skew = __builtin_amdgcn_readfirstlane(misc[3 + par]) != 0;
#pragma unroll
        for (int j = 0; j < kScE; j++) {
            const uint32_t qq = q[j] & 2047u, sl = q[j] >> 11;
            const bool     ok = full || qq < F;
            stg[ok && sl < kPayDepth ? qq * kPayDepth + sl : dummy] = make_uint2(w[j], p[j]);
            pq[j]  = ok && sl >= kPayDepth ? q[j] : kNoPend;
            pw[j]  = w[j];
            pp[j]  = p[j];
        }
        pskew = skew;
        {  // one thread per partition (F <= 1024): flush plan
            const uint32_t qq   = tid;
            const uint32_t f    = qq < F ? fill[qq] : 0u;
            const uint32_t nh   = f >> 4;
            const uint32_t cs   = qq < F ? cst[qq] : 0u;
            const uint32_t hcur = cs & 1u;
            const uint32_t newc = nh ? ((hcur + nh + 1u) >> 1) - hcur : 0u;  // chunks to allocate
            const uint32_t v    = newc | (nh ? (1u << 16) : 0u);
            const uint32_t incl = wave_incl_scan_dpp(v);
            const uint32_t tot  = __builtin_amdgcn_readlane(incl, 63);
            uint32_t       wbc = 0, wbf = 0;
            if (lane == 0 && tot) {
                wbc = atomicAdd(&misc[0], tot & 0xFFFFu);
                wbf = atomicAdd(&misc[1 + par], tot >> 16);
            }
            wbc = __builtin_amdgcn_readfirstlane(wbc);
            wbf = __builtin_amdgcn_readfirstlane(wbf);
            if (nh) {
                const uint32_t cb = wbc + (incl & 0xFFFFu) - newc;
                const uint32_t H0 = hcur ? cs | 1u : cb * 2u;  // (cs = chunk << 1 | 1)
                const uint32_t Bk = cb * 2u - hcur;            // half of further half k: Bk + k
                pl0[qq] = H0;
                pl1[qq] = Bk | (nh << 22);
                flq[wbf + (incl >> 16) - 1] = qq;
                fill[qq] = f & (kPayDepth - 1u);
                tel[qq] += nh * kPayDepth;
                for (uint32_t k = 1; k < nh; k++)  // chunks completed by a direct half
                    if ((Bk + k) & 1u) meta[(Bk + k) >> 1] = meta16(qq, 32u);
                const uint32_t Hl = nh == 1 ? H0 : Bk + nh - 1u;  // last half written
                cst[qq] = (Hl & 1u) ? 0u : (Hl | 1u);
            }
        }
        __syncthreads();  // B2: plan visible
        par ^= 1u;
    };
    for (uint32_t base = 0; base < len; base += kScRound) round(base);
    // ---- tail: last plan, the last pending words, then every partial stage as a partial half
    {
        flush_copy();
        resolve_pending();
        __syncthreads();
        write_pending();
        __syncthreads();
        {
            const uint32_t qq   = tid;
            const uint32_t f    = qq < F ? fill[qq] : 0u;
            const uint32_t cs   = qq < F ? cst[qq] : 0u;
            const uint32_t hcur = cs & 1u;
            const uint32_t need = f > 0 && !hcur ? 1u : 0u;
            const uint32_t incl = wave_incl_scan_dpp(need);
            const uint32_t tot  = __builtin_amdgcn_readlane(incl, 63);
            uint32_t       wb   = 0;
            if (lane == 0 && tot) wb = atomicAdd(&misc[0], tot);
            wb = __builtin_amdgcn_readfirstlane(wb);
            if (f > 0 || hcur) {
                const uint32_t ch = hcur ? cs >> 1 : wb + incl - 1u;
                meta[ch] = meta16(qq, hcur * kPayDepth + f);
                pl0[qq]  = ch * 2u + hcur;
                tel[qq] += f;
            }
        }
        __syncthreads();
        for (uint32_t k = tid; k < F * 4; k += kScPayThreads) {
            const uint32_t qq = k >> 2, l4 = k & 3;
            const uint32_t o  = fill[qq] > 0 ? (hword(pl0[qq]) + l4 * 4) * 4 : kOob;
            const v4u      x0 = *(const v4u*) &stg[qq * kPayDepth + l4 * 4];
            const v4u      x1 = *(const v4u*) &stg[qq * kPayDepth + l4 * 4 + 2];
            v4u            vw, vp;
            vw.x = x0.x; vw.y = x0.z; vw.z = x1.x; vw.w = x1.z;
            vp.x = x0.y; vp.y = x0.w; vp.z = x1.y; vp.w = x1.w;
            __builtin_amdgcn_raw_buffer_store_b128(vw, rpool, o, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(vp, rppool, o, 0, 0);
        }
        __syncthreads();
        if (tid == 0) P.wg_used[wg] = misc[0];
        for (uint32_t qq = tid; qq < F; qq += kScPayThreads) {
            P.wgq_chunks[wg * F + qq] = (tel[qq] + 31u) >> 5;
            P.wgq_elems[wg * F + qq]  = tel[qq];
        }
    }
}

// ====================================================== K4: planning scan and chunk lists
// List entries carry the chunk's element count, so consumers never read `meta`:
//   entry = chunk_id | (count - 1) << kListIdBits   (count 1..32)
constexpr uint32_t kListIdBits = 27;
constexpr uint32_t kListIdMask = (1u << kListIdBits) - 1u;
constexpr uint32_t kNoEntry    = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t list_count(uint32_t e) { return (e >> kListIdBits) + 1u; }

// LDS byte addresses as integers (address arithmetic the compiler cannot fold into a select)
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
__device__ __forceinline__ uint32_t lds_byte_addr(const uint32_t* p) {
    return (uint32_t) (uintptr_t) (const lds_u32_t*) p;
}
__device__ __forceinline__ void lds_store_u32(uint32_t byte_addr, uint32_t v) {
    *(lds_u32_t*) (uintptr_t) byte_addr = v;
}
// a * b + c for a, b < 2^24 (v_mad_u32_u24): the caller guarantees the ranges, which the compiler
// cannot see (it would mask the operands or fall back to v_mul_lo_u32)
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// (a << s) + b as one v_lshl_add_u32 (keeps a running sum the compiler would re-derive per use)
__device__ __forceinline__ uint32_t shl_add(uint32_t a, uint32_t s, uint32_t b) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(s), "v"(b));
    return r;
}

// Column-wise exclusive scan of the scatter's (workgroup x partition) matrices: every (wg, q) gets
// its offset inside q's chunk list, and every partition its chunk / element totals. A block takes
// kPlanCols partitions x 64 row groups (thread t: column t % kPlanCols, row group t / kPlanCols):
// every row is loaded by an independent load, so the scan costs one memory latency instead of one
// per workgroup row, and F / kPlanCols blocks share the 2 x G x F x 4 bytes (64 CUs at F = 1024).
#ifndef HWBRJ_PLANCOLS
#define HWBRJ_PLANCOLS 16
#endif
constexpr uint32_t kPlanCols  = HWBRJ_PLANCOLS;
constexpr uint32_t kPlanRGs   = 1024 / kPlanCols;   // row groups per block
constexpr uint32_t kPlanMaxRG = 512 / kPlanRGs;     // rows per row group: G <= 512 scatter workgroups

__global__ __launch_bounds__(1024) void k_plan(const uint32_t* __restrict__ wgq_chunks,
                                               const uint32_t* __restrict__ wgq_elems, uint32_t G,
                                               uint32_t log2F, uint32_t* __restrict__ wgq_off,
                                               uint32_t* __restrict__ colc,
                                               uint64_t* __restrict__ cole) {
    __shared__ uint32_t tc[16][kPlanCols];  // per wave and column: chunk sum of its row groups
    __shared__ uint64_t te[16][kPlanCols];
    const uint32_t F = 1u << log2F;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t cl = threadIdx.x % kPlanCols, rg = threadIdx.x / kPlanCols;
    const uint32_t col = blockIdx.x * kPlanCols + cl;
    const bool     okc = col < F;
    const uint32_t RG  = (G + kPlanRGs - 1) / kPlanRGs;
    const uint32_t r0  = min(G, rg * RG), r1 = min(G, r0 + RG);
    uint32_t       pre[kPlanMaxRG];
    uint32_t       c = 0;
    uint64_t       e = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPlanMaxRG; j++) {
        const uint32_t r  = r0 + j;
        const bool     ok = okc && r < r1;
        const uint32_t cc = ok ? wgq_chunks[(uint64_t) r * F + col] : 0u;
        const uint32_t ee = ok ? wgq_elems[(uint64_t) r * F + col] : 0u;
        pre[j] = c;
        c += cc;
        e += ee;
    }
    // inclusive scan of c over the wave's 4 row groups (lanes 16 apart), sum of e
    uint32_t inc = c;
#pragma unroll
    for (uint32_t d = kPlanCols; d < 64; d *= 2) {
        const uint32_t y = __shfl_up(inc, d);
        if (lane >= d) inc += y;
        e += __shfl_xor(e, d);
    }
    if (lane >= 64 - kPlanCols) tc[w][cl] = inc;
    if (lane < kPlanCols) te[w][cl] = e;
    __syncthreads();
    uint32_t base = inc - c;
    for (uint32_t v = 0; v < w; v++) base += tc[v][cl];
#pragma unroll
    for (uint32_t j = 0; j < kPlanMaxRG; j++) {
        const uint32_t r = r0 + j;
        if (okc && r < r1) wgq_off[(uint64_t) r * F + col] = base + pre[j];
    }
    if (w == 0 && lane < kPlanCols && okc) {
        uint32_t tcs = 0;
        uint64_t tes = 0;
        for (int v = 0; v < 16; v++) {
            tcs += tc[v][cl];
            tes += te[v][cl];
        }
        colc[col] = tcs;
        cole[col] = tes;
    }
}

// One block per scatter region: every chunk of the region gets its slot in its partition's list
// (slots of (wg, q) start at list_start[q] + wgq_off[wg][q]). The region's metas are taken in
// batches of kLfBatch, counting-sorted by partition in LDS and written out as contiguous runs per
// partition, so the list stores are coalesced.
constexpr uint32_t kLfThreads = 1024;
#ifndef HWBRJ_LFPER
#define HWBRJ_LFPER 28
#endif
constexpr uint32_t kLfPer     = HWBRJ_LFPER;
constexpr uint32_t kLfBatch   = kLfThreads * kLfPer;
static_assert(kLfBatch <= (1u << 17), "batch-local index in 17 bits of a packed entry");

__global__ __launch_bounds__(kLfThreads) void k_list_fill(const uint32_t* __restrict__ meta,
                                                          const uint32_t* __restrict__ wg_used,
                                                          uint64_t cap, uint32_t log2F,
                                                          const uint32_t* __restrict__ wgq_off,
                                                          const uint32_t* __restrict__ colc,
                                                          const uint64_t* __restrict__ cole,
                                                          uint32_t CH, uint32_t nseg,
                                                          uint32_t* __restrict__ list_start,
                                                          uint64_t* __restrict__ elem_start,
                                                          uint32_t* __restrict__ item_start,
                                                          uint32_t* __restrict__ list) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t F    = 1u << log2F;
    // sorted batch entries, packed: partition | (count - 1) << 10 | batch-local index << 15
    // (F <= 1024, kLfBatch <= 2^15)
    uint32_t*      pk   = lds;                // [kLfBatch]
    uint32_t*      cnt  = pk + kLfBatch;      // [F]
    uint32_t*      off  = cnt + F;            // [F] batch offsets
    uint32_t*      cur  = off + F;            // [F] next list slot
    uint32_t*      dcur = cur + F;            // [F] cur - off: the entry sorted to pos goes to list[dcur[q] + pos]
    uint32_t*      wtot = dcur + F;           // [16] wave totals of the scan
    const uint32_t tid  = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wg   = blockIdx.x;
    {
        // exclusive scans over the F <= 1024 partitions of the column totals (k_plan): list starts
        // (every block), element and probe-item starts (block 0 publishes all three)
        __shared__ uint32_t sc_c[16], sc_i[16];
        __shared__ uint64_t sc_e[16];
        const uint32_t c  = tid < F ? colc[tid] : 0u;
        const uint32_t it = ((c + CH - 1) / CH) * nseg;
        const uint64_t e  = tid < F ? cole[tid] : 0ull;
        uint32_t ic = wave_incl_scan(c), ii = wave_incl_scan(it);
        uint64_t ie = e;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t t = __shfl_up(ie, off, 64);
            if ((int) lane >= off) ie += t;
        }
        if (lane == 63) {
            sc_c[wave] = ic;
            sc_i[wave] = ii;
            sc_e[wave] = ie;
        }
        __syncthreads();
        for (uint32_t v = 0; v < wave; v++) {
            ic += sc_c[v];
            ii += sc_i[v];
            ie += sc_e[v];
        }
        if (tid < F) {
            cur[tid] = ic - c + wgq_off[wg * F + tid];
            cnt[tid] = 0;
            if (wg == 0) {
                list_start[tid + 1] = ic;
                item_start[tid + 1] = ii;
                elem_start[tid + 1] = ie;
            }
        }
        if (wg == 0 && tid == 0) {
            list_start[0] = 0;
            item_start[0] = 0;
            elem_start[0] = 0;
        }
    }
    __syncthreads();
    const uint64_t region = (uint64_t) wg * cap;
    const uint32_t used   = wg_used[wg];
    const uint16_t* __restrict__ rmeta = (const uint16_t*) meta + region;  // meta16 entries
    // the next batch's metas are loaded while the current one is sorted and written
    uint32_t nx[kLfPer];
#pragma unroll
    for (int j = 0; j < (int) kLfPer; j++) {
        const uint32_t i = tid + j * kLfThreads;
        nx[j]            = i < used ? rmeta[i] : kNoEntry;
    }
    for (uint32_t b0 = 0; b0 < used; b0 += kLfBatch) {
        const uint32_t nb = min(kLfBatch, used - b0);
        // p: partition | (count - 1) << 10 | rank in the partition's batch run << 15
        uint32_t p[kLfPer];
#pragma unroll
        for (int j = 0; j < (int) kLfPer; j++) {
            const uint32_t m = nx[j];
            p[j]             = kNoEntry;
            if (m != kNoEntry) p[j] = m | (atomicAdd(&cnt[m & 1023u], 1u) << 15);  // (m: meta16)
        }
        if (b0 + kLfBatch < used) {
#pragma unroll
            for (int j = 0; j < (int) kLfPer; j++) {
                const uint32_t i = b0 + kLfBatch + tid + j * kLfThreads;
                nx[j]            = i < used ? rmeta[i] : kNoEntry;
            }
        }
        __syncthreads();
        // exclusive scan of cnt over F (<= 1024) partitions: one per thread, wave scans + totals
        const uint32_t c    = tid < F ? cnt[tid] : 0u;
        const uint32_t incl = wave_incl_scan(c);
        if (lane == 63) wtot[wave] = incl;
        __syncthreads();
        uint32_t wbase = 0;
        for (uint32_t w = 0; w < wave; w++) wbase += wtot[w];
        if (tid < F) {
            const uint32_t o = wbase + incl - c;
            off[tid]  = o;
            dcur[tid] = cur[tid] - o;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < (int) kLfPer; j++) {
            if (p[j] == kNoEntry) continue;
            const uint32_t q = p[j] & 1023u;
            pk[off[q] + (p[j] >> 15)] = (p[j] & 0x7FFFu) | ((tid + j * kLfThreads) << 15);
        }
        __syncthreads();
        for (uint32_t pos = tid; pos < nb; pos += kLfThreads) {
            const uint32_t v = pk[pos];
            list[dcur[v & 1023u] + pos] = (uint32_t) (region + b0 + (v >> 15)) | (((v >> 10) & 31u) << kListIdBits);
        }
        __syncthreads();
        if (tid < F) {
            cur[tid] += cnt[tid];
            cnt[tid] = 0;
        }
        __syncthreads();
    }
}

// ======================================================== chunk-walking helpers (8 lanes)
// A sweep covers 128 * NPQ chunks of a chunk list: 8 threads share a chunk (16 B each) and every
// thread issues NPQ independent list loads, then NPQ independent chunk loads.
template <int NPQ>
struct Sweep {
    uint4    v[NPQ];
    uint32_t n[NPQ];   // valid words of this thread's quad (0..4)
    uint32_t id[NPQ];  // list entries' chunk ids (load_chunks_u; read by the materializing probe)
};

template <int NPQ>
__device__ __forceinline__ void load_list(const uint32_t* __restrict__ list, uint32_t lb, uint32_t le,
                                          uint32_t (&ent)[NPQ]) {
    const uint32_t cslot = threadIdx.x >> 3;
#pragma unroll
    for (int j = 0; j < NPQ; j++) {
        const uint32_t l = lb + cslot + (uint32_t) j * 128u;
        ent[j]           = l < le ? list[l] : kNoEntry;
    }
}

template <int NPQ>
__device__ __forceinline__ void load_chunks(const uint32_t* __restrict__ pool, const uint32_t (&ent)[NPQ],
                                            Sweep<NPQ>& S) {
    const uint32_t l8 = threadIdx.x & 7;
#pragma unroll
    for (int j = 0; j < NPQ; j++) {
        if (ent[j] != kNoEntry) {
            const uint32_t cnt = list_count(ent[j]);
            const uint32_t first = l8 * 4;
            S.n[j] = cnt > first ? min(cnt - first, 4u) : 0u;
            S.v[j] = *(const uint4*) &pool[(uint64_t) (ent[j] & kListIdMask) * 32 + l8 * 4];
        } else {
            S.n[j] = 0;
            S.v[j] = make_uint4(0, 0, 0, 0);
        }
    }
}

// Branch-free variants (a fixed number of vector-memory instructions per call, so the compiler
// can wait for exactly the loads it needs instead of vmcnt(0)). lb < le is required: slots past le
// re-read entry le-1; load_chunks_u gives them count 0 (validity comes from lb/le, not from the
// loaded value, so nothing forces an early wait on the list load).
template <int NPQ>
__device__ __forceinline__ void load_list_u(const uint32_t* __restrict__ list, uint32_t lb, uint32_t le,
                                            uint32_t (&ent)[NPQ]) {
    const uint32_t cslot = threadIdx.x >> 3;
#pragma unroll
    for (int j = 0; j < NPQ; j++) ent[j] = list[min(lb + cslot + (uint32_t) j * 128u, le - 1u)];
}

// NT: non-temporal chunk loads (the chunks are read once)
template <int NPQ, bool NT = false>
__device__ __forceinline__ void load_chunks_u(const uint32_t* __restrict__ pool, const uint32_t (&ent)[NPQ],
                                              uint32_t lb, uint32_t le, Sweep<NPQ>& S) {
    const uint32_t l8 = threadIdx.x & 7, cslot = threadIdx.x >> 3;
#pragma unroll
    for (int j = 0; j < NPQ; j++) {
        if (NT) {
            const v4u v = __builtin_nontemporal_load((const v4u*) &pool[(uint64_t) (ent[j] & kListIdMask) * 32 + l8 * 4]);
            S.v[j]      = make_uint4(v.x, v.y, v.z, v.w);
        } else
            S.v[j] = *(const uint4*) &pool[(uint64_t) (ent[j] & kListIdMask) * 32 + l8 * 4];
        // valid words of this thread's quad: clamp(count - 4 * l8, 0, 4), 0 past le
        const int32_t  d     = (int32_t) (ent[j] >> kListIdBits) + 1 - (int32_t) (l8 * 4);
        S.n[j]  = lb + cslot + (uint32_t) j * 128u < le ? (uint32_t) min(max(d, 0), 4) : 0u;
        S.id[j] = ent[j] & kListIdMask;
    }
}

template <int NPQ>
__device__ __forceinline__ uint32_t sweep_word(const Sweep<NPQ>& S, int j, int t) {
    return t == 0 ? S.v[j].x : t == 1 ? S.v[j].y : t == 2 ? S.v[j].z : S.v[j].w;
}


// ======================================================================== K6: R build
// One workgroup per partition q, one pass over q's chunk list per slice segment. The list is
// walked in groups of kBPQ sweeps (kBSweep chunks each); a group's list entries and chunks are
// loaded while the previous group is processed:
//   * every word sets its filter bits in the LDS slice segment (ds_or), the segment is written
//     once at the end (bloom add, src/bloom_filter.c:73-132);
//   * in the last segment's pass every sweep's codes are counting-sorted by join sub-partition in
//     an LDS stage and written coalesced to the sweep's own kBSlot-word slot of out_codes, with a
//     (sweep, sub) run table (pass-2 of R, src/parallel_radix_join_bloom.c:703-748). The join reads
//     (q, sub) as the sub's runs in the slots of q's sweeps.
#ifndef HWBRJ_BPQ
#define HWBRJ_BPQ 2
#endif
constexpr int      kBPQ    = HWBRJ_BPQ;       // sweeps per group (chunk quads per thread)
#ifndef HWBRJ_BD_NT
#define HWBRJ_BD_NT 0
#endif
constexpr bool     kBdNT   = HWBRJ_BD_NT != 0;  // non-temporal chunk loads in the build
constexpr uint32_t kBSweep = 128u;            // chunks per sweep (8 threads per chunk)
constexpr uint32_t kBSlot  = kBSweep * 32u;   // out_codes words per sweep (4096)

// PAY (materialization): the payload of every R word (ppool, same chunk positions) is written to
// out_pay at the word's sorted position.
template <int KIND, bool PAY = false>
__global__ __launch_bounds__(1024) void k_build(BuildParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const Geometry& g      = P.g;
    const uint32_t  NSUB   = 1u << g.log2NSUB;
    constexpr bool  slices = KIND != KIND_PASS;
    const bool      wr     = slices && !P.no_slices;  // this rank builds the slices (uniform)
    const uint32_t  segw   = slices ? g.seg_words : 0;  // multiple of 4
    uint32_t*       slice  = lds;
    uint32_t*       inv    = slice + segw;
    uint32_t*       stage  = inv + 128;       // kBSlot
    uint32_t*       cnt    = stage + kBSlot;  // 2 x 64: ranks of a sweep by sub (by sweep parity)
    const uint32_t  ql     = blockIdx.x;       // list / sweep tables are indexed by ql
    const uint32_t  q      = P.q_base + ql;    // the partition (codes, slices)
    const int       tid    = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    load_tab(inv, &P.tabs->inv[0][0]);
    if (tid < 128) cnt[tid] = 0;
    uint32_t nsw = 0;  // sweeps sorted so far (selects the counter buffer)
    const uint32_t l0 = P.list_start[ql], l1 = P.list_start[ql + 1];
    const uint32_t sw0  = P.sweep_start[ql];
    const uint32_t nseg = wr ? g.nseg : 1;
    constexpr uint32_t GRP = kBSweep * kBPQ;
    for (uint32_t seg = 0; seg < nseg; seg++) {
        for (uint32_t i = tid; i < segw; i += blockDim.x) slice[i] = 0;
        __syncthreads();
        const bool  last = seg + 1 == nseg;
        // list entries two groups ahead, chunks one group ahead: a group's chunk loads never wait
        // for the list loads just issued (one exposed memory latency per group otherwise)
        uint32_t    eB[kBPQ], eC[kBPQ];
        Sweep<kBPQ> SA, SB, PA, PB;  // words; payloads (PAY)
        if (l0 < l1) {
            uint32_t eA[kBPQ];
            load_list_u<kBPQ>(P.list, l0, l1, eA);
            const uint32_t n1 = min(l0 + GRP, l1 - 1u);
            load_list_u<kBPQ>(P.list, n1, min(n1 + GRP, l1), eB);
            load_chunks_u<kBPQ, kBdNT>(P.pool, eA, l0, l1, SA);
            if (PAY) load_chunks_u<kBPQ>(P.ppool, eA, l0, l1, PA);
        }
        for (uint32_t lb = l0; lb < l1; lb += GRP) {
            const uint32_t nb = min(lb + GRP, l1 - 1u);  // next group (re-reads the last entry past the end)
            const uint32_t ne = min(nb + GRP, l1);
            const uint32_t nnb = min(nb + GRP, l1 - 1u);  // the group after it (its list entries)
            load_chunks_u<kBPQ, kBdNT>(P.pool, eB, nb, ne, SB);
            if (PAY) load_chunks_u<kBPQ>(P.ppool, eB, nb, ne, PB);
            load_list_u<kBPQ>(P.list, nnb, min(nnb + GRP, l1), eC);
#pragma unroll
            for (int jj = 0; jj < kBPQ; jj++) {
                const uint32_t sb = lb + (uint32_t) jj * kBSweep;  // first list position of the sweep
                if (sb >= l1) break;  // uniform
                uint32_t c[4], rk[4];
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const bool     ok = (uint32_t) t < SA.n[jj];
                    const uint32_t w  = sweep_word(SA, jj, t);
#ifndef HWBRJ_ABL_BNOBITS
                    if (wr && ok) {
                        const Loc L = locate<KIND>(w, g, inv, q);
                        if (L.seg == seg) apply_bits<KIND, true>(L, g, slice);
                    }
#endif
                    c[t]  = decode_k<KIND>(w, q, g);
                    rk[t] = 0xFFFFFFFFu;
#ifndef HWBRJ_ABL_BNOSORT
                    if (last && ok) rk[t] = atomicAdd(&cnt[(nsw & 1u) * 64 + ((c[t] >> g.sub_shift) & (NSUB - 1u))], 1u);
#else
                    if (ok && c[t] == 0x12345678u) P.out_codes[0] = c[t];  // dev ablation: keep the loads live
#endif
                }
#ifdef HWBRJ_ABL_BNOSORT
                if (last && (uint32_t) tid < NSUB) {  // dev ablation (results invalid): empty runs
                    const uint64_t r = (uint64_t) (sw0 + (sb - l0) / kBSweep) * NSUB + tid;
                    P.run_cnt[r]     = 0;
                    P.run_off[r]     = 0;
                }
                continue;
#endif
                if (!last) continue;
                const uint32_t sw = sw0 + (sb - l0) / kBSweep;
                __syncthreads();  // B1: every rank of the sweep taken (and the last sweep copied out)
                // every wave: run offsets of the sweep (DPP scan over the NSUB counters), so no
                // second barrier; wave 0 writes the (sweep, sub) run table and clears the other
                // counter buffer (last read before this B1, next used after B3)
                uint32_t* cb = cnt + (nsw & 1u) * 64;
                const uint32_t cs   = (uint32_t) lane < NSUB ? cb[lane] : 0u;
                const uint32_t incl = wave_incl_scan_dpp(cs);
                const uint32_t tot  = __builtin_amdgcn_readlane(incl, 63);
                if (wave == 0) {
                    if ((uint32_t) lane < NSUB) {
                        const uint64_t r = (uint64_t) sw * NSUB + lane;
                        P.run_cnt[r]     = cs;
                        P.run_off[r]     = incl - cs;
                    }
                    cnt[((nsw & 1u) ^ 1u) * 64 + lane] = 0;
                }
#pragma unroll
                for (int t = 0; t < 4; t++) {
                    const uint32_t sub = (c[t] >> g.sub_shift) & (NSUB - 1u);
                    const uint32_t o   = (uint32_t) __shfl((int) (incl - cs), (int) sub, 64) + rk[t];
                    if (rk[t] != 0xFFFFFFFFu) {
                        stage[o] = c[t];
                        if (PAY) P.out_pay[(uint64_t) sw * kBSlot + o] = sweep_word(PA, jj, t);
                    }
                }
                nsw++;
                __syncthreads();  // B3: the sweep is sorted
                uint32_t* __restrict__ dst = P.out_codes + (uint64_t) sw * kBSlot;
                if (!PAY && P.kbits == 18) {  // 18-bit keys: 36 bytes per 16 codes (uniform)
                    const uint32_t i = tid;   // (kBSlot / 16 groups: threads below 256)
                    if (i < kBSlot / 16) {
                        uint32_t o[9];
                        pack18x16((const v4u*) stage + 4 * i, g.hash_shift, o);
                        const auto rd = buf_rsrc(dst, (tot + 15u) / 16u * 36u);  // (inside the slot)
                        __builtin_amdgcn_raw_buffer_store_b128(v4u{o[0], o[1], o[2], o[3]}, rd, i * 36u, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(v4u{o[4], o[5], o[6], o[7]}, rd, i * 36u + 16u, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b32(o[8], rd, i * 36u + 32u, 0, 0);
                    }
                } else if (!PAY && P.kbits) {  // 24-bit keys: one 12-byte store per 4 codes (uniform)
                    const uint32_t i = tid;  // kBSlot / 4 == blockDim.x quads
                    const v4u      v = ((const v4u*) stage)[i];
                    __builtin_amdgcn_raw_buffer_store_b96(pack3x4(v, g.hash_shift), buf_rsrc(dst, (tot + 3u) / 4u * 12u),
                                                          i * 12u, 0, 0);
                } else {
                    for (uint32_t i = tid; i < tot; i += blockDim.x) dst[i] = stage[i];
                }
            }
#pragma unroll
            for (int jj = 0; jj < kBPQ; jj++) {
                SA.v[jj] = SB.v[jj];
                SA.n[jj] = SB.n[jj];
                if (PAY) PA.v[jj] = PB.v[jj];
                eB[jj]   = eC[jj];
            }
        }
        __syncthreads();
        if (wr) {
            uint4*       dst = (uint4*) (P.slices + ((uint64_t) q * g.nseg + seg) * segw);
            const uint4* src = (const uint4*) slice;
            for (uint32_t i = tid; i < segw / 4; i += blockDim.x) dst[i] = src[i];
        }
        __syncthreads();
    }
}

// ======================================================================== K7: S probe
// Items = (partition q, slice segment, range of <= kProbeCH chunks of q's list); workgroups take
// contiguous item ranges, so a slice segment is (re)loaded only when (q, seg) changes. The next
// item's list entries and chunks are loaded while the current one is tested. Survivors are
// written into the item's own region grouped by join sub-partition (LDS counters + one scan), so
// the join reads them in place: surv_cnt[it][sub] / surv_off[it][sub] describe the runs.
#ifndef HWBRJ_PC
#define HWBRJ_PC 3
#endif
#ifndef HWBRJ_SCR1
#define HWBRJ_SCR1 128
#endif
constexpr int      kPC      = HWBRJ_PC;       // chunk quads per thread per item
#ifndef HWBRJ_PR_NT
#define HWBRJ_PR_NT 0
#endif
constexpr bool     kPrNT    = HWBRJ_PR_NT != 0;  // non-temporal chunk loads in the probe
constexpr uint32_t kProbeCH = 128u * kPC;     // chunks per probe item (1024 threads, 8 per chunk)
// compacted survivors (first-bit candidates for KIND_BLOCK_PKK, whose rate is higher) per wave
// and item in the LDS scratch, and the dense ranking rounds per wave
#ifndef HWBRJ_SCRK
#define HWBRJ_SCRK 256
#endif
template <int KIND> constexpr uint32_t scr_cap() {
    return KIND == KIND_BLOCK_PKK || KIND == KIND_BASIC_KK ? (uint32_t) HWBRJ_SCRK
                                                                                     : (uint32_t) HWBRJ_SCR1;
}
// Dev ablations of the probe's parts (dev builds only; results invalid except `filtered`):
// 1 = loads + test + barrier only, 2 = + the compaction, 3 = everything but the copy-out.
#ifndef HWBRJ_ABL_PROBE
#define HWBRJ_ABL_PROBE 0
#endif
constexpr int kAblProbe = HWBRJ_ABL_PROBE;
// The counting probe's copy-out: b128 stores per thread per piece (a fixed count: vmcnt), so its
// stage holds at most kPco * 4096 words. Every store instruction costs its whole wave's issue and
// data path even when its lanes are out of range (the copy-out of 3 per thread was 0.21 ms of the
// north star's 1.08 ms probe while its stage held 648 quads: profiles/r04/probe_split.txt).
#ifndef HWBRJ_PCO
#define HWBRJ_PCO 1
#endif
#ifndef HWBRJ_PCO_AUX
#define HWBRJ_PCO_AUX 0
#endif
constexpr int kPco = HWBRJ_PCO < kPC ? HWBRJ_PCO : kPC;
// without slices (PRO, the global-bitmap fallback) the stage can hold a whole item: kPC stores
template <int KIND> constexpr int probe_pco() { return KIND == KIND_PASS ? kPC : kPco; }

__device__ __forceinline__ uint32_t find_q(const uint32_t* item_start, uint32_t F, uint32_t it) {
    uint32_t lo = 0, hi = F - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (item_start[mid] <= it) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Items of partition q are numbered segment-major: local = seg * npieces + piece, where piece p
// covers list positions [lq0 + p * CH, min(lq1, lq0 + (p + 1) * CH)). Survivors of an item are
// written at seg * surv_seg_stride + lb * 32 (lb = first list position of the piece).

// PAY (materialization): every survivor's chunk position goes to surv_pos beside its code (the
// words are ranked one by one and stored directly, no LDS stage).
template <int KIND, bool SEG1, bool PAY = false>
__global__ __launch_bounds__(1024) void k_probe(ProbeParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr uint32_t NT  = 1024;
    const Geometry& g      = P.g;
    const uint32_t  F      = 1u << g.log2F;
    const uint32_t  NSUB   = 1u << g.log2NSUB;
    constexpr bool  slices = KIND != KIND_PASS;
    constexpr bool  onebit = KIND == KIND_BLOCK_PK1 || KIND == KIND_BASIC_K1 || KIND == KIND_BLOCK_PKK ||
                             KIND == KIND_BASIC_KK;
    // onebit tests only the first bit: test the rest (basic: from the global bitmap)
    constexpr bool  refine = KIND == KIND_BLOCK_PKK || KIND == KIND_BASIC_KK;
    constexpr int   NW     = kPC * 4;   // words per thread per item
    const uint32_t  segw   = slices ? g.seg_words : 0;  // multiple of 4
    const uint32_t  scap   = P.stage_cap;               // survivor words per stage buffer
    const uint32_t  sstr   = scap + 64;                 // stage buffer stride (64 dummy slots)
    __shared__ uint32_t zinv[128];           // static, at LDS address 0: inverse nibble table
    uint32_t*       slice  = lds;
    uint32_t*       inv    = zinv;
    uint32_t*       subc   = slice + segw;    // 3 x 128: per-sub counters (+64 dummies), by item
    uint32_t*       subow  = subc + 3 * 128;  // 16 waves x NSUB: each wave's copy of the offsets
    constexpr uint32_t kScrCap = scr_cap<KIND>();
    constexpr int      kDense  = kScrCap / 64 > 0 ? kScrCap / 64 : 1;
    // 64 garbage slots shared by all waves, below the scratch (the compaction's address arithmetic
    // needs scratch slots above them)
    uint32_t*       scrdum  = subow + 16 * NSUB;
    uint32_t*       scratch = scrdum + 64;            // 16 waves x kScrCap: compacted survivors (not PAY)
    uint32_t*       stage  = scratch + (PAY ? 0u : 16 * kScrCap);  // 2 x sstr, double-buffered by item
    const uint32_t  hp     = scap / 2;                // PAY: codes at [0, hp), positions at [hp, scap)
    const int       tid    = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    load_tab(inv, &P.tabs->inv[0][0]);
    for (uint32_t i = tid; i < 3 * 128; i += NT) subc[i] = 0;
    const uint32_t I    = P.item_start[F];
    // uniform values computed on the VALU are pinned to SGPRs (readfirstlane)
    const uint32_t it0  = __builtin_amdgcn_readfirstlane((uint32_t) ((uint64_t) blockIdx.x * I / gridDim.x));
    const uint32_t it1  = __builtin_amdgcn_readfirstlane((uint32_t) ((uint64_t) (blockIdx.x + 1) * I / gridDim.x));
    const uint32_t nseg = SEG1 || !slices ? 1u : g.nseg;
    uint64_t tph[6] = {0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
    (void) tlast;
    auto stamp = [&](int k) {  // dev-only phase stamps (build with -DHWBRJ_STAMPS, run with HWBRJ_DBG)
#ifdef HWBRJ_STAMPS
        if (P.dbg) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tph[k] += t - tlast;
            tlast = t;
        }
#else
        (void) k;
#endif
    };
    // Copy-out of the previous item's staged survivors and its run table: a fixed number of
    // buffer stores whatever the counts (out-of-range ones are dropped), so the compiler never has
    // to wait for them (vmcnt counts stores on gfx9).
    constexpr uint32_t kNoItem = 0x80000000u;
    uint32_t  prev_total = 0, prev_it = kNoItem, prev_buf = 0, subc_v = 0, subo_v = 0, prev_q = 0;
    uint32_t* prev_out   = P.surv;
    const bool pk3       = !PAY && P.kbits != 0;  // packed join keys for staged items
    const bool pk18      = pk3 && P.kbits == 18;
    bool       prev_pk   = false;  // the previous item's run is staged and stored as 3-byte keys
    uint32_t   n_unst    = 0;      // items of this workgroup too large for the stage (32-bit runs)
    auto copy_out = [&]() {
        const uint32_t nbytes = ((prev_total + 3u) & ~3u) * 4u;  // item region holds round_up(total, 4)
        const auto     ro     = buf_rsrc(prev_out, nbytes);
        const v4u*     src    = (const v4u*) (stage + prev_buf * sstr);
        if (kAblProbe != 0) {  // (ablations: the run table only; 1 and 2 write empty runs)
        } else if (PAY) {  // codes and their chunk positions (half a stage buffer each)
            const auto rp = buf_rsrc(P.surv_pos + (prev_out - P.surv), nbytes);
#pragma unroll
            for (int k = 0; k < (kPC + 1) / 2; k++) {
                const uint32_t i = tid + k * NT;
                const uint32_t j = min(i, hp / 4 - 1);  // reads past the half are never stored
                __builtin_amdgcn_raw_buffer_store_b128(src[j], ro, i * 16, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(src[hp / 4 + j], rp, i * 16, 0, 0);
            }
        } else if (prev_pk && pk18) {  // 18-bit keys: one 16-byte store per 4 stream dwords (whole
                                       // quads: the region holds round_up(total, 4) words, more)
            const uint32_t nq = ((prev_total * 18u + 31u) / 32u + 3u) / 4u;
            const auto     rp = buf_rsrc(prev_out, nq * 16u);
            const uint32_t* c = (const uint32_t*) src;
            for (uint32_t i = tid; i < nq; i += NT)
                __builtin_amdgcn_raw_buffer_store_b128(pack18_quad(c, i, g.hash_shift), rp, i * 16u, 0, HWBRJ_PCO_AUX);
        } else if (prev_pk) {  // 24-bit keys: 12 bytes per staged quad (whole quads: the item
                               // region holds round_up(total, 4) words, more than these bytes)
            const auto rp3 = buf_rsrc(prev_out, (prev_total + 3u) / 4u * 12u);
#pragma unroll
            for (int k = 0; k < probe_pco<KIND>(); k++) {
                const uint32_t i = tid + k * NT;
                const v4u      v = src[min(i, scap / 4 - 1)];
                __builtin_amdgcn_raw_buffer_store_b96(pack3x4(v, g.hash_shift), rp3, i * 12, 0, HWBRJ_PCO_AUX);
            }
        } else {
#pragma unroll
        for (int k = 0; k < probe_pco<KIND>(); k++) {
            const uint32_t i = tid + k * NT;
            const v4u      v = src[min(i, scap / 4 - 1)];  // reads past the stage are never stored
            __builtin_amdgcn_raw_buffer_store_b128(v, ro, i * 16, 0, HWBRJ_PCO_AUX);
        }
        }
        const uint32_t tb = prev_it == kNoItem ? 0u : NSUB * 4;  // run table (wave 0 holds it)
        const auto rc = buf_rsrc(P.surv_cnt + (uint64_t) (prev_it & ~kNoItem) * NSUB, tb);
        const auto rf = buf_rsrc(P.surv_off + (uint64_t) (prev_it & ~kNoItem) * NSUB, tb);
        __builtin_amdgcn_raw_buffer_store_b32(subc_v, rc, tid * 4, 0, 0);
        // survivors per join job (q, sub), for the join's skew split (every wave issues the one
        // atomic; only wave 0's first NSUB lanes are in range)
        const auto rj = buf_rsrc(P.job_surv + (uint64_t) prev_q * NSUB, tb);
        __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32((int) subc_v, rj, tid * 4, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(subo_v | (prev_pk ? 0x80000000u : 0u), rf, tid * 4, 0, 0);
    };
    uint64_t filtered = 0;  // wave 0: survivors of this workgroup's items
    uint32_t nstep    = 0;  // items processed (selects the counter / stage buffers)
    uint64_t abl_n    = 0;  // (probe ablations 1 and 2: this wave's survivors)
    // Outer loop: runs of items with one (q, seg), i.e. one slice segment in LDS. Inner loop:
    // the pieces of the run, software-pipelined: piece p is tested while p+1 and p+2 are in flight
    // (three register buffers rotate, so no load result is ever copied; past the end the loads
    // re-read the last piece). One barrier per piece: every wave scans the per-sub counters itself,
    // counters are triple-buffered and the stage double-buffered.
    uint32_t it = it0;
    while (it < it1) {
        const uint32_t q    = __builtin_amdgcn_readfirstlane(find_q(P.item_start, F, it));
        const uint32_t qi0  = __builtin_amdgcn_readfirstlane(P.item_start[q]);
        const uint32_t qi1  = __builtin_amdgcn_readfirstlane(P.item_start[q + 1]);
        const uint32_t lq0  = __builtin_amdgcn_readfirstlane(P.list_start[q]);
        const uint32_t lq1  = __builtin_amdgcn_readfirstlane(P.list_start[q + 1]);
        const uint32_t npc  = (qi1 - qi0) / nseg;  // pieces of q
        const uint32_t seg  = (it - qi0) / npc;
        const uint32_t p0   = (it - qi0) - seg * npc;
        const uint32_t rend = min(it1, qi0 + (seg + 1) * npc);  // end of this (q, seg) run
        const uint32_t p1   = p0 + (rend - it);
        const uint32_t rit0 = it;  // item index of piece p0
        auto lb_of = [&](uint32_t p) { return lq0 + p * kProbeCH; };
        auto le_of = [&](uint32_t p) { return min(lq1, lq0 + (p + 1) * kProbeCH); };
        uint32_t   eA[kPC], eB[kPC], eC[kPC];
        Sweep<kPC> SA, SB, SC;
        {  // the run's first loads are issued before the slice copy, so the two latencies overlap
            const uint32_t pa = min(p0 + 1, p1 - 1), pb = min(p0 + 2, p1 - 1);
            load_list_u<kPC>(P.list, lb_of(p0), le_of(p0), eA);
            load_list_u<kPC>(P.list, lb_of(pa), le_of(pa), eB);
            load_list_u<kPC>(P.list, lb_of(pb), le_of(pb), eC);
            load_chunks_u<kPC, kPrNT>(P.pool, eA, lb_of(p0), le_of(p0), SA);
            load_chunks_u<kPC, kPrNT>(P.pool, eB, lb_of(pa), le_of(pa), SB);
        }
        if (slices) {
            __syncthreads();  // every wave is done with the previous slice
            slice_to_lds(slice, P.slices + ((uint64_t) q * nseg + seg) * segw, segw);
            __syncthreads();
        }
        // Sc: words of piece p (registers); en: list entries of p+2 -> Sl; enn <- list of p+3.
        auto step = [&](uint32_t p, Sweep<kPC>& Sc, Sweep<kPC>& Sl, const uint32_t (&en)[kPC],
                        uint32_t (&enn)[kPC]) {
            const uint32_t p2  = min(p + 2, p1 - 1);
            const uint32_t p3  = min(p + 3, p1 - 1);
            const uint32_t cb3 = nstep % 3;  // counter buffer of this piece
            load_chunks_u<kPC, kPrNT>(P.pool, en, lb_of(p2), le_of(p2), Sl);
            load_list_u<kPC>(P.list, lb_of(p3), le_of(p3), enn);
            stamp(0);
            uint32_t* cnt = subc + cb3 * 128;
            uint32_t* scr = scratch + wave * kScrCap;
            // ---- test. One-bit kinds: all slice reads first, then per word slot the pass bit, its
            // wave ballot and the compaction of the wave's survivors into its scratch (no exec
            // masking: non-survivors write a per-lane dummy slot).
            uint32_t pass = 0;  // bit i: word i survives
            uint32_t nsv  = 0;  // survivors of this wave (uniform)
            if (onebit) {
                uint32_t wv[NW], bb[NW];  // slice word, bit index inside the segment
                // packed words: the low log2(m / F) bits are the first bit's position in the slice
                // (block in slice << log2B | bit in block), so its byte in LDS is one shift and mask
                constexpr bool pk = (KIND == KIND_BLOCK_PK1 || KIND == KIND_BLOCK_PKK) && SEG1;
                const uint32_t lw = (uint32_t) __builtin_ctz(g.slice_bits) - 5u;  // slice words: 2^lw
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    const uint32_t w = sweep_word(Sc, i >> 2, i & 3);
                    if (pk) {
                        bb[i] = w;  // (the test below uses only its low 5 bits)
                        wv[i] = slice[__builtin_amdgcn_ubfe(w, 5u, lw)];
                        continue;
                    } else {
                        const Loc L = locate<KIND>(w, g, inv, q);
                        bb[i]       = L.base + L.h;
                    }
                    wv[i] = slice[bb[i] >> 5];
                }
                // pass 1: this lane's survivor bits; the wave's survivor count by one DPP sum
                if (pk) {  // bit = one bfe at the word's low 5 bits; the chunk quads' fill as one mask each
#pragma unroll
                    for (int i = 0; i < NW; i++) pass |= __builtin_amdgcn_ubfe(wv[i], bb[i], 1u) << i;
                    uint32_t vm = 0;  // valid words: (1 << n) - 1 per quad, by one bfe each
#pragma unroll
                    for (int j = 0; j < kPC; j++) vm |= __builtin_amdgcn_ubfe(0xFu, 0u, Sc.n[j]) << (4 * j);
                    pass &= vm;
                } else {
#pragma unroll
                    for (int i = 0; i < NW; i++) {
                        uint32_t ok = (wv[i] >> (bb[i] & 31u)) & ((uint32_t) (i & 3) < Sc.n[i >> 2] ? 1u : 0u);
                        if (!SEG1) ok &= locate<KIND>(sweep_word(Sc, i >> 2, i & 3), g, inv, q).seg == seg ? 1u : 0u;
                        pass |= ok << i;
                    }
                }
                const uint32_t pcnt = (uint32_t) __builtin_popcount(pass);
                const uint32_t pinc = wave_incl_scan_dpp(pcnt);
                nsv = __builtin_amdgcn_readlane(pinc, 63);
                // pass 2, only when they fit the wave's scratch (dense ranking below): per slot, the
                // wave ballot compacts the survivors there (no exec masking: the others write a
                // shared garbage slot). Otherwise no scratch write at all (high selectivity: the
                // words are ranked one by one, and 12 LDS writes per thread would buy nothing)
                if (!PAY && kScrCap > 0 && nsv <= kScrCap && kAblProbe != 1) {  // wave-uniform
                    // lane-major: this lane's survivors from its exclusive prefix (the scan above) on.
                    // Word i goes to byte address dmy + t_i * x (t_i its pass bit, x = the next
                    // survivor slot - dmy, dmy the lane's garbage slot below the scratch): one bfe,
                    // one mad_u24 and one shift-add per word
                    const uint32_t dmy = lds_byte_addr(&scrdum[lane]);
                    uint32_t       x   = lds_byte_addr(&scr[pinc - pcnt]) - dmy;
#pragma unroll
                    for (int i = 0; i < NW; i++) {
                        const uint32_t t = __builtin_amdgcn_ubfe(pass, (uint32_t) i, 1u);
                        lds_store_u32(mad_u24(t, x, dmy), sweep_word(Sc, i >> 2, i & 3));
                        x = shl_add(t, 2, x);
                    }
                }
            } else {
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    bool ok = (uint32_t) (i & 3) < Sc.n[i >> 2];
                    if (slices && ok) {
                        const Loc L = locate<KIND>(sweep_word(Sc, i >> 2, i & 3), g, inv, q);
                        ok          = (SEG1 || L.seg == seg) && apply_bits<KIND, false>(L, g, slice);
                    }
                    pass |= (ok ? 1u : 0u) << i;
                }
                nsv = kScrCap + 1;  // (word-by-word ranking)
            }
            // ---- ranks inside the piece's sub runs
            const bool dense = !PAY && kScrCap > 0 && nsv <= kScrCap;  // wave-uniform
            // dense: rank << 16 | sub of scratch entry lane + 64 k (kNoRank: not a survivor); the
            // code itself is re-read from the wave's scratch after the barrier (fewer live VGPRs)
            constexpr uint32_t kNoRank = 0xFFFFFFFFu;
            uint32_t   dr[kDense];
            uint32_t   rank2[NW / 2];            // word by word: two 16-bit ranks per register
            if (kAblProbe == 1 || kAblProbe == 2) {
                abl_n += nsv;
            } else if (dense) {
                // KIND_BASIC_KK: bits 2..k of every slot's candidate from the slices in HBM, bit by
                // bit, each bit loaded for all of the wave's live slots before any is tested
                // (kDense loads in flight instead of one at a time); stops when no slot is live
                constexpr int KD = KIND == KIND_BASIC_KK ? kDense : 1;
                uint32_t      live[KD];
                if (KIND == KIND_BASIC_KK) {
                    const uint32_t msz = (uint32_t) g.m;
                    uint32_t       hh[KD], yy[KD], wv[KD];
#pragma unroll
                    for (int k = 0; k < kDense; k++) {
                        const uint32_t j   = lane + 64u * k;
                        const uint32_t key = bunmix(scr[j]);  // (the word is bmix(key))
                        const uint32_t y0  = mod_m(key + kSeed, msz);
                        hh[k]   = mod_m(mod_m(crapwow(kSeed, key), msz) + y0, msz);  // bit 2
                        yy[k]   = mod_m(y0 + 1u, msz);
                        live[k] = j < nsv ? 1u : 0u;
                    }
                    for (uint32_t i = 1; i < g.k; i++) {
#pragma unroll
                        for (int k = 0; k < kDense; k++) wv[k] = live[k] ? *basic_word(P.slices, g, hh[k]) : 0u;
                        uint32_t any = 0;
#pragma unroll
                        for (int k = 0; k < kDense; k++) {
                            live[k] &= (wv[k] >> ((hh[k] >> g.log2F) & 31u)) & 1u;
                            hh[k] = mod_m(hh[k] + yy[k], msz);
                            yy[k] = mod_m(yy[k] + i + 1u, msz);
                            any |= live[k];
                        }
                        if (__builtin_amdgcn_ballot_w64(any != 0) == 0) break;  // wave-uniform
                    }
                }
#pragma unroll
                for (int k = 0; k < kDense; k++) {
                    const uint32_t j  = lane + 64u * k;
                    const uint32_t w  = scr[j];
                    const uint32_t c  = decode_k<KIND>(w, q, g);
                    const uint32_t s  = (c >> g.sub_shift) & (NSUB - 1u);
                    bool           ok = j < nsv;
                    if (KIND == KIND_BASIC_KK)
                        ok = ok && live[k] != 0;
                    else if (refine) ok = ok && apply_bits<KIND, false>(locate<KIND>(w, g, inv, q), g, slice);
                    const uint32_t r = atomicAdd(&cnt[ok ? s : 64u + lane], 1u);  // dummies: 64..127
                    dr[k]            = ok ? (s | (r << 16)) : kNoRank;
                }
            } else {
                if (refine) {  // too many first-bit candidates: the full test of every word
                    const uint32_t pass1 = pass;
                    pass = 0;
#pragma unroll
                    for (int i = 0; i < NW; i++) {
                        bool ok = (uint32_t) (i & 3) < Sc.n[i >> 2];
                        if (KIND == KIND_BASIC_KK) {
                            ok = ok && ((pass1 >> i) & 1u) && basic_rest(bunmix(sweep_word(Sc, i >> 2, i & 3)), g, inv, P.slices);
                        } else if (ok) {
                            const Loc L = locate<KIND>(sweep_word(Sc, i >> 2, i & 3), g, inv, q);
                            ok          = (SEG1 || L.seg == seg) && apply_bits<KIND, false>(L, g, slice);
                        }
                        pass |= (ok ? 1u : 0u) << i;
                    }
                }
#pragma unroll
                for (int i = 0; i < NW; i += 2) {
                    uint32_t r[2] = {0, 0};
#pragma unroll
                    for (int u = 0; u < 2; u++) {
                        const uint32_t c = decode_k<KIND>(sweep_word(Sc, (i + u) >> 2, (i + u) & 3), q, g);
                        const uint32_t s = (c >> g.sub_shift) & (NSUB - 1u);
                        if ((pass >> (i + u)) & 1u) r[u] = atomicAdd(&cnt[s], 1u);
                    }
                    rank2[i / 2] = r[0] | (r[1] << 16);
                }
            }
            stamp(1);
#ifndef HWBRJ_ABL_PNOB1  // (dev ablation, results invalid: the probe without its per-piece barrier)
            __syncthreads();  // B1: every rank of this piece taken; the previous piece staged
#endif
            stamp(2);
            // ---- every wave: run offsets of this piece (DPP scan over the NSUB counters)
            const uint32_t cs    = lane < (int) NSUB ? cnt[lane] : 0u;
            const uint32_t incl  = wave_incl_scan_dpp(cs);
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            uint32_t*      subo  = subow + wave * NSUB;
            if (lane < (int) NSUB) subo[lane] = incl - cs;  // wave-private copy
            if (wave == 0) subc[((nstep + 2) % 3) * 128 + lane] = 0;  // read two pieces ago
            copy_out();  // previous piece (its stage buffer is complete: barrier B1)
            if (wave == 0) {
                subc_v = cs;
                subo_v = incl - cs;
                filtered += total;
            }
            stamp(3);
            uint32_t* __restrict__ out = P.surv + (uint64_t) seg * P.surv_seg_stride + (uint64_t) lb_of(p) * 32;
            const uint32_t buf    = nstep & 1u;
            const bool     staged = PAY ? total <= hp : total <= scap;
            uint32_t*      stg    = stage + buf * sstr;
            const auto     ro     = buf_rsrc(out, total * 4);
            if (kAblProbe == 1 || kAblProbe == 2) {
            } else if (dense) {
#pragma unroll
                for (int k = 0; k < kDense; k++) {
                    const bool     ok = dr[k] != kNoRank;
                    const uint32_t c  = decode_k<KIND>(scr[lane + 64u * k], q, g);
                    const uint32_t o  = subo[dr[k] & 0xFFFFu] + (dr[k] >> 16);
                    if (staged) stg[ok ? o : scap + lane] = c;
                    else __builtin_amdgcn_raw_buffer_store_b32(c, ro, ok ? o * 4 : 0x7FFFFFF0u, 0, 0);
                }
            } else if (staged) {  // LDS stage (copied out coalesced at the next piece)
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    const uint32_t c = decode_k<KIND>(sweep_word(Sc, i >> 2, i & 3), q, g);
                    const uint32_t o = subo[(c >> g.sub_shift) & (NSUB - 1u)] + ((rank2[i / 2] >> (16 * (i & 1))) & 0xFFFFu);
                    stg[(pass >> i) & 1u ? o : scap + lane] = c;
                    if (PAY)  // the survivor's chunk position beside it
                        stg[(pass >> i) & 1u ? hp + o : scap + lane] =
                            Sc.id[i >> 2] * 32u + ((uint32_t) tid & 7u) * 4u + (uint32_t) (i & 3);
                }
            } else {  // more survivors than a stage buffer holds: scattered global (buffer) stores
                const auto rpo = buf_rsrc(PAY ? P.surv_pos + (out - P.surv) : nullptr, PAY ? total * 4 : 0u);
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    const uint32_t c  = decode_k<KIND>(sweep_word(Sc, i >> 2, i & 3), q, g);
                    const uint32_t o  = subo[(c >> g.sub_shift) & (NSUB - 1u)] + ((rank2[i / 2] >> (16 * (i & 1))) & 0xFFFFu);
                    const uint32_t oo = ((pass >> i) & 1u) ? o * 4 : 0x7FFFFFF0u;
                    __builtin_amdgcn_raw_buffer_store_b32(c, ro, oo, 0, 0);
                    if (PAY)
                        __builtin_amdgcn_raw_buffer_store_b32(Sc.id[i >> 2] * 32u + ((uint32_t) tid & 7u) * 4u + (uint32_t) (i & 3),
                                                              rpo, oo, 0, 0);
                }
            }
            stamp(4);
            prev_total = staged ? total : 0u;
            prev_pk    = pk3 && staged;
            n_unst += staged ? 0u : 1u;
            prev_out   = out;
            prev_buf   = buf;
            prev_it    = rit0 + (p - p0);
            prev_q     = q;
            nstep++;
            stamp(5);
        };
        for (uint32_t p = p0; p < p1; p += 3) {
            step(p, SA, SC, eC, eA);
            if (p + 1 < p1) step(p + 1, SB, SA, eA, eB);
            if (p + 2 < p1) step(p + 2, SC, SB, eB, eC);
        }
        it = rend;
    }
    __syncthreads();  // the last piece is staged
    copy_out();
    if (tid == 0 && filtered) atomicAdd((unsigned long long*) P.filtered, (unsigned long long) filtered);
    if (tid == 0 && n_unst && P.fmt_cnt) atomicAdd(P.fmt_cnt, n_unst);
    if (kAblProbe == 1 || kAblProbe == 2)
        if (lane == 0 && abl_n) atomicAdd((unsigned long long*) P.filtered, (unsigned long long) abl_n);
    if (P.dbg && tid == 0)
        for (int k = 0; k < 6; k++) P.dbg[blockIdx.x * 8 + k] = tph[k];
}

// ================================================ K7b: basic k >= 2, one bit per pass
// The words (bmix(key)) are partitioned by the slice of add_basic's bit j (MODE_SLICE_BASIC's
// scatter for j = 0, MODE_BASIC_BITJ's for j > 0); every item tests bit j of its words in the LDS
// slice, and the passing words go to the workgroup's own region of surv (dense, no atomics;
// wg_cnt[w] = its count, filtered += the sum). The next pass's scatter partitions workgroup w's
// region by the slice of bit j + 1 in its workgroup w, so every bit of every key is tested in LDS
// (bloom contains, src/bloom_filter.c:92-111), never by a random HBM read. Items are numbered as
// in k_probe (segment-major inside a partition); the next item's chunks (and the one after's list
// entries) are loaded while the current one is tested; one barrier per item (double-buffered
// wave sums).
__global__ __launch_bounds__(1024) void k_probe_bitj(ProbeParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr uint32_t NT = 1024;
    constexpr int      NW = kPC * 4;
    const Geometry&    g  = P.g;
    const uint32_t     F  = 1u << g.log2F, segw = g.seg_words, nseg = g.nseg;
    uint32_t*          slice = lds;
    uint32_t*          wsum  = slice + segw;  // 2 x 16, by item parity
    const int      tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t I   = P.item_start[F];
    const uint32_t it0 = __builtin_amdgcn_readfirstlane((uint32_t) ((uint64_t) blockIdx.x * I / gridDim.x));
    const uint32_t it1 = __builtin_amdgcn_readfirstlane((uint32_t) ((uint64_t) (blockIdx.x + 1) * I / gridDim.x));
    uint32_t* __restrict__ out = P.surv + (uint64_t) blockIdx.x * P.surv_seg_stride;
    uint32_t cursor = 0;  // words appended (uniform)
    if (it0 < it1) {  // (uniform)
        struct ItemG {
            uint32_t q, seg, lb, le;
            uint32_t qi0, qi1, lq0, lq1, npc;  // partition q's items and list range
        };
        auto at_q = [&](ItemG& r, uint32_t q) {
            r.q   = q;
            r.qi0 = __builtin_amdgcn_readfirstlane(P.item_start[q]);
            r.qi1 = __builtin_amdgcn_readfirstlane(P.item_start[q + 1]);
            r.lq0 = __builtin_amdgcn_readfirstlane(P.list_start[q]);
            r.lq1 = __builtin_amdgcn_readfirstlane(P.list_start[q + 1]);
            r.npc = (r.qi1 - r.qi0) / nseg;
        };
        auto place = [&](ItemG& r, uint32_t it) {
            r.seg             = (it - r.qi0) / r.npc;
            const uint32_t pc = (it - r.qi0) - r.seg * r.npc;
            r.lb              = r.lq0 + pc * kProbeCH;
            r.le              = min(r.lq1, r.lb + kProbeCH);
        };
        // item it's geometry from that of an earlier item (a binary search only for the first)
        auto next = [&](const ItemG& prev, uint32_t it) {
            ItemG r = prev;
            if (it >= r.qi1) {  // (uniform) a later partition: step over empty ones
                uint32_t q = r.q + 1;
                while (__builtin_amdgcn_readfirstlane(P.item_start[q + 1]) <= it) q++;
                at_q(r, q);
            }
            place(r, it);
            return r;
        };
        ItemG g0;
        at_q(g0, __builtin_amdgcn_readfirstlane(find_q(P.item_start, F, it0)));
        place(g0, it0);
        const uint32_t msz = (uint32_t) g.m, F1 = F - 1u;
        const auto     rout = buf_rsrc(out, (uint32_t) (P.surv_seg_stride * 4));
        // geometry of items it .. it + 3 (gi[0] = it), rolled as the items advance (scalars)
        ItemG gi[4];
        gi[0] = g0;
        gi[1] = next(gi[0], min(it0 + 1, it1 - 1));
        gi[2] = next(gi[1], min(it0 + 2, it1 - 1));
        gi[3] = next(gi[2], min(it0 + 3, it1 - 1));
        uint32_t   eA[kPC], eB[kPC], eC[kPC];
        Sweep<kPC> SA, SB, SC;
        load_list_u<kPC>(P.list, gi[0].lb, gi[0].le, eA);
        load_list_u<kPC>(P.list, gi[1].lb, gi[1].le, eB);
        load_list_u<kPC>(P.list, gi[2].lb, gi[2].le, eC);
        load_chunks_u<kPC>(P.pool, eA, gi[0].lb, gi[0].le, SA);
        load_chunks_u<kPC>(P.pool, eB, gi[1].lb, gi[1].le, SB);
        uint32_t cq = 0xFFFFFFFFu, cs = 0xFFFFFFFFu, par = 0;  // the (partition, segment) in LDS
        // Sc: chunks of item it (loaded); the chunks of it + 1 are in flight; en: list entries of
        // it + 2 -> chunks into Sf; ef <- list entries of it + 3. Three buffers rotate (no load
        // result is ever copied, so no wait is forced before its use).
        auto step = [&](uint32_t it, Sweep<kPC>& Sc, Sweep<kPC>& Sf, const uint32_t (&en)[kPC], uint32_t (&ef)[kPC]) {
            const ItemG ga = gi[0];
            load_chunks_u<kPC>(P.pool, en, gi[2].lb, gi[2].le, Sf);
            load_list_u<kPC>(P.list, gi[3].lb, gi[3].le, ef);
            if (ga.q != cq || ga.seg != cs) {  // (uniform)
                __syncthreads();  // every wave is done with the previous slice
                slice_to_lds(slice, P.slices + ((uint64_t) ga.q * nseg + ga.seg) * segw, segw);
                cq = ga.q;
                cs = ga.seg;
                __syncthreads();
            }
            // bit j of every word: add_basic's sequence stepped j times (uniform loop)
            uint32_t h[NW], y[NW];
#pragma unroll
            for (int i = 0; i < NW; i++) {
                const uint32_t key = bunmix(sweep_word(Sc, i >> 2, i & 3));
                h[i] = mod_m(crapwow(kSeed, key), msz);
                y[i] = mod_m(key + kSeed, msz);
            }
            for (uint32_t t = 0; t < g.bitj; t++) {
#pragma unroll
                for (int i = 0; i < NW; i++) {
                    h[i] = mod_m(h[i] + y[i], msz);
                    y[i] = mod_m(y[i] + t + 1u, msz);
                }
            }
            uint32_t pass = 0;
#pragma unroll
            for (int i = 0; i < NW; i++) {
                const uint32_t lb = h[i] >> g.log2F;
                const uint32_t x  = lb & (g.seg_bits - 1u);
                const uint32_t in = ((uint32_t) (i & 3) < Sc.n[i >> 2] ? 1u : 0u) & ((h[i] & F1) == ga.q ? 1u : 0u) &
                                    ((lb >> g.log2seg) == ga.seg ? 1u : 0u);
                pass |= (in & (slice[x >> 5] >> (x & 31u))) << i;
            }
            const uint32_t c    = (uint32_t) __builtin_popcount(pass);
            const uint32_t incl = wave_incl_scan_dpp(c);
            uint32_t*      ws   = wsum + par * 16;
            if (lane == 63) ws[wave] = incl;
            __syncthreads();
            uint32_t before = 0, total = 0;
#pragma unroll
            for (int w = 0; w < (int) (NT / 64); w++) {
                const uint32_t x = ws[w];
                before += w < wave ? x : 0u;
                total += x;
            }
            uint32_t o = cursor + before + incl - c;
#pragma unroll
            for (int i = 0; i < NW; i++) {  // a fixed number of stores (the others are dropped)
                const uint32_t pi = (pass >> i) & 1u;
                __builtin_amdgcn_raw_buffer_store_b32(sweep_word(Sc, i >> 2, i & 3), rout, pi ? o * 4 : kOob, 0, 0);
                o += pi;
            }
            cursor += __builtin_amdgcn_readfirstlane(total);
            par ^= 1u;
            gi[0] = gi[1];
            gi[1] = gi[2];
            gi[2] = gi[3];
            gi[3] = next(gi[2], min(it + 4, it1 - 1));
        };
        for (uint32_t it = it0; it < it1; it += 3) {
            step(it, SA, SC, eC, eA);
            if (it + 1 < it1) step(it + 1, SB, SA, eA, eB);
            if (it + 2 < it1) step(it + 2, SC, SB, eB, eC);
        }
    }
    if (tid == 0) {
        P.wg_cnt[blockIdx.x] = cursor;
        if (cursor) atomicAdd((unsigned long long*) P.filtered, (unsigned long long) cursor);
    }
}

size_t probe_bitj_lds_bytes(const Geometry& g) { return (g.seg_words + 32) * sizeof(uint32_t); }

void launch_probe_bitj(const ProbeParams& p, uint32_t grid, hipStream_t st) {
    const size_t lds = probe_bitj_lds_bytes(p.g);
    (void) hipFuncSetAttribute((const void*) &k_probe_bitj, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_probe_bitj<<<grid, 1024, lds, st>>>(p);
}

// ========================================================================= K10: join
// One workgroup per (partition q, sub-partition s) job (bucket_chaining_join per task,
// src/parallel_radix_join_bloom.c:259-329). The R codes of (q, s) are known to share their low
// hash_shift bits, so v = code >> hash_shift identifies the key inside the job.
//  * bitmap path (v < 2^18): every R key sets bit v of a 32 KiB LDS bitmap (ds_or_rtn); a bit
//    that was already set means a duplicate R key, and the job falls back to the hash path
//    (multiplicities). Each survivor then costs one LDS read.
//  * hash path: LDS open-addressing table (linear probing, ds_cmpswap) holding pieces of <= 4096
//    R keys; survivors count equal keys (S re-streamed per piece).
// Survivor runs of (q, s) -- one per probe item of q, written in place by k_probe -- are taken a
// wave per run, several runs in flight per wave.
#ifndef HWBRJ_JT
#define HWBRJ_JT 256  // threads per join workgroup (A/B)
#endif
constexpr int      kJoinThreads = HWBRJ_JT;
constexpr int      kJoinWaves   = kJoinThreads / 64;
#ifndef HWBRJ_JBM
#define HWBRJ_JBM 18  // bitmap path: keys v < 2^HWBRJ_JBM (17: half the LDS, with 32 subs; dev A/B)
#endif
constexpr uint32_t kJoinBmLog2  = HWBRJ_JBM;           // bitmap path: v < 2^18
constexpr uint32_t kJoinWords   = 1u << (kJoinBmLog2 - 5);  // 8192 LDS words (32 KiB)
constexpr uint32_t kJoinLog2T   = kJoinBmLog2 - 5;     // hash path: 8192 slots in the same words
constexpr uint32_t kJoinT       = 1u << kJoinLog2T;
constexpr uint32_t kJoinPiece   = kJoinT / 2;
constexpr uint32_t kJoinDesc    = 256;                 // run descriptors per batch
#ifndef HWBRJ_JTU
#define HWBRJ_JTU 8
#endif
constexpr uint32_t kJoinTailU   = HWBRJ_JTU;           // loads in flight per lane in a long run
#ifndef HWBRJ_JTS
#define HWBRJ_JTS 2
#endif
constexpr uint32_t kJoinTailS   = HWBRJ_JTS;           // ... in the rest of a run (< 64 kJoinTailU words)
constexpr uint32_t kEmpty       = 0xFFFFFFFFu;  // codes of one job share their low hash_shift >= 1
                                                // bits, so (code >> hash_shift) never equals it

__device__ __forceinline__ uint32_t join_slot(uint32_t v) {
    return (v * 0x9E3779B1u) >> (32 - kJoinLog2T);
}

// The table is probed by buckets of 4 slots (one 16-byte LDS read compares four keys): a key lives
// in the first bucket from its home that had a free slot when it was inserted. Slots are never
// freed, so every bucket before it stays full, and a lookup can stop at the first bucket that
// has a free slot (every copy of a key lies at or before it).
__device__ __forceinline__ uint32_t join_count(const uint32_t* keys, uint32_t v) {
    uint32_t b = join_slot(v) & ~3u, cnt = 0;
    for (;;) {
        const uint4 k = *(const uint4*) &keys[b];
        cnt += (k.x == v) + (k.y == v) + (k.z == v) + (k.w == v);
        if (k.x == kEmpty || k.y == kEmpty || k.z == kEmpty || k.w == kEmpty) return cnt;
        b = (b + 4u) & (kJoinT - 1u);
    }
}

__device__ __forceinline__ void join_insert(uint32_t* keys, uint32_t v) {
    uint32_t b = join_slot(v) & ~3u;
    for (;;) {
        const uint4 k = *(const uint4*) &keys[b];  // (a free slot may be taken meanwhile: then CAS fails)
        if (k.x == kEmpty && atomicCAS(&keys[b], kEmpty, v) == kEmpty) return;
        if (k.y == kEmpty && atomicCAS(&keys[b + 1], kEmpty, v) == kEmpty) return;
        if (k.z == kEmpty && atomicCAS(&keys[b + 2], kEmpty, v) == kEmpty) return;
        if (k.w == kEmpty && atomicCAS(&keys[b + 3], kEmpty, v) == kEmpty) return;
        b = (b + 4u) & (kJoinT - 1u);
    }
}

// Join tasks. A (q, sub) job whose survivors exceed kJoinTaskSurv (probe-side skew, e.g. the
// hot keys of a Zipf S) is split into parts over q's probe items; every part rebuilds the job's
// small R table and counts its share of the survivors. k_probe sums the survivors of every job
// (job_surv); k_join_split gives part 0 of job j to workgroup j and appends the further parts to
// a table read by kJoinExtra extra workgroups (first come, first served: the table bounds the
// added parts). It also clears job_surv for the next join.
constexpr uint32_t kJoinTaskSurv = 1u << 17;
constexpr uint32_t kJoinExtra    = 2048;

// Match counts: every join workgroup adds its count to one of kJoinSumSlots partial sums (each in
// its own 128-byte line, so the adds are not serialised on one address); the host sums them.
constexpr uint32_t kJoinSumSlots = 64;
constexpr uint32_t kJoinSumStride = 16;  // u64 words per slot (128 bytes)

__global__ __launch_bounds__(256) void k_join_split(const uint32_t* __restrict__ item_start,
                                                     uint32_t* __restrict__ job_surv,
                                                     uint32_t log2NSUB, uint32_t NJ, uint32_t split,
                                                     uint32_t* __restrict__ nparts,
                                                     uint2* __restrict__ extra, uint32_t* nextra,
                                                     uint64_t* __restrict__ jsum) {
    if (blockIdx.x == 0 && threadIdx.x < kJoinSumSlots)
        for (int w = 0; w < 3; w++) jsum[threadIdx.x * kJoinSumStride + w] = 0;
    const uint32_t job = blockIdx.x * blockDim.x + threadIdx.x;  // one thread per job
    if (job >= NJ) return;
    const uint32_t q = job >> log2NSUB, items = item_start[q + 1] - item_start[q];
    const uint32_t tot = job_surv[job];
    job_surv[job]      = 0;
    const uint32_t want = min(max((uint32_t) (((uint64_t) tot + split - 1) / split), 1u), max(items, 1u));
    uint32_t       np   = 1;
    if (want > 1) {
        const uint32_t base = atomicAdd(nextra, want - 1);
        if (base < kJoinExtra) {
            np = 1 + min(want - 1, kJoinExtra - base);
            for (uint32_t p = 1; p < np; p++) extra[base + p - 1] = make_uint2(job, p);
        }
    }
    nparts[job] = np;
}

// One (job, part) of the join on workgroup slot blk; MIXED: survivor runs of both formats (below).
// Adds this thread's matches to cnt_acc and (P.timing) the workgroup's probe ticks to tp_acc.
// A join workgroup's LDS, declared once by the kernel: both join_job instantiations (uniform and
// mixed formats) in one kernel share it (a static __shared__ array per instantiation would be
// allocated twice).
struct JoinShared {
    __attribute__((aligned(16))) uint32_t tab[kJoinWords];  // bitmap or hash table
    uint64_t dbase[kJoinDesc];  // run starts (byte offsets) of a batch: S survivor runs
    __attribute__((aligned(16))) uint32_t dcnt[kJoinDesc];
    uint64_t rbase[kJoinDesc];  // R runs (one per build sweep of q)
    __attribute__((aligned(16))) uint32_t rcnt[kJoinDesc];
    __attribute__((aligned(16))) uint32_t pend[kJoinDesc + 1];  // hash path: piece boundaries in an R batch
    uint32_t dupflag, npieces;
};

// KW: the launch's packed key width, 18 / 24 (every run packed), 32 (every run 32-bit codes), or 0
// (P.r_kbits at run time: the mixed launches, k_join_mixed)
template <bool MIXED, int KW = 0>
__device__ __forceinline__ void join_job(const JoinParams& P, const uint32_t blk, JoinShared& L, uint64_t& cnt_acc,
                                         uint64_t& tp_acc) {
    uint32_t* const tab   = L.tab;
    uint64_t* const dbase = L.dbase;
    uint32_t* const dcnt  = L.dcnt;
    uint64_t* const rbase = L.rbase;
    uint32_t* const rcnt  = L.rcnt;
    uint32_t* const pend  = L.pend;
    uint32_t&       dupflag = L.dupflag;
    uint32_t&       npieces = L.npieces;
    const uint32_t NSUB = 1u << P.log2NSUB;
    uint32_t       job = blk, part = 0;  // workgroup j < jobs: part 0 of job j
#ifndef HWBRJ_JXCD
#define HWBRJ_JXCD 1
#endif
    // XCD-aware job order: blocks b, b + 8, ... share an XCD (dealt round-robin), so they take
    // consecutive jobs -- the 16 subs of a partition run on one XCD, where the lines their runs
    // share (adjacent sub runs in every sweep slot and item region) are fetched into its L2 once
    if (HWBRJ_JXCD && blk < P.jobs && (P.jobs & 7u) == 0) job = (blk & 7u) * (P.jobs >> 3) + (blk >> 3);
    if (blk >= P.jobs) {                 // extra workgroups: further parts of skewed jobs
        const uint32_t e = blk - P.jobs;
        if (e >= min(*P.nextra, kJoinExtra)) return;
        const uint2 x = P.extra[e];
        job           = x.x;
        part          = x.y;
    }
    const uint32_t q = job >> P.log2NSUB, s = job & (NSUB - 1u);
    const uint32_t w0 = P.r_sweep_start[q], w1 = P.r_sweep_start[q + 1];
    const uint32_t qi0 = P.item_start[q], qi1 = P.item_start[q + 1];  // q's items (segment-major)
    const uint32_t np  = P.nparts[job];
    const bool     rpk = KW ? KW != 32 : P.r_kbits != 0;
    const uint32_t i0  = qi0 + (uint32_t) ((uint64_t) (qi1 - qi0) * part / np);
    const uint32_t i1  = qi0 + (uint32_t) ((uint64_t) (qi1 - qi0) * (part + 1) / np);
    if (w1 == w0 || i1 == i0) return;
    const uint32_t lq0 = P.item_base ? 0u : P.list_start[q];
    const uint32_t npc = (qi1 - qi0) / P.nseg;  // probe pieces of q
    const uint32_t sh  = P.hash_shift;
    const int      tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    uint64_t       cnt = 0;
    // probe share of the join (the reference's per-thread probe timers, :289-321): the 100 MHz
    // ticks of the survivor-probing sections of this workgroup (synchronous joins only, P.timing)
    uint64_t t_probe = 0, t_mark = 0;
    auto probe_begin = [&]() {
        if (P.timing) t_mark = wall_clock64();
    };
    auto probe_end = [&]() {
        if (P.timing) t_probe += wall_clock64() - t_mark;
    };
    // dev-only phase stamps of wave 0 (build with -DHWBRJ_STAMPS, run with HWBRJ_DBG): fused path
    // 0 descriptors, 1 R loads + bit sets, 2 popcount, 3 first survivor runs, 4 further runs, 5 sum
    uint64_t tph[6] = {0, 0, 0, 0, 0, 0}, tlast = __builtin_amdgcn_s_memtime();
    (void) tlast;
    (void) tph;
    auto stamp = [&](int k) {
#ifdef HWBRJ_STAMPS
        if (P.dbg) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            tph[k] += t - tlast;
            tlast = t;
        }
#else
        (void) k;
#endif
    };
    // Run formats. A run is addressed by a tag tb from its array's base: bit 63 set = packed keys
    // (P.r_kbits = kw bits each: 18 or 24), tb their bit address, key o the kw bits at tb + kw o
    // (the unaligned dword at byte (tb + kw o) >> 3, shifted by (tb + kw o) & 7); else 32-bit codes at
    // byte tb + 4 o, key = code >> sh. R runs share one format (the build's); survivor runs are
    // packed when their probe item was staged (bit 31 of surv_off). P.fmt_cnt counts the unstaged
    // items: with none (or no packing at all) every run of the launch has one format, whose width,
    // shift and mask are uniform (k_join); otherwise the survivor runs are mixed and read with a
    // per-run format (k_join_mixed: only where probe items overflow their stage), R runs packed.
    // Loads stay raw until used (key()): ALU work on a conditionally loaded value would make the
    // wave wait for it at once.
    // Packed runs are tagged by their bit address in the stream (bit 63 set): key o at bit
    // tb + kw o, read as the dword at byte (tb + kw o) >> 3 shifted by (tb + kw o) & 7; code runs by
    // their byte address, key o the code at tb + 4 o shifted by hash_shift.
    constexpr uint64_t kPk = 1ull << 63;
    const uint32_t kw = KW ? (uint32_t) KW : rpk ? P.r_kbits : 32u, kw7 = kw & 7u;
    const uint32_t ksh = rpk ? 0u : sh, kmk = rpk ? (1u << kw) - 1u : 0xFFFFFFFFu;
    // (24-bit keys start on byte boundaries: a run's tb & 7 is 0, key o at byte 3 o)
    constexpr bool kB8 = KW == 24 || KW == 32;
    const uint8_t* const r8 = (const uint8_t*) P.r_codes;
    const uint8_t* const s8 = (const uint8_t*) P.surv;
    using SideR = std::integral_constant<int, 0>;
    using SideS = std::integral_constant<int, 1>;
    // R run of (sweep, sub) at key offset off of the sweep's slot; survivor run at key offset off of
    // the item region at element e0 (regions and slots keep their 4-byte-per-key sizes)
    auto rtag = [&](uint32_t sweep, uint32_t off) -> uint64_t {
        return rpk ? kPk | ((uint64_t) sweep * P.slot * 32u + (uint64_t) off * kw) : ((uint64_t) sweep * P.slot + off) * 4u;
    };
    auto stag = [&](uint64_t e0, uint32_t offw) -> uint64_t {
        const uint64_t off = offw & 0x7FFFFFFFu;
        return (offw >> 31) ? kPk | (e0 * 32u + off * kw) : (e0 + off) * 4u;
    };
    auto ldv = [&](auto side_c, uint64_t tb, uint32_t o) -> uint32_t {
        constexpr int SIDE = decltype(side_c)::value;
        bool          pk   = rpk;
        if constexpr (MIXED) pk = (tb & kPk) != 0;
        // (the run's byte base once per run, the key's byte inside it in 32 bits)
        const uint8_t* rb = (SIDE == 0 ? r8 : s8) + (pk ? (tb & ~kPk) >> 3 : tb);
        const uint32_t ob = pk ? (kB8 ? (kw >> 3) * o : (((uint32_t) tb & 7u) + kw * o) >> 3) : 4u * o;
        return *(const u32_unaligned*) (rb + ob);
    };
    // the key of raw word x = key o of a run whose tag has low bits b7 (tb & 7 of a packed run, 0
    // else). Only o mod 8 matters (kw o mod 8), and every caller's o is its lane plus a multiple of
    // 64: callers pass the lane, so the shift is one value per run and lane, not one per key.
    auto key = [&](auto side_c, uint32_t x, bool pk, uint32_t b7, uint32_t o) -> uint32_t {  // (side_c: as ldv's, unused)
        (void) side_c;
        if constexpr (MIXED) return pk ? (x >> ((b7 + kw7 * o) & 7u)) & kmk : x >> sh;
        (void) pk;
        if constexpr (kB8) return (x >> ksh) & kmk;
        return (x >> (((b7 + kw7 * o) & 7u) + ksh)) & kmk;
    };
    auto b7_of = [&](uint64_t tb) -> uint32_t { return !kB8 && (tb & kPk) ? (uint32_t) tb & 7u : 0u; };
    // The words [from, n) of one run (long runs: high-selectivity survivors, large R runs): whole
    // rounds of kJoinTailU loads in flight per lane (no per-load predicate) while the run has them,
    // then the rest kJoinTailS per lane, not a predicated full-width round (q = 1 join 0.99 ->
    // 0.96 ms, PRO 1.03 -> 0.97 ms, the north star within 0.002 ms: profiles/r06/join_tail_ab.txt).
    // b stays a multiple of 64 (from is), so word b + lane + 64 u is lane mod 8 for the packed keys.
    auto tail_run = [&](auto side_c, uint64_t bb, uint32_t from, uint32_t n, auto&& op) {
        const bool     pk = (bb & kPk) != 0;
        const uint32_t b7 = b7_of(bb);
        uint32_t       b  = from;  // (uniform)
        for (; b + 64u * kJoinTailU <= n; b += 64u * kJoinTailU) {
            uint32_t v[kJoinTailU];
#pragma unroll
            for (int u = 0; u < (int) kJoinTailU; u++) v[u] = ldv(side_c, bb, b + lane + 64u * u);
#pragma unroll
            for (int u = 0; u < (int) kJoinTailU; u++) op(key(side_c, v[u], pk, b7, lane));
        }
        for (; b < n; b += 64u * kJoinTailS) {
            uint32_t v[kJoinTailS];
#pragma unroll
            for (int u = 0; u < (int) kJoinTailS; u++) {
                const uint32_t oo = b + lane + 64u * u;
                v[u]              = oo < n ? ldv(side_c, bb, oo) : 0u;
            }
#pragma unroll
            for (int u = 0; u < (int) kJoinTailS; u++)
                if (b + lane + 64u * u < n) op(key(side_c, v[u], pk, b7, lane));
        }
    };
    // Every word of runs [da, db) of a descriptor batch through op(word): a wave per run, RUNS runs
    // in flight per wave with WPL words per lane each; longer runs finish in a tail loop.
    auto walk = [&](auto runs_c, auto wpl_c, auto side_c, const uint32_t* nc,
                    const uint64_t* nb, uint32_t da, uint32_t db, auto&& op) {
        constexpr int RUNS = decltype(runs_c)::value, WPL = decltype(wpl_c)::value;
        static_assert(3 * RUNS <= 32, "b7m holds 3 bits per run in flight (HWBRJ_JRR / HWBRJ_JSR <= 10)");
        for (uint32_t d = da + wave; d < db; d += kJoinWaves * RUNS) {
            uint32_t v[RUNS][WPL], n[RUNS], pkm = 0, b7m = 0;  // pkm bit r: run r packed; b7m: its tb & 7
#pragma unroll
            for (int r = 0; r < RUNS; r++) {
                const uint32_t dd = d + r * kJoinWaves;
                n[r]              = dd < db ? nc[dd] : 0u;
                const uint64_t bb = dd < db ? nb[dd] : 0ull;
                pkm |= (uint32_t) (bb >> 63) << r;
                b7m |= b7_of(bb) << (3 * r);
#pragma unroll
                for (int j = 0; j < WPL; j++) {
                    const uint32_t o = lane + 64u * j;
                    v[r][j]          = o < n[r] ? ldv(side_c, bb, o) : 0u;
                }
            }
#pragma unroll
            for (int r = 0; r < RUNS; r++) {
#pragma unroll
                for (int j = 0; j < WPL; j++)
                    if (lane + 64u * j < n[r]) op(key(side_c, v[r][j], (pkm >> r) & 1u, (b7m >> (3 * r)) & 7u, lane));
                if (n[r] > 64u * WPL) {
                    const uint64_t bb = nb[d + r * kJoinWaves];
                    tail_run(side_c, bb, 64u * WPL, n[r], op);
                }
            }
        }
    };
#ifndef HWBRJ_JRR
#define HWBRJ_JRR 4
#define HWBRJ_JRW 4
#define HWBRJ_JSR 8
#define HWBRJ_JSW 2
#endif
    using RR = std::integral_constant<int, HWBRJ_JRR>;  // R runs in flight per wave
    using RW = std::integral_constant<int, HWBRJ_JRW>;  // R words per lane per run
    using SR = std::integral_constant<int, HWBRJ_JSR>;  // survivor runs in flight per wave
    using SW = std::integral_constant<int, HWBRJ_JSW>;
    // the survivors of (q, s), batch by batch, against the table: bitmap (BM) or hash table
    auto probe_survivors = [&](auto&& op) {
        probe_begin();
        for (uint32_t d0 = i0; d0 < i1; d0 += kJoinDesc) {
            const uint32_t nd = min(kJoinDesc, i1 - d0);
            __syncthreads();  // previous descriptors consumed
            if ((uint32_t) tid < nd) {
                const uint32_t it    = d0 + tid;
                const uint32_t local = it - qi0;
                const uint32_t seg   = local / npc;
                const uint32_t piece = local - seg * npc;
                dcnt[tid]  = P.surv_cnt[(uint64_t) it * NSUB + s];
                dbase[tid] = stag(P.item_base ? P.item_base[it]  // (the partitioned multi-GPU join)
                                              : (uint64_t) seg * P.surv_seg_stride + (uint64_t) (lq0 + piece * P.CH) * 32,
                                  P.surv_off[(uint64_t) it * NSUB + s]);
            }
            __syncthreads();
            walk(SR{}, SW{}, SideS{}, dcnt, dbase, 0, nd, op);
        }
        probe_end();
    };
    // R run descriptors of a batch
    auto load_r = [&](uint32_t d0, uint32_t nd) {
        __syncthreads();  // previous R descriptors consumed
        uint32_t c = 0;
        if ((uint32_t) tid < nd) {
            const uint64_t r = (uint64_t) (d0 + tid) * NSUB + s;
            c                = P.r_cnt[r];
            rcnt[tid]        = c;
            rbase[tid]       = rtag(d0 + tid, P.r_off[r]);
        }
        (void) c;
        __syncthreads();
    };
    // PRH / PRHO (P.jkind 1 / 2): the histogram join of every job, below
    bool hashed = !P.bitmap || P.jkind != 0;
    bool done   = false;
#ifndef HWBRJ_JFR
#define HWBRJ_JFR 8  // fused path: R runs per wave
#define HWBRJ_JFW 5  // fused path: R words per lane per run (runs average slot / NSUB words)
#endif
    constexpr int FR = HWBRJ_JFR, FW = HWBRJ_JFW;
    const uint32_t nRd = w1 - w0, nSd = i1 - i0;
    if (!hashed && nRd <= (uint32_t) (kJoinWaves * FR) && nSd <= kJoinDesc) {
        // Fused bitmap path (every job of the north star): both descriptor sets in one phase, then
        // the loads of all R runs and of the first survivor runs are issued before any is used, so
        // a job costs two memory latencies (descriptors, data) instead of one per batch.
        for (uint32_t i = tid; i < kJoinWords / 4; i += kJoinThreads) ((uint4*) tab)[i] = make_uint4(0, 0, 0, 0);
        if (tid == 0) dupflag = 0;
        uint32_t rc = 0;
        if ((uint32_t) tid < nRd) {
            const uint64_t r = (uint64_t) (w0 + tid) * NSUB + s;
            rcnt[tid]        = P.r_cnt[r];
            rbase[tid]       = rtag(w0 + tid, P.r_off[r]);
            rc = rcnt[tid];
        }
        stamp(0);
        if (wave == 0) {  // the job's R keys (nRd <= 64: every R descriptor is in wave 0)
            const uint32_t t = __builtin_amdgcn_readlane(wave_incl_scan_dpp(rc), 63);
            if (lane == 0) npieces = t;
        }
        if ((uint32_t) tid < nSd) {
            const uint32_t it    = i0 + tid;
            const uint32_t local = it - qi0;
            const uint32_t seg   = local / npc;
            const uint32_t piece = local - seg * npc;
            dcnt[tid]  = P.surv_cnt[(uint64_t) it * NSUB + s];
            dbase[tid] = stag(P.item_base ? P.item_base[it]  // (the partitioned multi-GPU join)
                                          : (uint64_t) seg * P.surv_seg_stride + (uint64_t) (lq0 + piece * P.CH) * 32,
                              P.surv_off[(uint64_t) it * NSUB + s]);
        }
        __syncthreads();
#ifndef HWBRJ_JFS
#define HWBRJ_JFS 5  // (round 6: 5 of 8 -> join 0.294 -> 0.284 ms, profiles/r06/join_fs_ab.txt)
#endif
        constexpr int FS = HWBRJ_JFS, FSW = HWBRJ_JSW;  // survivor runs per wave loaded with R's
        static_assert(3 * FR <= 32 && 3 * FS <= 32, "r7m / s7m hold 3 bits per run (HWBRJ_JFR / HWBRJ_JFS <= 10)");
        uint32_t rv[FR][FW], rn[FR], sv[FS][FSW], sn[FS], spk = 0;  // spk bit r: survivor run r packed
        uint32_t r7m = 0, s7m = 0;  // tb & 7 of the packed runs (3 bits per run)
#pragma unroll
        for (int r = 0; r < FR; r++) {
            const uint32_t dd = wave + r * kJoinWaves;
            rn[r]             = dd < nRd ? rcnt[dd] : 0u;
#ifdef HWBRJ_ABL_JNOR
            rn[r] = 0;  // dev ablation (results invalid)
#endif
            const uint64_t bb = dd < nRd ? rbase[dd] : 0ull;
            r7m |= b7_of(bb) << (3 * r);
#pragma unroll
            for (int j = 0; j < FW; j++) {
                const uint32_t o = lane + 64u * j;
                rv[r][j]         = o < rn[r] ? ldv(SideR{}, bb, o) : 0u;
            }
        }
#pragma unroll
        for (int r = 0; r < FS; r++) {
            const uint32_t dd = wave + r * kJoinWaves;
            sn[r]             = dd < nSd ? dcnt[dd] : 0u;
#ifdef HWBRJ_ABL_JNOS
            sn[r] = 0;  // dev ablation (results invalid)
#endif
            const uint64_t bb = dd < nSd ? dbase[dd] : 0ull;
            spk |= (uint32_t) (bb >> 63) << r;
            s7m |= b7_of(bb) << (3 * r);
#pragma unroll
            for (int j = 0; j < FSW; j++) {
                const uint32_t o = lane + 64u * j;
                sv[r][j]         = o < sn[r] ? ldv(SideS{}, bb, o) : 0u;
            }
        }
        // bits set without returns (no wave waits on them); a duplicate R key shows as fewer set
        // bits than the job's R keys (popcount after the barrier)
        auto set = [&](uint32_t x) { __hip_atomic_fetch_or(&tab[x >> 5], 1u << (x & 31u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); };
#pragma unroll
        for (int r = 0; r < FR; r++) {
#pragma unroll
            for (int j = 0; j < FW; j++)
                if (lane + 64u * j < rn[r]) set(key(SideR{}, rv[r][j], rpk, (r7m >> (3 * r)) & 7u, lane));
            if (rn[r] > 64u * FW) {  // (rare) longer run
                const uint64_t bb = rbase[wave + r * kJoinWaves];
                tail_run(SideR{}, bb, 64u * FW, rn[r], set);
            }
        }
        __syncthreads();
        stamp(1);
        {
            uint32_t pc = 0;
            for (uint32_t i = tid; i < kJoinWords / 4; i += kJoinThreads) {
                const uint4 v = ((const uint4*) tab)[i];
                pc += __builtin_popcount(v.x) + __builtin_popcount(v.y) + __builtin_popcount(v.z) + __builtin_popcount(v.w);
            }
            pc = __builtin_amdgcn_readlane(wave_incl_scan_dpp(pc), 63);
            if (lane == 0 && pc) atomicAdd(&dupflag, pc);  // (dupflag: the set bits)
        }
        __syncthreads();
        hashed = dupflag != npieces;  // uniform
        stamp(2);
        if (!hashed) {
            probe_begin();
            auto test = [&](uint32_t x) { cnt += (tab[x >> 5] >> (x & 31u)) & 1u; };
#pragma unroll
            for (int r = 0; r < FS; r++) {
#pragma unroll
                for (int j = 0; j < FSW; j++)
                    if (lane + 64u * j < sn[r]) test(key(SideS{}, sv[r][j], (spk >> r) & 1u, (s7m >> (3 * r)) & 7u, lane));
                if (sn[r] > 64u * FSW) {
                    const uint64_t bb = dbase[wave + r * kJoinWaves];
                    tail_run(SideS{}, bb, 64u * FSW, sn[r], test);
                }
            }
            stamp(3);
#ifndef HWBRJ_ABL_JNOS
            walk(SR{}, SW{}, SideS{}, dcnt, dbase, (uint32_t) (kJoinWaves * FS), nSd, test);
#endif
            stamp(4);
            probe_end();
            done = true;
        }
    }
    if (!hashed && !done) {  // every R key sets bit v; a bit already set means a duplicate key
        for (uint32_t i = tid; i < kJoinWords / 4; i += kJoinThreads) ((uint4*) tab)[i] = make_uint4(0, 0, 0, 0);
        if (tid == 0) dupflag = 0;
        uint32_t dup = 0;
        for (uint32_t d0 = w0; d0 < w1; d0 += kJoinDesc) {
            const uint32_t nd = min(kJoinDesc, w1 - d0);
            load_r(d0, nd);
            walk(RR{}, RW{}, SideR{}, rcnt, rbase, 0, nd, [&](uint32_t x) {
                const uint32_t bit = 1u << (x & 31u);
                dup |= atomicOr(&tab[x >> 5], bit) & bit;
            });
        }
        if (dup) dupflag = 1;
        __syncthreads();
        hashed = dupflag != 0;  // uniform
        if (!hashed) probe_survivors([&](uint32_t x) { cnt += (tab[x >> 5] >> (x & 31u)) & 1u; });
    }
    if (hashed) {  // duplicate R keys (or keys too wide for the bitmap): counting hash table over
                   // pieces of consecutive R runs holding <= kJoinPiece keys (a run has <= slot)
        for (uint32_t d0 = w0; d0 < w1; d0 += kJoinDesc) {
            const uint32_t nd = min(kJoinDesc, w1 - d0);
            load_r(d0, nd);
            if (tid == 0) {
                uint32_t np = 0, acc = 0;
                pend[0] = 0;
                for (uint32_t d = 0; d < nd; d++) {
                    if (acc + rcnt[d] > kJoinPiece && acc > 0) {
                        pend[++np] = d;
                        acc        = 0;
                    }
                    acc += rcnt[d];
                }
                pend[++np] = nd;
                npieces    = np;
            }
            __syncthreads();
            const uint32_t np = npieces;
            for (uint32_t pc = 0; pc < np; pc++) {
                const uint32_t da = pend[pc], db = pend[pc + 1];
                __syncthreads();
                if (P.jkind == 0) {  // counting hash table (bucket_chaining_join's role)
                    for (uint32_t i = tid; i < kJoinT / 4; i += kJoinThreads)
                        ((uint4*) tab)[i] = make_uint4(kEmpty, kEmpty, kEmpty, kEmpty);
                    __syncthreads();
                    walk(RR{}, RW{}, SideR{}, rcnt, rbase, da, db, [&](uint32_t x) { join_insert(tab, x); });
                    probe_survivors([&](uint32_t x) { cnt += join_count(tab, x); });  // (starts with a barrier)
                    continue;
                }
                // Histogram join of Kim et al. (histogram_join / histogram_optimized_join,
                // src/parallel_radix_join_bloom.c:350-419, :441-555): a histogram of the piece's R
                // keys over NH = max(4, next_pow2(n) / 4) buckets, its prefix sum, the keys
                // reordered by bucket (keys = tab[0, kJoinPiece), hist = tab[kJoinPiece, +NH + 2));
                // every survivor compares the keys of its bucket -- one by one (PRH), or 4 per
                // 16-byte LDS read (PRHO, the reference's SIMD compare).
                uint32_t n = 0;
                for (uint32_t d = da; d < db; d++) n += rcnt[d];
                uint32_t NH = 4;
                while (NH * 4 < n) NH <<= 1;
                uint32_t* keys = tab;
                uint32_t* hist = tab + kJoinPiece;
                for (uint32_t i = tid; i < NH + 2; i += kJoinThreads) hist[i] = 0;
                __syncthreads();
                walk(RR{}, RW{}, SideR{}, rcnt, rbase, da, db, [&](uint32_t x) { atomicAdd(&hist[(x & (NH - 1u)) + 2], 1u); });
                __syncthreads();
                if (wave == 0) {  // inclusive prefix sum of hist[2, NH + 2): 16 buckets per lane
                    const uint32_t per = (NH + 63) / 64, b0 = 2 + lane * per;
                    uint32_t       loc = 0;
                    for (uint32_t i = 0; i < per; i++)
                        if (b0 + i < NH + 2) loc += hist[b0 + i];
                    uint32_t run = wave_incl_scan(loc) - loc;
                    for (uint32_t i = 0; i < per; i++)
                        if (b0 + i < NH + 2) {
                            run += hist[b0 + i];
                            hist[b0 + i] = run;
                        }
                }
                __syncthreads();
                walk(RR{}, RW{}, SideR{}, rcnt, rbase, da, db, [&](uint32_t x) {
                    keys[atomicAdd(&hist[(x & (NH - 1u)) + 1], 1u)] = x;  // bucket b: [hist[b], hist[b + 1])
                });
                if (P.jkind == 1) {
                    probe_survivors([&](uint32_t x) {
                        const uint32_t b = x & (NH - 1u);
                        for (uint32_t j = hist[b], e = hist[b + 1]; j < e; j++) cnt += keys[j] == x;
                    });
                } else {
                    probe_survivors([&](uint32_t x) {
                        const uint32_t b = x & (NH - 1u), j0 = hist[b], e = hist[b + 1];
                        for (uint32_t j = j0 & ~3u; j < e; j += 4) {
                            const uint4 k = *(const uint4*) &keys[j];
                            cnt += (k.x == x && j >= j0) + (k.y == x && j + 1 >= j0 && j + 1 < e) +
                                   (k.z == x && j + 2 >= j0 && j + 2 < e) + (k.w == x && j + 3 < e);
                        }
                    });
                }
            }
        }
    }
    cnt_acc += cnt;
    tp_acc += t_probe;
    stamp(5);
#ifdef HWBRJ_STAMPS
    if (P.dbg && tid == 0)
        for (int k = 0; k < 6; k++) atomicAdd((unsigned long long*) &P.dbg[(blk & 1023u) * 8 + k], (unsigned long long) tph[k]);
#endif
}

// The uniform-format join (every launch without unstaged probe items, the north star's) and the
// mixed one; both are launched, the one whose case this is not returns at once. The mixed one runs
// on a small grid of persistent workgroups (an empty launch of it costs ~1 us, a full grid ~14 us);
// it is rare: the Engine stops packing after a join that had unstaged items (pack3_hint_).
// The end of a join workgroup: its matches go to partial sum blk % kJoinSumSlots (each in its own
// 128-byte line, so the adds are not serialised on one address; with P.timing also its probe and
// total ticks). No kernel sums the slots: the host reads them with the other counts when it waits
// for the join (Engine::wait). (Summing them on the device was measured: a last-workgroup ticket
// per slot costs as much as the launch it saves, and with a __threadfence() -- an agent-scope
// release, which writes the XCD's L2 back -- the join took 0.84 instead of 0.29 ms.)
__device__ __forceinline__ void join_finish(const JoinParams& P, uint64_t cnt, uint64_t t_probe, uint64_t t_start) {
    __shared__ uint64_t wsum[kJoinWaves];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    cnt = wave_sum_u64(cnt);
    __syncthreads();  // (the previous job's LDS reads are done)
    if (lane == 0) wsum[wave] = cnt;
    __syncthreads();
    if (tid != 0) return;
    uint64_t t = 0;
    for (int w = 0; w < kJoinWaves; w++) t += wsum[w];
    uint64_t* slot = &P.jsum[(blockIdx.x % kJoinSumSlots) * kJoinSumStride];
    if (t) atomicAdd((unsigned long long*) slot, (unsigned long long) t);
    if (P.timing) {
        if (t_probe) atomicAdd((unsigned long long*) (slot + 1), (unsigned long long) t_probe);
        atomicAdd((unsigned long long*) (slot + 2), (unsigned long long) (wall_clock64() - t_start));
    }
}

template <int KW>
__global__ __launch_bounds__(kJoinThreads) void k_join(JoinParams P) {
    __shared__ JoinShared L;
    const bool mixed = __builtin_amdgcn_readfirstlane(P.r_kbits && P.fmt_cnt && *P.fmt_cnt ? 1u : 0u) != 0;
    if (mixed) return;  // (k_join_mixed's launch)
    const uint64_t t_start = P.timing ? wall_clock64() : 0;
    uint64_t       cnt = 0, t_probe = 0;
    join_job<false, KW>(P, blockIdx.x, L, cnt, t_probe);
    join_finish(P, cnt, t_probe, t_start);
}

__global__ __launch_bounds__(kJoinThreads) void k_join_mixed(JoinParams P) {
    __shared__ JoinShared L;
    if (!(P.r_kbits && P.fmt_cnt && *P.fmt_cnt)) return;
    const uint64_t t_start = P.timing ? wall_clock64() : 0;
    uint64_t       cnt = 0, t_probe = 0;
    for (uint32_t b = blockIdx.x; b < P.jobs + kJoinExtra; b += gridDim.x) {
        __syncthreads();  // the previous job's LDS reads are done
        join_job<true>(P, b, L, cnt, t_probe);
    }
    join_finish(P, cnt, t_probe, t_start);
}

// ============================================================ K10m: the materializing join
// One workgroup per (q, sub) job. The job's R codes and payloads (the sub's runs in q's build
// sweeps) go into an LDS open-addressing table, one slot per R tuple (linear probing; duplicate
// keys keep every payload), in pieces of <= kMatPiece tuples. The job's survivors are taken
// kMatPiece at a time: every thread loads its kMatU codes at once and counts their matches in the
// table; a workgroup scan gives every match its output row (one global atomic per batch); then the
// matching survivors' chunk positions and S payloads are gathered, kMatU loads in flight, and the
// {R.payload, S.payload} pairs written (bucket_chaining_join under JOIN_RESULT_MATERIALIZE,
// src/parallel_radix_join_bloom.c:259-329, :307-312).
constexpr int      kMatThreads = 512;
constexpr int      kMatU       = 4;                    // elements per thread per batch
constexpr uint32_t kMatLog2T   = 12;
constexpr uint32_t kMatT       = 1u << kMatLog2T;      // table slots
constexpr uint32_t kMatPiece   = kMatThreads * kMatU;  // R tuples per piece, survivors per batch
constexpr uint32_t kMatDesc    = 128;                  // run descriptors per batch
constexpr int      kMatUB      = 8;                    // bitmap path: elements per thread per batch
constexpr uint32_t kMatRCap    = kMatThreads * kMatUB; // bitmap path: R tuples of a job (at most)
constexpr uint32_t kMatBmWords = 1u << (17 - 5);       // bitmap path: keys v < 2^17
static_assert(2 * kMatPiece == kMatT, "the table is at most half full");

__device__ __forceinline__ uint32_t mat_jslot(uint32_t v) { return (v * 0x9E3779B1u) >> (32 - kMatLog2T); }

// Exclusive prefix of one value per thread over the workgroup (contains barriers).
__device__ __forceinline__ uint32_t mat_block_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const int      lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    total           = 0;
#pragma unroll
    for (int w = 0; w < kMatThreads / 64; w++) {
        const uint32_t x = wsum[w];
        before += w < wave ? x : 0u;
        total += x;
    }
    __syncthreads();  // (wsum reusable)
    return before + incl - v;
}

// the descriptor d of element e: pre[d] <= e < pre[d + 1] (n descriptors)
__device__ __forceinline__ uint32_t mat_find(const uint32_t* pre, uint32_t n, uint32_t e) {
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= e) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// insert an R tuple (linear probing, one slot per tuple)
__device__ __forceinline__ void mat_insert1(uint32_t* tk, uint32_t* tp, uint32_t v, uint32_t pay) {
    uint32_t h = mat_jslot(v);
    while (atomicCAS(&tk[h], kEmpty, v) != kEmpty) h = (h + 1) & (kMatT - 1);
    tp[h] = pay;
}

// matches of kMatU survivor keys (v = kEmpty: none)
__device__ __forceinline__ void mat_count(const uint32_t* tk, const uint32_t (&v)[kMatU], uint32_t (&m)[kMatU]) {
#pragma unroll
    for (int k = 0; k < kMatU; k++) {
        m[k] = 0;
        if (v[k] != kEmpty)
            for (uint32_t h = mat_jslot(v[k]);; h = (h + 1) & (kMatT - 1)) {
                const uint32_t x = tk[h];
                if (x == kEmpty) break;
                m[k] += x == v[k] ? 1u : 0u;
            }
    }
}

// Bitmap path (unique R keys v < 2^17, the blocked / sectorized join's jobs): every R key sets its
// bit (ds_or_rtn; a bit already set means duplicate keys, and the job takes the hash table);
// a prefix popcount per 64-bit word ranks the keys, and the R payloads are stored by rank. A
// survivor costs a bit test, and a match two more LDS reads: no probe sequences, no CAS.
__global__ __launch_bounds__(kMatThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_join_mat(MatJoinParams P) {
    // LDS union: hash table {keys (kEmpty: free) [kMatT], R payloads [kMatT]}, or the bitmap path's
    // {bitmap [kMatBmWords], rank prefix per 64-bit word (u16) [kMatBmWords / 2], payloads [kMatRCap]}
    __shared__ __attribute__((aligned(16))) uint32_t smem[kMatBmWords + kMatBmWords / 4 + kMatRCap];
    static_assert(kMatBmWords + kMatBmWords / 4 + kMatRCap >= 2 * kMatT, "LDS union");
    uint32_t* tk = smem;
    uint32_t* tp = smem + kMatT;
    __shared__ uint32_t dupf;
    __shared__ uint32_t rpre[kMatDesc + 1], spre[kMatDesc + 1];
    __shared__ uint64_t rbase[kMatDesc], sbase[kMatDesc];
    __shared__ uint32_t wsum[kMatThreads / 64];
    __shared__ unsigned long long obase;
    const int      tid  = threadIdx.x;
    const uint32_t NSUB = 1u << P.log2NSUB, hs = P.hash_shift;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs, so the jobs of partition q
    // (which read the same R sweeps and S payload lines) all go to XCD q mod 8 and share its L2
    uint32_t job = blockIdx.x;
    if (P.xcd8) {
        const uint32_t x = blockIdx.x & 7u, l = blockIdx.x >> 3;
        job = ((((l >> P.log2NSUB) << 3) | x) << P.log2NSUB) | (l & (NSUB - 1u));
    }
    const uint32_t q = job >> P.log2NSUB, s = job & (NSUB - 1u);
    const uint32_t r0 = P.r_sweep_start[q], r1 = P.r_sweep_start[q + 1];
    const uint32_t qi0 = P.item_start[q], qi1 = P.item_start[q + 1];
    if (r0 == r1 || qi0 == qi1) return;  // (uniform) no R or no survivors in q
    const uint32_t lq0 = P.list_start[q];
    const uint32_t npc = (qi1 - qi0) / P.nseg;  // probe pieces of q per segment
    auto s_desc = [&](uint32_t it, uint32_t& cnt, uint64_t& base) {  // survivor run of item it
        const uint32_t local = it - qi0, seg = local / npc, piece = local - seg * npc;
        cnt  = P.surv_cnt[(uint64_t) it * NSUB + s];
        base = (uint64_t) seg * P.surv_seg_stride + (uint64_t) (lq0 + piece * P.CH) * 32 +
               P.surv_off[(uint64_t) it * NSUB + s];
    };
    // ---- single-shot form (the usual job): every descriptor in one batch, R in one piece, the
    // survivors in one batch; R and S descriptors, then R tuples and survivor codes, are loaded
    // together, so the job costs four dependent global round trips
    if (r1 - r0 <= kMatDesc && qi1 - qi0 <= kMatDesc) {  // (uniform)
        const uint32_t nrd = r1 - r0, nsd = qi1 - qi0;
#ifdef HWBRJ_ABL_MJ_EMPTY  // dev ablation (results invalid): descriptors only
        if (nrd != 0x12345) {
            uint32_t c0 = (uint32_t) tid < nrd ? P.r_cnt[(uint64_t) (r0 + tid) * NSUB + s] : 0u, t0;
            c0 = mat_block_scan(c0, wsum, t0);
            if (t0 == 0x12345678u) P.out[0] = make_uint2(c0, 0);
            return;
        }
#endif
        uint32_t       rcn = 0, scn = 0;
        if ((uint32_t) tid < nrd) {
            const uint64_t r = (uint64_t) (r0 + tid) * NSUB + s;
            rcn        = P.r_cnt[r];
            rbase[tid] = (uint64_t) (r0 + tid) * P.slot + P.r_off[r];
        }
        if ((uint32_t) tid < nsd) s_desc(qi0 + tid, scn, sbase[tid]);
        uint32_t       rtot, stot;
        const uint32_t rx = mat_block_scan(rcn, wsum, rtot);
        const uint32_t sx = mat_block_scan(scn, wsum, stot);
        if ((uint32_t) tid < nrd) rpre[tid] = rx;
        if ((uint32_t) tid < nsd) spre[tid] = sx;
        if (tid == 0) {
            rpre[nrd] = rtot;
            spre[nsd] = stot;
            dupf      = 0;
        }
        if (P.bm && rtot <= kMatRCap) {  // (uniform) ---- bitmap path
            uint32_t*       bmw = smem;
            uint16_t*       pfx = (uint16_t*) (smem + kMatBmWords);
            uint32_t*       rpy = smem + kMatBmWords + kMatBmWords / 4;
            const uint64_t* bm64 = (const uint64_t*) smem;
            for (uint32_t i = tid; i < kMatBmWords; i += kMatThreads) bmw[i] = 0;
            __syncthreads();  // descriptors visible, bitmap cleared
            uint32_t rv[kMatUB], rp[kMatUB];
#pragma unroll
            for (int k = 0; k < kMatUB; k++) {
                const uint32_t e = tid + k * kMatThreads;
                rv[k] = kEmpty;
                if (e < rtot) {
                    const uint32_t d  = mat_find(rpre, nrd, e);
                    const uint64_t ra = rbase[d] + (e - rpre[d]);
                    rv[k] = P.r_codes[ra] >> hs;
                    rp[k] = P.r_pay[ra];
                }
            }
            uint32_t dup = 0;
#pragma unroll
            for (int k = 0; k < kMatUB; k++)
                if (rv[k] != kEmpty) dup |= (atomicOr(&bmw[rv[k] >> 5], 1u << (rv[k] & 31u)) >> (rv[k] & 31u)) & 1u;
            if (dup) dupf = 1;
            __syncthreads();
            if (!dupf) {  // (uniform)
                // rank prefix: thread t owns 64-bit words 4t .. 4t + 3
                uint32_t c4[4], c = 0;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    c4[j] = (uint32_t) __builtin_popcountll(bm64[tid * 4 + j]);
                    c += c4[j];
                }
                uint32_t       ntot;
                uint32_t       run = mat_block_scan(c, wsum, ntot);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    pfx[tid * 4 + j] = (uint16_t) run;
                    run += c4[j];
                }
                __syncthreads();
                auto rank = [&](uint32_t v) {
                    const uint64_t w = bm64[v >> 6];
                    return (uint32_t) pfx[v >> 6] + (uint32_t) __builtin_popcountll(w & ((1ull << (v & 63u)) - 1ull));
                };
#pragma unroll
                for (int k = 0; k < kMatUB; k++)
                    if (rv[k] != kEmpty) rpy[rank(rv[k])] = rp[k];
                __syncthreads();  // payloads by rank complete
                for (uint32_t e0 = 0; e0 < stot; e0 += kMatRCap) {  // survivors, batch by batch
                    uint64_t a[kMatUB];
                    uint32_t v[kMatUB], hit = 0;
#pragma unroll
                    for (int k = 0; k < kMatUB; k++) {
                        const uint32_t e = e0 + tid + k * kMatThreads;
                        v[k] = kEmpty;
                        a[k] = 0;
                        if (e < stot) {
                            const uint32_t d = mat_find(spre, nsd, e);
                            a[k] = sbase[d] + (e - spre[d]);
                            v[k] = P.surv[a[k]] >> hs;
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kMatUB; k++)
                        if (v[k] != kEmpty) hit |= ((bmw[v[k] >> 5] >> (v[k] & 31u)) & 1u) << k;
                    uint32_t pos[kMatUB], sp[kMatUB];
#pragma unroll
                    for (int k = 0; k < kMatUB; k++) pos[k] = (hit >> k) & 1u ? P.surv_pos[a[k]] : 0u;
                    uint32_t       tot;
                    const uint32_t off = mat_block_scan((uint32_t) __builtin_popcount(hit), wsum, tot);
                    if (tot == 0) continue;  // (uniform)
                    if (tid == 0) obase = atomicAdd(P.count, (unsigned long long) tot);
#pragma unroll
                    for (int k = 0; k < kMatUB; k++) sp[k] = (hit >> k) & 1u ? P.s_pay[pos[k]] : 0u;
                    __syncthreads();
                    uint64_t o = obase + off;
#pragma unroll
                    for (int k = 0; k < kMatUB; k++) {
                        if (!((hit >> k) & 1u)) continue;
                        if (o < P.cap) P.out[o] = make_uint2(rpy[rank(v[k])], sp[k]);
                        o++;
                    }
                }
                return;
            }
            // duplicate R keys: the hash table (over the same LDS)
        }
        if (rtot <= kMatPiece && stot <= kMatPiece) {  // (uniform)
            __syncthreads();  // descriptors visible; the bitmap path is done with the LDS
            for (uint32_t i = tid; i < kMatT; i += kMatThreads) tk[i] = kEmpty;
            __syncthreads();
            uint32_t rc[kMatU], rp[kMatU], v[kMatU], m[kMatU];
            uint64_t a[kMatU];
#pragma unroll
            for (int k = 0; k < kMatU; k++) {
                const uint32_t e = tid + k * kMatThreads;
                if (e < rtot) {
#ifdef HWBRJ_ABL_MJ_NOLOAD  // dev ablation (results invalid): no R loads
                    rc[k] = e * 2654435761u;
                    rp[k] = e;
#else
                    const uint32_t d  = mat_find(rpre, nrd, e);
                    const uint64_t ra = rbase[d] + (e - rpre[d]);
                    rc[k] = P.r_codes[ra];
                    rp[k] = P.r_pay[ra];
#endif
                }
                v[k] = kEmpty;
                a[k] = 0;
                if (e < stot) {
                    const uint32_t d = mat_find(spre, nsd, e);
                    a[k] = sbase[d] + (e - spre[d]);
                    v[k] = P.surv[a[k]] >> hs;
                }
            }
#ifdef HWBRJ_ABL_MJ_NOINS  // dev ablation (results invalid): R loaded, not inserted
            if (rc[0] + rc[1] + rc[2] + rc[3] + rp[0] + rp[1] + rp[2] + rp[3] == 0x12345678u) P.out[0] = make_uint2(0, 0);
            return;
#endif
#pragma unroll
            for (int k = 0; k < kMatU; k++)
                if (tid + k * kMatThreads < rtot) mat_insert1(tk, tp, rc[k] >> hs, rp[k]);
            __syncthreads();  // table complete
#ifdef HWBRJ_ABL_MJ_R  // dev ablation (results invalid): R table only
            if (v[0] != 0x12345678u) return;
#endif
            mat_count(tk, v, m);
            uint32_t cnt = 0;
#pragma unroll
            for (int k = 0; k < kMatU; k++) cnt += m[k];
            uint32_t pos[kMatU], sp[kMatU];
#pragma unroll
            for (int k = 0; k < kMatU; k++) pos[k] = m[k] ? P.surv_pos[a[k]] : 0u;  // (in flight over the scan)
            uint32_t       tot;
            const uint32_t off = mat_block_scan(cnt, wsum, tot);
            if (tot == 0) return;  // (uniform)
            if (tid == 0) obase = atomicAdd(P.count, (unsigned long long) tot);
#pragma unroll
            for (int k = 0; k < kMatU; k++) sp[k] = m[k] ? P.s_pay[pos[k]] : 0u;
            __syncthreads();
            uint64_t o = obase + off;
#pragma unroll
            for (int k = 0; k < kMatU; k++) {
                if (!m[k]) continue;
                for (uint32_t h = mat_jslot(v[k]);; h = (h + 1) & (kMatT - 1)) {
                    const uint32_t x = tk[h];
                    if (x == kEmpty) break;
                    if (x == v[k]) {
                        if (o < P.cap) P.out[o] = make_uint2(tp[h], sp[k]);
                        o++;
                    }
                }
            }
            return;
        }
    }
    // ---- general form: R descriptor batches x R pieces x survivor batches
    for (uint32_t rd0 = r0; rd0 < r1; rd0 += kMatDesc) {  // R run descriptors, batch by batch
        const uint32_t nrd = min(kMatDesc, r1 - rd0);
        __syncthreads();  // previous descriptors consumed
        uint32_t c = 0;
        if ((uint32_t) tid < nrd) {
            const uint64_t r = (uint64_t) (rd0 + tid) * NSUB + s;
            c          = P.r_cnt[r];
            rbase[tid] = (uint64_t) (rd0 + tid) * P.slot + P.r_off[r];
        }
        uint32_t       rtot;
        const uint32_t rx = mat_block_scan(c, wsum, rtot);
        if ((uint32_t) tid < nrd) rpre[tid] = rx;
        if (tid == 0) rpre[nrd] = rtot;
        __syncthreads();
        for (uint32_t pb = 0; pb < rtot; pb += kMatPiece) {
            const uint32_t pe = min(rtot, pb + kMatPiece);
            __syncthreads();  // the previous piece's survivors are done with the table
            for (uint32_t i = tid; i < kMatT; i += kMatThreads) tk[i] = kEmpty;
            uint32_t rc[kMatU], rp[kMatU];  // this thread's R tuples of the piece (loads in flight)
#pragma unroll
            for (int k = 0; k < kMatU; k++) {
                const uint32_t e = pb + tid + k * kMatThreads;
                rc[k] = kEmpty;
                if (e < pe) {
                    const uint32_t d = mat_find(rpre, nrd, e);
                    const uint64_t a = rbase[d] + (e - rpre[d]);
                    rc[k] = P.r_codes[a];
                    rp[k] = P.r_pay[a];
                }
            }
            __syncthreads();  // table cleared
#pragma unroll
            for (int k = 0; k < kMatU; k++)
                if (pb + tid + k * kMatThreads < pe) mat_insert1(tk, tp, rc[k] >> hs, rp[k]);
            for (uint32_t sd0 = qi0; sd0 < qi1; sd0 += kMatDesc) {  // survivor runs of the job
                const uint32_t nsd = min(kMatDesc, qi1 - sd0);
                __syncthreads();  // table complete; previous descriptors consumed
                uint32_t sc = 0;
                if ((uint32_t) tid < nsd) s_desc(sd0 + tid, sc, sbase[tid]);
                uint32_t       stot;
                const uint32_t sx = mat_block_scan(sc, wsum, stot);
                if ((uint32_t) tid < nsd) spre[tid] = sx;
                if (tid == 0) spre[nsd] = stot;
                __syncthreads();
                for (uint32_t e0 = 0; e0 < stot; e0 += kMatPiece) {
                    uint64_t a[kMatU];
                    uint32_t v[kMatU], m[kMatU];
#pragma unroll
                    for (int k = 0; k < kMatU; k++) {
                        const uint32_t e = e0 + tid + k * kMatThreads;
                        a[k] = ~0ull;
                        v[k] = kEmpty;
                        if (e < stot) {
                            const uint32_t d = mat_find(spre, nsd, e);
                            a[k] = sbase[d] + (e - spre[d]);
                            v[k] = P.surv[a[k]] >> hs;
                        }
                    }
                    mat_count(tk, v, m);
                    uint32_t cnt = 0;
#pragma unroll
                    for (int k = 0; k < kMatU; k++) cnt += m[k];
                    uint32_t       tot;
                    const uint32_t off = mat_block_scan(cnt, wsum, tot);
                    if (tot == 0) continue;  // (uniform)
                    if (tid == 0) obase = atomicAdd(P.count, (unsigned long long) tot);
                    __syncthreads();
                    uint64_t o = obase + off;
                    uint32_t pos[kMatU], sp[kMatU];
#pragma unroll
                    for (int k = 0; k < kMatU; k++) pos[k] = m[k] ? P.surv_pos[a[k]] : 0u;
#pragma unroll
                    for (int k = 0; k < kMatU; k++) sp[k] = m[k] ? P.s_pay[pos[k]] : 0u;
#pragma unroll
                    for (int k = 0; k < kMatU; k++) {
                        if (!m[k]) continue;
                        for (uint32_t h = mat_jslot(v[k]);; h = (h + 1) & (kMatT - 1)) {
                            const uint32_t x = tk[h];
                            if (x == kEmpty) break;
                            if (x == v[k]) {
                                if (o < P.cap) P.out[o] = make_uint2(tp[h], sp[k]);
                                o++;
                            }
                        }
                    }
                }
            }
        }
    }
}

void launch_join_mat(const MatJoinParams& p0, uint32_t jobs, hipStream_t st) {
    MatJoinParams p = p0;
    p.xcd8          = ((jobs >> p.log2NSUB) % 8 == 0 && !dev_knobs().noxcd) ? 1u : 0u;
    k_join_mat<<<jobs, kMatThreads, 0, st>>>(p);
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

// ======================================== K11b: basic k >= 2, partition slices without atomics
// The reference sets all k bits of every R key anywhere in the m-bit filter (add_basic,
// src/bloom_filter.c:73-89). Here every bit position becomes an element (k_bitpos), the SWWC
// scatter partitions the positions by their low log2F bits (the slice they belong to, SRC_CODES),
// and one workgroup per partition ORs its positions into the slice in LDS (k_slice_fill).
__global__ void k_bitpos(const uint2* __restrict__ R, uint64_t n, Geometry g, uint32_t* __restrict__ out) {
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    const uint32_t msz    = (uint32_t) g.m;
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint32_t key = R[i].x;
        uint32_t       h = mod_m(crapwow(kSeed, key), msz), y = mod_m(key + kSeed, msz);
        for (uint32_t j = 0; j < g.k; j++) {  // element j * n + i: coalesced per bit
            out[(uint64_t) j * n + i] = h;
            h = mod_m(h + y, msz);
            y = mod_m(y + j + 1u, msz);
        }
    }
}

__global__ __launch_bounds__(1024) void k_slice_fill(const uint32_t* __restrict__ pool,
                                                     const uint32_t* __restrict__ list,
                                                     const uint32_t* __restrict__ list_start, Geometry g,
                                                     uint32_t* __restrict__ slices) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t q = blockIdx.x, segw = g.seg_words;
    const uint32_t l0 = list_start[q], l1 = list_start[q + 1];
    const uint64_t nw = (uint64_t) (l1 - l0) * 32u;
    for (uint32_t seg = 0; seg < g.nseg; seg++) {
        for (uint32_t i = threadIdx.x; i < segw; i += blockDim.x) lds[i] = 0;
        __syncthreads();
        // 32 lanes per chunk (coalesced); kFillU list entries, then kFillU words, in flight per thread
        constexpr int kFillU = 8;
        for (uint64_t i0 = threadIdx.x; i0 < nw; i0 += (uint64_t) blockDim.x * kFillU) {
            uint32_t e[kFillU], v[kFillU], okm = 0;
#pragma unroll
            for (int u = 0; u < kFillU; u++) {
                const uint64_t i = i0 + (uint64_t) u * blockDim.x;
                e[u]             = i < nw ? list[l0 + (uint32_t) (i >> 5)] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kFillU; u++) {
                const uint64_t i  = i0 + (uint64_t) u * blockDim.x;
                const bool     ok = i < nw && (uint32_t) (i & 31u) < list_count(e[u]);
                v[u]              = ok ? pool[(uint64_t) (e[u] & kListIdMask) * 32 + (i & 31u)] : 0u;
                okm |= (ok ? 1u : 0u) << u;
            }
#pragma unroll
            for (int u = 0; u < kFillU; u++) {
                const uint32_t lb = v[u] >> g.log2F;
                if (!((okm >> u) & 1u) || (lb >> g.log2seg) != seg) continue;
                const uint32_t off = lb & (g.seg_bits - 1u);
                atomicOr(&lds[off >> 5], 1u << (off & 31u));
            }
        }
        __syncthreads();
        uint4*       dst = (uint4*) (slices + ((uint64_t) q * g.nseg + seg) * segw);
        const uint4* src = (const uint4*) lds;
        for (uint32_t i = threadIdx.x; i < segw / 4; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
}

void launch_bitpos(const uint2* R, uint64_t n, const Geometry& g, uint32_t* out, hipStream_t st) {
    k_bitpos<<<4096, 256, 0, st>>>(R, n, g, out);
}

void launch_slice_fill(const uint32_t* pool, const uint32_t* list, const uint32_t* list_start,
                       const Geometry& g, uint32_t* slices, hipStream_t st) {
    const size_t lds = (size_t) g.seg_words * 4;
    (void) hipFuncSetAttribute((const void*) &k_slice_fill, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_slice_fill<<<1u << g.log2F, 1024, lds, st>>>(pool, list, list_start, g, slices);
}

// ================================================================ K12: result materialization
// (R.payload, S.payload) pairs of every match, the reference's JOIN_RESULT_MATERIALIZE output
// (src/parallel_radix_join_bloom.c:307-312: key = R rid, payload = S rid). A separate pass after
// the counting pipeline (which fixes the output size): an open-addressing table of R
// (entry = (row + 1) << 32 | key, 0 = empty, linear probing), then every S tuple walks its probe
// sequence; a wave takes its output range with one atomic and every matching lane writes its
// pairs there (a second walk, taken only by lanes that matched).
__device__ __forceinline__ uint32_t mat_slot(uint32_t key, uint64_t mask) {
    return (uint32_t) (mix32(key * 0x9E3779B1u + 0x7F4A7C15u) & mask);
}

__global__ __launch_bounds__(256) void k_mat_build(const uint2* __restrict__ R, uint64_t n,
                                                    unsigned long long* __restrict__ tab,
                                                    uint64_t mask) {
    uint64_t       i      = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n; i += stride) {
        const uint32_t           key = R[i].x;
        const unsigned long long e   = ((unsigned long long) (i + 1) << 32) | key;
        uint64_t                 h   = mat_slot(key, mask);
        while (atomicCAS(&tab[h], 0ull, e) != 0ull) h = (h + 1) & mask;
    }
}

// The last join's filter as a pre-test (no false negatives, so it only skips table walks): the
// reference bits of the key (src/bloom_filter.c:73-141) read from the partition slices (or the
// global bitmap of MODE_GLOBAL).
__device__ __forceinline__ bool mat_filter(uint32_t key, const Geometry& g, const uint32_t* slices,
                                           const uint32_t* bm, const CrcTables* tabs) {
    if (g.mode == MODE_NOBLOOM) return true;
    const uint32_t code = key_code(&tabs->fwd[0][0], key);
    if (g.mode == MODE_GLOBAL) return global_contains(key, code, g, bm);
    const uint32_t F1 = (1u << g.log2F) - 1u;
    auto bit = [&](uint32_t q, uint32_t sb) {  // bit sb of slice q
        const uint32_t* w = slices + ((uint64_t) q * g.nseg + (sb >> g.log2seg)) * g.seg_words;
        const uint32_t  o = sb & (g.seg_bits - 1u);
        return (w[o >> 5] >> (o & 31u)) & 1u;
    };
    if (g.mode == MODE_SLICE_BASIC) {  // bit b lives in slice b & F1 at b >> log2F
        const uint32_t msz = (uint32_t) g.m;
        uint32_t       h = mod_m(crapwow(kSeed, key), msz), y = mod_m(key + kSeed, msz);
        for (uint32_t i = 0; i < g.k; i++) {
            if (!bit(h & F1, h >> g.log2F)) return false;
            h = mod_m(h + y, msz);
            y = mod_m(y + i + 1u, msz);
        }
        return true;
    }
    const uint32_t q    = code & F1;
    const uint32_t base = ((code >> g.log2F) & g.lbmask) << g.log2B;
    const uint32_t mask = g.B - 1u;
    uint32_t       h = crapwow(kSeed, key) & mask, y = (key + kSeed) & mask;
    const uint32_t s0 = h >> g.log2secw;
    for (uint32_t i = 0; i < g.k; i++) {
        const uint32_t pos = g.variant == VAR_SECTORIZED
                                 ? (((s0 + i) & g.nsecmask) << g.log2secw) | (h & ((1u << g.log2secw) - 1u))
                                 : h;
        if (!bit(q, base + pos)) return false;
        h = (h + y) & mask;
        y = (y + i + 1u) & mask;
    }
    return true;
}

constexpr uint32_t kMatBuf = 4096;  // pairs staged in LDS per workgroup before one output atomic

__global__ __launch_bounds__(256) void k_mat_probe(const uint2* __restrict__ S, uint64_t n,
                                                    const uint2* __restrict__ R,
                                                    const unsigned long long* __restrict__ tab,
                                                    uint64_t mask, uint2* __restrict__ out,
                                                    uint64_t cap, unsigned long long* __restrict__ count,
                                                    Geometry g, const uint32_t* __restrict__ slices,
                                                    const uint32_t* __restrict__ bm,
                                                    const CrcTables* __restrict__ tabs) {
    // Pairs are staged in LDS and appended to `out` with one atomic per flush (a single global
    // counter taken per wave serialises at the L2); a burst beyond the stage takes one atomic per
    // pair.
    __shared__ uint2              buf[kMatBuf];
    __shared__ uint32_t           nbuf;
    __shared__ unsigned long long obase;
    const uint64_t e0 = n * blockIdx.x / gridDim.x, e1 = n * (blockIdx.x + 1) / gridDim.x;
    if (threadIdx.x == 0) nbuf = 0;
    __syncthreads();
    auto flush = [&]() {
        const uint32_t c = min(nbuf, kMatBuf);
        if (threadIdx.x == 0) obase = c ? atomicAdd(count, (unsigned long long) c) : 0ull;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x)
            if (obase + i < cap) out[obase + i] = buf[i];
        __syncthreads();
        if (threadIdx.x == 0) nbuf = 0;
        __syncthreads();
    };
    for (uint64_t t0 = e0; t0 < e1; t0 += blockDim.x) {
        const uint64_t i  = t0 + threadIdx.x;
        if (i < e1) {
            const uint2 st = S[i];
            if (mat_filter(st.x, g, slices, bm, tabs)) {
                for (uint64_t h = mat_slot(st.x, mask);; h = (h + 1) & mask) {
                    const unsigned long long e = tab[h];
                    if (e == 0ull) break;
                    if ((uint32_t) e != st.x) continue;
                    const uint2    pr   = make_uint2(R[(e >> 32) - 1].y, st.y);  // (R rid, S rid)
                    const uint32_t slot = atomicAdd(&nbuf, 1u);
                    if (slot < kMatBuf) {
                        buf[slot] = pr;
                    } else {  // burst beyond the stage
                        const unsigned long long o = atomicAdd(count, 1ull);
                        if (o < cap) out[o] = pr;
                    }
                }
            }
        }
        __syncthreads();
        if (nbuf >= kMatBuf / 2) flush();  // uniform (read after the barrier)
    }
    flush();
}

void launch_mat_build(const uint2* R, uint64_t n, unsigned long long* tab, uint64_t mask, hipStream_t st) {
    k_mat_build<<<8192, 256, 0, st>>>(R, n, tab, mask);
}

void launch_mat_probe(const uint2* S, uint64_t n, const uint2* R, const unsigned long long* tab,
                      uint64_t mask, uint2* out, uint64_t cap, unsigned long long* count,
                      const Geometry& g, const uint32_t* slices, const uint32_t* bm,
                      const CrcTables* tabs, hipStream_t st) {
    k_mat_probe<<<2048, 256, 0, st>>>(S, n, R, tab, mask, out, cap, count, g, slices, bm, tabs);
}

// ================================= K13: partitioned multi-GPU join (R and survivors exchanged)
// Rank r of G owns partitions [r F / G, (r + 1) F / G). Its R shard is scattered locally; every
// partition's chunks go to the owner (k_pj_gather: all chunks in list order, so each destination's
// chunks are one contiguous block), the owner rebuilds its partitions' lists from what every
// source sent (k_pj_relist) and builds their slices and join runs; the slices are all-gathered.
// The S shard is scattered and probed locally against the full filter, and each item's survivors
// go to the owner of its partition (k_pj_surv_pack), which joins them (k_join with item_base).

// out chunk p (8 lanes of 16 B) = pool chunk of list entry p; ent[p] = p | the entry's count bits.
// Chunks p in [own.lo, own.hi) -- this rank's block to itself -- go to own.out / own.ent at p +
// own.delta instead (the receive buffer: the exchange skips the copy to itself).
__global__ __launch_bounds__(256) void k_pj_gather(const uint32_t* __restrict__ pool,
                                                   const uint32_t* __restrict__ list, uint32_t n,
                                                   uint4* __restrict__ out, uint32_t* __restrict__ ent, PjOwn own) {
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t t = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; t < (uint64_t) n * 8; t += stride) {
        const uint32_t p = (uint32_t) (t >> 3), l8 = (uint32_t) (t & 7);
        const uint32_t e = list[p];
        const bool     me = p >= own.lo && p < own.hi;
        const uint64_t d  = me ? (uint64_t) ((int64_t) p + own.delta) : p;
        (me ? (uint4*) own.out : out)[d * 8 + l8] = ((const uint4*) pool)[(uint64_t) (e & kListIdMask) * 8 + l8];
        if (l8 == 0) (me ? own.ent : ent)[d] = p | (e & ~kListIdMask);
    }
}

// One block per (source, owned partition) pair: tab[4 pair + {0, 1, 2, 3}] = first received
// entry, count, destination list position, chunk id adjustment (source block base in the received
// chunks minus the source's id of its block's first chunk).
__global__ __launch_bounds__(256) void k_pj_relist(const uint32_t* __restrict__ rent,
                                                   const int64_t* __restrict__ tab,
                                                   uint32_t* __restrict__ list) {
    const int64_t* t = tab + 4 * (uint64_t) blockIdx.x;
    const uint64_t so = (uint64_t) t[0], n = (uint64_t) t[1], dl = (uint64_t) t[2];
    const int64_t  adj = t[3];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t e = rent[so + i];
        list[dl + i]     = (uint32_t) ((int64_t) (e & kListIdMask) + adj) | (e & ~kListIdMask);
    }
}

// One wave per item: its `tot` survivor words (contiguous from the item region's start, grouped
// by sub) to out + soff[it]; items in [own.lo, own.hi) to own.out + soff[it] + own.delta instead.
__global__ __launch_bounds__(256) void k_pj_surv_pack(const uint32_t* __restrict__ surv,
                                                      const uint64_t* __restrict__ region,
                                                      const uint32_t* __restrict__ tot,
                                                      const uint64_t* __restrict__ soff, uint32_t n,
                                                      uint32_t* __restrict__ out, PjOwn own) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv   = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw   = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t it = wv; it < n; it += nw) {
        const bool     me  = it >= own.lo && it < own.hi;
        const uint64_t src = region[it], dst = me ? (uint64_t) ((int64_t) soff[it] + own.delta) : soff[it];
        uint32_t*      o   = me ? (uint32_t*) own.out : out;
        const uint32_t c   = tot[it];
        for (uint32_t i = lane; i < c; i += 64) o[dst + i] = surv[src + i];
    }
}

// ---- device-side item tables (no host round trip for per-item counts)
constexpr uint32_t kPjScanBlock = 1024;  // items per scan block

// Block-wide exclusive scan of one u32 per thread (1024 threads): returns this thread's exclusive
// prefix and the block total.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan(v);
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    total         = 0;
    for (uint32_t w = 0; w < 16; w++) {
        const uint32_t x = wsum[w];
        if (w < wave) base += x;
        total += x;
    }
    __syncthreads();
    return base + incl - v;
}

// Probe items of this rank (it < I): the survivor region of the item (seg * LS * 32 + first list
// position * 32, as k_probe wrote it), its survivor total over the NSUB sub runs, and the total of
// each block of kPjScanBlock items.
// (I = item_start[F], read on the device: the grid covers the items' upper bound, so no host round
// trip is needed before the launch)
__global__ __launch_bounds__(1024) void k_pj_items(const uint32_t* __restrict__ item_start,
                                                   const uint32_t* __restrict__ list_start,
                                                   const uint32_t* __restrict__ cnt, uint32_t F,
                                                   uint32_t nseg, uint32_t CH, uint64_t seg_words,
                                                   uint32_t NSUB, uint64_t* __restrict__ region,
                                                   uint32_t* __restrict__ tot, uint64_t* __restrict__ bsum) {
    __shared__ uint32_t wsum[16];
    const uint32_t I  = item_start[F];
    const uint32_t it = blockIdx.x * kPjScanBlock + threadIdx.x;
    uint32_t       t  = 0;
    if (it < I) {
        const uint32_t q     = find_q(item_start, F, it);
        const uint32_t i0    = item_start[q];
        const uint32_t npc   = (item_start[q + 1] - i0) / nseg;
        const uint32_t local = it - i0, seg = local / npc, piece = local - seg * npc;
        region[it] = (uint64_t) seg * seg_words + (uint64_t) (list_start[q] + piece * CH) * 32;
        for (uint32_t s = 0; s < NSUB; s++) t += cnt[(uint64_t) it * NSUB + s];
        tot[it] = t;
    }
    uint32_t total;
    (void) block_excl_scan(t, wsum, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// Received items (it < n, in received order): survivor total over the NSUB counts, block totals.
// (BI > 0: received items in blocks of BI per source, of which the first ritems[j] are valid; the
// others -- the block's padding -- count 0)
__global__ __launch_bounds__(1024) void k_pj_recv_tot(const uint32_t* __restrict__ cnt, uint32_t n,
                                                      uint32_t NSUB, uint32_t* __restrict__ tot,
                                                      uint64_t* __restrict__ bsum, uint32_t BI,
                                                      const uint32_t* __restrict__ ritems) {
    __shared__ uint32_t wsum[16];
    const uint32_t it = blockIdx.x * kPjScanBlock + threadIdx.x;
    uint32_t       t  = 0;
    if (it < n && (BI == 0 || it % BI < ritems[it / BI]))
        for (uint32_t s = 0; s < NSUB; s++) t += cnt[(uint64_t) it * NSUB + s];
    if (it < n) tot[it] = t;
    uint32_t total;
    (void) block_excl_scan(t, wsum, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// out[it] = exclusive prefix of tot over [0, it) for it <= n (block b adds the totals of blocks < b;
// the grid has n / kPjScanBlock + 1 blocks).
__global__ __launch_bounds__(1024) void k_pj_scan(const uint32_t* __restrict__ tot, uint32_t n_host,
                                                  const uint32_t* __restrict__ n_dev,
                                                  const uint64_t* __restrict__ bsum,
                                                  uint64_t* __restrict__ out) {
    __shared__ uint32_t wsum[16];
    __shared__ uint64_t red[16];
    const uint32_t n = n_dev ? *n_dev : n_host;  // (n_dev: blocks past n / kPjScanBlock idle)
    if (blockIdx.x > n / kPjScanBlock) return;
    uint64_t p = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 1024) p += bsum[b];
    p = wave_sum_u64(p);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = p;
    __syncthreads();
    uint64_t base = 0;
    for (int w = 0; w < 16; w++) base += red[w];
    const uint32_t it = blockIdx.x * kPjScanBlock + threadIdx.x;
    uint32_t       total;
    const uint32_t ex = block_excl_scan(it < n ? tot[it] : 0u, wsum, total);
    if (it <= n) out[it] = base + ex;  // (the grid covers it = n: out[n] is the grand total)
}

// sofs at the first item of every partition (q <= F): the host's per-destination word counts.
__global__ void k_pj_bound(const uint32_t* __restrict__ item_start, uint32_t F,
                           const uint64_t* __restrict__ sofs, uint64_t* __restrict__ out) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q <= F) out[q] = sofs[item_start[q]];
}

// The owner's join tables from the received per-item counts. One block per (owned partition i,
// source j) pair: tab[3 pair + {0, 1, 2}] = first received item, items, first output item. Output
// item out of received item src: ibase = its first word in the received survivors (wscan[src]),
// icnt / ioff its NSUB run counts and offsets; jobs[i][s] += the counts (every output order: items
// of partition i from source 0, 1, ...).
// (BI > 0: received survivors in blocks of BW words per source: ibase = the source block's base plus
// the item's offset in it)
__global__ __launch_bounds__(256) void k_pj_item_tables(const uint32_t* __restrict__ tab, uint32_t W,
                                                        const uint32_t* __restrict__ rcnt,
                                                        const uint64_t* __restrict__ wscan, uint32_t NSUB,
                                                        uint64_t* __restrict__ ibase, uint32_t* __restrict__ icnt,
                                                        uint32_t* __restrict__ ioff, uint32_t* __restrict__ jobs,
                                                        uint32_t BI, uint64_t BW) {
    __shared__ uint32_t js[64];
    const uint32_t* t  = tab + 3 * (uint64_t) blockIdx.x;
    const uint32_t  i  = blockIdx.x / W;
    const uint32_t  s0 = t[0], n = t[1], o0 = t[2];
    if (threadIdx.x < 64) js[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
        const uint32_t src = s0 + k, out = o0 + k;
        ibase[out] = BI ? (src / BI) * BW + (wscan[src] - wscan[(src / BI) * BI]) : wscan[src];
        uint32_t o = 0;
        for (uint32_t s = 0; s < NSUB; s++) {
            const uint32_t c = rcnt[(uint64_t) src * NSUB + s];
            icnt[(uint64_t) out * NSUB + s] = c;
            ioff[(uint64_t) out * NSUB + s] = o;
            o += c;
            if (c) atomicAdd(&js[s], c);
        }
    }
    __syncthreads();
    if (threadIdx.x < NSUB && js[threadIdx.x]) atomicAdd(&jobs[(uint64_t) i * NSUB + threadIdx.x], js[threadIdx.x]);
}

void launch_pj_items(const uint32_t* item_start, const uint32_t* list_start, const uint32_t* cnt,
                     uint32_t items_max, uint32_t F, uint32_t nseg, uint32_t CH, uint64_t seg_words, uint32_t NSUB,
                     uint64_t* region, uint32_t* tot, uint64_t* bsum, uint64_t* sofs, uint64_t* bound,
                     hipStream_t st) {
    const uint32_t nb = (items_max + kPjScanBlock) / kPjScanBlock;  // (covers it == I for sofs[I])
    k_pj_items<<<nb, 1024, 0, st>>>(item_start, list_start, cnt, F, nseg, CH, seg_words, NSUB, region, tot, bsum);
    k_pj_scan<<<nb, 1024, 0, st>>>(tot, 0, item_start + F, bsum, sofs);
    k_pj_bound<<<(F + 256) / 256, 256, 0, st>>>(item_start, F, sofs, bound);
}

void launch_pj_recv_scan(const uint32_t* cnt, uint32_t n, uint32_t NSUB, uint32_t* tot, uint64_t* bsum,
                         uint64_t* wscan, hipStream_t st, uint32_t BI, const uint32_t* ritems) {
    const uint32_t nb = (n + kPjScanBlock) / kPjScanBlock;
    k_pj_recv_tot<<<nb, 1024, 0, st>>>(cnt, n, NSUB, tot, bsum, BI, ritems);
    k_pj_scan<<<nb, 1024, 0, st>>>(tot, n, nullptr, bsum, wscan);
}

void launch_pj_item_tables(const uint32_t* tab, uint32_t pairs, uint32_t W, const uint32_t* rcnt,
                           const uint64_t* wscan, uint32_t NSUB, uint64_t* ibase, uint32_t* icnt, uint32_t* ioff,
                           uint32_t* jobs, hipStream_t st, uint32_t BI, uint64_t BW) {
    if (pairs) k_pj_item_tables<<<pairs, 256, 0, st>>>(tab, W, rcnt, wscan, NSUB, ibase, icnt, ioff, jobs, BI, BW);
}


// The native transport's counts message to every destination j (out[j NC .. (j + 1) NC)), packed on
// the device so no host read precedes its exchange: the item (or chunk) counts of j's QL partitions
// from starts[], then words = bound[(j + 1) QL] - bound[j QL] when bound is given (survivors), else
// starts[j QL] (the position of j's first chunk), then this rank's status and `extra`.
__global__ void k_pj_counts(const uint32_t* __restrict__ starts, const uint64_t* __restrict__ bound, uint32_t W,
                            uint32_t QL, uint32_t NC, uint64_t status, uint64_t extra, uint64_t extra2,
                            uint64_t* __restrict__ out) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= W * NC) return;
    const uint32_t j = t / NC, i = t % NC;
    uint64_t v;
    if (i < QL) v = starts[j * QL + i + 1] - starts[j * QL + i];
    else if (i == QL) v = bound ? bound[(j + 1) * QL] - bound[j * QL] : starts[j * QL];
    else if (i == QL + 1) v = status;
    else if (i == QL + 2) v = extra;
    else v = extra2;
    out[t] = v;
}

void launch_pj_counts(const uint32_t* starts, const uint64_t* bound, uint32_t W, uint32_t QL, uint32_t NC,
                      uint64_t status, uint64_t extra, uint64_t extra2, uint64_t* out, hipStream_t st) {
    k_pj_counts<<<(W * NC + 255) / 256, 256, 0, st>>>(starts, bound, W, QL, NC, status, extra, extra2, out);
}

void launch_pj_gather(const uint32_t* pool, const uint32_t* list, uint32_t n, void* out, uint32_t* ent,
                      hipStream_t st, const PjOwn& own) {
    if (n) k_pj_gather<<<4096, 256, 0, st>>>(pool, list, n, (uint4*) out, ent, own);
}

void launch_pj_relist(const uint32_t* rent, const int64_t* tab, uint32_t pairs, uint32_t* list,
                      hipStream_t st) {
    if (pairs) k_pj_relist<<<pairs, 256, 0, st>>>(rent, tab, list);
}

void launch_pj_surv_pack(const uint32_t* surv, const uint64_t* region, const uint32_t* tot,
                         const uint64_t* soff, uint32_t n, uint32_t* out, hipStream_t st, const PjOwn& own) {
    if (n) k_pj_surv_pack<<<2048, 256, 0, st>>>(surv, region, tot, soff, n, out, own);
}

// ---- the async partitioned join (hwbrj_join_partitioned_rccl_async): fixed exchange blocks
// Every (source, destination) block of the three variable all-to-alls is padded to the plan's
// bound (R chunks BR, survivor items BI, survivor words BW; agreed by all ranks, host-known), so the
// RCCL calls need no host-read counts. What does not fit sets flag[0]; the ranks all-reduce it at
// the end of the join and rerun it synchronously when it is set (Engine::pj_wait).
constexpr uint32_t kPjOverflow = 1u, kPjPeerFailed = 2u;

// R chunks in list order into destination j's block at j * BR (entries: their index in the block
// plus the list entry's count bits). n = lstart[F] (on the device). The block of destination `own`
// (this rank; -1: none) goes straight to own_out / own_ent at the same position: the receive
// buffer's block of this source, so the exchange skips the rank's copy to itself.
__global__ __launch_bounds__(256) void k_pjx_gather(const uint32_t* __restrict__ pool, const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ lstart, uint32_t F, uint32_t QL,
                                                    uint32_t W, uint64_t BR, uint4* __restrict__ out,
                                                    uint32_t* __restrict__ ent, int own, uint4* __restrict__ own_out,
                                                    uint32_t* __restrict__ own_ent, uint64_t* flag) {
    const uint32_t n      = lstart[F];
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    bool           over   = false;
    for (uint64_t t = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; t < (uint64_t) n * 8; t += stride) {
        const uint32_t p = (uint32_t) (t >> 3), l8 = (uint32_t) (t & 7);
        // destination: the last block start at or below p (W starts, not F: empty blocks skipped)
        uint32_t lo = 0, hi = W;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (lstart[mid * QL] <= p) lo = mid;
            else hi = mid;
        }
        const uint64_t k = p - lstart[lo * QL];  // index in the destination's block
        if (k >= BR) {
            over = true;
            continue;
        }
        const uint32_t e   = list[p];
        const bool     me  = (int) lo == own;
        const uint64_t pos = lo * BR + k;
        (me ? own_out : out)[pos * 8 + l8] = ((const uint4*) pool)[(uint64_t) (e & kListIdMask) * 8 + l8];
        if (l8 == 0) (me ? own_ent : ent)[pos] = (uint32_t) k | (e & ~kListIdMask);
    }
    if (over) atomicOr((unsigned long long*) flag, (unsigned long long) kPjOverflow);
}

// The counts c(i, j) of the (owned partition i, source j) pairs from the received counts messages
// rc[j NC + i] (F = W QL <= 1024 pairs, in LDS), each clamped to what fits in source j's block of
// B, so that nothing downstream leaves the padded receive buffers when a block overflowed (the flag
// then reruns the join), and the pair's first element in the block (partition-major within each
// source: one block scan per source). Flags a source whose block overflowed (wb > 0: its words, at
// QL, must fit wb too) or whose status (at QL + 1) is nonzero. All 1024 threads take part.
__device__ __forceinline__ void pjx_pairs(const uint64_t* __restrict__ rc, uint32_t W, uint32_t QL, uint32_t NC,
                                          uint64_t B, uint64_t wb, uint32_t* cnt, uint32_t* first, uint32_t* wsum,
                                          uint64_t* flag) {
    const uint32_t i = threadIdx.x;
    for (uint32_t j = 0; j < W; j++) {
        const uint32_t v = i < QL ? (uint32_t) rc[(uint64_t) j * NC + i] : 0u;
        uint32_t       total;
        const uint32_t c = block_excl_scan(v, wsum, total);
        if (i < QL) {
            cnt[i * W + j]   = (uint32_t) (c < B ? min<uint64_t>(v, B - c) : 0u);
            first[i * W + j] = (uint32_t) min<uint64_t>(c, B);
        }
        if (i == 0) {
            uint64_t f = 0;
            if (total > B || (wb && rc[(uint64_t) j * NC + QL] > wb)) f |= kPjOverflow;
            if (rc[(uint64_t) j * NC + QL + 1]) f |= kPjPeerFailed;
            if (f) atomicOr((unsigned long long*) flag, (unsigned long long) f);
        }
    }
    __syncthreads();
}

// The owner's R tables (one block of 1024 threads): per (owned partition i, source j) pair tab =
// {first received entry, count, list position, chunk id adjustment} (source j's chunks sit at
// j * BR of the received ones and their entries carry their index in that block), list starts
// lsO[QL + 1] and sweep starts swO[QL + 1] (bsw chunks per sweep).
__global__ __launch_bounds__(1024) void k_pjx_rtab(const uint64_t* __restrict__ rc, uint32_t W, uint32_t QL,
                                                   uint32_t NC, uint64_t BR, uint32_t bsw, int64_t* __restrict__ tab,
                                                   uint32_t* __restrict__ lsO, uint32_t* __restrict__ swO,
                                                   uint64_t* flag) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t cnt[1024], first[1024];
    pjx_pairs(rc, W, QL, NC, BR, 0, cnt, first, wsum, flag);
    const uint32_t i = threadIdx.x;
    uint32_t       t = 0;
    if (i < QL)
        for (uint32_t j = 0; j < W; j++) t += cnt[i * W + j];
    uint32_t       total;
    const uint32_t pos = block_excl_scan(i < QL ? t : 0u, wsum, total);  // list start of partition i
    if (i < QL) {
        lsO[i]     = pos;
        uint32_t p = pos;
        for (uint32_t j = 0; j < W; j++) {
            int64_t* e = tab + 4 * ((uint64_t) i * W + j);
            e[0]       = (int64_t) (j * BR + first[i * W + j]);
            e[1]       = cnt[i * W + j];
            e[2]       = p;
            e[3]       = (int64_t) (j * BR);
            p += cnt[i * W + j];
        }
    }
    if (i == 0) lsO[QL] = total;
    const uint32_t sw = i < QL ? (t + bsw - 1) / bsw : 0u;
    const uint32_t so = block_excl_scan(sw, wsum, total);
    if (i < QL) swO[i] = so;
    if (i == 0) swO[QL] = total;
}

// Survivors of this rank's probe items, item it of destination j (j = its partition / QL, k its
// index among j's items) into j's blocks: its words at j * BW + (sofs[it] - bound[j QL]), its NSUB
// run counts at (j * BI + k) * NSUB; destination `own` (this rank; -1: none) straight into the
// receive buffers own_out / own_cnt at the same positions. One wave per item; I = item_start[F]
// on the device.
__global__ __launch_bounds__(256) void k_pjx_surv_pack(const uint32_t* __restrict__ surv, const uint64_t* __restrict__ region,
                                                       const uint32_t* __restrict__ tot, const uint64_t* __restrict__ sofs,
                                                       const uint32_t* __restrict__ item_start, const uint64_t* __restrict__ bound,
                                                       const uint32_t* __restrict__ cnt, uint32_t F, uint32_t QL, uint32_t NSUB,
                                                       uint64_t BI, uint64_t BW, uint32_t* __restrict__ out,
                                                       uint32_t* __restrict__ out_cnt, int own, uint32_t* __restrict__ own_out,
                                                       uint32_t* __restrict__ own_cnt, uint64_t* flag) {
    const uint32_t I    = item_start[F];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv   = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw   = (gridDim.x * blockDim.x) >> 6;
    bool           over = false;
    for (uint32_t it = wv; it < I; it += nw) {
        const uint32_t j  = find_q(item_start, F, it) / QL;
        const uint64_t k  = it - item_start[j * QL];
        const uint64_t w  = sofs[it] - bound[j * QL];  // the item's first word in j's block
        const uint32_t c  = tot[it];
        uint32_t*      oc = (int) j == own ? own_cnt : out_cnt;
        if (k >= BI || w + c > BW) {  // (does not fit: the item goes with no survivors, flagged)
            over = true;
            if (k < BI)
                for (uint32_t s = lane; s < NSUB; s += 64) oc[(j * BI + k) * NSUB + s] = 0;
            continue;
        }
        const uint64_t src = region[it], dst = j * BW + w;
        uint32_t*      o   = (int) j == own ? own_out : out;
        for (uint32_t x = lane; x < c; x += 64) o[dst + x] = surv[src + x];
        for (uint32_t s = lane; s < NSUB; s += 64) oc[(j * BI + k) * NSUB + s] = cnt[(uint64_t) it * NSUB + s];
    }
    if (over && lane == 0) atomicOr((unsigned long long*) flag, (unsigned long long) kPjOverflow);
}

// The owner's survivor tables (one block of 1024 threads): per (owned partition i, source j) pair
// tab2 = {first received item (in j's block of BI), items, first output item}, istart[QL + 1], and
// ritems[j] (the valid items of source j's block).
__global__ __launch_bounds__(1024) void k_pjx_stab(const uint64_t* __restrict__ rc, uint32_t W, uint32_t QL, uint32_t NC,
                                                   uint64_t BI, uint64_t BW, uint32_t* __restrict__ tab2,
                                                   uint32_t* __restrict__ istart, uint32_t* __restrict__ ritems,
                                                   uint64_t* flag) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t cnt[1024], first[1024];
    pjx_pairs(rc, W, QL, NC, BI, BW, cnt, first, wsum, flag);
    const uint32_t i = threadIdx.x;
    for (uint32_t j = 0; j < W; j++) {  // (block-uniform: every thread takes part in the scans)
        uint32_t total;
        (void) block_excl_scan(i < QL ? cnt[i * W + j] : 0u, wsum, total);
        if (i == 0) ritems[j] = total;
    }
    uint32_t t = 0;
    if (i < QL)
        for (uint32_t j = 0; j < W; j++) t += cnt[i * W + j];
    uint32_t       total;
    const uint32_t pos = block_excl_scan(i < QL ? t : 0u, wsum, total);
    if (i < QL) {
        istart[i]  = pos;
        uint32_t p = pos;
        for (uint32_t j = 0; j < W; j++) {
            uint32_t* e = tab2 + 3 * ((uint64_t) i * W + j);
            e[0]        = (uint32_t) (j * BI + first[i * W + j]);
            e[1]        = cnt[i * W + j];
            e[2]        = p;
            p += cnt[i * W + j];
        }
    }
    if (i == 0) istart[QL] = total;
}

// The join's exchange sizes, for the next join's plan: out = {flag, the largest R block (chunks),
// survivor item block and word block this rank sent or received} (all-reduced with MAX over the
// ranks afterwards). rc1 / rc2: the received counts messages; ls / is / bd: this rank's R list
// starts, item starts and survivor word bounds (what it sent). One block of 1024 threads.
__global__ __launch_bounds__(1024) void k_pjx_stat(const uint64_t* __restrict__ rc1, const uint64_t* __restrict__ rc2,
                                                   const uint32_t* __restrict__ ls, const uint32_t* __restrict__ is,
                                                   const uint64_t* __restrict__ bd, uint32_t W, uint32_t QL, uint32_t NC,
                                                   const uint64_t* flag, uint64_t* __restrict__ out) {
    __shared__ uint32_t wsum[16];
    const uint32_t i  = threadIdx.x;
    uint64_t       mr = 0, mi = 0, mw = 0;
    for (uint32_t j = 0; j < W; j++) {  // (block-uniform)
        uint32_t r, it;
        (void) block_excl_scan(i < QL ? (uint32_t) rc1[(uint64_t) j * NC + i] : 0u, wsum, r);
        (void) block_excl_scan(i < QL ? (uint32_t) rc2[(uint64_t) j * NC + i] : 0u, wsum, it);
        mr = max(mr, max((uint64_t) r, (uint64_t) (ls[(j + 1) * QL] - ls[j * QL])));
        mi = max(mi, max((uint64_t) it, (uint64_t) (is[(j + 1) * QL] - is[j * QL])));
        mw = max(mw, max(rc2[(uint64_t) j * NC + QL], bd[(j + 1) * QL] - bd[j * QL]));
    }
    if (i == 0) {
        out[0] = *flag;
        out[1] = mr;
        out[2] = mi;
        out[3] = mw;
    }
}

void launch_pjx_gather(const uint32_t* pool, const uint32_t* list, const uint32_t* lstart, uint32_t F, uint32_t QL,
                       uint32_t W, uint64_t BR, void* out, uint32_t* ent, int own, void* own_out, uint32_t* own_ent,
                       uint64_t* flag, hipStream_t st) {
    k_pjx_gather<<<4096, 256, 0, st>>>(pool, list, lstart, F, QL, W, BR, (uint4*) out, ent, own, (uint4*) own_out,
                                       own_ent, flag);
}

void launch_pjx_rtab(const uint64_t* rc, uint32_t W, uint32_t QL, uint32_t NC, uint64_t BR, uint32_t bsw,
                     int64_t* tab, uint32_t* lsO, uint32_t* swO, uint64_t* flag, hipStream_t st) {
    k_pjx_rtab<<<1, 1024, 0, st>>>(rc, W, QL, NC, BR, bsw, tab, lsO, swO, flag);
}

void launch_pjx_surv_pack(const uint32_t* surv, const uint64_t* region, const uint32_t* tot, const uint64_t* sofs,
                          const uint32_t* item_start, const uint64_t* bound, const uint32_t* cnt, uint32_t F,
                          uint32_t QL, uint32_t NSUB, uint64_t BI, uint64_t BW, uint32_t* out, uint32_t* out_cnt,
                          int own, uint32_t* own_out, uint32_t* own_cnt, uint64_t* flag, hipStream_t st) {
    k_pjx_surv_pack<<<2048, 256, 0, st>>>(surv, region, tot, sofs, item_start, bound, cnt, F, QL, NSUB, BI, BW, out,
                                          out_cnt, own, own_out, own_cnt, flag);
}

void launch_pjx_stab(const uint64_t* rc, uint32_t W, uint32_t QL, uint32_t NC, uint64_t BI, uint64_t BW,
                     uint32_t* tab2, uint32_t* istart, uint32_t* ritems, uint64_t* flag, hipStream_t st) {
    k_pjx_stab<<<1, 1024, 0, st>>>(rc, W, QL, NC, BI, BW, tab2, istart, ritems, flag);
}

void launch_pjx_stat(const uint64_t* rc1, const uint64_t* rc2, const uint32_t* ls, const uint32_t* is,
                     const uint64_t* bd, uint32_t W, uint32_t QL, uint32_t NC, const uint64_t* flag, uint64_t* out,
                     hipStream_t st) {
    k_pjx_stat<<<1, 1024, 0, st>>>(rc1, rc2, ls, is, bd, W, QL, NC, flag, out);
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
    return (F * 32 + 64 + F + 4 + 3 * F + 8) * sizeof(uint32_t);  // stage, dummies, fill, ncb x2, flq, misc (+512 B static)
}

// The R and S scatters are one body under two kernel names, so per-kernel profiles (rocprofv3
// --kernel-trace --stats) report the two phases separately.
// ---------------------------------------------------------- measured copy rate (hwbrj_copy_bandwidth)
// The roofline's "measured copy-kernel bandwidth" beside the spec peak: every
// workgroup streams its own contiguous range (the shape of the scatter's reads), 16-byte loads,
// four in flight per thread.
__global__ __launch_bounds__(1024) void k_copy_bw(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t) blockIdx.x * per, e = min(n, b + per);
    for (uint64_t i = b + threadIdx.x; i < e; i += 4u * 1024u) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t k = i + u * 1024u;
            v[u] = k < e ? src[k] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (i + u * 1024u < e) dst[i + u * 1024u] = v[u];
    }
}

void launch_copy_bw(const void* src, void* dst, uint64_t bytes, int grid, hipStream_t st) {
    k_copy_bw<<<grid, 1024, 0, st>>>((const uint4*) src, (uint4*) dst, bytes / 16);
}

template <int SRC, int MODE, int FMT>
__global__ __launch_bounds__(kScThreads) void k_scatter_r(ScatterParams P) { scatter_body<SRC, MODE, FMT, HWBRJ_SC_SAUX_R>(P); }
template <int SRC, int MODE, int FMT>
__global__ __launch_bounds__(kScThreads) void k_scatter_s(ScatterParams P) { scatter_body<SRC, MODE, FMT>(P); }

template <int SRC, int MODE, int FMT>
static void scatter_inst(const ScatterParams& p, int side, uint32_t grid, hipStream_t st) {
    const size_t lds = scatter_lds_bytes(p.g.log2F);
    const void*  fn  = side == SIDE_R ? (const void*) &k_scatter_r<SRC, MODE, FMT> : (const void*) &k_scatter_s<SRC, MODE, FMT>;
    (void) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    if (side == SIDE_R) k_scatter_r<SRC, MODE, FMT><<<grid, kScThreads, lds, st>>>(p);
    else k_scatter_s<SRC, MODE, FMT><<<grid, kScThreads, lds, st>>>(p);
}

size_t scatter_pay_lds_bytes(uint32_t log2F) {
    const size_t F = (size_t) 1 << log2F;
    return (2 * (F * kPayDepth + 64) + F + 4 + 5 * F + 8) * sizeof(uint32_t);  // (+512 B static)
}

template <int MODE, int FMT>
__global__ __launch_bounds__(kScPayThreads) void k_scatter_rp(ScatterParams P) { scatter_body_pay<MODE, FMT>(P); }
template <int MODE, int FMT>
__global__ __launch_bounds__(kScPayThreads) void k_scatter_sp(ScatterParams P) { scatter_body_pay<MODE, FMT>(P); }

template <int MODE, int FMT>
static void scatter_pay_inst(const ScatterParams& p, int side, uint32_t grid, hipStream_t st) {
    const size_t lds = scatter_pay_lds_bytes(p.g.log2F);
    const void*  fn  = side == SIDE_R ? (const void*) &k_scatter_rp<MODE, FMT> : (const void*) &k_scatter_sp<MODE, FMT>;
    (void) hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    if (side == SIDE_R) k_scatter_rp<MODE, FMT><<<grid, kScPayThreads, lds, st>>>(p);
    else k_scatter_sp<MODE, FMT><<<grid, kScPayThreads, lds, st>>>(p);
}

void launch_scatter(const ScatterParams& p, int src, int side, uint32_t grid, hipStream_t st) {
    const Geometry& g = p.g;
    if (p.ppool) {  // tuples with payloads (materialization): no global-mode codes
        switch (g.mode) {
            case MODE_SLICE_BLOCK:
                if (g.format == FMT_PACKED) return scatter_pay_inst<MODE_SLICE_BLOCK, FMT_PACKED>(p, side, grid, st);
                return scatter_pay_inst<MODE_SLICE_BLOCK, FMT_CODE>(p, side, grid, st);
            case MODE_SLICE_BASIC: return scatter_pay_inst<MODE_SLICE_BASIC, FMT_CODE>(p, side, grid, st);
            default: return scatter_pay_inst<MODE_NOBLOOM, FMT_CODE>(p, side, grid, st);
        }
    }
    if (src == SRC_CODES) {
        if (g.mode == MODE_BASIC_BITJ) return scatter_inst<SRC_CODES, MODE_BASIC_BITJ, FMT_CODE>(p, side, grid, st);
        if (g.mode == MODE_CODE_OF_KEY) return scatter_inst<SRC_CODES, MODE_CODE_OF_KEY, FMT_CODE>(p, side, grid, st);
        return scatter_inst<SRC_CODES, MODE_GLOBAL, FMT_CODE>(p, side, grid, st);
    }
    switch (g.mode) {
        case MODE_SLICE_BLOCK:
            if (g.format == FMT_PACKED)
                return scatter_inst<SRC_TUPLES, MODE_SLICE_BLOCK, FMT_PACKED>(p, side, grid, st);
            return scatter_inst<SRC_TUPLES, MODE_SLICE_BLOCK, FMT_CODE>(p, side, grid, st);
        case MODE_SLICE_BASIC:
            return scatter_inst<SRC_TUPLES, MODE_SLICE_BASIC, FMT_CODE>(p, side, grid, st);
        case MODE_BASIC_POS: return scatter_inst<SRC_TUPLES, MODE_BASIC_POS, FMT_CODE>(p, side, grid, st);
        default: return scatter_inst<SRC_TUPLES, MODE_NOBLOOM, FMT_CODE>(p, side, grid, st);
    }
}

void launch_list_fill(const uint32_t* meta, const uint32_t* wg_used, uint64_t cap, uint32_t log2F,
                      const uint32_t* wgq_off, const uint32_t* colc, const uint64_t* cole,
                      uint32_t CH, uint32_t nseg, uint32_t* list_start, uint64_t* elem_start,
                      uint32_t* item_start, uint32_t* list, uint32_t grid, hipStream_t st) {
    const size_t lds = (kLfBatch + 4 * (1u << log2F) + 16) * sizeof(uint32_t);
    (void) hipFuncSetAttribute((const void*) &k_list_fill, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_list_fill<<<grid, kLfThreads, lds, st>>>(meta, wg_used, cap, log2F, wgq_off, colc, cole, CH,
                                               nseg, list_start, elem_start, item_start, list);
}

bool launch_plan(const uint32_t* wgq_chunks, const uint32_t* wgq_elems, uint32_t G, uint32_t log2F,
                 uint32_t* wgq_off, uint32_t* colc, uint64_t* cole, hipStream_t st) {
    if (G > kPlanRGs * kPlanMaxRG) return false;
    const uint32_t F = 1u << log2F;
    k_plan<<<(F + kPlanCols - 1) / kPlanCols, 1024, 0, st>>>(wgq_chunks, wgq_elems, G, log2F, wgq_off, colc, cole);
    return true;
}

size_t slice_lds_bytes(const Geometry& g) {
    const bool slices = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    return ((slices ? g.seg_words : 0) + 128 + kBSlot + 128) * sizeof(uint32_t);
}

uint32_t build_chunks_per_sweep() { return kBSweep; }
uint32_t build_sweep_slot() { return kBSlot; }

int consumer_kind(const Geometry& g) {
    if (g.mode == MODE_SLICE_BASIC) return g.k == 1 ? KIND_BASIC_K1 : KIND_BASIC_KK;
    if (g.mode == MODE_SLICE_BLOCK)
        return g.format == FMT_PACKED ? (g.k == 1 ? KIND_BLOCK_PK1 : KIND_BLOCK_PKK) : KIND_BLOCK;
    return KIND_PASS;
}


template <int KIND>
static void build_inst(const BuildParams& p, uint32_t F, size_t lds, hipStream_t st) {
    if (p.ppool) {
        (void) hipFuncSetAttribute((const void*) &k_build<KIND, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
        k_build<KIND, true><<<F, 1024, lds, st>>>(p);
        return;
    }
    (void) hipFuncSetAttribute((const void*) &k_build<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
    k_build<KIND><<<F, 1024, lds, st>>>(p);
}

template <int KIND>
static void probe_inst(const ProbeParams& p, uint32_t grid, size_t lds, hipStream_t st) {
    if (p.surv_pos) {
        if (KIND == KIND_PASS || p.g.nseg == 1) {
            (void) hipFuncSetAttribute((const void*) &k_probe<KIND, true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
            k_probe<KIND, true, true><<<grid, 1024, lds, st>>>(p);
        } else {
            (void) hipFuncSetAttribute((const void*) &k_probe<KIND, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
            k_probe<KIND, false, true><<<grid, 1024, lds, st>>>(p);
        }
        return;
    }
    if (KIND == KIND_PASS || p.g.nseg == 1) {  // one slice segment per partition: no per-word segment check
        (void) hipFuncSetAttribute((const void*) &k_probe<KIND, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
        k_probe<KIND, true><<<grid, 1024, lds, st>>>(p);
    } else {
        (void) hipFuncSetAttribute((const void*) &k_probe<KIND, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int) lds);
        k_probe<KIND, false><<<grid, 1024, lds, st>>>(p);
    }
}

void launch_build(const BuildParams& p, uint32_t F, hipStream_t st) {
    const size_t lds = slice_lds_bytes(p.g);
    switch (consumer_kind(p.g)) {
        case KIND_BLOCK_PK1: return build_inst<KIND_BLOCK_PK1>(p, F, lds, st);
        case KIND_BLOCK_PKK: return build_inst<KIND_BLOCK_PKK>(p, F, lds, st);
        case KIND_BLOCK: return build_inst<KIND_BLOCK>(p, F, lds, st);
        case KIND_BASIC_K1: return build_inst<KIND_BASIC_K1>(p, F, lds, st);
        case KIND_BASIC_KK: return build_inst<KIND_PASS>(p, F, lds, st);  // (KK: k_slice_fill sets the bits)
        default: return build_inst<KIND_PASS>(p, F, lds, st);
    }
}

// Probe LDS: slice segment + tables + a survivor stage using what is left of the CU's 160 KiB.
size_t probe_lds_bytes(const Geometry& g, uint32_t* stage_cap, bool pay) {
    const bool   slices = g.mode == MODE_SLICE_BLOCK || g.mode == MODE_SLICE_BASIC;
    const size_t NSUB   = (size_t) 1 << g.log2NSUB;
    const int    kind   = consumer_kind(g);
    const size_t scap   = pay ? 0 : kind == KIND_BLOCK_PKK || kind == KIND_BASIC_KK
                              ? scr_cap<KIND_BLOCK_PKK>() : scr_cap<KIND_PASS>();
    const size_t base   = ((slices ? g.seg_words : 0) + 3 * 128 + 16 * NSUB + 16 * scap + 64) * sizeof(uint32_t);
    // 2 buffers of cap words + 64 dummy slots each, in what the 512-byte static table leaves
    // (pay: codes and positions, half a buffer each)
    size_t cap = std::min<size_t>(kProbeCH * 32, (163840 - 512 - base) / 8 - 64) & ~(size_t) 7;
    if (!pay) cap = std::min<size_t>(cap, (size_t) (slices ? kPco : kPC) * 4096);  // what the copy-out's stores cover
    if (stage_cap) *stage_cap = (uint32_t) cap;
    return base + 2 * (cap + 64) * 4;
}

void launch_probe(const ProbeParams& p0, uint32_t grid, hipStream_t st) {
    ProbeParams p = p0;
    const size_t lds = probe_lds_bytes(p.g, &p.stage_cap, p.surv_pos != nullptr);
    switch (consumer_kind(p.g)) {
        case KIND_BLOCK_PK1: return probe_inst<KIND_BLOCK_PK1>(p, grid, lds, st);
        case KIND_BLOCK_PKK: return probe_inst<KIND_BLOCK_PKK>(p, grid, lds, st);
        case KIND_BLOCK: return probe_inst<KIND_BLOCK>(p, grid, lds, st);
        case KIND_BASIC_K1: return probe_inst<KIND_BASIC_K1>(p, grid, lds, st);
        case KIND_BASIC_KK: return probe_inst<KIND_BASIC_KK>(p, grid, lds, st);
        default: return probe_inst<KIND_PASS>(p, grid, lds, st);
    }
}

uint32_t probe_chunks_per_item() { return kProbeCH; }

void launch_join(const JoinParams& p0, uint32_t jobs, uint32_t* job_surv, hipStream_t st) {
    JoinParams p = p0;
    p.jobs       = jobs;
    const uint32_t split = p.split_surv ? p.split_surv : kJoinTaskSurv;
    k_join_split<<<(jobs + 255) / 256, 256, 0, st>>>(p.item_start, job_surv, p.log2NSUB, jobs, split,
                                                     p.nparts, p.extra, p.nextra, p.jsum);
    // (one key width per launch: k_join's key reads are compile-time for it)
    if (p.r_kbits == 18) k_join<18><<<jobs + kJoinExtra, kJoinThreads, 0, st>>>(p);
    else if (p.r_kbits == 24) k_join<24><<<jobs + kJoinExtra, kJoinThreads, 0, st>>>(p);
    else k_join<32><<<jobs + kJoinExtra, kJoinThreads, 0, st>>>(p);
    k_join_mixed<<<std::min<uint32_t>(jobs + kJoinExtra, 1024u), kJoinThreads, 0, st>>>(p);
}

uint32_t join_extra_tasks() { return kJoinExtra; }
uint32_t join_sum_slots() { return kJoinSumSlots; }
uint32_t join_sum_stride() { return kJoinSumStride; }
uint32_t join_bitmap_log2() { return kJoinBmLog2; }

void launch_export(const uint32_t* slices, const Geometry& g, uint32_t* out, uint64_t nwords,
                   hipStream_t st) {
    k_export<<<2048, 256, 0, st>>>(slices, g, out, nwords);
}

// ---------------------------------------------------------------- build knobs (hwbrj_version)
// Every compile-time switch of this file whose value differs from the product default, as
// "NAME=value" words; empty for the product build (tests/test_abi.py pins that).
const char* kernel_build_knobs() {
    static const std::string s = [] {
        std::string r;
        auto num = [&](const char* n, long v, long d) {
            if (v != d) r += std::string(r.empty() ? "" : " ") + n + "=" + std::to_string(v);
        };
        auto flag = [&](const char* n) { r += std::string(r.empty() ? "" : " ") + n; };
        (void) flag;
#ifdef HWBRJ_DEV_BUILD
        flag("HWBRJ_DEV_BUILD");
#endif
        num("HWBRJ_SC_T", HWBRJ_SC_T, 1024);
        num("HWBRJ_SC_E", HWBRJ_SC_E, 8);
        num("HWBRJ_SC_K", HWBRJ_SC_K, 2);
        num("HWBRJ_SC_PRE", HWBRJ_SC_PRE, 1);
        num("HWBRJ_SC_KEEPY", HWBRJ_SC_KEEPY, 1);
        num("HWBRJ_SC_LAUX", HWBRJ_SC_LAUX, 2);
        num("HWBRJ_SC_SAUX", HWBRJ_SC_SAUX, 2);
        num("HWBRJ_SC_SAUX_R", HWBRJ_SC_SAUX_R, 2);
        num("HWBRJ_SC_SB", HWBRJ_SC_SB, 2);
        num("HWBRJ_SC_KP", HWBRJ_SC_KP, 3);
        num("HWBRJ_PLANCOLS", HWBRJ_PLANCOLS, 16);
        num("HWBRJ_LFPER", HWBRJ_LFPER, 28);
        num("HWBRJ_BPQ", HWBRJ_BPQ, 2);
        num("HWBRJ_BD_NT", HWBRJ_BD_NT, 0);
        num("HWBRJ_PC", HWBRJ_PC, 3);
        num("HWBRJ_SCR1", HWBRJ_SCR1, 128);
        num("HWBRJ_PR_NT", HWBRJ_PR_NT, 0);
        num("HWBRJ_SCRK", HWBRJ_SCRK, 256);
        num("HWBRJ_JTU", HWBRJ_JTU, 8);
        num("HWBRJ_JTS", HWBRJ_JTS, 2);
        num("HWBRJ_JT", HWBRJ_JT, 256);
        num("HWBRJ_JXCD", HWBRJ_JXCD, 1);
        num("HWBRJ_PACK3", HWBRJ_PACK3, 1);
        num("HWBRJ_PACK18", HWBRJ_PACK18, 1);
        num("HWBRJ_JRR", HWBRJ_JRR, 4);
        num("HWBRJ_JRW", HWBRJ_JRW, 4);
        num("HWBRJ_JSR", HWBRJ_JSR, 8);
        num("HWBRJ_JFS", HWBRJ_JFS, 5);
        num("HWBRJ_JSW", HWBRJ_JSW, 2);
        num("HWBRJ_JFR", HWBRJ_JFR, 8);
        num("HWBRJ_JFW", HWBRJ_JFW, 5);
        num("HWBRJ_JBM", HWBRJ_JBM, 18);
        num("HWBRJ_OVL_ASYNC", HWBRJ_OVL_ASYNC, 1);
        num("HWBRJ_PJ_OVL", HWBRJ_PJ_OVL, 1);
        num("HWBRJ_ABL_PROBE", HWBRJ_ABL_PROBE, 0);
        num("HWBRJ_PCO", HWBRJ_PCO, 1);
        num("HWBRJ_PCO_AUX", HWBRJ_PCO_AUX, 0);
#define HWBRJ_FLAG_KNOB(X) flag(#X)
#ifdef HWBRJ_STAMPS
        HWBRJ_FLAG_KNOB(HWBRJ_STAMPS);
#endif
#ifdef HWBRJ_ABL_NOCRC
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_NOCRC);
#endif
#ifdef HWBRJ_ABL_NOCRAP
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_NOCRAP);
#endif
#ifdef HWBRJ_ABL_NOSTORE
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_NOSTORE);
#endif
#ifdef HWBRJ_ABL_SPLITH
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_SPLITH);
#endif
#ifdef HWBRJ_ABL_PNOPST
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_PNOPST);
#endif
#ifdef HWBRJ_ABL_BNOBITS
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_BNOBITS);
#endif
#ifdef HWBRJ_ABL_BNOSORT
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_BNOSORT);
#endif
#ifdef HWBRJ_ABL_PNOB1
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_PNOB1);
#endif
#ifdef HWBRJ_ABL_JNOR
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_JNOR);
#endif
#ifdef HWBRJ_ABL_JNOS
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_JNOS);
#endif
#ifdef HWBRJ_ABL_MJ_EMPTY
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_MJ_EMPTY);
#endif
#ifdef HWBRJ_ABL_MJ_NOLOAD
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_MJ_NOLOAD);
#endif
#ifdef HWBRJ_ABL_MJ_NOINS
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_MJ_NOINS);
#endif
#ifdef HWBRJ_ABL_MJ_R
        HWBRJ_FLAG_KNOB(HWBRJ_ABL_MJ_R);
#endif
#undef HWBRJ_FLAG_KNOB
        return r;
    }();
    return s.c_str();
}

}  // namespace hwbrj
