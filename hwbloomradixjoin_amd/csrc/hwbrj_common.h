// hwbrj_common.h -- host+device definitions shared by the MI355X kernels, the C-ABI shim and the
// host generator. gfx950 only; no CUDA/HIP dual paths.
//
// Hash and filter semantics restate Briimbo/HwBloomRadixJoin exactly:
//   crc32c          src/hash.c:6-10      (_mm_crc32_u32: reflected CRC32-C, 0x82F63B78, no inversion)
//   crapwow         src/hash.c:26-47
//   mod_m           src/bloom_filter.c:59-63
//   add/contains    src/bloom_filter.c:73-141 (basic, blocked), seed 42 (parallel_radix_join_bloom.c:1583)
//   generator       src/generator.c:304-415, :161-221 (key multiset; our shuffle is a seeded Feistel
//                   permutation where the reference uses a time-seeded Knuth shuffle, :173-176)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define HWBRJ_HD __host__ __device__ __forceinline__

namespace hwbrj {

constexpr uint32_t kSeed     = 42u;          // parallel_radix_join_bloom.c:1583
constexpr uint32_t kCrcPoly  = 0x82F63B78u;  // CRC32-C reflected
constexpr uint32_t kCrapN    = 0x5052acdbu;  // hash.c:29

enum Variant : int { VAR_BASIC = 0, VAR_BLOCKED = 1, VAR_SECTORIZED = 2 };

// ---------------------------------------------------------------------------------- hashing
// The 32 reflected CRC steps as a GF(2)-linear map f; crc32c(seed, key) = f(seed ^ key).
inline uint32_t crc_f_bitwise(uint32_t x) {
    for (int i = 0; i < 32; i++) x = (x >> 1) ^ (kCrcPoly & (0u - (x & 1u)));
    return x;
}

// Nibble tables: f(x) = XOR_j T[j][nibble_j(x)]; finv likewise. 2 x 8 x 16 u32 = 1 KiB.
struct CrcTables {
    uint32_t fwd[8][16];
    uint32_t inv[8][16];
};

// Builds f's tables and inverts f over GF(2) (f is a bijection: x^32 is a unit mod the CRC-32C
// polynomial), so a key can be recovered from its code. Returns false if inversion fails.
bool build_crc_tables(CrcTables* t);

HWBRJ_HD uint32_t crapwow(uint32_t seed, uint32_t key) {  // hash.c:26-47
    uint32_t h = 4u;
    uint32_t k = h + seed + kCrapN;
    uint64_t p = (uint64_t) key * (uint64_t) kCrapN;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    p = (uint64_t) (h ^ (k + kCrapN)) * (uint64_t) kCrapN;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    return k ^ h;
}

// tab = 8 x 16 nibble table (LDS or host memory). code(key) = crc32c(42, key).
HWBRJ_HD uint32_t nibble_map(const uint32_t* tab, uint32_t x) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) r ^= tab[j * 16 + ((x >> (4 * j)) & 15u)];
    return r;
}
HWBRJ_HD uint32_t key_code(const uint32_t* fwd, uint32_t key) { return nibble_map(fwd, key ^ kSeed); }
HWBRJ_HD uint32_t code_key(const uint32_t* inv, uint32_t code) { return nibble_map(inv, code) ^ kSeed; }

HWBRJ_HD uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x85ebca6bu;
    x ^= x >> 13;
    x *= 0xc2b2ae35u;
    x ^= x >> 16;
    return x;
}

// MODE_SLICE_BASIC partition words: an invertible mix of the key (not the key itself), so the
// join's sub-partition digit (the word's low bits) is spread even when keys share their low bits
// (e.g. all multiples of 64), and equal words still mean equal keys.
constexpr uint32_t kBMixC    = 0x9E3779B1u;  // odd: invertible mod 2^32
constexpr uint32_t kBMixCinv = 0x0E8B2F51u;  // kBMixC * kBMixCinv == 1 (mod 2^32)
HWBRJ_HD uint32_t bmix(uint32_t key) {
    const uint32_t h = key * kBMixC;
    return h ^ (h >> 16);
}
static_assert(kBMixC * kBMixCinv == 1u, "kBMixCinv inverts kBMixC");
HWBRJ_HD uint32_t bunmix(uint32_t w) { return (w ^ (w >> 16)) * kBMixCinv; }

// ------------------------------------------------------------------------- filter geometry
// Everything the kernels need about the filter and the partitioning, computed on the host.
enum Mode : int {
    MODE_NOBLOOM      = 0,  // PRO: no filter
    MODE_SLICE_BLOCK  = 1,  // blocked/sectorized: S partitioned by block bits, probed from LDS slices
    MODE_SLICE_BASIC  = 2,  // basic: partitioned by the first bit's index bits, element word = the key,
                            // LDS slices (k >= 2:
                            // bits 2..k of the first-bit candidates from the global bitmap)
    MODE_GLOBAL       = 3,  // basic k = 0 or B < 8: global atomics build + direct probe (fallback)
    // scatter modes of basic k >= 2's repartitioning passes (words = bmix(key) in, SRC_CODES):
    MODE_BASIC_BITJ   = 4,  // partition = the slice of bit j (Geometry::bitj) of add_basic; word kept
    MODE_CODE_OF_KEY  = 5,  // partition = code & (F-1), word = code = crc32c(42, key) (join layout)
    MODE_BASIC_POS    = 6,  // R tuples read as k * |R| elements (bit j of tuple t = element j |R| + t):
                            // word = bit j's position, partition = its slice (the slice build)
};

enum Format : int {
    FMT_CODE   = 0,  // element word = code = crc32c(42, key) (MODE_SLICE_BASIC: bmix(key))
    FMT_PACKED = 1,  // blocked, log2B <= log2F: (first bit-in-block) | (code >> log2F) << log2B (low bits: the slice bit)
                     // into a 22-dword (88-byte) chunk; the probe recomputes the bit-in-block from
                     // the key (inverse CRC + CrapWow)
};

struct Geometry {
    int      mode;
    int      variant;
    int      format;
    uint32_t k;            // hashes per key
    uint64_t m;            // filter bits
    uint32_t B;            // block bits (blocked/sectorized)
    uint32_t nblocks;      // m / B
    uint32_t block_span;   // (B/8)*8: bit distance between blocks (src/bloom_filter.c:128 B/8 quirk)
    uint32_t log2F;        // radix partitions F = 1 << log2F (<= 1024)
    uint32_t log2NSUB;     // join sub-partitions per partition
    uint32_t sub_shift;    // sub = (code >> sub_shift) & (NSUB-1)
    uint32_t hash_shift;   // join table hash input = code >> hash_shift
    uint32_t slice_bits;   // filter bits per partition slice (m / F)
    uint32_t seg_bits;     // bits per LDS-resident slice segment (<= kSliceMaxBits)
    uint32_t seg_words;    // 32-bit words per stored segment (>= seg_bits/32, multiple of 4)
    uint32_t nseg;         // slice_bits / seg_bits
    // derived constants (no per-element loops or divisions on the device)
    uint32_t log2B;        // blocked family
    uint32_t log2seg;      // log2(seg_bits)
    uint32_t lbmask;       // (nblocks >> log2F) - 1: slice-local block index mask
    uint32_t log2secw;     // sectorized: log2(min(B, 64))
    uint32_t nsecmask;     // sectorized: B / secw - 1
    int      s_format;     // element format of the S partitions (format: the R partitions)
    uint32_t bitj;         // MODE_BASIC_BITJ / k_probe_bitj: which bit of add_basic's sequence (0-based)
};

// Consumer-kernel specializations (selected on the host from Geometry).
enum Kind : int {
    KIND_PASS        = 0,  // no filter test (PRO, or the global-bitmap fallback already filtered)
    KIND_BLOCK_PK1   = 1,  // blocked/sectorized, k = 1, packed words
    KIND_BLOCK       = 2,  // blocked/sectorized, code words, any k
    KIND_BASIC_K1    = 3,  // basic, k = 1
    KIND_BLOCK_PKK   = 4,  // blocked/sectorized, k >= 2, packed words: the first bit is tested from
                           // the word, the key (for the rest) is recovered only for those that pass
    KIND_BASIC_KK    = 5,  // basic, k >= 2: the first bit from the LDS slice, bits 2..k of the
                           // candidates from the global bitmap (slices = its transpose)
};

constexpr uint32_t kMaxLog2F     = 10;
constexpr uint32_t kSliceMaxBits = 1u << 20;  // 128 KiB of LDS per slice segment
constexpr uint32_t kChunk        = 32;        // elements per 128-byte chunk

HWBRJ_HD uint32_t ilog2u(uint64_t v) {
    uint32_t r = 0;
    while ((1ull << (r + 1)) <= v) r++;
    return r;
}

// ----------------------------------------------------------- reference filter arithmetic
// Bit positions of `key` inside its block / the whole bitmap, following add_generic
// (src/bloom_filter.c:73-89): h = crapwow & (size-1), y = (key+seed) & (size-1),
// h_{i+1} = (h_i + y_i) & (size-1), y_{i+1} = (y_i + i + 1) & (size-1). `size` arrives as uint32
// and is widened (mod_m), so size = 0 means "no masking".
HWBRJ_HD uint32_t mod_m(uint32_t v, uint32_t size) { return (uint32_t) (v & ((uint64_t) size - 1ull)); }

// Bit j (0-based) of add_basic's sequence for key (src/bloom_filter.c:73-111): the position in
// the whole m-bit filter.
HWBRJ_HD uint32_t basic_bit(uint32_t key, uint32_t j, uint32_t msz) {
    uint32_t h = mod_m(crapwow(kSeed, key), msz), y = mod_m(key + kSeed, msz);
    for (uint32_t i = 0; i < j; i++) {
        h = mod_m(h + y, msz);
        y = mod_m(y + i + 1u, msz);
    }
    return h;
}

// SECTORIZED (the build's extension): bit i of the sequence is moved into 64-bit sector
// (s0 + i) mod nsec, s0 = sector of the first bit. k = 1 is bit-identical to BLOCKED.
HWBRJ_HD uint32_t sectorize(uint32_t h, uint32_t s0, uint32_t i, uint32_t B) {
    const uint32_t secw = B < 64u ? B : 64u;
    const uint32_t nsec = B / secw;
    return ((s0 + i) % nsec) * secw + (h & (secw - 1u));
}

// ---------------------------------------------------------------------- generator (exact)
// One reference generator thread's chunk (src/generator.c:363-395).
struct GenChunk {
    uint64_t start;      // first tuple index of the chunk
    uint64_t n;          // tuples in the chunk
    uint64_t n_below;    // tuples with keys cycling in [1, threshold]
    int64_t  firstkey;
    int64_t  firstabove;
};

constexpr int kMaxGenChunks = 1024;

struct GenPlan {
    uint32_t nchunks;
    uint64_t num_tuples;
    uint64_t threshold;
    GenChunk chunk[kMaxGenChunks];
};

// Restates parallel_create_relation's sizing (src/generator.c:331-395). Returns 0 on success.
int make_gen_plan(GenPlan* plan, uint64_t num_tuples, uint32_t nthreads, uint64_t maxid,
                  uint64_t threshold, double selectivity);

// Key of generation-order tuple g (before the shuffle), per random_unique_gen_thread (:178-194).
HWBRJ_HD int32_t gen_key_at(const GenPlan& plan, uint64_t g) {
    uint32_t lo = 0, hi = plan.nchunks - 1;
    while (lo < hi) {  // last chunk with start <= g
        uint32_t mid = (lo + hi + 1) >> 1;
        if (plan.chunk[mid].start <= g) lo = mid; else hi = mid - 1;
    }
    const GenChunk& c = plan.chunk[lo];
    uint64_t j = g - c.start;
    const int64_t T = (int64_t) plan.threshold;
    if (j < c.n_below) {
        // x_0 = f; x_{j+1} = (x_j == T) ? 1 : x_j + 1
        // f = (offset + 1) % T lies in [0, T-1]
        int64_t f = c.firstkey;
        if (f == 0) return j == 0 ? 0 : (int32_t) (((int64_t) (j - 1) % T) + 1);
        return (int32_t) (((f - 1 + (int64_t) j) % T) + 1);
    }
    j -= c.n_below;
    // y_0 = fa; y_{j+1} = (y_j == INT_MAX) ? T + 1 : y_j + 1
    const int64_t span = 2147483647LL - T;  // values T+1 .. INT_MAX
    int64_t fa = c.firstabove;
    if (span <= 0) return (int32_t) (fa + (int64_t) j);
    if (fa <= T) {  // fa == T: first value is T, then T+1 ...
        if (j == 0) return (int32_t) fa;
        return (int32_t) (T + 1 + ((int64_t) (j - 1) % span));
    }
    return (int32_t) (T + 1 + ((fa - T - 1 + (int64_t) j) % span));
}

// Seeded bijection on [0, n): 4-round Feistel network on 2h bits with cycle walking.
struct Perm {
    uint64_t n;
    uint32_t half_bits;
    uint32_t keys[4];
};

inline Perm make_perm(uint64_t n, uint64_t seed) {
    Perm p;
    p.n = n;
    uint32_t bits = 2;
    while (bits < 64 && (1ull << bits) < n) bits += 2;
    p.half_bits = bits / 2;
    uint64_t s = seed * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
    for (int r = 0; r < 4; r++) {
        s ^= s >> 31;
        s *= 0xBF58476D1CE4E5B9ull;
        s ^= s >> 29;
        p.keys[r] = (uint32_t) (s >> 16) | 1u;
    }
    return p;
}

HWBRJ_HD uint64_t perm_apply(const Perm& p, uint64_t i) {
    const uint64_t mask = (p.half_bits >= 64) ? ~0ull : ((1ull << p.half_bits) - 1ull);
    uint64_t x = i;
    do {
        uint64_t L = x >> p.half_bits, R = x & mask;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            uint64_t fr = (uint64_t) mix32((uint32_t) R ^ p.keys[r]) |
                          ((uint64_t) mix32((uint32_t) (R >> 32) + p.keys[r] * 3u) << 32);
            uint64_t nl = R;
            R = (L ^ fr) & mask;
            L = nl;
        }
        x = (L << p.half_bits) | R;
    } while (x >= p.n);
    return x;
}

}  // namespace hwbrj
