/*
 * oracle.c -- CPU restatement of the reference BPRO path. TEST INFRASTRUCTURE ONLY
 * (see oracle.h). Plain C11 + pthreads; the multithreaded orc_bpro doubles as the "port"
 * CPU baseline that bench.py times on the GPU host.
 *
 * Reference citations are relative to the Briimbo/HwBloomRadixJoin root.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <pthread.h>
#include <sched.h>
#include <unistd.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <string.h>
#ifdef __SSE4_2__
#include <nmmintrin.h>
#endif
#include <time.h>

/* ------------------------------------------------------------------ hashes */

/* src/hash.c:6-10: _mm_crc32_u32(seed, key), the SSE4.2 instruction the reference uses (the build
 * targets x86-64-v2). Without SSE4.2: the same function as 32 reflected CRC32-C steps on seed ^ key. */
uint32_t
orc_crc32c(uint32_t seed, int32_t key)
{
#ifdef __SSE4_2__
    return _mm_crc32_u32(seed, (uint32_t) key);
#else
    uint32_t x = seed ^ (uint32_t) key;
    for (int i = 0; i < 32; i++) x = (x >> 1) ^ (0x82F63B78u & (0u - (x & 1u)));
    return x;
#endif
}

/* src/hash.c:26-47 (CrapWow, n = 0x5052acdb, h = sizeof(intkey_t) = 4). */
uint32_t
orc_crapwow(uint32_t seed, int32_t key)
{
    const uint32_t n = 0x5052acdbu;
    uint32_t       h = 4u;
    uint32_t       k = h + seed + n;
    uint64_t       p;
    p = (uint64_t) (uint32_t) key * (uint64_t) n;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    p = (uint64_t) (uint32_t) (h ^ (k + n)) * (uint64_t) n;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    return k ^ h;
}

/* ------------------------------------------------------------ bloom filter */

/* src/bloom_filter.c:59-63: size arrives as uint32_t and is widened to uint64_t. */
static inline uint32_t
mod_m(uint32_t val, uint64_t m)
{
    return (uint32_t) (val & (m - 1));
}

int
orc_bloom_args_invalid(int variant, uint64_t m, uint64_t B)
{
    /* src/bloom_filter.c:25-34 */
    if (m == 0 || (m & (m - 1)) != 0) return 1;
    if (variant != ORC_BASIC) {
        if (B == 0 || (B & (B - 1)) != 0) return 1;
        if (m % B != 0) return 1;
    }
    return 0;
}

int
orc_bloom_init(orc_bloom_t * f, int variant, uint64_t m, uint64_t k, uint64_t B, uint32_t seed)
{
    /* src/bloom_filter.c:143-171 */
    f->variant = variant;
    f->m       = m;
    f->k       = k;
    f->B       = B;
    f->nblocks = B ? m / B : 0;
    f->seed    = seed;
    f->bitmap  = (uint8_t *) calloc(m / 8 ? m / 8 : 1, 1);
    return f->bitmap ? 0 : 1;
}

void
orc_bloom_free(orc_bloom_t * f)
{
    free(f->bitmap);
    f->bitmap = NULL;
}

/* src/bloom_filter.c:73-89 add_generic; the atomic_fetch_or becomes a plain OR in the
 * single-threaded helpers and an atomic OR in orc_bpro's threads. */
static inline void
add_generic(const orc_bloom_t * f, int32_t key, uint8_t * bitmap, uint32_t size, int atomic)
{
    uint32_t h = orc_crapwow(f->seed, key);
    uint32_t y = (uint32_t) key + f->seed;
    h          = mod_m(h, size);
    y          = mod_m(y, size);
    for (int i = 0; (uint64_t) i < f->k; i++) {
        if (atomic)
            __atomic_fetch_or(bitmap + (h >> 3), (uint8_t) (1u << (h & 7)), __ATOMIC_RELAXED);
        else
            bitmap[h >> 3] |= (uint8_t) (1u << (h & 7));
        h = mod_m(h + y, size);
        y = mod_m(y + (uint32_t) i + 1u, size);
    }
}

/* src/bloom_filter.c:92-111 contains_generic */
static inline int
contains_generic(const orc_bloom_t * f, int32_t key, const uint8_t * bitmap, uint32_t size)
{
    uint32_t h = orc_crapwow(f->seed, key);
    uint32_t y = (uint32_t) key + f->seed;
    h          = mod_m(h, size);
    y          = mod_m(y, size);
    for (int i = 0; (uint64_t) i < f->k; i++) {
        if (!(bitmap[h >> 3] & (1u << (h & 7)))) return 0;
        h = mod_m(h + y, size);
        y = mod_m(y + (uint32_t) i + 1u, size);
    }
    return 1;
}

/* SECTORIZED (the build's extension, DESIGN.md "Filter variants"): the block is chosen exactly
 * like BLOCKED; the B-bit block is cut into 64-bit sectors; hash i keeps the double-hashing
 * sequence of add_generic for the bit offset but lands in sector (s0 + i) mod nsec, where s0 is
 * the sector of the first hash. k = 1 is therefore bit-identical to BLOCKED. */
static inline void
sector_positions(const orc_bloom_t * f, int32_t key, uint32_t * pos, int kmax)
{
    const uint32_t B    = (uint32_t) f->B;
    const uint32_t secw = B < 64u ? B : 64u;
    const uint32_t nsec = B / secw;
    uint32_t       h    = mod_m(orc_crapwow(f->seed, key), B);
    uint32_t       y    = mod_m((uint32_t) key + f->seed, B);
    const uint32_t s0   = h / secw;
    for (int i = 0; i < kmax; i++) {
        uint32_t sector = (s0 + (uint32_t) i) % nsec;
        pos[i]          = sector * secw + (h & (secw - 1u));
        h               = mod_m(h + y, B);
        y               = mod_m(y + (uint32_t) i + 1u, B);
    }
}

static inline uint8_t *
block_of(const orc_bloom_t * f, int32_t key)
{
    /* src/bloom_filter.c:125-141 */
    uint32_t block_idx = mod_m(orc_crc32c(f->seed, key), f->nblocks);
    return f->bitmap + (uint64_t) block_idx * (f->B / 8);
}

static inline void
bloom_add_impl(const orc_bloom_t * f, int32_t key, int atomic)
{
    switch (f->variant) {
        case ORC_BASIC: add_generic(f, key, f->bitmap, (uint32_t) f->m, atomic); break;
        case ORC_BLOCKED: add_generic(f, key, block_of(f, key), (uint32_t) f->B, atomic); break;
        default: {
            uint8_t *  blk = block_of(f, key);
            int        kk  = (int) f->k;
            uint32_t   stackpos[64];
            uint32_t * pos = kk <= 64 ? stackpos : (uint32_t *) malloc(sizeof(uint32_t) * kk);
            sector_positions(f, key, pos, kk);
            for (int j = 0; j < kk; j++) {
                uint32_t h = pos[j];
                if (atomic)
                    __atomic_fetch_or(blk + (h >> 3), (uint8_t) (1u << (h & 7)), __ATOMIC_RELAXED);
                else
                    blk[h >> 3] |= (uint8_t) (1u << (h & 7));
            }
            if (pos != stackpos) free(pos);
        }
    }
}

void
orc_bloom_add(const orc_bloom_t * f, int32_t key)
{
    bloom_add_impl(f, key, 0);
}

int
orc_bloom_contains(const orc_bloom_t * f, int32_t key)
{
    switch (f->variant) {
        case ORC_BASIC: return contains_generic(f, key, f->bitmap, (uint32_t) f->m);
        case ORC_BLOCKED: return contains_generic(f, key, block_of(f, key), (uint32_t) f->B);
        default: {
            const uint8_t * blk = block_of(f, key);
            int             kk  = (int) f->k;
            uint32_t        stackpos[64];
            uint32_t *      pos = kk <= 64 ? stackpos : (uint32_t *) malloc(sizeof(uint32_t) * kk);
            sector_positions(f, key, pos, kk);
            int ok = 1;
            for (int j = 0; j < kk && ok; j++)
                if (!(blk[pos[j] >> 3] & (1u << (pos[j] & 7)))) ok = 0;
            if (pos != stackpos) free(pos);
            return ok;
        }
    }
}

uint64_t
orc_bloom_popcount(const orc_bloom_t * f)
{
    uint64_t c = 0;
    for (uint64_t i = 0; i < f->m / 8; i++) c += (uint64_t) __builtin_popcount(f->bitmap[i]);
    return c;
}

void
orc_bloom_add_all(orc_bloom_t * f, const int32_t * keys, uint64_t n)
{
    for (uint64_t i = 0; i < n; i++) orc_bloom_add(f, keys[i]);
}

/* the add loop of orc_bpro's R pass-1 (atomic OR, :794-797), for several threads at once */
void
orc_bloom_add_all_atomic(orc_bloom_t * f, const int32_t * keys, uint64_t n)
{
    for (uint64_t i = 0; i < n; i++) bloom_add_impl(f, keys[i], 1);
}

uint64_t
orc_count_filtered(const orc_bloom_t * f, const int32_t * keys, uint64_t n)
{
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; i++) c += (uint64_t) orc_bloom_contains(f, keys[i]);
    return c;
}

/* --------------------------------------------------------------- generator */

/* src/generator.c:304-415 (parallel_create_relation) and :161-221 (random_unique_gen_thread),
 * restated sequentially per "thread" chunk. Only the keys before the shuffle are produced. */
int
orc_gen_keys(int32_t * keys, uint64_t num_tuples, uint32_t nthreads, uint64_t maxid,
             uint64_t threshold, double selectivity)
{
    if (nthreads == 0 || threshold == 0) return 1;
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
    for (uint32_t t = 0; t < nthreads; t++) {
        uint64_t span       = maxid > threshold ? maxid - threshold : 0;
        int64_t  firstkey   = (int64_t) ((offset + 1) % threshold);
        int64_t  firstabove = (int64_t) (threshold + (offset_above + 1) % (span > 1 ? span : 1));
        uint64_t n_above    = (t == nthreads - 1) ? ntuples_above_lastthr : ntuples_above_perthr;
        uint64_t n_t        = (t == nthreads - 1) ? ntuples_lastthr : ntuples_perthr;
        uint64_t start      = offset + offset_above;
        if (n_above > n_t || start + n_t > num_tuples) return 2; /* reference would overrun */
        uint64_t n_below = n_t - n_above;
        int32_t * out    = keys + start;
        uint64_t  i;
        for (i = 0; i < n_below; i++) {
            out[i] = (int32_t) firstkey;
            if (firstkey == (int64_t) threshold) firstkey = 0;
            firstkey++;
        }
        for (; i < n_t; i++) {
            out[i] = (int32_t) firstabove;
            if (firstabove == 2147483647LL) firstabove = (int64_t) threshold;
            firstabove++;
        }
        offset += ntuples_perthr - ntuples_above_perthr;
        offset_above += ntuples_above_perthr;
    }
    return 0;
}

static inline uint64_t
splitmix64(uint64_t * s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z          = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z          = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void
orc_shuffle_keys(int32_t * keys, uint64_t n, uint64_t seed)
{
    uint64_t s = seed;
    for (uint64_t i = n; i > 1; i--) {
        uint64_t j   = (uint64_t) (((unsigned __int128) splitmix64(&s) * i) >> 64);
        int32_t  tmp = keys[i - 1];
        keys[i - 1]  = keys[j];
        keys[j]      = tmp;
    }
}

/* ------------------------------------------- rand()-driven generators (libc rand itself) */
/* The reference calls glibc srand()/rand() (src/generator.c:75-81); so does this restatement, so
 * the draws are the reference's by construction. Not thread-safe (libc's global state), like the
 * reference's generator. */
#define ORC_RAND_RANGE(O, N) ((O) + ((double) rand() / ((double) RAND_MAX + 1) * ((N) - (O))))

/* src/generator.c:271-279 */
static void
orc_random_gen(orc_tuple_t * rel, uint64_t n, int64_t minid, int64_t maxid)
{
    for (uint64_t i = 0; i < n; i++) {
        rel[i].key     = ORC_RAND_RANGE(minid, maxid);
        rel[i].payload = i;
    }
}

/* src/generator.c:99-109 */
static void
orc_knuth_shuffle(orc_tuple_t * rel, uint64_t n)
{
    int i;
    for (i = n - 1; i > 0; i--) {
        int64_t j    = ORC_RAND_RANGE(0, i);
        int32_t tmp  = rel[i].key;
        rel[i].key   = rel[j].key;
        rel[j].key   = tmp;
    }
}

/* src/generator.c:585-605 after srand(seed) (src/main.c:410) */
void
orc_gen_nonunique(orc_tuple_t * out, uint64_t n, int64_t maxid, uint32_t seed)
{
    srand(seed);
    orc_random_gen(out, n, 0, maxid);
}

/* src/generator.c:608-646 */
void
orc_gen_nonunique_from_pk(orc_tuple_t * out, uint64_t n, const orc_tuple_t * pk, uint64_t npk,
                          int64_t threshold, double selectivity, uint32_t seed)
{
    srand(seed);
    uint64_t ntuples_above = n * (1 - selectivity);
    orc_random_gen(out, ntuples_above, threshold + 1, 2147483647);
    int i, j;
    for (i = ntuples_above; i < (int) n; i++) {
        j              = ORC_RAND_RANGE(0, npk);
        out[i].key     = pk[j].key;
        out[i].payload = i;
    }
    orc_knuth_shuffle(out, n);
}

/* src/generator.c:531-582 */
void
orc_gen_fk_from_pk(orc_tuple_t * out, uint64_t n, const orc_tuple_t * pk, uint64_t npk,
                   int64_t threshold, double selectivity, uint32_t seed)
{
    srand(seed);
    uint64_t ntuples_above = n * (1 - selectivity);
    uint64_t ntuples_below = n - ntuples_above;
    orc_random_gen(out + ntuples_below, ntuples_above, threshold + 1, 2147483647);
    int iters = ntuples_below / npk, i;
    for (i = 0; i < iters; i++) memcpy(out + i * npk, pk, npk * sizeof(orc_tuple_t));
    int64_t remainder = ntuples_below % npk;
    if (remainder > 0) memcpy(out + i * npk, pk, remainder * sizeof(orc_tuple_t));
    orc_knuth_shuffle(out, n);
}

/* src/genzipf.c:28-158 (gen_alphabet, gen_zipf_lut, gen_zipf) via create_relation_zipf
 * (src/generator.c:659-676). Payload = row (the reference leaves it uninitialised). */
int
orc_gen_zipf(orc_tuple_t * out, uint64_t n, unsigned int alphabet_size, double zipf_factor,
             uint32_t seed)
{
    srand(seed);
    uint32_t * alphabet = malloc(alphabet_size * sizeof(*alphabet));
    double *   lut      = malloc(alphabet_size * sizeof(*lut));
    if (!alphabet || !lut) {
        free(alphabet);
        free(lut);
        return 1;
    }
    for (unsigned int i = 0; i < alphabet_size; i++) alphabet[i] = i + 1;
    for (unsigned int i = alphabet_size - 1; i > 0; i--) {
        unsigned int k   = (unsigned long) i * rand() / RAND_MAX;
        unsigned int tmp = alphabet[i];
        alphabet[i]      = alphabet[k];
        alphabet[k]      = tmp;
    }
    double scaling_factor = 0.0, sum = 0.0;
    for (unsigned int i = 1; i <= alphabet_size; i++) scaling_factor += 1.0 / pow(i, zipf_factor);
    for (unsigned int i = 1; i <= alphabet_size; i++) {
        sum += 1.0 / pow(i, zipf_factor);
        lut[i - 1] = sum / scaling_factor;
    }
    for (uint64_t i = 0; i < n; i++) {
        double       r    = ((double) rand()) / RAND_MAX;
        unsigned int left = 0, right = alphabet_size - 1, m, pos;
        if (lut[0] >= r)
            pos = 0;
        else {
            while (right - left > 1) {
                m = (left + right) / 2;
                if (lut[m] < r)
                    left = m;
                else
                    right = m;
            }
            pos = right;
        }
        out[i].key     = alphabet[pos];
        out[i].payload = i;
    }
    free(lut);
    free(alphabet);
    return 0;
}

/* -------------------------------------------------- materialized join result */
static int
orc_key_cmp(const void * a, const void * b)
{
    const orc_tuple_t *x = a, *y = b;
    return (x->key > y->key) - (x->key < y->key);
}

/* JOIN_RESULT_MATERIALIZE (src/parallel_radix_join_bloom.c:307-312): for every S tuple and every
 * R tuple with an equal key, the pair {R.payload, S.payload}. Order-free restatement (sorted R,
 * binary search); writes min(total, cap) pairs, returns the total (-1: out of memory). */
int64_t
orc_join_pairs(const orc_tuple_t * R, uint64_t nR, const orc_tuple_t * S, uint64_t nS,
               orc_tuple_t * out, uint64_t cap)
{
    orc_tuple_t * r = malloc((nR ? nR : 1) * sizeof(orc_tuple_t));
    if (!r) return -1;
    memcpy(r, R, nR * sizeof(orc_tuple_t));
    qsort(r, nR, sizeof(orc_tuple_t), orc_key_cmp);
    int64_t n = 0;
    for (uint64_t i = 0; i < nS; i++) {
        uint64_t lo = 0, hi = nR;
        while (lo < hi) {
            uint64_t mid = (lo + hi) / 2;
            if (r[mid].key < S[i].key) lo = mid + 1; else hi = mid;
        }
        for (uint64_t j = lo; j < nR && r[j].key == S[i].key; j++, n++)
            if ((uint64_t) n < cap) {
                out[n].key     = r[j].payload;
                out[n].payload = S[i].payload;
            }
    }
    free(r);
    return n;
}

/* ------------------------------------------------------------- radix join */

#define NUM_RADIX_BITS 10 /* src/prj_params.h:16 */
#define PASS1_BITS 5      /* :72 */
#define FANOUT1 32        /* :76 */
#define FANOUT2 32        /* :78 */
#define SMALL_PADDING 24  /* :86: 3 * 64 / sizeof(tuple_t) */
#define PADDING (SMALL_PADDING * (FANOUT2 + 1)) /* :87 */

typedef struct task_t {
    const orc_tuple_t * R;
    orc_tuple_t *       outR;
    uint32_t            nR;
    const orc_tuple_t * S;
    orc_tuple_t *       outS;
    uint32_t            nS;
} task_t;

typedef struct shared_t {
    int                 nthreads;
    pthread_barrier_t   barrier;
    const orc_tuple_t * R;
    const orc_tuple_t * S;
    uint64_t            nR, nS;
    orc_tuple_t *       tmpR;
    orc_tuple_t *       tmpS;
    orc_tuple_t *       tmp2R;
    orc_tuple_t *       tmp2S;
    int                 use_bloom;
    orc_bloom_t         bloom;
    uint32_t *          histR; /* [nthreads][FANOUT1] counts */
    uint32_t *          histS;
    task_t              part_tasks[FANOUT1];
    int                 n_part_tasks;
    atomic_int          next_part;
    task_t *            join_tasks;
    atomic_int          n_join_tasks;
    atomic_int          next_join;
    uint64_t            filtered;
    struct timespec     t_start, t_part, t_end;
    struct timespec     t_ph[5];  /* thread 0: R loop 1, R scatter, S loop 1, S scatter, pass-2 */
} shared_t;

typedef struct thr_t {
    shared_t * sh;
    int        tid;
    int64_t    result;
} thr_t;

static inline uint32_t
hash_bit_modulo(int32_t key, uint32_t mask, int nbits)
{
    /* src/parallel_radix_join_bloom.c:74 */
    return ((uint32_t) key & mask) >> nbits;
}

/* src/parallel_radix_join_bloom.c:758-852 (parallel_radix_partition, pass-1, R=0, D=5). */
static void
pass1_partition(shared_t * sh, int tid, const orc_tuple_t * rel, uint64_t num, uint32_t * hist,
                orc_tuple_t * tmp, int relidx)
{
    const uint32_t MASK  = FANOUT1 - 1;
    uint32_t *     my    = hist + (size_t) tid * FANOUT1;
    uint8_t *      cache = NULL;
    if (sh->use_bloom && relidx == 1) cache = (uint8_t *) calloc((num + 7) / 8 + 1, 1);
    memset(my, 0, sizeof(uint32_t) * FANOUT1);
    for (uint64_t i = 0; i < num; i++) {
        int32_t key = rel[i].key;
        if (sh->use_bloom) {
            if (relidx == 0) {
                bloom_add_impl(&sh->bloom, key, 1);
            } else if (!orc_bloom_contains(&sh->bloom, key)) {
                continue;
            } else {
                cache[i >> 3] |= (uint8_t) (1u << (i & 7));
            }
        }
        my[hash_bit_modulo(key, MASK, 0)]++;
    }
    pthread_barrier_wait(&sh->barrier);
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_ph[relidx * 2]);
    /* :820-837 -- global start of each partition + this thread's offset inside it */
    uint64_t dst[FANOUT1];
    uint64_t base = 0;
    for (int j = 0; j < FANOUT1; j++) {
        uint64_t before = 0, total = 0;
        for (int t = 0; t < sh->nthreads; t++) {
            uint32_t c = hist[(size_t) t * FANOUT1 + j];
            if (t < tid) before += c;
            total += c;
        }
        dst[j] = base + before + (uint64_t) j * PADDING;
        base += total;
    }
    /* :842-849 */
    for (uint64_t i = 0; i < num; i++) {
        if (cache && !(cache[i >> 3] & (1u << (i & 7)))) continue;
        orc_tuple_t t = rel[i];
        tmp[dst[hash_bit_modulo(t.key, MASK, 0)]++] = t;
    }
    free(cache);
}

/* src/parallel_radix_join_bloom.c:573-608 radix_cluster (R=5, D=5, SMALL_PADDING) and
 * :703-748 serial_radix_partition. */
static void
pass2_partition(shared_t * sh, const task_t * task)
{
    const int      R   = PASS1_BITS;
    const uint32_t M   = (uint32_t) (FANOUT2 - 1) << R;
    uint32_t       hR[FANOUT2] = {0}, hS[FANOUT2] = {0};
    uint32_t       dR[FANOUT2], dS[FANOUT2];
    for (uint32_t i = 0; i < task->nR; i++) hR[hash_bit_modulo(task->R[i].key, M, R)]++;
    for (uint32_t i = 0; i < task->nS; i++) hS[hash_bit_modulo(task->S[i].key, M, R)]++;
    uint32_t oR = 0, oS = 0;
    for (int i = 0; i < FANOUT2; i++) {
        dR[i] = oR + (uint32_t) i * SMALL_PADDING;
        dS[i] = oS + (uint32_t) i * SMALL_PADDING;
        oR += hR[i];
        oS += hS[i];
    }
    uint32_t startR[FANOUT2], startS[FANOUT2];
    memcpy(startR, dR, sizeof dR);
    memcpy(startS, dS, sizeof dS);
    for (uint32_t i = 0; i < task->nR; i++)
        task->outR[dR[hash_bit_modulo(task->R[i].key, M, R)]++] = task->R[i];
    for (uint32_t i = 0; i < task->nS; i++)
        task->outS[dS[hash_bit_modulo(task->S[i].key, M, R)]++] = task->S[i];
    for (int i = 0; i < FANOUT2; i++) {
        if (hR[i] > 0 && hS[i] > 0) {
            int     slot = atomic_fetch_add(&sh->n_join_tasks, 1);
            task_t *t    = &sh->join_tasks[slot];
            t->R         = task->outR + startR[i];
            t->nR        = hR[i];
            t->S         = task->outS + startS[i];
            t->nS        = hS[i];
            t->outR = t->outS = NULL;
        }
    }
}

/* src/parallel_radix_join_bloom.c:259-329 bucket_chaining_join (count only). */
static int64_t
bucket_chaining_join(const task_t * t)
{
    uint32_t N = t->nR;
    N--;
    N |= N >> 1;
    N |= N >> 2;
    N |= N >> 4;
    N |= N >> 8;
    N |= N >> 16;
    N++;
    const uint32_t MASK    = (N - 1) << NUM_RADIX_BITS;
    int *          next    = (int *) malloc(sizeof(int) * t->nR);
    int *          bucket  = (int *) calloc(N, sizeof(int));
    int64_t        matches = 0;
    for (uint32_t i = 0; i < t->nR;) {
        uint32_t idx = hash_bit_modulo(t->R[i].key, MASK, NUM_RADIX_BITS);
        next[i]      = bucket[idx];
        bucket[idx]  = (int) ++i;
    }
    for (uint32_t i = 0; i < t->nS; i++) {
        uint32_t idx = hash_bit_modulo(t->S[i].key, MASK, NUM_RADIX_BITS);
        for (int hit = bucket[idx]; hit > 0; hit = next[hit - 1])
            if (t->S[i].key == t->R[hit - 1].key) matches++;
    }
    free(bucket);
    free(next);
    return matches;
}

static double
usec_between(const struct timespec * a, const struct timespec * b)
{
    return (double) (b->tv_sec - a->tv_sec) * 1e6 + (double) (b->tv_nsec - a->tv_nsec) / 1e3;
}

/* src/parallel_radix_join_bloom.c:1059-1506 prj_thread (default build: no SWWC, no skew). */
static void *
prj_thread(void * arg)
{
    thr_t *    me  = (thr_t *) arg;
    shared_t * sh  = me->sh;
    int        tid = me->tid;
    int        n   = sh->nthreads;

    uint64_t perR = sh->nR / (uint64_t) n, perS = sh->nS / (uint64_t) n;
    uint64_t numR = tid == n - 1 ? sh->nR - (uint64_t) tid * perR : perR;
    uint64_t numS = tid == n - 1 ? sh->nS - (uint64_t) tid * perS : perS;

    /* Before the timer, like the reference's setup: its bitmap is memset (src/bloom_filter.c:36-49,
     * calloc_aligned) and its pass-2 writes into the caller's (already touched) input relations
     * (:1240-1245), so the bitmap and our separate pass-2 buffers are pre-faulted here. */
    {
        uint64_t padR = sh->nR + (uint64_t) PADDING * FANOUT1, padS = sh->nS + (uint64_t) PADDING * FANOUT1;
        uint64_t bR = padR * tid / n, eR = padR * (tid + 1) / n;
        uint64_t bS = padS * tid / n, eS = padS * (tid + 1) / n;
        memset(sh->tmp2R + bR, 0, (eR - bR) * sizeof(orc_tuple_t));
        memset(sh->tmp2S + bS, 0, (eS - bS) * sizeof(orc_tuple_t));
        if (sh->use_bloom) {
            uint64_t nb = sh->bloom.m / 8, b = nb * tid / n, e = nb * (tid + 1) / n;
            memset(sh->bloom.bitmap + b, 0, e - b);
        }
    }
    pthread_barrier_wait(&sh->barrier); /* :1107 */
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_start);

    pass1_partition(sh, tid, sh->R + (uint64_t) tid * perR, numR, sh->histR, sh->tmpR, 0);
    pthread_barrier_wait(&sh->barrier); /* :1153 bitmap complete */
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_ph[1]);
    pass1_partition(sh, tid, sh->S + (uint64_t) tid * perS, numS, sh->histS, sh->tmpS, 1);
    pthread_barrier_wait(&sh->barrier); /* :1171 */
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_ph[3]);

    if (tid == 0) { /* :1183-1253 */
        uint64_t offR = 0, offS = 0, filtered = 0, offS2 = 0;
        sh->n_part_tasks = 0;
        for (int j = 0; j < FANOUT1; j++) {
            uint64_t ntR = 0, ntS = 0;
            for (int t = 0; t < n; t++) {
                ntR += sh->histR[(size_t) t * FANOUT1 + j];
                ntS += sh->histS[(size_t) t * FANOUT1 + j];
            }
            filtered += ntS;
            if (ntR > 0 && ntS > 0) {
                task_t * t = &sh->part_tasks[sh->n_part_tasks++];
                t->R       = sh->tmpR + offR + (uint64_t) j * PADDING;
                t->outR    = sh->tmp2R + offR + (uint64_t) j * PADDING;
                t->nR      = (uint32_t) ntR;
                t->S       = sh->tmpS + offS + (uint64_t) j * PADDING;
                t->outS    = sh->tmp2S + offS2;
                t->nS      = (uint32_t) ntS;
            }
            offR += ntR;
            offS += ntS;
            if (ntR > 0 && ntS > 0) offS2 += ntS + PADDING;
        }
        sh->filtered = filtered;
    }
    pthread_barrier_wait(&sh->barrier); /* :1264 */

    int i;
    while ((i = atomic_fetch_add(&sh->next_part, 1)) < sh->n_part_tasks) /* :1280-1283 */
        pass2_partition(sh, &sh->part_tasks[i]);
    pthread_barrier_wait(&sh->barrier); /* :1424 */
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_part);

    int64_t results = 0;
    int     nj      = atomic_load(&sh->n_join_tasks);
    while ((i = atomic_fetch_add(&sh->next_join, 1)) < nj) /* :1456-1464 */
        results += bucket_chaining_join(&sh->join_tasks[i]);
    me->result = results;
    pthread_barrier_wait(&sh->barrier); /* :1479 */
    if (tid == 0) clock_gettime(CLOCK_MONOTONIC, &sh->t_end);
    return NULL;
}

int64_t
orc_bpro(const orc_tuple_t * R, uint64_t nR, const orc_tuple_t * S, uint64_t nS, int nthreads,
         int variant, uint64_t m, uint64_t k, uint64_t B, int use_bloom, uint64_t * filtered,
         orc_timing_t * timing)
{
    if (nthreads < 1) nthreads = 1;
    shared_t sh;
    memset(&sh, 0, sizeof sh);
    sh.nthreads  = nthreads;
    sh.R         = R;
    sh.S         = S;
    sh.nR        = nR;
    sh.nS        = nS;
    sh.use_bloom = use_bloom;
    if (use_bloom && orc_bloom_init(&sh.bloom, variant, m, k, B, 42u)) return -1; /* :1583 */
    size_t padR = (nR + (uint64_t) PADDING * FANOUT1);
    size_t padS = (nS + (uint64_t) PADDING * FANOUT1);
    sh.tmpR     = (orc_tuple_t *) malloc(sizeof(orc_tuple_t) * padR);
    sh.tmpS     = (orc_tuple_t *) malloc(sizeof(orc_tuple_t) * padS);
    sh.tmp2R    = (orc_tuple_t *) malloc(sizeof(orc_tuple_t) * padR);
    sh.tmp2S    = (orc_tuple_t *) malloc(sizeof(orc_tuple_t) * padS);
    /* one 128-byte histogram row per thread on lines of its own: the reference allocates every
     * thread's histogram separately, cache-line aligned (:1624-1627, alloc_aligned at
     * CACHE_LINE_SIZE); rows packed into a 16-byte-aligned calloc shared lines between neighbour
     * threads, whose per-tuple increments then ping-ponged those lines (2.8x slower pass-1 loops) */
    sh.histR    = (uint32_t *) aligned_alloc(64, (size_t) nthreads * FANOUT1 * sizeof(uint32_t));
    sh.histS    = (uint32_t *) aligned_alloc(64, (size_t) nthreads * FANOUT1 * sizeof(uint32_t));
    if (sh.histR) memset(sh.histR, 0, (size_t) nthreads * FANOUT1 * sizeof(uint32_t));
    if (sh.histS) memset(sh.histS, 0, (size_t) nthreads * FANOUT1 * sizeof(uint32_t));
    sh.join_tasks = (task_t *) calloc((size_t) FANOUT1 * FANOUT2, sizeof(task_t));
    if (!sh.tmpR || !sh.tmpS || !sh.tmp2R || !sh.tmp2S || !sh.histR || !sh.histS || !sh.join_tasks)
        return -1;
    atomic_init(&sh.next_part, 0);
    atomic_init(&sh.n_join_tasks, 0);
    atomic_init(&sh.next_join, 0);
    pthread_barrier_init(&sh.barrier, NULL, (unsigned) nthreads);

    pthread_t tids[nthreads];
    thr_t     args[nthreads];
    for (int t = 0; t < nthreads; t++) {
        args[t].sh     = &sh;
        args[t].tid    = t;
        args[t].result = 0;
        /* one thread per core, like the reference's cpu mapping (src/parallel_radix_join_bloom.c
         * :1673-1693, get_cpu_id) */
        pthread_attr_t attr;
        cpu_set_t      set;
        pthread_attr_init(&attr);
        CPU_ZERO(&set);
        CPU_SET(t % CPU_SETSIZE, &set);
        if (t < (int) sysconf(_SC_NPROCESSORS_ONLN)) pthread_attr_setaffinity_np(&attr, sizeof(set), &set);
        pthread_create(&tids[t], &attr, prj_thread, &args[t]);
        pthread_attr_destroy(&attr);
    }
    int64_t result = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(tids[t], NULL);
        result += args[t].result; /* :1696-1707 */
    }
    if (filtered) *filtered = use_bloom ? sh.filtered : nS;
    if (timing) {
        timing->total_usec     = usec_between(&sh.t_start, &sh.t_end);
        timing->partition_usec = usec_between(&sh.t_start, &sh.t_part);
        timing->join_usec      = usec_between(&sh.t_part, &sh.t_end);
        const struct timespec * tp[7] = {&sh.t_start, &sh.t_ph[0], &sh.t_ph[1], &sh.t_ph[2],
                                         &sh.t_ph[3], &sh.t_part, &sh.t_end};
        for (int j = 0; j < 6; j++) timing->phase_usec[j] = usec_between(tp[j], tp[j + 1]);
    }
    pthread_barrier_destroy(&sh.barrier);
    free(sh.tmpR);
    free(sh.tmpS);
    free(sh.tmp2R);
    free(sh.tmp2S);
    free(sh.histR);
    free(sh.histS);
    free(sh.join_tasks);
    if (use_bloom) orc_bloom_free(&sh.bloom);
    return result;
}

/* ------------------------------------------------------------ FPR known answers (F6) */

/* src/unit_tests.c:154-173 random_unique_gen_range: Knuth's selection sampling of n keys out of
 * [min, max) with libc rand(), in increasing order */
static void
fpr_unique_range(int32_t * keys, uint64_t n, int32_t min, int32_t max)
{
    uint32_t inserted  = 0;
    int32_t  m_options = max - min;
    for (uint32_t i = 0; i < (uint32_t) m_options && inserted < n; ++i) {
        int rn = (int) (n - inserted);
        int rm = m_options - (int32_t) i;
        if (rand() % rm < rn) keys[inserted++] = min + (int32_t) i;
    }
}

/* src/unit_tests.c:191-283 (test_bloom_fpr_wrapper, test_bloom_fpr): R and S drawn from disjoint
 * key ranges, then for the blocked filter (B = 512) and the basic filter, k = 1 .. kmax: a filter
 * seeded with rand() after srand(seed), R added, S probed. pos[v * kmax + k - 1] = positives of S
 * (all false: fpr_emp = pos / n_samples), v = 0 blocked, 1 basic. */
int
orc_fpr_test(int seed, uint64_t m, uint64_t kmax, uint32_t n_samples, uint32_t n_insertions,
             uint64_t * pos)
{
    srand((unsigned) (seed + 1));
    int32_t * R = (int32_t *) malloc(sizeof(int32_t) * (n_insertions ? n_insertions : 1));
    int32_t * S = (int32_t *) malloc(sizeof(int32_t) * (n_samples ? n_samples : 1));
    if (!R || !S) return 1;
    int32_t threshold = (int32_t) (INT32_MAX * (n_insertions / (double) (n_insertions + n_samples)));
    fpr_unique_range(R, n_insertions, 0, threshold);
    fpr_unique_range(S, n_samples, threshold + 1, INT32_MAX);
    for (int v = 0; v < 2; v++) {
        for (uint64_t k = 1; k <= kmax; k++) {
            srand((unsigned) seed);
            orc_bloom_t f;
            if (orc_bloom_init(&f, v == 0 ? 1 : 0, m, k, 512, (uint32_t) rand())) return 1;
            orc_bloom_add_all(&f, R, n_insertions);
            pos[v * kmax + k - 1] = orc_count_filtered(&f, S, n_samples);
            orc_bloom_free(&f);
        }
    }
    free(R);
    free(S);
    return 0;
}
