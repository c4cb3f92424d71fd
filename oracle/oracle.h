/*
 * oracle.h -- CPU restatement of the reference's BPRO path. TEST INFRASTRUCTURE ONLY.
 *
 * This is the parity checker for the MI355X product in hwbloomradixjoin_amd/. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product never
 * links, loads or falls back to it.
 *
 * Every function restates one piece of Briimbo/HwBloomRadixJoin (paths relative to the
 * reference root). Parity is pinned by:
 *   - the reference's own hash.c/bloom_filter.c, compiled unmodified into oracle/_ref
 *     (scalar KATs and bitmap popcounts; tests/test_oracle.py);
 *   - the reference binary's published/measured counts recorded in SURVEY.md s8c
 *     (tests/golden/ fixtures).
 */
#ifndef HWBRJ_ORACLE_H
#define HWBRJ_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/types.h:37-40 (8-byte tuple, KEY_8B off) */
typedef struct orc_tuple_t {
    int32_t key;
    int32_t payload;
} orc_tuple_t;

/* src/bloom_filter.h:10 plus the build's documented SECTORIZED extension. */
enum { ORC_BASIC = 0, ORC_BLOCKED = 1, ORC_SECTORIZED = 2 };

typedef struct orc_bloom_t {
    int       variant;
    uint32_t  seed;
    uint64_t  m, k, B, nblocks;
    uint8_t * bitmap; /* m/8 bytes, byte-addressed exactly like src/bloom_filter.c */
} orc_bloom_t;

/* src/hash.c:6-10  (_mm_crc32_u32: CRC32-C, reflected 0x82F63B78, no inversion) */
uint32_t orc_crc32c(uint32_t seed, int32_t key);
/* src/hash.c:26-47 */
uint32_t orc_crapwow(uint32_t seed, int32_t key);

/* src/bloom_filter.c:143-171 (calloc'd bitmap of m/8 bytes). Returns 0 on success. */
int      orc_bloom_init(orc_bloom_t * f, int variant, uint64_t m, uint64_t k, uint64_t B,
                        uint32_t seed);
void     orc_bloom_free(orc_bloom_t * f);
/* src/bloom_filter.c:73-89,113-132 */
void     orc_bloom_add(const orc_bloom_t * f, int32_t key);
/* src/bloom_filter.c:92-111,118-141 */
int      orc_bloom_contains(const orc_bloom_t * f, int32_t key);
uint64_t orc_bloom_popcount(const orc_bloom_t * f);
/* src/bloom_filter.c:25-34: returns 0 if args are valid, else 1 (the reference exits(1)) */
int      orc_bloom_args_invalid(int variant, uint64_t m, uint64_t B);

/* src/generator.c:304-415 + :161-221 -- the exact key multiset (order: generation order, i.e.
 * before the reference's time-seeded shuffle). keys[i] for i < num_tuples. */
int      orc_gen_keys(int32_t * keys, uint64_t num_tuples, uint32_t nthreads, uint64_t maxid,
                      uint64_t threshold, double selectivity);
/* Seeded Fisher-Yates of keys (splitmix64). The reference shuffles with a time seed
 * (src/generator.c:173-176), so any fixed seed is an equally valid order. */
void     orc_shuffle_keys(int32_t * keys, uint64_t n, uint64_t seed);

/* The rand()-driven generators (src/generator.c:531-646, :659-676, src/genzipf.c:28-158), calling
 * libc srand(seed)/rand() exactly as the reference does. Payload = row (zipf: the reference leaves
 * it uninitialised). */
void     orc_gen_nonunique(orc_tuple_t * out, uint64_t n, int64_t maxid, uint32_t seed);
void     orc_gen_nonunique_from_pk(orc_tuple_t * out, uint64_t n, const orc_tuple_t * pk,
                                   uint64_t npk, int64_t threshold, double selectivity,
                                   uint32_t seed);
void     orc_gen_fk_from_pk(orc_tuple_t * out, uint64_t n, const orc_tuple_t * pk, uint64_t npk,
                            int64_t threshold, double selectivity, uint32_t seed);
int      orc_gen_zipf(orc_tuple_t * out, uint64_t n, unsigned int alphabet_size,
                      double zipf_factor, uint32_t seed);

typedef struct orc_timing_t {
    double total_usec;     /* src/parallel_radix_join_bloom.c:1521-1522 */
    double partition_usec; /* :1525-1527 */
    double join_usec;      /* :1528-1530 */
    /* thread 0's phases (for the CPU-baseline calibration): R loop 1 (histogram +
     * bloom add) and its barrier, R scatter (+ barrier :1153), S loop 1 (histogram + contains),
     * S scatter (+ barrier :1171), pass-2 (+ task creation), join */
    double phase_usec[6];
} orc_timing_t;

/* src/parallel_radix_join_bloom.c:1560-1787 (BPRO -> join_init_run -> prj_thread):
 * 2-pass radix partition (5+5 bits), bloom add fused in R pass-1, bloom contains fused in S
 * pass-1, bucket-chaining join per partition (:259-329). bloom == NULL gives PRO
 * (src/parallel_radix_join.c:1697). Inputs are not modified. Returns the match count; stores
 * the "S-tuples after filter" count in *filtered (= |S| without bloom). */
int64_t  orc_bpro(const orc_tuple_t * R, uint64_t nR, const orc_tuple_t * S, uint64_t nS,
                  int nthreads, int variant, uint64_t m, uint64_t k, uint64_t B, int use_bloom,
                  uint64_t * filtered, orc_timing_t * timing);

/* src/parallel_radix_join_bloom.c:307-312 (JOIN_RESULT_MATERIALIZE): {R.payload, S.payload} of
 * every match, order-free; writes min(total, cap) pairs, returns the total. */
int64_t  orc_join_pairs(const orc_tuple_t * R, uint64_t nR, const orc_tuple_t * S, uint64_t nS,
                        orc_tuple_t * out, uint64_t cap);

void     orc_bloom_add_all_atomic(orc_bloom_t * f, const int32_t * keys, uint64_t n);
/* Scalar helpers for tests (single-threaded, small inputs). */
uint64_t orc_count_filtered(const orc_bloom_t * f, const int32_t * keys, uint64_t n);
/* src/unit_tests.c:191-283: false-positive counts of the FPR unit test (blocked B=512, then
 * basic, k = 1 .. kmax) */
int      orc_fpr_test(int seed, uint64_t m, uint64_t kmax, uint32_t n_samples, uint32_t n_insertions,
                      uint64_t * pos);
void     orc_bloom_add_all(orc_bloom_t * f, const int32_t * keys, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
