/*
 * hwbrj.h -- C-ABI of libhwbrj.so, the MI355X drop-in for the reference's bloom radix join.
 *
 * Reference interfaces replaced (paths relative to the Briimbo/HwBloomRadixJoin root):
 *   tuple_t, relation_t, threadresult_t, result_t   src/types.h:37-63 (KEY_8B off: 8-byte tuples)
 *   bloom_filter_variant_t, bloom_filter_args_t     src/bloom_filter.h:10, :50-55
 *   BPRO                                            src/parallel_radix_join_bloom.h:34-36
 *                                                   (impl. src/parallel_radix_join_bloom.c:1781-1787)
 *   PRO                                             src/parallel_radix_join.h:33-34 (impl. :1697-1700)
 *   assert_args                                     src/bloom_filter.h:80-81 (impl. bloom_filter.c:25-34)
 *
 * BPRO/PRO keep the reference's contract: caller-owned host relations, a malloc'd result_t the
 * caller frees, the reference's stdout lines ("S-tuples after filter", the timing block), and
 * print + exit(EXIT_FAILURE) on fatal errors. Inputs are copied to HBM (hipMemcpy) outside the
 * timed region, like the reference allocates its tmp buffers before its timer starts.
 *
 * The hwbrj_* entry points are this build's additions: the same join on device-resident data,
 * generators, and test hooks. They return 0 on success and a nonzero code otherwise
 * (message in hwbrj_last_error()).
 */
#ifndef HWBRJ_H
#define HWBRJ_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference-compatible types (layouts identical to src/types.h, src/bloom_filter.h) ----
 * A translation unit may include the reference's own headers beside this one (its src/main.c
 * relinked against this library): each type is then defined once.
 *   - src/types.h (guard TYPES_H), in either order: this block defines TYPES_H, so a later
 *     types.h is empty, and an earlier one makes this block empty.
 *   - src/bloom_filter.h (guard BLOOM_FILTER_H): include it BEFORE this header (main.c's include
 *     order); its BASIC/BLOCKED enum and bloom_filter_args_t are then used as they are, and the
 *     sectorized variant is HWBRJ_SECTORIZED.
 * This library is the reference's default build (32-bit keys, 8-byte tuples): KEY_8B is refused. */
#ifdef KEY_8B
#error "libhwbrj joins 8-byte tuples (src/types.h without KEY_8B); KEY_8B is not supported"
#endif
#ifndef TYPES_H
#define TYPES_H
typedef int32_t intkey_t;
typedef int32_t value_t;

typedef struct tuple_t    tuple_t;
typedef struct relation_t relation_t;
typedef struct result_t       result_t;
typedef struct threadresult_t threadresult_t;

struct tuple_t {
    intkey_t key;
    value_t  payload;
};

struct relation_t {
    tuple_t * tuples;
    uint64_t  num_tuples;
};

struct threadresult_t {
    int64_t  nresults;
    void *   results;
    uint32_t threadid;
};

struct result_t {
    int64_t          totalresults;
    threadresult_t * resultlist; /* NULL: results are counted, not materialized (reference default) */
    int              nthreads;
};
#endif /* TYPES_H */

#ifndef BLOOM_FILTER_H
/* BASIC = 0 and BLOCKED = 1 as in the reference. SECTORIZED is this build's extension
 * (DESIGN.md "Filter variants"); the reference has no such variant. */
typedef enum { BASIC = 0, BLOCKED = 1, SECTORIZED = 2 } bloom_filter_variant_t;

typedef struct bloom_filter_args_t {
    bloom_filter_variant_t variant;
    uint64_t               m; /* filter size in bits (power of 2, <= 2^32) */
    uint64_t               k; /* hashes per key */
    uint64_t               B; /* block size in bits (power of 2, divides m) */
} bloom_filter_args_t;

void assert_args(bloom_filter_args_t * args);
#endif /* BLOOM_FILTER_H */
#define HWBRJ_SECTORIZED ((bloom_filter_variant_t) 2)

/* ---- drop-in operator boundary ---- */
result_t * BPRO(relation_t * relR, relation_t * relS, int nthreads,
                bloom_filter_args_t * bloom_filter_args);
result_t * PRO(relation_t * relR, relation_t * relS, int nthreads);
/* The reference's other partitioned-join entries (src/main.c:331-339). They differ in the
 * per-partition join function plugged into join_init_run: the histogram join (Kim et al.) for
 * BPRH / PRH, with SIMD compares for BPRHO / PRHO (here: k_join's histogram variants, see
 * hwbrj_join_device_algo), or in running single-threaded (BRJ / RJ: the BPRO / PRO operator on
 * the MI355X). The counts are the same.
 *   BPRH, BPRHO   src/parallel_radix_join_bloom.h:68-87 (impl. :1789-1804)
 *   BRJ           src/parallel_radix_join_bloom.c:1806-1930
 *   PRH, PRHO, RJ src/parallel_radix_join.h:49-82 */
result_t * BPRH(relation_t * relR, relation_t * relS, int nthreads,
                bloom_filter_args_t * bloom_filter_args);
result_t * BPRHO(relation_t * relR, relation_t * relS, int nthreads,
                 bloom_filter_args_t * bloom_filter_args);
result_t * BRJ(relation_t * relR, relation_t * relS, int nthreads,
               bloom_filter_args_t * bloom_filter_args);
result_t * PRH(relation_t * relR, relation_t * relS, int nthreads);
result_t * PRHO(relation_t * relR, relation_t * relS, int nthreads);
result_t * RJ(relation_t * relR, relation_t * relS, int nthreads);
/* The same two operators under prefixed names, for linking next to the reference's own
 * parallel_radix_join*.o (which also define BPRO/PRO): see INTEGRATION.md. */
result_t * hwbrj_BPRO(relation_t * relR, relation_t * relS, int nthreads,
                      bloom_filter_args_t * bloom_filter_args);
result_t * hwbrj_PRO(relation_t * relR, relation_t * relS, int nthreads);

/* ---- device-resident entry points (this build) ---- */
typedef struct hwbrj_stats_t {
    uint64_t filtered;      /* "S-tuples after filter" (= |S| without a filter) */
    int64_t  matches;       /* "Results" */
    int      mode;          /* 0 nobloom, 1 slice-blocked, 2 slice-basic, 3 global fallback */
    int      format;        /* S partition words: 0 codes, 1 packed (code + bit) */
    uint32_t partitions;    /* F */
    uint32_t subparts;      /* join sub-partitions per partition */
    uint32_t slice_segments;
    /* device time (ms, HIP events on the join stream) */
    double   ms_total;
    double   ms_r_scatter;  /* R -> partitions */
    double   ms_r_index;
    double   ms_build;      /* filter slices + R sub-partitioning (or global build) */
    double   ms_s_scatter;  /* S -> partitions (the dominant, HBM-bound kernel) */
    double   ms_s_index;
    double   ms_probe;      /* filter probe + survivor compaction */
    double   ms_surv;       /* survivor sub-partitioning: fused into the probe (k_probe), ~0 */
    double   ms_join;
    double   ms_join_probe; /* the survivor-probing share of ms_join (k_join's probe sections),
                               printed as PROBE-TIME-USECS; synchronous joins only (0 for async) */
    /* The key format between the build / probe and the join ("Join keys"):
     * HWBRJ_JOIN_KEYS_32 32-bit codes, _PACKED packed keys (join_key_bits each), _MIXED packed keys with the survivor
     * runs of unstaged probe items in 32-bit codes. It follows the last waited join on the device
     * (after a join with unstaged items the next one does not pack). */
    int      join_keys;
    uint32_t unstaged_items; /* probe items whose survivors overflowed the probe's LDS stage */
    uint32_t join_key_bits;  /* bits per packed join key: 18 (the bitmap path's keys, hash_shift 14;
                                the north star), 24, or 32 for 32-bit codes */
} hwbrj_stats_t;
enum { HWBRJ_JOIN_KEYS_32 = 0, HWBRJ_JOIN_KEYS_PACKED = 1, HWBRJ_JOIN_KEYS_MIXED = 2 };

/* Join device-resident tuple arrays (tuple_t layout). args == NULL runs PRO (no filter).
 * stream: a hipStream_t (NULL = the library's own stream). The call is synchronous. */
int hwbrj_join_device(const tuple_t * d_R, uint64_t nR, const tuple_t * d_S, uint64_t nS,
                      const bloom_filter_args_t * args, void * stream, hwbrj_stats_t * stats);
/* The same join with the reference's per-partition join function chosen (join_init_run's
 * JoinFunction, src/parallel_radix_join_bloom.c:1789-1804): HWBRJ_ALGO_PRO bucket chaining
 * (:259-329; here an LDS bitmap or counting hash table), HWBRJ_ALGO_PRH the histogram join of
 * Kim et al. (:350-419), HWBRJ_ALGO_PRHO its SIMD form (:441-555; 16-byte LDS compares). The host
 * entries BPRH / BPRHO / PRH / PRHO use them. Counts are identical. */
enum { HWBRJ_ALGO_PRO = 0, HWBRJ_ALGO_PRH = 1, HWBRJ_ALGO_PRHO = 2 };
int hwbrj_join_device_algo(const tuple_t * d_R, uint64_t nR, const tuple_t * d_S, uint64_t nS,
                           const bloom_filter_args_t * args, int algorithm, void * stream,
                           hwbrj_stats_t * stats);
/* The same join, enqueued on `stream` without waiting (back-to-back joins then run without host
 * gaps); the inputs must stay valid until it completes. hwbrj_join_wait() waits for the last join
 * enqueued on this device and fills stats with its counts. An async join records no phase events
 * (each would idle the GPU between the kernels around it), so its ms_* fields are 0; the
 * synchronous entry points measure the phases. */
int hwbrj_join_device_async(const tuple_t * d_R, uint64_t nR, const tuple_t * d_S, uint64_t nS,
                            const bloom_filter_args_t * args, void * stream);
int hwbrj_join_wait(hwbrj_stats_t * stats);
/* Every join enqueued on this device since the last hwbrj_join_wait / hwbrj_join_wait_all (or
 * synchronous join), oldest first, each with its own counts: stats[i] is join i's filtered /
 * matches / mode / join_keys (ms_* only for the last one, and only if it was synchronous). The
 * reference checks every run's count (src/parallel_radix_join_bloom.c:1696-1707 sums each thread's);
 * here every join of a back-to-back run keeps its counts in a device ring of 64 result slots, and an
 * enqueue that finds all 64 in use first collects them on the host (one wait). *n_joins = the
 * number of joins; returns 7 when it exceeds capacity (the oldest `capacity` are written). */
int hwbrj_join_wait_all(hwbrj_stats_t * stats, int capacity, int * n_joins);
/* on != 0: async joins bracket their S scatter (k_scatter_s, the dominant kernel) with timing
 * events on the side stream that runs it beside the R side, and hwbrj_join_wait / _wait_all report
 * its device time as ms_s_scatter of every async join (the other ms_* stay 0). For measuring the
 * kernel in the schedule the back-to-back joins run (bench.py's roofline); off by default, so the
 * timed joins carry no markers. */
int hwbrj_set_async_timing(int on);

/* The join with result materialization (the reference's JOIN_RESULT_MATERIALIZE output,
 * src/parallel_radix_join_bloom.c:307-312): d_out[i] = {R.payload, S.payload} of every match, in
 * no particular order. One pass of the partitioned pipeline with every tuple's payload carried
 * beside its word (stats: its counts and phase times); the global-bitmap configurations (basic
 * k = 0, B < 8) run the counting join and a pairs pass instead. capacity is in pairs; with too
 * small a capacity the first `capacity` pairs are written and 7 is returned with *n_out = the
 * match count. ms_materialize (optional) receives the device time of the pairs' production. */
int hwbrj_join_materialize_device(const tuple_t * d_R, uint64_t nR, const tuple_t * d_S,
                                  uint64_t nS, const bloom_filter_args_t * args, tuple_t * d_out,
                                  uint64_t capacity, uint64_t * n_out, void * stream,
                                  hwbrj_stats_t * stats, double * ms_materialize);
/* Host BPRO/PRO (and the PRH/PRHO/RJ entries) fill result_t.resultlist with the reference's
 * chained result buffers (src/tuple_buffer.h) when on (default: on iff HWBRJ_MATERIALIZE is set). */
void hwbrj_set_materialize(int on);
/* Host BPRO/PRO (and the PRH/PRHO/BRJ/RJ entries) range-shard S into `gpus` shards, shard g on
 * visible device g mod hwbrj_device_count(), R replicated (the reference's per-thread chunking of S,
 * src/parallel_radix_join_bloom.c:1646-1670, one host thread per device); counts are summed.
 * 0 (default) takes HWBRJ_GPUS from the environment, else 1. More shards than devices run one after
 * the other on each device (a G-GPU rehearsal on fewer GPUs). Returns 0, or 2 for gpus < 0. */
int  hwbrj_set_gpus(int gpus);

/* ---- partitioned multi-GPU join (this build) ----
 * Rank `rank` of `world` holds an R shard and an S shard (any split, e.g. range shards). Radix
 * partition q of the F partitions belongs to rank q / (F / world). Every rank scatters its R shard,
 * sends each partition's chunks to the owner, which builds that partition's filter slice and join
 * runs; the slices are all-gathered (the filter bitmap broadcast, in 1/world pieces), every rank
 * scatters and probes its S shard against the whole filter and sends each partition's survivors
 * to the owner, which joins them. stats->filtered: this rank's S survivors; stats->matches: the
 * matches of its partitions (the sums over ranks are the join's counts). nR_total = |R| over all
 * ranks (the filter geometry depends on it). Supported: blocked/sectorized filters, basic k = 1
 * and no filter (args NULL); returns 9 otherwise. world must divide F (a power of two <= F).
 *
 * The transport is the caller's (RCCL through torch.distributed, gloo, peer copies). Every call is
 * synchronous; device buffers are the caller's, named by slot (hwbrj_pj_slot_t). */
typedef enum {
    HWBRJ_PJ_R_SEND = 0, HWBRJ_PJ_R_SEND_ENT, HWBRJ_PJ_R_RECV, HWBRJ_PJ_R_RECV_ENT,
    HWBRJ_PJ_SLICES, HWBRJ_PJ_S_SEND, HWBRJ_PJ_S_RECV, HWBRJ_PJ_M_SEND, HWBRJ_PJ_M_RECV,
    HWBRJ_PJ_NSLOTS
} hwbrj_pj_slot_t;

typedef struct hwbrj_exchange_t {
    void * ctx;
    /* device buffer `slot` of at least `bytes` bytes (kept until the next request for the slot) */
    void * (*buffer)(void * ctx, int slot, uint64_t bytes);
    /* host all-to-all: send[j n .. (j + 1) n) goes to rank j, recv[j n ..) comes from rank j */
    int (*alltoall_u64)(void * ctx, const uint64_t * send, uint64_t * recv, uint64_t n);
    /* device all-to-all of byte blocks between slot buffers: [soff[j], soff[j] + sbytes[j]) of
     * send_slot goes to rank j; rank j's block lands at roff[j] of recv_slot (rbytes[j] bytes) */
    int (*alltoallv)(void * ctx, int send_slot, const uint64_t * soff, const uint64_t * sbytes,
                     int recv_slot, const uint64_t * roff, const uint64_t * rbytes);
    /* device all-gather in place: block j = [j bytes, (j + 1) bytes) of slot, from rank j */
    int (*allgather)(void * ctx, int slot, uint64_t bytes);
} hwbrj_exchange_t;

int hwbrj_join_partitioned(const hwbrj_exchange_t * x, int rank, int world, const tuple_t * d_R,
                           uint64_t nR, uint64_t nR_total, const tuple_t * d_S, uint64_t nS,
                           const bloom_filter_args_t * args, hwbrj_stats_t * stats);

/* ---- native RCCL transport (this build) ----
 * One communicator per device (one rank per GPU). hwbrj_comm_unique_id fills the 128-byte
 * ncclUniqueId on one rank; the caller hands the bytes to every rank (torch.distributed, MPI, a
 * file), and each calls hwbrj_comm_init on its device. librccl.so.1 is loaded at the first call
 * (HWBRJ_RCCL_LIB overrides the path); 31 = it could not be loaded, 30 = an RCCL error, 32 = no
 * communicator.
 *   hwbrj_join_partitioned_rccl  hwbrj_join_partitioned over the communicator: the R-chunk and
 *                                survivor all-to-alls (grouped ncclSend / ncclRecv) and the slice
 *                                all-gather (in-place ncclAllGather) run on the join's stream;
 *                                only the per-rank counts that size the all-to-alls reach the host.
 *   hwbrj_set_filter_broadcast   the replicated design (hwbrj_join_device*, S sharded, R on every
 *                                rank) with the north_star's bitmap broadcast: rank 0 builds the
 *                                filter slices, ncclBroadcast sends them to every rank on the join
 *                                stream; the other ranks only sub-partition R for the join. Off by
 *                                default (every rank rebuilds the slices from its R).
 *                                Slice modes only (blocked/sectorized, basic k = 1); a collective:
 *                                every rank must enqueue the same joins. */
int hwbrj_comm_unique_id(uint8_t * unique_id_out /* 128 bytes */);
int hwbrj_comm_init(const uint8_t * unique_id /* 128 bytes */, int world, int rank);
int hwbrj_comm_destroy(void);
int hwbrj_comm_info(int * world, int * rank);
int hwbrj_set_filter_broadcast(int on);
int hwbrj_join_partitioned_rccl(const tuple_t * d_R, uint64_t nR, uint64_t nR_total,
                                const tuple_t * d_S, uint64_t nS, const bloom_filter_args_t * args,
                                hwbrj_stats_t * stats);
/* The same join enqueued without host waits (no reference counterpart; the reference joins one
 * relation pair per process run). Every variable all-to-all is padded to a plan's block bounds
 * (the largest blocks of an earlier synchronous join of the same shapes + 12.5 % + 64, agreed by
 * all ranks), so counts messages, padded exchanges, the owner's tables, build, probe and join are
 * all enqueued on the join stream and up to 8 joins can be in flight. The first call (and the call
 * after a plan was dropped) runs synchronously and makes the plan. A block that does not fit sets
 * a device flag that is max-reduced over the ranks at the end of the join: its wait reruns it
 * synchronously on every rank (same counts; a new plan). A rank whose shard sizes or filter
 * differ from the plan's takes part with empty messages and flags the join the same way.
 * A collective: every rank makes the same calls in the same order (hwbrj_release and
 * hwbrj_comm_destroy included: they drop the joins in flight and the plan's buffers). The inputs
 * must stay valid and unchanged until the join's wait returns.
 *   hwbrj_join_partitioned_wait  collects the oldest enqueued join (FIFO): 0 or its error; stats:
 *                                counts, and ms_total = its device time between its first and last
 *                                operation on the join stream (0 phase times)
 *   hwbrj_pj_async_info          out[16]: plan valid, BR (chunks), BI (items), BW (words), async
 *                                joins, synchronous plan joins, overflow reruns, plans made, joins
 *                                in flight, the last rerun's flag (1 overflow, 2 a rank in the
 *                                failed mode), the last join's largest R / item / word block. */
int hwbrj_join_partitioned_rccl_async(const tuple_t * d_R, uint64_t nR, uint64_t nR_total,
                                      const tuple_t * d_S, uint64_t nS,
                                      const bloom_filter_args_t * args);
/* The async join over the caller's transport (the hwbrj_exchange_t callbacks of
 * hwbrj_join_partitioned): the same plan, padded layout, device tables, overflow flag and failed
 * mode, with the exchanges made by the callbacks (host-synchronous, so this form has host waits;
 * it is what lets several ranks share one GPU in tests). The exchange's callbacks and context must
 * stay valid until the join's wait returns. Collected by hwbrj_join_partitioned_wait. */
int hwbrj_join_partitioned_async(const hwbrj_exchange_t * x, int rank, int world, const tuple_t * d_R,
                                 uint64_t nR, uint64_t nR_total, const tuple_t * d_S, uint64_t nS,
                                 const bloom_filter_args_t * args);
int hwbrj_join_partitioned_wait(hwbrj_stats_t * stats);
int hwbrj_pj_async_info(uint64_t * out /* 16 */);

/* Fill d_out / out with the reference generator's key multiset (src/generator.c:304-415 with
 * `nthreads` generator threads) in a seeded permuted order; payload = row index. */
int hwbrj_generate_device(tuple_t * d_out, uint64_t n, uint32_t nthreads, uint64_t maxid,
                          uint64_t threshold, double selectivity, uint64_t seed, void * stream);
/* Rows [offset, offset + count) of the same n-row relation (for range-sharding S over ranks). */
int hwbrj_generate_device_range(tuple_t * d_out, uint64_t n, uint64_t offset, uint64_t count,
                                uint32_t nthreads, uint64_t maxid, uint64_t threshold,
                                double selectivity, uint64_t seed, void * stream);
int hwbrj_generate_host(tuple_t * out, uint64_t n, uint32_t nthreads, uint64_t maxid,
                        uint64_t threshold, double selectivity, uint64_t seed, int host_threads);

/* ---- the reference's rand()-driven generators, on the host, bit-exact ----
 * Each seeds its own restatement of glibc rand() (srand(seed), src/generator.c:75-81) and draws in
 * the reference's order, so keys AND order equal the reference's relation for the same seed.
 *   hwbrj_create_relation_nonunique          src/generator.c:585-605 (random_gen, :271-279):
 *                                            keys in [0, maxid), payload = row
 *   hwbrj_create_relation_nonunique_from_pk  src/generator.c:608-646 (--non-unique S)
 *   hwbrj_create_relation_fk_from_pk         src/generator.c:531-582 (--full-range S)
 *   hwbrj_create_relation_zipf               src/generator.c:659-676 + src/genzipf.c:28-158 (-z S);
 *                                            payload = row (the reference leaves it uninitialised)
 *   hwbrj_nonunique_threshold                src/main.c:421-427 (threshold for R and S) */
uint64_t hwbrj_nonunique_threshold(uint64_t r_size, double selectivity, int full_range);
int      hwbrj_create_relation_nonunique(tuple_t * out, uint64_t n, int64_t maxid, uint32_t seed);
int      hwbrj_create_relation_nonunique_from_pk(tuple_t * out, uint64_t n, const tuple_t * pk,
                                                 uint64_t npk, int64_t threshold,
                                                 double selectivity, uint32_t seed);
int      hwbrj_create_relation_fk_from_pk(tuple_t * out, uint64_t n, const tuple_t * pk,
                                          uint64_t npk, int64_t threshold, double selectivity,
                                          uint32_t seed);
int      hwbrj_create_relation_zipf(tuple_t * out, uint64_t n, uint64_t alphabet_size,
                                    double theta, uint32_t seed, int host_threads);
/* The -z relation generated straight into HBM (binary searches on the GPU): selectivity = 1 gives
 * exactly hwbrj_create_relation_zipf's relation. selectivity < 1 is this build's extension for
 * BASELINE config 5 (the reference ignores -q with -z): floor(n (1 - q)) rows chosen by a seeded
 * permutation get unique keys above the alphabet. stream: hipStream_t or NULL. */
int      hwbrj_create_relation_zipf_device(tuple_t * d_out, uint64_t n, uint64_t alphabet_size,
                                           double theta, uint32_t seed, double selectivity,
                                           int host_threads, void * stream);
/* The first n values rand() returns after srand(seed) (test hook for the restatement). */
int      hwbrj_rand_stream(uint32_t seed, int32_t * out, uint64_t n);

/* Relation files, the reference's PERSIST_RELATIONS output (the only on-disk format; the CLI's
 * --persist writes R.tbl / S.tbl / Out.tbl like a -DPERSIST_RELATIONS reference build):
 *   hwbrj_write_relation         src/generator.c:250-263 write_relation ("#KEY, VAL" header,
 *                                "key payload" lines); -R / -S read it back
 *   hwbrj_write_result_relation  src/tuple_buffer.h:155-236 write_result_relation: the pairs of a
 *                                materializing BPRO / PRO result ("R.payload S.payload", no header) */
int hwbrj_write_relation(const relation_t * rel, const char * filename);
int hwbrj_write_result_relation(const result_t * res, const char * filename);

/* The filter built by the last join, in the reference's byte layout (src/bloom_filter.c:143-171:
 * m/8 bytes, bit h of a block at byte h>>3, bit h&7). nbytes must be m/8. */
int hwbrj_export_filter(uint8_t * host_out, uint64_t nbytes);

/* Cycles per second of the counter behind BPRO's "RUNTIME TOTAL, BUILD, PART (cycles)" line (the
 * reference's rdtsc timers, src/rdtsc.h:35-68), calibrated once against the steady clock. */
uint64_t hwbrj_tsc_hz(void);

/* Measurement utility (no reference counterpart): the device's streaming copy rate, for the
 * roofline's measured-copy figure beside the spec peak. Copies `bytes` (a
 * multiple of 16) between two fresh device buffers `reps` times; *gbps = (read + write bytes) /
 * the median copy time. Returns 0, or an error code (device memory). */
int hwbrj_copy_bandwidth(uint64_t bytes, int reps, double * gbps);

/* Scalar hashes on the host (test hooks): crc32c(seed,key) and CrapWow(seed,key). */
uint32_t hwbrj_hash_crc(uint32_t seed, int32_t key);
uint32_t hwbrj_hash_crapwow(uint32_t seed, int32_t key);

int          hwbrj_device_count(void);
int          hwbrj_set_device(int device);
void         hwbrj_release(void); /* free all device buffers */
const char * hwbrj_last_error(void);
/* "hwbloomradixjoin_amd <version> (gfx950)"; a build whose kernels were compiled with any
 * non-default switch (tuning A/Bs, dev ablations) appends " knobs: NAME=value ..." naming them,
 * and so does every test hook that is set (hwbrj_set_test_hook). */
const char * hwbrj_version(void);

/* Test hooks (no reference counterpart): process-wide settings that force rarely taken paths or
 * inject a failure, so tests can reach them on one GPU. All are off (0 / -1) by default; none
 * changes a result except HWBRJ_HOOK_BCAST_NONROOT = 2, which exists to show that it would.
 *   HWBRJ_HOOK_JOIN_SPLIT     value > 0: the join's skew split cuts every (partition, sub) job
 *                             above `value` survivors into parts (counts unchanged).
 *   HWBRJ_HOOK_PJ_FAIL_RANK   rank `value` of a partitioned join fails its shard-size check
 *                             (code 3), as an oversized shard would; -1 = off.
 *   HWBRJ_HOOK_BCAST_NONROOT  with hwbrj_set_filter_broadcast(1): this rank runs the broadcast
 *                             join's non-root side (k_build writes no filter slices; they come
 *                             from ncclBroadcast, which at world 1 leaves the buffer as it is).
 *                             1 = as is, 2 = the slice buffer zeroed first (the filter is then
 *                             empty unless something writes it: the counts must drop). Honoured
 *                             only on a communicator of world 1 (a test setting; ignored by a
 *                             real multi-rank broadcast).
 *   HWBRJ_HOOK_PJ_PLAN_DIV    value > 0: the async partitioned join's plans get their block bounds
 *                             divided by `value`, so the next async join overflows and is rerun
 *                             synchronously (counts unchanged).
 *   HWBRJ_HOOK_PJ_ASYNC_FAIL  1: this rank runs every async partitioned join in the failed mode
 *                             (empty messages, failed status), as after a shape change: every rank
 *                             reruns the join synchronously (counts unchanged).
 * Returns 0, or 2 for an unknown hook or a value out of range. */
enum {
    HWBRJ_HOOK_JOIN_SPLIT     = 1,
    HWBRJ_HOOK_PJ_FAIL_RANK   = 2,
    HWBRJ_HOOK_BCAST_NONROOT  = 3,
    HWBRJ_HOOK_PJ_PLAN_DIV    = 4,
    HWBRJ_HOOK_PJ_ASYNC_FAIL  = 5
};
int          hwbrj_set_test_hook(int hook, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* HWBRJ_H */
