// hwbrj_api.cpp -- the C-ABI of libhwbrj.so (include/hwbrj.h): the drop-in BPRO / PRO operator
// boundary with the reference's stdout contract, plus device-resident entry points.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <x86intrin.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "hwbrj_engine.h"

namespace hwbrj {

static thread_local std::string g_last_error;
void set_last_error(const std::string& s) { g_last_error = s; }

}  // namespace hwbrj

using namespace hwbrj;

extern "C" {

const char* hwbrj_last_error(void) { return g_last_error.c_str(); }
// "<name> <version> (gfx950) src <hash>", then " knobs: ..." naming every compile-time switch of
// the kernels and every dev environment knob (dev builds only) that differs from the product
// default. The hash is the Makefile's stamp of the product sources and flags ("dev" otherwise).
#ifndef HWBRJ_SRC_SHA
#define HWBRJ_SRC_SHA "dev"
#endif
// Test hooks that are set (hwbrj_set_test_hook) are named too, so a bench line or a PMC stamp of a
// process that set one shows it.
const char* hwbrj_version(void) {
    static const std::string base = [] {
        std::string k = kernel_build_knobs();
        const std::string d = dev_knobs_string();
        if (!d.empty()) k += (k.empty() ? "" : " ") + d;
        return k;
    }();
    // one immutable string per distinct hook state, never freed: a pointer returned earlier stays
    // valid whatever hooks are set later
    static std::mutex            mu;
    static std::set<std::string> interned;
    std::lock_guard<std::mutex>  lk(mu);
    std::string        k = base;
    const TestHooks&   h = test_hooks();
    auto add = [&](const std::string& w) { k += (k.empty() ? "" : " ") + w; };
    if (h.join_split) add("HWBRJ_HOOK_JOIN_SPLIT=" + std::to_string(h.join_split));
    if (h.pj_fail_rank >= 0) add("HWBRJ_HOOK_PJ_FAIL_RANK=" + std::to_string(h.pj_fail_rank));
    if (h.bcast_nonroot) add("HWBRJ_HOOK_BCAST_NONROOT=" + std::to_string(h.bcast_nonroot));
    if (h.pj_plan_div) add("HWBRJ_HOOK_PJ_PLAN_DIV=" + std::to_string(h.pj_plan_div));
    if (h.pj_async_fail) add("HWBRJ_HOOK_PJ_ASYNC_FAIL=" + std::to_string(h.pj_async_fail));
    const std::string v = std::string("hwbloomradixjoin_amd 0.6 (gfx950) src " HWBRJ_SRC_SHA) +
                          (k.empty() ? "" : " knobs: " + k);
    return interned.insert(v).first->c_str();
}

int hwbrj_set_test_hook(int hook, int64_t value) {
    TestHooks& h = test_hooks();
    switch (hook) {
        case HWBRJ_HOOK_JOIN_SPLIT:
            if (value < 0 || value > 0xFFFFFFFFll) break;
            h.join_split = (uint32_t) value;
            return 0;
        case HWBRJ_HOOK_PJ_FAIL_RANK:
            h.pj_fail_rank = (int) value;
            return 0;
        case HWBRJ_HOOK_BCAST_NONROOT:
            if (value < 0 || value > 2) break;
            h.bcast_nonroot = (int) value;
            return 0;
        case HWBRJ_HOOK_PJ_PLAN_DIV:
            if (value < 0 || value > 1000000) break;
            h.pj_plan_div = (int) value;
            return 0;
        case HWBRJ_HOOK_PJ_ASYNC_FAIL:
            if (value < 0 || value > 1) break;
            h.pj_async_fail = (int) value;
            return 0;
        default:
            set_last_error("unknown test hook");
            return 2;
    }
    set_last_error("test hook value out of range");
    return 2;
}

int hwbrj_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hwbrj_set_device(int device) {
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        set_last_error(std::string("hipSetDevice: ") + hipGetErrorString(e));
        return 1;
    }
    return 0;
}

void hwbrj_release(void) {
    Engine* e = engine_for_current_device();
    if (e) e->release();
}

// The rate of the cycle counter behind "RUNTIME TOTAL, BUILD, PART (cycles)" (the reference's
// rdtsc timers, src/rdtsc.h:35-68), measured once against the steady clock over 50 ms.
uint64_t hwbrj_tsc_hz(void) {
    static const uint64_t hz = [] {
        const auto     t0 = std::chrono::steady_clock::now();
        const uint64_t c0 = __rdtsc();
        std::this_thread::sleep_for(std::chrono::milliseconds(50));
        const uint64_t c1 = __rdtsc();
        const double   s  = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return (uint64_t) ((double) (c1 - c0) / s);
    }();
    return hz;
}

int hwbrj_copy_bandwidth(uint64_t bytes, int reps, double* gbps) {
    if (!gbps || reps < 1 || bytes < 16 || bytes % 16) {
        set_last_error("hwbrj_copy_bandwidth: bytes must be a positive multiple of 16, reps >= 1");
        return 1;
    }
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) {
        if (a) (void) hipFree(a);
        set_last_error("hwbrj_copy_bandwidth: hipMalloc failed");
        return 6;
    }
    hipStream_t st = nullptr;
    hipEvent_t  e0 = nullptr, e1 = nullptr;
    int         rc = 0;
    std::vector<float> ms;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
        hipEventCreate(&e1) != hipSuccess || hipMemsetAsync(a, 1, bytes, st) != hipSuccess) {
        rc = 3;
    } else {
        int dev = 0, cus = 256;
        (void) hipGetDevice(&dev);
        (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        launch_copy_bw(a, b, bytes, cus, st);  // warm-up (page mapping, clocks)
        for (int r = 0; r < reps && rc == 0; r++) {
            float t = 0;
            (void) hipEventRecord(e0, st);
            launch_copy_bw(a, b, bytes, cus, st);
            (void) hipEventRecord(e1, st);
            if (hipEventSynchronize(e1) != hipSuccess || hipEventElapsedTime(&t, e0, e1) != hipSuccess) rc = 3;
            ms.push_back(t);
        }
    }
    if (rc == 0) {
        std::sort(ms.begin(), ms.end());
        *gbps = 2.0 * (double) bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
    } else {
        set_last_error(std::string("hwbrj_copy_bandwidth: ") + hipGetErrorString(hipGetLastError()));
    }
    if (e0) (void) hipEventDestroy(e0);
    if (e1) (void) hipEventDestroy(e1);
    if (st) (void) hipStreamDestroy(st);
    (void) hipFree(a);
    (void) hipFree(b);
    return rc;
}

uint32_t hwbrj_hash_crc(uint32_t seed, int32_t key) { return crc_f_bitwise(seed ^ (uint32_t) key); }
uint32_t hwbrj_hash_crapwow(uint32_t seed, int32_t key) { return crapwow(seed, (uint32_t) key); }

int hwbrj_join_device(const tuple_t* d_R, uint64_t nR, const tuple_t* d_S, uint64_t nS,
                      const bloom_filter_args_t* args, void* stream, hwbrj_stats_t* stats) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    return e->run((const uint2*) d_R, nR, (const uint2*) d_S, nS, args, (hipStream_t) stream, stats);
}

int hwbrj_join_device_algo(const tuple_t* d_R, uint64_t nR, const tuple_t* d_S, uint64_t nS,
                           const bloom_filter_args_t* args, int algorithm, void* stream,
                           hwbrj_stats_t* stats) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->run((const uint2*) d_R, nR, (const uint2*) d_S, nS, args, (hipStream_t) stream, stats, algorithm);
}

int hwbrj_join_device_async(const tuple_t* d_R, uint64_t nR, const tuple_t* d_S, uint64_t nS,
                            const bloom_filter_args_t* args, void* stream) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    return e->run_async((const uint2*) d_R, nR, (const uint2*) d_S, nS, args, (hipStream_t) stream);
}

int hwbrj_join_partitioned(const hwbrj_exchange_t* x, int rank, int world, const tuple_t* d_R,
                           uint64_t nR, uint64_t nR_total, const tuple_t* d_S, uint64_t nS,
                           const bloom_filter_args_t* args, hwbrj_stats_t* stats) {
    if (!x || !x->buffer || !x->alltoall_u64 || !x->alltoallv || !x->allgather) {
        set_last_error("incomplete exchange (hwbrj_exchange_t)");
        return 2;
    }
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->join_partitioned(x, rank, world, (const uint2*) d_R, nR, nR_total, (const uint2*) d_S, nS,
                               args, stats);
}

int hwbrj_join_wait(hwbrj_stats_t* stats) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->wait(stats);
}

int hwbrj_set_async_timing(int on) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    e->set_async_timing(on != 0);
    return 0;
}

int hwbrj_join_wait_all(hwbrj_stats_t* stats, int capacity, int* n_joins) {
    if (capacity < 0 || (capacity > 0 && !stats)) {
        set_last_error("stats must hold capacity >= 0 entries");
        return 2;
    }
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    return e->wait_all(stats, capacity, n_joins);
}

// The materializing join: the partitioned pipeline carrying payloads (Engine::run_mat); the
// global-bitmap mode (basic k = 0 or B < 8) falls back to a counting join plus the side pass.
// *n = all pairs (also beyond cap); *ms = the device time of the pairs' production.
static int materialize_pairs(Engine* e, const tuple_t* d_R, uint64_t nR, const tuple_t* d_S, uint64_t nS,
                             const bloom_filter_args_t* args, tuple_t* d_out, uint64_t cap, uint64_t* n,
                             hipStream_t stream, hwbrj_stats_t* st, double* ms) {
    int rc = e->run_mat((const uint2*) d_R, nR, (const uint2*) d_S, nS, args, stream,
                        MatReq{(uint2*) d_out, cap}, st);
    if (rc == 0) {
        *n = (uint64_t) st->matches;
        if (ms) *ms = st->ms_total;
        return 0;
    }
    if (rc != kRcMatGlobal) return rc;
    rc = e->run((const uint2*) d_R, nR, (const uint2*) d_S, nS, args, stream, st);
    if (rc) return rc;
    *n = (uint64_t) st->matches;
    if (*n > cap) return 0;  // (the caller reports the capacity)
    uint64_t m = 0;
    rc = e->materialize((const uint2*) d_R, nR, (const uint2*) d_S, nS, (uint2*) d_out, cap, &m, stream, ms);
    if (rc) return rc;
    if (m != *n) {
        set_last_error("materialized pairs differ from the counted matches");
        return 8;
    }
    return 0;
}

int hwbrj_join_materialize_device(const tuple_t* d_R, uint64_t nR, const tuple_t* d_S, uint64_t nS,
                                  const bloom_filter_args_t* args, tuple_t* d_out,
                                  uint64_t capacity, uint64_t* n_out, void* stream,
                                  hwbrj_stats_t* stats, double* ms_materialize) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    hwbrj_stats_t st;
    uint64_t      n  = 0;
    const int     rc = materialize_pairs(e, d_R, nR, d_S, nS, args, d_out, capacity, &n, (hipStream_t) stream,
                                         &st, ms_materialize);
    if (rc) return rc;
    if (stats) *stats = st;
    if (n_out) *n_out = n;
    if (n > capacity) {
        set_last_error("output capacity below the match count (*n_out holds the count)");
        return 7;
    }
    return 0;
}

static int g_materialize = -1;  // -1: from HWBRJ_MATERIALIZE
static int g_gpus        = 0;   // shards of a host BPRO/PRO (0: from HWBRJ_GPUS, default 1)
void hwbrj_set_materialize(int on) { g_materialize = on ? 1 : 0; }

int hwbrj_set_gpus(int g) {
    if (g < 0 || g > 4096) {
        set_last_error("gpus must be in [0, 4096]");
        return 2;
    }
    g_gpus = g;
    return 0;
}

int hwbrj_generate_device(tuple_t* d_out, uint64_t n, uint32_t nthreads, uint64_t maxid,
                          uint64_t threshold, double selectivity, uint64_t seed, void* stream) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    return e->generate((uint2*) d_out, n, 0, n, nthreads, maxid, threshold, selectivity, seed,
                       (hipStream_t) stream);
}

int hwbrj_generate_device_range(tuple_t* d_out, uint64_t n, uint64_t offset, uint64_t count,
                                uint32_t nthreads, uint64_t maxid, uint64_t threshold,
                                double selectivity, uint64_t seed, void* stream) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    return e->generate((uint2*) d_out, n, offset, count, nthreads, maxid, threshold, selectivity,
                       seed, (hipStream_t) stream);
}

int hwbrj_generate_host(tuple_t* out, uint64_t n, uint32_t nthreads, uint64_t maxid,
                        uint64_t threshold, double selectivity, uint64_t seed, int host_threads) {
    std::vector<GenPlan> plan(1);
    if (make_gen_plan(&plan[0], n, nthreads, maxid, threshold, selectivity)) {
        set_last_error("invalid generator parameters");
        return 2;
    }
    const Perm perm = make_perm(n, seed);
    int        T    = host_threads > 0 ? host_threads : (int) std::thread::hardware_concurrency();
    if (T < 1) T = 1;
    if ((uint64_t) T > n / 4096 + 1) T = (int) (n / 4096 + 1);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) {
        th.emplace_back([&, t] {
            const uint64_t b = n * t / T, e = n * (t + 1) / T;
            for (uint64_t i = b; i < e; i++) {
                out[i].key     = gen_key_at(plan[0], perm_apply(perm, i));
                out[i].payload = (int32_t) i;
            }
        });
    }
    for (auto& x : th) x.join();
    return 0;
}

int hwbrj_export_filter(uint8_t* host_out, uint64_t nbytes) {
    Engine* e = engine_for_current_device();
    if (!e) return 10;  // (last error set by engine_for_current_device)
    return e->export_filter(host_out, nbytes);
}

// src/bloom_filter.c:25-34 -- prints the reference's message and exits(1).
void assert_args(bloom_filter_args_t* args) {
    if ((args->m & (args->m - 1)) != 0) {
        printf("m must be a power of 2");
        exit(1);
    }
    if (args->variant != BASIC) {
        const uint64_t B = args->B;
        if (B == 0 || (B & (B - 1)) != 0) {
            printf("B must be a power 2");
            exit(1);
        }
        if (args->m % B != 0) {
            printf("m must be a multiple of B");
            exit(1);
        }
    }
}

}  // extern "C"

// ------------------------------------------------------------------ BPRO / PRO (host data)
static void fatal(const char* what) {
    printf("[ERROR] %s: %s\n", what, hwbrj_last_error());
    exit(EXIT_FAILURE);  // the reference's convention (src/parallel_radix_join_bloom.c:64-71)
}

// src/parallel_radix_join_bloom.c:1509-1547 print_timing, fed with device times.
static void print_timing(uint64_t total_cyc, uint64_t build_cyc, uint64_t part_cyc,
                         uint64_t numtuples, int64_t result, double total_usec,
                         double part_usec, double probe_usec, double join_usec) {
    const double nsec_per_tuple = total_usec * 1000.0 / (double) (numtuples ? numtuples : 1);
    fprintf(stdout, "RUNTIME TOTAL, BUILD, PART (cycles): \n");
    fprintf(stdout, "%llu \t %llu \t %llu ", (unsigned long long) total_cyc,
            (unsigned long long) build_cyc, (unsigned long long) part_cyc);
    fprintf(stdout, "\n");
    fprintf(stdout, "TOTAL-TIME-USECS, TOTAL-TUPLES, NSEC-PER-TUPLE: \n");
    fprintf(stdout, "%.4lf \t %llu \t ", total_usec, (unsigned long long) result);
    fprintf(stdout, "%.4lf ", nsec_per_tuple);
    fprintf(stdout, "\n");
    fprintf(stdout, "PARTITION-TIME-USECS, PROBE-TIME-USECS, JOIN-TIME-USECS: \n");
    fprintf(stdout, "%.4lf \t %.4lf\t %.4lf \n", part_usec, probe_usec, join_usec);
    fflush(stdout);
}

// src/tuple_buffer.h:27-126: the reference's chained result buffers. The newest buffer is the
// head (cb->buf, `writepos` tuples); older, full buffers of CHAINEDBUFF_NUMTUPLESPERBUF follow
// through `next`, so cb_begin / cb_read_next walk every pair.
namespace {
constexpr uint32_t kCbTuples = 1024 * 1024;  // CHAINEDBUFF_NUMTUPLESPERBUF
struct TupleBuffer {
    tuple_t*     tuples;
    TupleBuffer* next;
};
struct ChainedTupleBuffer {
    TupleBuffer* buf;
    TupleBuffer* readcursor;
    TupleBuffer* writecursor;
    uint32_t     writepos, readpos, readlen, numbufs;
};

ChainedTupleBuffer* chained_from(const tuple_t* pairs, uint64_t n) {
    ChainedTupleBuffer* cb   = (ChainedTupleBuffer*) calloc(1, sizeof(ChainedTupleBuffer));
    TupleBuffer*        head = nullptr;
    uint64_t            off  = 0;
    do {
        const uint64_t c = n - off < kCbTuples ? n - off : kCbTuples;
        TupleBuffer*   b = (TupleBuffer*) malloc(sizeof(TupleBuffer));
        if (posix_memalign((void**) &b->tuples, 64, sizeof(tuple_t) * kCbTuples)) b->tuples = nullptr;
        if (!b->tuples) {
            set_last_error("out of host memory (result buffers)");
            return nullptr;
        }
        if (c) memcpy(b->tuples, pairs + off, c * sizeof(tuple_t));
        b->next      = head;
        head         = b;
        cb->writepos = (uint32_t) c;
        cb->numbufs++;
        off += c;
    } while (off < n);
    cb->buf = cb->readcursor = cb->writecursor = head;
    return cb;
}
}  // namespace

// JOIN_RESULT_MATERIALIZE (src/parallel_radix_join_bloom.c:1450-1472): resultlist[t] of every
// worker; here all pairs are thread 0's, the others hold empty buffers.
static threadresult_t* materialize_to_host(const tuple_t* dR, uint64_t nR, const tuple_t* dS,
                                           uint64_t nS, const bloom_filter_args_t* args,
                                           uint64_t matches, int nthreads) {
    tuple_t* dout = nullptr;
    if (hipMalloc((void**) &dout, (matches ? matches : 1) * sizeof(tuple_t)) != hipSuccess) {
        set_last_error("hipMalloc of the result pairs failed");
        fatal("BPRO");
    }
    Engine*       e = engine_for_current_device();
    uint64_t      n = 0;
    hwbrj_stats_t st;
    if (!e || materialize_pairs(e, dR, nR, dS, nS, args, dout, matches, &n, nullptr, &st, nullptr) != 0 ||
        n != matches)
        fatal("BPRO (materialize)");
    std::vector<tuple_t> host(matches ? matches : 1);
    if (matches && hipMemcpy(host.data(), dout, matches * sizeof(tuple_t), hipMemcpyDeviceToHost) != hipSuccess) {
        set_last_error("D2H of the result pairs failed");
        fatal("BPRO");
    }
    (void) hipFree(dout);
    const int       T    = nthreads > 0 ? nthreads : 1;
    threadresult_t* tres = (threadresult_t*) calloc(T, sizeof(threadresult_t));
    for (int t = 0; t < T; t++) {
        tres[t].threadid = (uint32_t) t;
        tres[t].nresults = t == 0 ? (int64_t) matches : 0;
        tres[t].results  = chained_from(host.data(), t == 0 ? matches : 0);
        if (!tres[t].results) fatal("BPRO");
    }
    return tres;
}

static int host_shards() {
    if (g_gpus > 0) return g_gpus;
    const char* e = getenv("HWBRJ_GPUS");
    const int   v = e ? atoi(e) : 1;
    return v > 0 ? v : 1;
}

// One shard of a host join: R replicated, S rows [s0, s1) (the reference's per-thread chunking of
// S, src/parallel_radix_join_bloom.c:1646-1670, with a GPU per chunk).
struct Shard {
    uint64_t      s0 = 0, s1 = 0;
    hwbrj_stats_t st{};
    double        h2d_usec = 0;
    tuple_t*      dS = nullptr;  // this shard's S rows in HBM (staged before the timed region)
};

// The device copies of one device's shards (first, first + step, ...): R once, every shard's S.
struct DeviceStage {
    int      dev = 0;
    tuple_t* dR  = nullptr;
};

static void free_stage(DeviceStage& ds, std::vector<Shard>& shards, int first, int step) {
    (void) hipSetDevice(ds.dev);
    (void) hipFree(ds.dR);
    ds.dR = nullptr;
    for (size_t g = first; g < shards.size(); g += step) {
        (void) hipFree(shards[g].dS);
        shards[g].dS = nullptr;
    }
}

// Everything the reference does before its timer starts (src/parallel_radix_join_bloom.c:1560-1640:
// allocations, the zeroed bitmap and tmp buffers): device allocations, the H2D copies of R and of
// every shard's S rows, and the join's scratch (Engine::reserve). Returns 0 or an error code.
static int stage_device_shards(DeviceStage& ds, int first, int step, const relation_t* relR,
                               const relation_t* relS, const bloom_filter_args_t* args,
                               std::vector<Shard>& shards, int algo) {
    if (hipSetDevice(ds.dev) != hipSuccess) {
        set_last_error("hipSetDevice failed");
        return 11;
    }
    const uint64_t nR = relR->num_tuples;
    if (hipMalloc((void**) &ds.dR, (nR ? nR : 1) * sizeof(tuple_t)) != hipSuccess) {
        set_last_error("hipMalloc of the input relations failed");
        return 12;
    }
    const auto h0 = std::chrono::steady_clock::now();
    if (nR && hipMemcpy(ds.dR, relR->tuples, nR * sizeof(tuple_t), hipMemcpyHostToDevice) != hipSuccess) {
        set_last_error("H2D copy failed");
        return 13;
    }
    double h2d_r = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
    for (size_t g = first; g < shards.size(); g += step) {
        Shard&         sh = shards[g];
        const uint64_t n  = sh.s1 - sh.s0;
        if (hipMalloc((void**) &sh.dS, (n ? n : 1) * sizeof(tuple_t)) != hipSuccess) {
            set_last_error("hipMalloc of the input relations failed");
            return 12;
        }
        const auto h1 = std::chrono::steady_clock::now();
        if (n && hipMemcpy(sh.dS, relS->tuples + sh.s0, n * sizeof(tuple_t), hipMemcpyHostToDevice) != hipSuccess) {
            set_last_error("H2D copy failed");
            return 13;
        }
        sh.h2d_usec = h2d_r + std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h1).count();
        h2d_r       = 0;
    }
    Engine* e = engine_for_current_device();
    if (!e) return 10;
    for (size_t g = first; g < shards.size(); g += step) {  // grow-only: the largest shard decides
        const int rc = e->reserve((const uint2*) ds.dR, nR, (const uint2*) shards[g].dS,
                                  shards[g].s1 - shards[g].s0, args, algo);
        if (rc) return rc;
    }
    return hipDeviceSynchronize() == hipSuccess ? 0 : 14;
}

// The timed part: the device's shards joined one after the other on its Engine.
static int join_device_shards(const DeviceStage& ds, int first, int step, uint64_t nR,
                              const bloom_filter_args_t* args, std::vector<Shard>& shards, int algo) {
    if (hipSetDevice(ds.dev) != hipSuccess) {
        set_last_error("hipSetDevice failed");
        return 11;
    }
    for (size_t g = first; g < shards.size(); g += step) {
        Shard&    sh = shards[g];
        const int rc = hwbrj_join_device_algo(ds.dR, nR, sh.dS, sh.s1 - sh.s0, args, algo, nullptr, &sh.st);
        if (rc) return rc;
    }
    return 0;
}

// algo: the per-partition join (HWBRJ_ALGO_PRO / PRH / PRHO, the reference's join_init_run
// JoinFunction: bucket_chaining_join / histogram_join / histogram_optimized_join)
static result_t* run_host_join(relation_t* relR, relation_t* relS, int nthreads,
                               bloom_filter_args_t* args, bool print_filtered = true, int algo = 0) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        set_last_error("no MI355X device visible");
        fatal("BPRO");
    }
    int cur = 0;
    (void) hipGetDevice(&cur);
    const uint64_t nR = relR->num_tuples, nS = relS->num_tuples;
    // G shards of S over the visible devices (shard g on device g mod ndev; G > ndev runs several
    // shards per device one after the other, e.g. to rehearse G = 8 on one GPU)
    const int          G    = host_shards();
    const int          nuse = std::min(G, ndev);
    std::vector<Shard> shards(G);
    for (int g = 0; g < G; g++) {
        shards[g].s0 = nS * (uint64_t) g / (uint64_t) G;
        shards[g].s1 = nS * (uint64_t) (g + 1) / (uint64_t) G;
    }
    std::vector<int> rcs(nuse, 0);
    std::vector<std::string> errs(nuse);
    std::vector<DeviceStage> stage(nuse);
    for (int d = 0; d < nuse; d++) stage[d].dev = nuse == 1 ? cur : d;
    // one host thread per device (the reference's nthreads workers, one per GPU); phase 0 stages
    // the inputs and scratch, phase 1 is the timed join
    auto each_device = [&](int phase) {
        auto work = [&](int d) {
            rcs[d] = phase == 0 ? stage_device_shards(stage[d], d, nuse, relR, relS, args, shards, algo)
                                : join_device_shards(stage[d], d, nuse, nR, args, shards, algo);
            errs[d] = hwbrj_last_error();
        };
        if (nuse == 1) {
            work(0);
        } else {
            std::vector<std::thread> th;
            for (int d = 0; d < nuse; d++) th.emplace_back(work, d);
            for (auto& t : th) t.join();
        }
        for (int d = 0; d < nuse; d++)
            if (rcs[d]) {
                for (int d2 = 0; d2 < nuse; d2++) free_stage(stage[d2], shards, d2, nuse);
                (void) hipSetDevice(cur);
                set_last_error(errs[d]);
                fatal("BPRO");
            }
    };
    each_device(0);
    // The timed region (src/parallel_radix_join_bloom.c:1107-1131 to :1477-1484): the joins only,
    // so RUNTIME TOTAL (cycles) and TOTAL-TIME-USECS cover the same work.
    const uint64_t c0 = __rdtsc();
    each_device(1);
    const uint64_t c1 = __rdtsc();
    for (int d = 0; d < nuse; d++) free_stage(stage[d], shards, d, nuse);
    (void) hipSetDevice(cur);
    // counts summed over shards; device times: the slowest device (its shards back to back)
    hwbrj_stats_t st{};
    std::vector<double> dev_ms(nuse, 0.0), dev_join(nuse, 0.0), dev_probe(nuse, 0.0);
    double h2d_usec = 0;
    for (int g = 0; g < G; g++) {
        const hwbrj_stats_t& s = shards[g].st;
        st.filtered += s.filtered;
        st.matches += s.matches;
        st.mode = s.mode, st.format = s.format, st.partitions = s.partitions;
        st.subparts = s.subparts, st.slice_segments = s.slice_segments;
        dev_ms[g % nuse] += s.ms_total;
        dev_join[g % nuse] += s.ms_join;
        dev_probe[g % nuse] += s.ms_join_probe;
        h2d_usec = std::max(h2d_usec, shards[g].h2d_usec);
        st.ms_r_scatter += s.ms_r_scatter, st.ms_r_index += s.ms_r_index, st.ms_build += s.ms_build;
        st.ms_s_scatter += s.ms_s_scatter, st.ms_s_index += s.ms_s_index, st.ms_probe += s.ms_probe;
        st.ms_surv += s.ms_surv;
    }
    const int slow = (int) (std::max_element(dev_ms.begin(), dev_ms.end()) - dev_ms.begin());
    st.ms_total      = dev_ms[slow];
    st.ms_join       = dev_join[slow];
    st.ms_join_probe = dev_probe[slow];
    // materialization (JOIN_RESULT_MATERIALIZE) runs on one device over the whole relations
    const bool mat = g_materialize == 1 || (g_materialize < 0 && getenv("HWBRJ_MATERIALIZE"));
    threadresult_t* tres = nullptr;
    if (mat) {
        tuple_t *dR = nullptr, *dS = nullptr;
        if (hipMalloc((void**) &dR, (nR ? nR : 1) * sizeof(tuple_t)) != hipSuccess ||
            hipMalloc((void**) &dS, (nS ? nS : 1) * sizeof(tuple_t)) != hipSuccess ||
            (nR && hipMemcpy(dR, relR->tuples, nR * sizeof(tuple_t), hipMemcpyHostToDevice) != hipSuccess) ||
            (nS && hipMemcpy(dS, relS->tuples, nS * sizeof(tuple_t), hipMemcpyHostToDevice) != hipSuccess)) {
            set_last_error("device copies of the relations for materialization failed");
            fatal("BPRO");
        }
        hwbrj_stats_t one;
        if (G > 1 && hwbrj_join_device_algo(dR, nR, dS, nS, args, algo, nullptr, &one) != 0) fatal("BPRO");
        tres = materialize_to_host(dR, nR, dS, nS, args, (uint64_t) st.matches, nthreads);
        (void) hipFree(dR);
        (void) hipFree(dS);
    }
    // "S-tuples after filter" is printed by BPRO/BPRH/BPRHO's thread 0 (:1253); BRJ has no such line
    if (args && print_filtered) fprintf(stdout, "S-tuples after filter: %d\n", (int) st.filtered);
    // print_timing (:1730-1742): PARTITION = start -> partitioned (both partition passes, filter
    // build and probe), JOIN = partitioned -> end, PROBE = the probe share of the join (the
    // reference's per-thread probe timers, bucket_chaining_join :289-321), cycles likewise
    const double total_cyc = (double) (c1 - c0);
    const double part_ms   = st.ms_total - st.ms_join;
    const double frac_part = st.ms_total > 0 ? part_ms / st.ms_total : 0.0;
    const double frac_prob = st.ms_total > 0 ? st.ms_join_probe / st.ms_total : 0.0;
    const uint64_t part_cyc  = (uint64_t) (total_cyc * frac_part);
    const uint64_t probe_cyc = (uint64_t) (total_cyc * frac_prob);
    print_timing((uint64_t) total_cyc, (uint64_t) total_cyc - part_cyc - probe_cyc, part_cyc, nS,
                 st.matches, st.ms_total * 1e3, part_ms * 1e3, st.ms_join_probe * 1e3, st.ms_join * 1e3);
    if (getenv("HWBRJ_VERBOSE"))
        fprintf(stderr,
                "[hwbrj] shards=%d devices=%d mode=%d format=%d F=%u NSUB=%u nseg=%u h2d_usec=%.1f | "
                "ms (summed over shards): r_scatter %.3f r_index %.3f build %.3f s_scatter %.3f "
                "s_index %.3f probe %.3f surv %.3f | join (slowest device) %.3f\n",
                G, nuse, st.mode, st.format, st.partitions, st.subparts, st.slice_segments, h2d_usec,
                st.ms_r_scatter, st.ms_r_index, st.ms_build, st.ms_s_scatter, st.ms_s_index,
                st.ms_probe, st.ms_surv, st.ms_join);
    result_t* res = (result_t*) malloc(sizeof(result_t));
    if (!res) {
        set_last_error("malloc");
        fatal("BPRO");
    }
    res->totalresults = st.matches;
    res->resultlist   = tres;
    res->nthreads     = nthreads;
    return res;
}

extern "C" {

// src/parallel_radix_join_bloom.h:34-36
result_t* BPRO(relation_t* relR, relation_t* relS, int nthreads,
               bloom_filter_args_t* bloom_filter_args) {
    return run_host_join(relR, relS, nthreads, bloom_filter_args);
}

// src/parallel_radix_join.h:33-34
result_t* PRO(relation_t* relR, relation_t* relS, int nthreads) {
    return run_host_join(relR, relS, nthreads, nullptr);
}

// The other entries of the reference's algorithm table (src/main.c:331-339). BPRH / BPRHO plug a
// different per-partition join function into the same join_init_run
// (src/parallel_radix_join_bloom.c:1789-1804): the histogram join of Kim et al. (histogram_join,
// :350-419) and its SIMD + prefetch form (histogram_optimized_join, :441-555); here k_join runs
// them (JoinParams::jkind 1 / 2) instead of its bitmap / hash table. BRJ is the single-threaded
// form of BPRO (:1806-1930) with bucket chaining: the same operator on the MI355X.
result_t* BPRH(relation_t* relR, relation_t* relS, int nthreads, bloom_filter_args_t* a) {
    return run_host_join(relR, relS, nthreads, a, true, 1);
}
result_t* BPRHO(relation_t* relR, relation_t* relS, int nthreads, bloom_filter_args_t* a) {
    return run_host_join(relR, relS, nthreads, a, true, 2);
}
result_t* BRJ(relation_t* relR, relation_t* relS, int nthreads, bloom_filter_args_t* a) {
    return run_host_join(relR, relS, nthreads, a, false);
}
result_t* PRH(relation_t* relR, relation_t* relS, int nthreads) {
    return run_host_join(relR, relS, nthreads, nullptr, true, 1);
}
result_t* PRHO(relation_t* relR, relation_t* relS, int nthreads) {
    return run_host_join(relR, relS, nthreads, nullptr, true, 2);
}
result_t* RJ(relation_t* relR, relation_t* relS, int nthreads) {
    return run_host_join(relR, relS, nthreads, nullptr);
}

result_t* hwbrj_BPRO(relation_t* relR, relation_t* relS, int nthreads,
                     bloom_filter_args_t* bloom_filter_args) {
    return run_host_join(relR, relS, nthreads, bloom_filter_args);
}

result_t* hwbrj_PRO(relation_t* relR, relation_t* relS, int nthreads) {
    return run_host_join(relR, relS, nthreads, nullptr);
}

}  // extern "C"
