// hwbrj_gen.cpp -- the reference's rand()-driven relation generators on the host, bit-exact.
//
// The reference builds these relations with glibc rand() after srand(-x / -y seed)
// (src/main.c:410-466):
//   --non-unique  R: create_relation_nonunique          src/generator.c:585-605 (random_gen :271-279)
//                 S: create_relation_nonunique_from_pk  :608-646
//   --full-range  R: create_relation_nonunique          (threshold = ceil(INT_MAX * q))
//                 S: create_relation_fk_from_pk         :531-582
//   -z <theta>    S: create_relation_zipf -> gen_zipf   :659-676, src/genzipf.c:28-158
// Their counts depend on the exact rand() sequence, so rand() is restated here (glibc's TYPE_3
// additive feedback generator behind rand(), with its own state instead of libc's global one) and
// every draw happens in the reference's order, including the Knuth shuffles. The only deliberate
// difference: gen_zipf leaves payloads uninitialised (genzipf.c:147-148); here payload = row index.
//
// Host code, compiled without floating-point contraction: RAND_RANGE's a*b+c must round like the
// reference's x86-64 build (no FMA).
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <climits>
#include <thread>
#include <vector>

#include "hwbrj_engine.h"

#pragma clang fp contract(off)

namespace hwbrj {

// glibc stdlib/random_r.c, TYPE_3 (degree 31, separation 3): srandom_r seeds the 31 words with
// the Park-Miller LCG (Schrage's method), then discards 310 outputs; random_r adds the lagged word
// and returns the sum >> 1. RAND_MAX = 2^31 - 1.
void GlibcRand::seed(uint32_t s) {
    if (s == 0) s = 1;
    int32_t word = (int32_t) s;
    st[0]        = word;
    for (int i = 1; i < 31; i++) {
        const int64_t hi = word / 127773, lo = word % 127773;
        int64_t       w  = 16807 * lo - 2836 * hi;
        if (w < 0) w += 2147483647;
        word  = (int32_t) w;
        st[i] = word;
    }
    f = 3;
    r = 0;
    for (int i = 0; i < 310; i++) (void) next();
}

// ------------------------------------------------------------------ src/generator.c helpers
static constexpr double kRandMaxP1 = (double) 2147483647 + 1;  // (double) RAND_MAX + 1

// RAND_RANGE(O, N) = O + (double) rand() / ((double) RAND_MAX + 1) * (N - O)   (generator.c:25)
static inline double rand_range(GlibcRand& g, double O, double N) {
    const double x = (double) g.next() / kRandMaxP1;
    const double s = x * (N - O);
    return O + s;
}

// random_gen (generator.c:271-279): keys in [minid, maxid), payload = index in `rel`.
static void random_gen(GlibcRand& g, tuple_t* rel, uint64_t n, int64_t minid, int64_t maxid) {
    for (uint64_t i = 0; i < n; i++) {
        rel[i].key     = (int32_t) rand_range(g, (double) minid, (double) maxid);
        rel[i].payload = (int32_t) i;
    }
}

// knuth_shuffle (generator.c:99-109): keys only; the loop index is an int.
static void knuth_shuffle(GlibcRand& g, tuple_t* rel, uint64_t n) {
    for (int i = (int) n - 1; i > 0; i--) {
        const int64_t j   = (int64_t) rand_range(g, 0.0, (double) i);
        const int32_t tmp = rel[i].key;
        rel[i].key        = rel[j].key;
        rel[j].key        = tmp;
    }
}

// gen_alphabet (genzipf.c:28-53: 1..size permuted by rand() after srand(seed)) and gen_zipf_lut
// (:60-92: the two sequential sums of 1 / pow(i, theta); the pow terms are computed in parallel,
// the sums in the reference's order). Leaves *g positioned for the stream. Returns the thread count.
static int zipf_tables(GlibcRand* g, unsigned int size, double theta, uint32_t seed, int host_threads,
                       std::vector<uint32_t>* alphabet, std::vector<double>* lut) {
    g->seed(seed);
    int T = host_threads > 0 ? host_threads : (int) std::thread::hardware_concurrency();
    T     = std::max(1, std::min(T, 64));
    alphabet->resize(size);
    uint32_t* a = alphabet->data();
    for (unsigned int i = 0; i < size; i++) a[i] = i + 1;
    for (unsigned int i = size - 1; i > 0; i--) {
        const unsigned int k   = (unsigned int) ((unsigned long) i * (unsigned long) g->next() /
                                                 (unsigned long) 2147483647);
        const uint32_t     tmp = a[i];
        a[i]                   = a[k];
        a[k]                   = tmp;
    }
    lut->resize(size);
    double* l = lut->data();
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([=] {
            const uint64_t b = (uint64_t) size * t / T, e = (uint64_t) size * (t + 1) / T;
            for (uint64_t i = b; i < e; i++) l[i] = 1.0 / pow((double) (unsigned int) (i + 1), theta);
        });
    for (auto& x : th) x.join();
    double scaling = 0.0;
    for (unsigned int i = 0; i < size; i++) scaling += l[i];
    double sum = 0.0;
    for (unsigned int i = 0; i < size; i++) {
        sum += l[i];
        l[i] = sum / scaling;
    }
    return T;
}

}  // namespace hwbrj

using namespace hwbrj;

extern "C" {

uint64_t hwbrj_nonunique_threshold(uint64_t r_size, double selectivity, int full_range) {
    // src/main.c:421-427
    const double t = ceil((double) INT_MAX * selectivity);
    if (full_range) return (uint64_t) t;
    return (double) r_size < t ? r_size : (uint64_t) t;
}

int hwbrj_rand_stream(uint32_t seed, int32_t* out, uint64_t n) {
    GlibcRand g;
    g.seed(seed);
    for (uint64_t i = 0; i < n; i++) out[i] = g.next();
    return 0;
}

int hwbrj_create_relation_nonunique(tuple_t* out, uint64_t n, int64_t maxid, uint32_t seed) {
    if (!out && n) {
        set_last_error("null output");
        return 2;
    }
    GlibcRand g;
    g.seed(seed);  // seed_generator (generator.c:75-81, main.c:410)
    random_gen(g, out, n, 0, maxid);
    return 0;
}

int hwbrj_create_relation_nonunique_from_pk(tuple_t* out, uint64_t n, const tuple_t* pk,
                                            uint64_t npk, int64_t threshold, double selectivity,
                                            uint32_t seed) {
    if ((!out && n) || (!pk && npk) || (npk == 0 && n > 0) || n > (uint64_t) INT_MAX) {
        set_last_error("invalid arguments (|S| must be < 2^31 and the pk relation non-empty)");
        return 2;
    }
    GlibcRand g;
    g.seed(seed);
    const uint64_t above = (uint64_t) ((double) n * (1 - selectivity));  // generator.c:616
    if (above > n) {
        set_last_error("selectivity out of range");
        return 2;
    }
    random_gen(g, out, above, threshold + 1, INT_MAX);
    for (int i = (int) above; i < (int) n; i++) {  // :632-637
        const int j    = (int) rand_range(g, 0.0, (double) npk);
        out[i].key     = pk[j].key;
        out[i].payload = i;
    }
    knuth_shuffle(g, out, n);
    return 0;
}

int hwbrj_create_relation_fk_from_pk(tuple_t* out, uint64_t n, const tuple_t* pk, uint64_t npk,
                                     int64_t threshold, double selectivity, uint32_t seed) {
    if ((!out && n) || (!pk && npk) || n > (uint64_t) INT_MAX) {
        set_last_error("invalid arguments (|S| must be < 2^31)");
        return 2;
    }
    GlibcRand g;
    g.seed(seed);
    const uint64_t above = (uint64_t) ((double) n * (1 - selectivity));  // generator.c:548
    if (above > n) {
        set_last_error("selectivity out of range");
        return 2;
    }
    const uint64_t below = n - above;
    if (below > 0 && npk == 0) {
        set_last_error("empty pk relation");
        return 2;
    }
    random_gen(g, out + below, above, threshold + 1, INT_MAX);  // unmatched tuples last
    uint64_t off = 0;
    while (off < below) {  // whole copies of pk, then the remainder (:560-571)
        const uint64_t c = std::min(npk, below - off);
        memcpy(out + off, pk, c * sizeof(tuple_t));
        off += c;
    }
    knuth_shuffle(g, out, n);
    return 0;
}

// src/genzipf.c:28-158 via create_relation_zipf (generator.c:659-676). The rand() stream is drawn
// in order on one thread; the binary searches over the CDF run on `host_threads` threads.
int hwbrj_create_relation_zipf(tuple_t* out, uint64_t n, uint64_t alphabet_size, double theta,
                               uint32_t seed, int host_threads) {
    if ((!out && n) || alphabet_size == 0 || alphabet_size > (uint64_t) UINT_MAX ||
        n > (uint64_t) UINT_MAX) {
        set_last_error("invalid arguments (alphabet and |S| must be in [1, 2^32))");
        return 2;
    }
    const unsigned int    size = (unsigned int) alphabet_size;
    GlibcRand             g;
    std::vector<uint32_t> alphabet;
    std::vector<double>   lut;
    const int             T = zipf_tables(&g, size, theta, seed, host_threads, &alphabet, &lut);
    auto par = [&](uint64_t total, auto&& fn) {
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] { fn(total * t / T, total * (t + 1) / T); });
        for (auto& x : th) x.join();
    };
    // the stream (:119-150): r = rand() / RAND_MAX, binary search, key = alphabet[pos]
    for (uint64_t i = 0; i < n; i++) out[i].key = g.next();
    par(n, [&](uint64_t b, uint64_t e) {
        for (uint64_t i = b; i < e; i++) {
            const double r     = ((double) out[i].key) / 2147483647;
            unsigned int left  = 0, right = size - 1, pos;
            if (lut[0] >= r) {
                pos = 0;
            } else {
                while (right - left > 1) {
                    const unsigned int m = (left + right) / 2;
                    if (lut[m] < r) left = m;
                    else right = m;
                }
                pos = right;
            }
            out[i].key     = (int32_t) alphabet[pos];
            out[i].payload = (int32_t) i;
        }
    });
    return 0;
}

// The same Zipf relation generated into HBM (the binary searches run on the GPU; the rand() stream
// is drawn on the host in order and shipped in chunks). selectivity < 1 is this build's extension
// for BASELINE config 5 (the reference ignores -q under -z, src/main.c:457-466): floor(n (1 - q))
// rows, chosen by a seeded permutation, get unique keys above the alphabet, so exactly the other
// rows match. selectivity = 1 gives the reference's relation.
int hwbrj_create_relation_zipf_device(tuple_t* d_out, uint64_t n, uint64_t alphabet_size,
                                      double theta, uint32_t seed, double selectivity,
                                      int host_threads, void* stream) {
    if ((!d_out && n) || alphabet_size == 0 || alphabet_size > (uint64_t) UINT_MAX ||
        n > (uint64_t) UINT_MAX || selectivity < 0 || selectivity > 1) {
        set_last_error("invalid arguments (alphabet and |S| in [1, 2^32), q in [0, 1])");
        return 2;
    }
    const uint64_t n_above = (uint64_t) ((double) n * (1 - selectivity));
    if (alphabet_size + 1 + n_above > (uint64_t) INT_MAX) {
        set_last_error("alphabet + unmatched keys exceed INT_MAX");
        return 2;
    }
    hipStream_t st = (hipStream_t) stream;
    GlibcRand             g;
    std::vector<uint32_t> alphabet;
    std::vector<double>   lut;
    zipf_tables(&g, (unsigned int) alphabet_size, theta, seed, host_threads, &alphabet, &lut);
    const uint64_t kChunk = 1ull << 26;
    uint32_t* d_alpha = nullptr;
    double*   d_lut   = nullptr;
    int32_t*  d_rnd   = nullptr;
    auto fail = [&](const char* what) {
        set_last_error(what);
        (void) hipFree(d_alpha);
        (void) hipFree(d_lut);
        (void) hipFree(d_rnd);
        return 4;
    };
    if (hipMalloc((void**) &d_alpha, alphabet.size() * 4) != hipSuccess ||
        hipMalloc((void**) &d_lut, lut.size() * 8) != hipSuccess ||
        hipMalloc((void**) &d_rnd, kChunk * 4) != hipSuccess)
        return fail("hipMalloc failed (zipf tables)");
    if (hipMemcpy(d_alpha, alphabet.data(), alphabet.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_lut, lut.data(), lut.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        return fail("H2D of the zipf tables failed");
    std::vector<int32_t> rnd(std::min(n, kChunk));
    const Perm           perm = make_perm(n ? n : 1, seed ^ 0x5A17F00Dull);
    for (uint64_t r0 = 0; r0 < n; r0 += kChunk) {
        const uint64_t c = std::min(kChunk, n - r0);
        for (uint64_t i = 0; i < c; i++) rnd[i] = g.next();
        if (hipStreamSynchronize(st) != hipSuccess ||  // the previous chunk's kernel read d_rnd
            hipMemcpy(d_rnd, rnd.data(), c * 4, hipMemcpyHostToDevice) != hipSuccess)
            return fail("H2D of the rand() stream failed");
        launch_zipf(d_rnd, c, r0, d_lut, d_alpha, (uint32_t) alphabet_size, (uint2*) d_out + r0, n_above,
                    (uint32_t) (alphabet_size + 1), perm, st);
        if (hipGetLastError() != hipSuccess) return fail("zipf kernel launch failed");
    }
    if (hipStreamSynchronize(st) != hipSuccess) return fail("zipf kernel failed");
    (void) hipFree(d_alpha);
    (void) hipFree(d_lut);
    (void) hipFree(d_rnd);
    return 0;
}

// ---- relation files (the reference's PERSIST_RELATIONS output, the only on-disk format) ----
// "%d %d\n" lines through a large buffer (fprintf per tuple is slow for 10^9 tuples).
// backwards: t[n-1] first (write_result_relation's cb_read_backwards order, tuple_buffer.h:77-90)
static int write_pairs(FILE* fp, const tuple_t* t, uint64_t n, bool backwards = false) {
    std::vector<char> buf(1 << 20);
    size_t            used = 0;
    auto put_int = [&](int32_t v, char end) {
        char     tmp[16];
        int      len = 0;
        uint32_t u   = v < 0 ? 0u - (uint32_t) v : (uint32_t) v;
        do {
            tmp[len++] = (char) ('0' + u % 10);
            u /= 10;
        } while (u);
        if (v < 0) buf[used++] = '-';
        while (len) buf[used++] = tmp[--len];
        buf[used++] = end;
    };
    for (uint64_t i = 0; i < n; i++) {
        if (used + 32 > buf.size()) {
            if (fwrite(buf.data(), 1, used, fp) != used) return 1;
            used = 0;
        }
        const tuple_t& x = t[backwards ? n - 1 - i : i];
        put_int(x.key, ' ');
        put_int(x.payload, '\n');
    }
    return used && fwrite(buf.data(), 1, used, fp) != used ? 1 : 0;
}

// src/generator.c:250-263 write_relation: a "#KEY, VAL" header, then "key payload" lines.
int hwbrj_write_relation(const relation_t* rel, const char* filename) {
    FILE* fp = fopen(filename, "w");
    if (!fp) {
        set_last_error(std::string("cannot open ") + filename);
        return 2;
    }
    int rc = fputs("#KEY, VAL\n", fp) < 0 ? 1 : write_pairs(fp, rel->tuples, rel->num_tuples);
    if (fclose(fp) != 0) rc = 1;
    if (rc) set_last_error(std::string("write failed: ") + filename);
    return rc;
}

// src/tuple_buffer.h:155-236 write_result_relation (SORTED_MATERIALIZE_TO_FILE 0, its default):
// every worker's chained result buffers, "R.payload S.payload" lines, no header. The buffers are
// this library's (result_t.resultlist of a materializing BPRO / PRO, hwbrj_api.cpp).
int hwbrj_write_result_relation(const result_t* res, const char* filename) {
    struct Buf {
        tuple_t* tuples;
        Buf*     next;
    };
    struct Chain {
        Buf*     buf;
        Buf*     readcursor;
        Buf*     writecursor;
        uint32_t writepos, readpos, readlen, numbufs;
    };
    constexpr uint64_t kPer = 1024 * 1024;  // CHAINEDBUFF_NUMTUPLESPERBUF (tuple_buffer.h)
    if (!res || !res->resultlist) {
        set_last_error("the result holds no materialized pairs (hwbrj_set_materialize)");
        return 2;
    }
    FILE* fp = fopen(filename, "w");
    if (!fp) {
        set_last_error(std::string("cannot open ") + filename);
        return 2;
    }
    int rc = 0;
    for (int t = 0; t < res->nthreads && rc == 0; t++) {
        const Chain* cb = (const Chain*) res->resultlist[t].results;
        if (!cb) continue;
        uint64_t left = (uint64_t) res->resultlist[t].nresults;
        bool     head = true;  // the newest buffer holds writepos pairs, the older ones are full
        // the reference's order exactly: newest buffer first, each read from its last pair to its
        // first (cb_begin_backwards / cb_read_backwards, src/tuple_buffer.h:58-90, :221-226)
        for (const Buf* b = cb->buf; b && left && rc == 0; b = b->next, head = false) {
            const uint64_t n = std::min<uint64_t>(left, head ? cb->writepos : kPer);
            rc = write_pairs(fp, b->tuples, n, true);
            left -= n;
        }
    }
    if (fclose(fp) != 0) rc = 1;
    if (rc) set_last_error(std::string("write failed: ") + filename);
    return rc;
}

}  // extern "C"
