// mchashjoins.cpp -- CLI driver with the reference's flags and stdout (src/main.c:351-731),
// running the join through libhwbrj.so's BPRO / PRO on an MI355X.
//
// Differences from the reference driver (DESIGN.md "CLI"):
//   -b sectorized    selects this build's SECTORIZED filter (the reference silently runs BASIC);
//   -a               PRO, PRH, PRHO and RJ all run the MI355X partitioned join (their CPU join
//                    functions differ, their counts do not); NPO / NPO_st print an error;
//   --gpus=G         S range-sharded into G shards over the visible devices (R replicated);
//   -z / --non-unique / --full-range relations are the reference's exactly (restated glibc
//   rand() after srand(-x / -y), hwbrj_gen.cpp); the default PK/FK relations have the reference's
//   key multiset in a seeded (-x / -y) Feistel order instead of the time-seeded Knuth shuffle
//   (src/generator.c:173-176).
#include <getopt.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <climits>
#include <cmath>
#include <string>
#include <thread>

#include "hwbrj.h"

struct Params {
    std::string algo        = "PRO";
    uint32_t    nthreads    = 2;
    uint64_t    r_size      = 128000000;
    uint64_t    s_size      = 128000000;
    uint32_t    r_seed      = 12345;
    uint32_t    s_seed      = 54321;
    double      skew        = 0.0;
    double      selectivity = 1.0;
    const char* loadR       = nullptr;
    const char* loadS       = nullptr;
    bool        bloom       = false;
    bloom_filter_args_t bf  = {BASIC, 256ull << 20, 8, 1024};  // src/main.c:389-393
    int         gpus        = 1;
};

static void print_help(const char* prog) {
    printf("Usage: %s [options]\n", prog);
    printf(
        "    Join algorithm selection, algorithms : PRO, PRH, PRHO, RJ (MI355X)          \n"
        "       -a --algo=<name>    Run the hash join algorithm named <name> [PRO]      \n"
        "                                                                               \n"
        "    Other join configuration options, with default values in [] :              \n"
        "       -n --nthreads=<N>  Number of threads to use <N> [2]                     \n"
        "       -r --r-size=<R>    Number of tuples in build relation R <R> [128000000] \n"
        "       -s --s-size=<S>    Number of tuples in probe relation S <S> [128000000] \n"
        "       -x --r-seed=<x>    Seed value for generating relation R <x> [12345]     \n"
        "       -y --s-seed=<y>    Seed value for generating relation S <y> [54321]     \n"
        "       -q --s-sel=<q>     Selectivity for %% of S-tuples with a match in R [1.0]\n"
        "       -z --skew=<z>      Zipf skew parameter for probe relation S <z> [0.0]   \n"
        "       --non-unique       Use non-unique (duplicated) keys in input relations  \n"
        "       --full-range       Spread keys in relns. in full 32-bit integer range   \n"
        "       --persist          Write R.tbl / S.tbl (and Out.tbl when materializing) \n"
        "                          as a -DPERSIST_RELATIONS reference build does        \n"
        "       -R --r-file=<Rf>   The file to load build relation R from <Rf> [R.tbl]  \n"
        "       -S --s-file=<Sf>   The file to load probe relation S from <Sf> [S.tbl]  \n"
        "                                                                               \n"
        "    Bloom Filter options:                                                      \n"
        "       -b --bloom-filter=<b>     no, basic, blocked, sectorized (this build)   \n"
        "       -k --bloom-hashes=<k>     number of bits set per tuple                  \n"
        "       -m --bloom-size=<m>       number of filter entries in bits              \n"
        "       -B --bloom-block-size=<B> number of bits per block (B = 2^x)            \n"
        "       --gpus=<G>                S shards over the MI355X devices [1]          \n"
        "        -h --help         Show this message                                    \n"
        "        --version         Show version                                         \n");
}

// src/generator.c:685-741 (read_relation): the first line is a header and is skipped; data lines
// are "key payload", "key,payload" or a bare key (payload 0). Reads at most n tuples; a shorter
// file gives a shorter relation (the reference would repeat its last tuple).
static int load_relation(relation_t* rel, const char* path, uint64_t n) {
    FILE* fp = fopen(path, "r");
    if (!fp) {
        perror(path);
        return -1;
    }
    rel->tuples     = (tuple_t*) malloc(sizeof(tuple_t) * (n ? n : 1));
    rel->num_tuples = n;
    char     line[256];
    uint64_t i = 0;
    if (!fgets(line, sizeof line, fp)) line[0] = 0;  // header
    bool warn = true;
    while (i < n && fgets(line, sizeof line, fp)) {
        for (char* c = line; *c; c++)
            if (*c == ',' || *c == '|') *c = ' ';
        long long k = 0, p = 0;
        const int got = sscanf(line, "%lld %lld", &k, &p);
        if (got < 1) continue;
        if (got == 1) p = 0;
        if (warn && k < 0) {  // :732-735
            warn = false;
            printf("[WARN ] key=%d, payload=%d\n", (int32_t) k, (int32_t) p);
        }
        rel->tuples[i].key     = (int32_t) k;
        rel->tuples[i].payload = (int32_t) p;
        i++;
    }
    fclose(fp);
    rel->num_tuples = i;
    return 0;
}

int main(int argc, char** argv) {
    Params         P;
    static int     nonunique = 0, fullrange = 0, basic_numa = 0, verbose = 0, persist = 0;
    static option  opts[] = {{"verbose", no_argument, &verbose, 1},
                            {"brief", no_argument, &verbose, 0},
                            {"non-unique", no_argument, &nonunique, 1},
                            {"full-range", no_argument, &fullrange, 1},
                            {"persist", no_argument, &persist, 1},
                            {"basic-numa", no_argument, &basic_numa, 1},
                            {"help", no_argument, 0, 'h'},
                            {"version", no_argument, 0, 'v'},
                            {"algo", required_argument, 0, 'a'},
                            {"nthreads", required_argument, 0, 'n'},
                            {"perfconf", required_argument, 0, 'p'},
                            {"r-size", required_argument, 0, 'r'},
                            {"s-size", required_argument, 0, 's'},
                            {"perfout", required_argument, 0, 'o'},
                            {"r-seed", required_argument, 0, 'x'},
                            {"s-seed", required_argument, 0, 'y'},
                            {"s-sel", required_argument, 0, 'q'},
                            {"skew", required_argument, 0, 'z'},
                            {"r-file", required_argument, 0, 'R'},
                            {"s-file", required_argument, 0, 'S'},
                            {"bloom-filter", required_argument, 0, 'b'},
                            {"bloom-size", required_argument, 0, 'm'},
                            {"bloom-hashes", required_argument, 0, 'k'},
                            {"bloom-block-size", required_argument, 0, 'B'},
                            {"gpus", required_argument, 0, 'G'},
                            {0, 0, 0, 0}};
    int c, idx = 0;
    while ((c = getopt_long(argc, argv, "a:n:p:q:r:s:o:x:y:z:R:S:b:m:k:B:Z:A:hv", opts, &idx)) != -1) {
        switch (c) {
            case 0: break;
            case 'a':  // src/main.c:331-339 (NPO / NPO_st do not partition: not in this build)
                if (strcmp(optarg, "PRO") != 0 && strcmp(optarg, "PRH") != 0 &&
                    strcmp(optarg, "PRHO") != 0 && strcmp(optarg, "RJ") != 0) {
                    printf("[ERROR] Join algorithm named `%s' does not exist in this build!\n",
                           optarg);
                    print_help(argv[0]);
                    exit(EXIT_SUCCESS);
                }
                P.algo = optarg;
                break;
            case 'h':
            case '?': print_help(argv[0]); exit(EXIT_SUCCESS);
            case 'v': printf("\n%s\n\n", hwbrj_version()); exit(EXIT_SUCCESS);
            case 'n': P.nthreads = (uint32_t) atoi(optarg); break;
            case 'q': P.selectivity = atof(optarg); break;
            case 'r': P.r_size = (uint64_t) atol(optarg); break;
            case 's': P.s_size = (uint64_t) atol(optarg); break;
            case 'x': P.r_seed = (uint32_t) atoi(optarg); break;
            case 'y': P.s_seed = (uint32_t) atoi(optarg); break;
            case 'z': P.skew = atof(optarg); break;
            case 'R': P.loadR = optarg; break;
            case 'S': P.loadS = optarg; break;
            case 'b':  // src/main.c:692-698 (+ sectorized)
                P.bloom = strcmp(optarg, "no") != 0;
                if (strcmp(optarg, "basic") == 0) P.bf.variant = BASIC;
                else if (strcmp(optarg, "blocked") == 0) P.bf.variant = BLOCKED;
                else if (strcmp(optarg, "sectorized") == 0) P.bf.variant = SECTORIZED;
                break;
            case 'm': P.bf.m = (uint64_t) atoll(optarg); break;
            case 'k': P.bf.k = (uint64_t) atoi(optarg); break;
            case 'B': P.bf.B = (uint64_t) atoi(optarg); break;
            case 'G': P.gpus = atoi(optarg); break;
            default: break;
        }
    }
    if (P.bloom) assert_args(&P.bf);  // src/main.c:730
    // --gpus=G: S range-sharded over G shards (shard g on device g mod #devices), R replicated
    if (hwbrj_set_gpus(P.gpus) != 0) {
        printf("[ERROR] --gpus=%d: %s\n", P.gpus, hwbrj_last_error());
        exit(EXIT_FAILURE);
    }
    if (P.nthreads == 0) P.nthreads = 1;
    const int hthreads = (int) std::thread::hardware_concurrency();

    // Relation creation in the order of src/main.c:402-468 (each relation seeded by -x / -y).
    relation_t relR, relS;
    auto alloc = [](relation_t* rel, uint64_t n) {
        rel->num_tuples = n;
        rel->tuples     = (tuple_t*) malloc(sizeof(tuple_t) * (n ? n : 1));
        if (!rel->tuples) {
            perror("out of memory");
            exit(EXIT_FAILURE);
        }
    };
    auto check = [](int rc, const char* what) {
        if (rc) {
            printf("[ERROR] generating %s: %s\n", what, hwbrj_last_error());
            exit(EXIT_FAILURE);
        }
    };
    fprintf(stdout, "[INFO ] %s relation R with size = %.3lf MiB, #tuples = %llu : ",
            P.loadR ? "Loading" : "Creating", 8.0 * P.r_size / 1024.0 / 1024.0,
            (unsigned long long) P.r_size);
    fflush(stdout);
    uint64_t threshold = 0;
    if (P.loadR) {
        if (load_relation(&relR, P.loadR, P.r_size)) exit(EXIT_FAILURE);
    } else if (fullrange || nonunique) {  // :421-427
        threshold = hwbrj_nonunique_threshold(P.r_size, P.selectivity, fullrange);
        alloc(&relR, P.r_size);
        check(hwbrj_create_relation_nonunique(relR.tuples, P.r_size, (int64_t) threshold, P.r_seed), "R");
    } else {
        alloc(&relR, P.r_size);
        check(hwbrj_generate_host(relR.tuples, P.r_size, P.nthreads, P.r_size, P.r_size, 1.0,
                                  P.r_seed, hthreads), "R");
    }
    printf("OK \n");
    // src/generator.c:408-412 (PERSIST_RELATIONS): every generated relation, R then S
    auto persist_rel = [&](const relation_t* rel, const char* name) {
        if (persist && hwbrj_write_relation(rel, name) != 0) {
            printf("[ERROR] %s\n", hwbrj_last_error());
            exit(EXIT_FAILURE);
        }
    };
    if (!P.loadR) persist_rel(&relR, "R.tbl");
    fprintf(stdout, "[INFO ] %s relation S with size = %.3lf MiB, #tuples = %lld : ",
            P.loadS ? "Loading" : "Creating", 8.0 * P.s_size / 1024.0 / 1024.0,
            (long long) P.s_size);
    fflush(stdout);
    if (P.loadS) {
        if (load_relation(&relS, P.loadS, P.s_size)) exit(EXIT_FAILURE);
    } else if (fullrange) {  // :448-450
        alloc(&relS, P.s_size);
        check(hwbrj_create_relation_fk_from_pk(relS.tuples, P.s_size, relR.tuples, relR.num_tuples,
                                               (int64_t) threshold, P.selectivity, P.s_seed), "S");
    } else if (nonunique) {  // :451-453
        alloc(&relS, P.s_size);
        check(hwbrj_create_relation_nonunique_from_pk(relS.tuples, P.s_size, relR.tuples,
                                                      relR.num_tuples, (int64_t) threshold,
                                                      P.selectivity, P.s_seed), "S");
    } else if (P.skew > 0) {  // :457-460 (-q is ignored, as in the reference)
        alloc(&relS, P.s_size);
        check(hwbrj_create_relation_zipf(relS.tuples, P.s_size, P.r_size, P.skew, P.s_seed, hthreads), "S");
    } else {
        alloc(&relS, P.s_size);
        check(hwbrj_generate_host(relS.tuples, P.s_size, P.nthreads, INT_MAX, P.r_size, P.selectivity,
                                  P.s_seed, hthreads), "S");
    }
    printf("OK \n");
    if (!P.loadS) persist_rel(&relS, "S.tbl");
    printf("[INFO ] Running join algorithm %s ...\n", P.algo.c_str());
    // src/main.c:331-339 algos[] and :473-478 (joinAlgoBloom when -b is not "no")
    struct Algo {
        const char* name;
        result_t* (*join)(relation_t*, relation_t*, int);
        result_t* (*bloom)(relation_t*, relation_t*, int, bloom_filter_args_t*);
    };
    static const Algo algos[] = {{"PRO", PRO, BPRO}, {"PRH", PRH, BPRH}, {"PRHO", PRHO, BPRHO}, {"RJ", RJ, BRJ}};
    const Algo* algo = &algos[0];
    for (const Algo& a : algos)
        if (P.algo == a.name) algo = &a;
    result_t* res = P.bloom ? algo->bloom(&relR, &relS, (int) P.nthreads, &P.bf)
                            : algo->join(&relR, &relS, (int) P.nthreads);
    printf("[INFO ] Results = %llu. DONE.\n", (unsigned long long) res->totalresults);
    if (persist && res->resultlist) {  // src/main.c:482-485 (PERSIST_RELATIONS + JOIN_RESULT_MATERIALIZE)
        printf("[INFO ] Persisting the join result to \"Out.tbl\" ...\n");
        if (hwbrj_write_result_relation(res, "Out.tbl") != 0) {
            printf("[ERROR] %s\n", hwbrj_last_error());
            exit(EXIT_FAILURE);
        }
    }
    free(relR.tuples);
    free(relS.tuples);
    free(res);
    return 0;
}
