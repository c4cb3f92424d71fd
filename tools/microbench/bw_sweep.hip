// bw_sweep.hip -- which streaming shapes reach the MI355X's ~6.3 TB/s (dev tool).
// Copy (1:1), the S scatter's read:write = 2:1 shape, and read-only, over:
//   layout   C: every workgroup its own contiguous range (the scatter's shape)
//            I: grid-stride interleaved (consecutive workgroups read consecutive blocks)
//   grid x threads, U 16-byte loads in flight per thread, cache policy (default / nt)
//   hipcc -O3 --offload-arch=gfx950 bw_sweep.hip -o bw_sweep && ./bw_sweep
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("err %s line %d\n", hipGetErrorString(e_), __LINE__);                       \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void st(T* p, T v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// KIND 0: copy 16 B -> 16 B; 1: read 16 B, write 8 B (2:1); 2: read only
template <int KIND, int U, bool NT, bool INTERLEAVE>
__global__ void k_bw(const v4u* __restrict__ in, void* __restrict__ out, uint64_t n, uint32_t* sink) {
    const uint64_t T = blockDim.x;
    uint64_t b, e, step, first;
    if (INTERLEAVE) {
        b = 0, e = n, step = T * U * gridDim.x, first = (uint64_t) blockIdx.x * T * U + threadIdx.x;
    } else {
        const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
        b = (uint64_t) blockIdx.x * per, e = min(n, b + per), step = T * U, first = b + threadIdx.x;
    }
    (void) b;
    uint32_t acc = 0;
    for (uint64_t i = first; i < e; i += step) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * T;
            v[u] = k < e ? ld<NT>(in + k) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * T;
            if (k >= e) continue;
            if (KIND == 0) st<NT>((v4u*) out + k, v[u]);
            else if (KIND == 1) st<NT>((v2u*) out + k, v2u{v[u].x ^ 0x9e3779b9u, v[u].z});
            else acc ^= v[u].x ^ v[u].z;
        }
    }
    if (KIND == 2 && acc == 0x12345678u) sink[0] = acc;
}

// rw21 software-pipelined: the next step's U loads are issued before this step's stores (the
// scatter's shape: loads one round ahead), each workgroup its own contiguous range
template <int U, bool NT>
__global__ void k_rw_pipe(const v4u* __restrict__ in, v2u* __restrict__ out, uint64_t n) {
    const uint64_t T = blockDim.x, per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t) blockIdx.x * per, e = min(n, b + per);
    v4u cur[U], nxt[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const uint64_t k = b + threadIdx.x + (uint64_t) u * T;
        cur[u] = k < e ? ld<NT>(in + k) : v4u{0, 0, 0, 0};
    }
    for (uint64_t i = b + threadIdx.x; i < e; i += T * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + T * U + (uint64_t) u * T;
            nxt[u] = k < e ? ld<NT>(in + k) : v4u{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * T;
            if (k < e) st<NT>(out + k, v2u{cur[u].x ^ 0x9e3779b9u, cur[u].z});
        }
#pragma unroll
        for (int u = 0; u < U; u++) cur[u] = nxt[u];
    }
}

template <int U, bool NT>
static void run_pipe(const v4u* in, void* out, uint64_t n, int grid, int thr);

template <class L>
static float timeit(L launch, int reps = 5) {
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 1; r++) {
        (void) hipEventRecord(a);
        launch();
        (void) hipEventRecord(b);
        (void) hipEventSynchronize(b);
        float ms = 0;
        (void) hipEventElapsedTime(&ms, a, b);
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

template <int KIND, int U, bool NT, bool IL>
static void run(const v4u* in, void* out, uint64_t n, uint32_t* sink, int grid, int thr) {
    const float ms = timeit([&] { k_bw<KIND, U, NT, IL><<<grid, thr>>>(in, out, n, sink); });
    const double rd = n * 16.0, wr = KIND == 0 ? n * 16.0 : KIND == 1 ? n * 8.0 : 0.0;
    printf("%-4s %c U=%d %-3s grid=%5d x %4d  %7.3f ms  %7.1f GB/s\n", KIND == 0 ? "copy" : KIND == 1 ? "rw21" : "read",
           IL ? 'I' : 'C', U, NT ? "nt" : "def", grid, thr, ms, (rd + wr) / ms / 1e6);
    fflush(stdout);
}

template <int U, bool NT>
static void run_pipe(const v4u* in, void* out, uint64_t n, int grid, int thr) {
    const float ms = timeit([&] { k_rw_pipe<U, NT><<<grid, thr>>>(in, (v2u*) out, n); });
    printf("rw21 P U=%d %-3s grid=%5d x %4d  %7.3f ms  %7.1f GB/s (pipelined: next loads before stores)\n", U,
           NT ? "nt" : "def", grid, thr, ms, (n * 24.0) / ms / 1e6);
    fflush(stdout);
}

template <int KIND>
static void sweep(const v4u* in, void* out, uint64_t n, uint32_t* sink) {
    const int cfg[][2] = {{256, 1024}, {512, 1024}, {1024, 256}, {2048, 256}, {4096, 256}, {8192, 256}};
    for (auto& c : cfg) {
        run<KIND, 4, false, false>(in, out, n, sink, c[0], c[1]);
        run<KIND, 4, true, false>(in, out, n, sink, c[0], c[1]);
        run<KIND, 4, false, true>(in, out, n, sink, c[0], c[1]);
        run<KIND, 4, true, true>(in, out, n, sink, c[0], c[1]);
    }
    run<KIND, 1, false, true>(in, out, n, sink, 8192, 256);
    run<KIND, 2, false, true>(in, out, n, sink, 8192, 256);
    run<KIND, 8, false, true>(in, out, n, sink, 4096, 256);
    run<KIND, 8, false, false>(in, out, n, sink, 256, 1024);
    run<KIND, 1, false, true>(in, out, n, sink, 16384, 256);
    run<KIND, 1, true, true>(in, out, n, sink, 16384, 256);
}

int main(int argc, char** argv) {
    (void) argv;
    const uint64_t bytes = 4ull << 30, n = bytes / 16;
    v4u*      in;
    void*     out;
    uint32_t* sink;
    CK(hipMalloc(&in, bytes));
    CK(hipMalloc(&out, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 1, bytes));
    CK(hipMemset(out, 2, bytes));
    if (argc > 1) {  // pipelined rw21 only
        for (int r = 0; r < 2; r++) {
            run<1, 4, true, false>(in, out, n, sink, 256, 1024);
            run<1, 4, true, false>(in, out, n, sink, 512, 1024);
            run_pipe<2, true>(in, out, n, 256, 1024);
            run_pipe<4, true>(in, out, n, 256, 1024);
            run_pipe<4, false>(in, out, n, 256, 1024);
            run_pipe<8, true>(in, out, n, 256, 1024);
            run_pipe<4, true>(in, out, n, 512, 1024);
            run_pipe<2, true>(in, out, n, 256, 512);
        }
        printf("done\n");
        return 0;
    }
    sweep<0>(in, out, n, sink);
    sweep<1>(in, out, n, sink);
    sweep<2>(in, out, n, sink);
    printf("done\n");
    return 0;
}
