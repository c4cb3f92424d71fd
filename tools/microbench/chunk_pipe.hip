// chunk_pipe.hip -- 128-byte chunk gathers through a list, software-pipelined as k_probe does them
// (list entries two steps ahead, chunks one step ahead), by locality of the list: consecutive list
// entries contiguous in runs of E chunks ("extents"), extents in random order. E = 1 is the
// probe's pattern today; E = all is a partition-contiguous layout. Dev tool:
//   hipcc -O3 --offload-arch=gfx950 chunk_pipe.hip -o chunk_pipe && ./chunk_pipe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
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

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// 8 lanes per chunk (16 B each); U chunk slots per thread-octet per step
template <int U, bool NT>
__global__ __launch_bounds__(1024) void k_read_pipe(const v4u* __restrict__ pool, const uint32_t* __restrict__ list,
                                                    uint32_t n, uint32_t* sink) {
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t b = blockIdx.x * per, e = min(n, b + per);
    if (b >= e) return;
    const uint32_t cs = threadIdx.x >> 3, l8 = threadIdx.x & 7;
    const uint32_t nst = (e - b + 128 * U - 1) / (128 * U);
    auto pos = [&](uint32_t s, int u) { return b + s * 128u * U + (uint32_t) u * 128u + cs; };
    uint32_t L0[U], L1[U];
    v4u      C[U];
#pragma unroll
    for (int u = 0; u < U; u++) L0[u] = list[min(pos(0, u), e - 1)];
#pragma unroll
    for (int u = 0; u < U; u++) L1[u] = list[min(pos(1, u), e - 1)];
#pragma unroll
    for (int u = 0; u < U; u++) C[u] = ld<NT>(pool + (uint64_t) L0[u] * 8 + l8);
    uint32_t acc = 0;
    for (uint32_t s = 0; s < nst; s++) {
        v4u Cn[U];
#pragma unroll
        for (int u = 0; u < U; u++) Cn[u] = ld<NT>(pool + (uint64_t) L1[u] * 8 + l8);
#pragma unroll
        for (int u = 0; u < U; u++) L0[u] = list[min(pos(s + 2, u), e - 1)];
#pragma unroll
        for (int u = 0; u < U; u++)
            if (pos(s, u) < e) acc ^= C[u].x ^ C[u].y ^ C[u].z ^ C[u].w;
#pragma unroll
        for (int u = 0; u < U; u++) {
            C[u]  = Cn[u];
            L1[u] = L0[u];
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint32_t n = 32u << 20;  // chunks: 4 GiB
    v4u*      pool;
    uint32_t *list, *sink;
    CK(hipMalloc(&pool, (size_t) n * 128));
    CK(hipMalloc(&list, (size_t) n * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(pool, 1, (size_t) n * 128));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    std::vector<uint32_t> h(n);
    std::mt19937_64       rng(7);
    printf("pipelined gathers: pool 4 GiB of 128-B chunks, %d workgroups x 1024 threads (GB/s incl. 4-B list reads)\n", cus);
    printf("%9s %10s %10s %10s %10s\n", "extent", "U=3 def", "U=3 nt", "U=6 def", "U=6 nt");
    for (uint32_t E : {1u, 4u, 16u, 122u, 1u << 25}) {
        const uint32_t        ne = n / E;
        std::vector<uint32_t> perm(ne);
        for (uint32_t i = 0; i < ne; i++) perm[i] = i;
        if (E < n) std::shuffle(perm.begin(), perm.end(), rng);
        for (uint32_t i = 0; i < n; i++) h[i] = perm[i / E] * E + i % E;
        CK(hipMemcpy(list, h.data(), (size_t) n * 4, hipMemcpyHostToDevice));
        float best[4] = {1e9f, 1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 4; rep++) {
            for (int v = 0; v < 4; v++) {
                float ms;
                CK(hipEventRecord(a));
                if (v == 0) k_read_pipe<3, false><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 1) k_read_pipe<3, true><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 2) k_read_pipe<6, false><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 3) k_read_pipe<6, true><<<cus, 1024>>>(pool, list, n, sink);
                CK(hipEventRecord(z));
                CK(hipEventSynchronize(z));
                CK(hipEventElapsedTime(&ms, a, z));
                best[v] = std::min(best[v], ms);
            }
        }
        const double bytes = (double) n * 132;
        printf("%9u %10.0f %10.0f %10.0f %10.0f\n", E, bytes / best[0] / 1e6, bytes / best[1] / 1e6,
               bytes / best[2] / 1e6, bytes / best[3] / 1e6);
        fflush(stdout);
    }
    return 0;
}
