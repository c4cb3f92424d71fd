// chunk_bw.hip -- HBM rate of 128-byte chunk reads and writes by locality, the access shape of the
// probe (reads chunks through a list) and of the scatter (writes chunks). A list visits every
// chunk of a 4 GiB pool once; consecutive list entries are contiguous in runs of E chunks (an
// "extent"), extents in random order. E = 1 is the probe's pattern today (chunks of one partition
// scattered over the scatter regions); larger E is what per-partition extents in the scatter
// regions would give. Dev tool:
//   hipcc -O3 --offload-arch=gfx950 chunk_bw.hip -o chunk_bw && ./chunk_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// U: list positions per thread per step (8 threads per chunk, 16 B each), i.e. loads in flight
// 8 lanes per chunk: a wave touches 8 consecutive list entries per load instruction
template <int U>
__global__ __launch_bounds__(1024) void k_read(const uint4* __restrict__ pool, const uint32_t* __restrict__ list,
                                               uint32_t n, uint32_t* sink) {
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t b = blockIdx.x * per, e = min(n, b + per);
    const uint32_t cs = threadIdx.x >> 3, l8 = threadIdx.x & 7;
    uint32_t acc = 0;
    for (uint32_t i = b + cs; i < e; i += 128 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t k = i + u * 128;
            v[u] = k < e ? pool[(uint64_t) list[k] * 8 + l8] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int U>
__global__ __launch_bounds__(1024) void k_write(uint4* __restrict__ pool, const uint32_t* __restrict__ list,
                                                uint32_t n) {
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t b = blockIdx.x * per, e = min(n, b + per);
    const uint32_t cs = threadIdx.x >> 3, l8 = threadIdx.x & 7;
    for (uint32_t i = b + cs; i < e; i += 128 * U) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t k = i + u * 128;
            if (k < e) pool[(uint64_t) list[k] * 8 + l8] = make_uint4(k, l8, k ^ l8, 7);
        }
    }
}

int main() {
    const uint32_t n = 32u << 20;  // chunks: 4 GiB
    uint4*    pool;
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
    printf("pool 4 GiB of 128-B chunks, %d workgroups x 1024 threads; U = 16-B loads in flight per thread\n", cus);
    printf("%8s %12s %12s %12s %12s\n", "extent", "read U=4", "read U=8", "read U=12", "write U=4");
    for (uint32_t E : {1u, 2u, 8u, 64u, 1u << 25}) {
        const uint32_t       ne = n / E;
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
                if (v == 0) k_read<4><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 1) k_read<8><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 2) k_read<12><<<cus, 1024>>>(pool, list, n, sink);
                if (v == 3) k_write<4><<<cus, 1024>>>(pool, list, n);
                CK(hipEventRecord(z));
                CK(hipEventSynchronize(z));
                CK(hipEventElapsedTime(&ms, a, z));
                best[v] = std::min(best[v], ms);
            }
        }
        // list reads (4 B per chunk) are counted too: they are part of the probe's traffic
        const double bytes = (double) n * 132;
        printf("%8u %12.0f %12.0f %12.0f %12.0f\n", E, bytes / best[0] / 1e6, bytes / best[1] / 1e6,
               bytes / best[2] / 1e6, bytes / best[3] / 1e6);
    }
    return 0;
}
