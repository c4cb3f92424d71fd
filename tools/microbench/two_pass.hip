// two_pass.hip -- model of a two-pass S partition: a histogram
// pass over S, then a scatter to precomputed offsets with no LDS stage (so no 128 KiB stage caps
// the kernel at one workgroup per CU). Dev tool: the access shapes of the real pass, with the
// product's per-key work (8 LDS nibble-table reads for the partition code, one LDS atomic rank).
//   hipcc -O3 --offload-arch=gfx950 two_pass.hip -o two_pass && ./two_pass
// S = 1.024e9 tuples (8.19 GB), F = 1024 partitions, 4-byte words out (4.1 GB), like k_scatter_s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr uint32_t kF = 1024;

// the partition code of a key from 8 x 16 nibble tables in LDS (the product's crc_nib shape)
__device__ __forceinline__ uint32_t code_of(const uint32_t* tab, uint32_t k) {
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) c ^= tab[j * 16 + ((k >> (4 * j)) & 15u)];
    return c;
}

__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load((const v4u*) p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// pass 1: per-workgroup histogram of the partition codes over its contiguous range of S
template <int U>
__global__ __launch_bounds__(1024) void k_hist(const uint4* __restrict__ S, uint64_t n2, const uint32_t* __restrict__ gtab,
                                               uint32_t* __restrict__ hist) {
    __shared__ uint32_t tab[128], h[kF];
    for (uint32_t i = threadIdx.x; i < 128; i += blockDim.x) tab[i] = gtab[i];
    for (uint32_t i = threadIdx.x; i < kF; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t per = (n2 + gridDim.x - 1) / gridDim.x, b = blockIdx.x * per, e = min(n2, b + per);
    for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t) blockDim.x * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * blockDim.x;
            v[u] = k < e ? ld_nt(S + k) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i + (uint64_t) u * blockDim.x >= e) continue;
            atomicAdd(&h[code_of(tab, v[u].x) & (kF - 1)], 1u);
            atomicAdd(&h[code_of(tab, v[u].z) & (kF - 1)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kF; i += blockDim.x) hist[(uint64_t) blockIdx.x * kF + i] = h[i];
}

// exclusive offsets, partition-major: off[wg][q] = sum of hist[*][q' < q] + sum of hist[wg' < wg][q]
__global__ void k_scan(const uint32_t* __restrict__ hist, uint32_t G, uint64_t* __restrict__ off) {
    __shared__ uint64_t col[kF];
    const uint32_t q = threadIdx.x;  // one thread per partition (kF threads)
    uint64_t s = 0;
    for (uint32_t w = 0; w < G; w++) s += hist[(uint64_t) w * kF + q];
    col[q] = s;
    __syncthreads();
    if (q == 0) {
        uint64_t a = 0;
        for (uint32_t i = 0; i < kF; i++) { const uint64_t t = col[i]; col[i] = a; a += t; }
    }
    __syncthreads();
    uint64_t a = col[q];
    for (uint32_t w = 0; w < G; w++) {
        off[(uint64_t) w * kF + q] = a;
        a += hist[(uint64_t) w * kF + q];
    }
}

// pass 2: every word to its precomputed position (LDS cursor per partition), 4-byte stores
template <int U, bool NT>
__global__ __launch_bounds__(1024) void k_place(const uint4* __restrict__ S, uint64_t n2, const uint32_t* __restrict__ gtab,
                                                const uint64_t* __restrict__ off, uint32_t* __restrict__ out) {
    __shared__ uint32_t tab[128];
    __shared__ uint64_t cur[kF];
    for (uint32_t i = threadIdx.x; i < 128; i += blockDim.x) tab[i] = gtab[i];
    for (uint32_t i = threadIdx.x; i < kF; i += blockDim.x) cur[i] = off[(uint64_t) blockIdx.x * kF + i];
    __syncthreads();
    const uint64_t per = (n2 + gridDim.x - 1) / gridDim.x, b = blockIdx.x * per, e = min(n2, b + per);
    for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t) blockDim.x * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * blockDim.x;
            v[u] = k < e ? ld_nt(S + k) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (i + (uint64_t) u * blockDim.x >= e) continue;
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const uint32_t key = t ? v[u].z : v[u].x;
                const uint32_t c   = code_of(tab, key);
                const uint64_t p   = atomicAdd((unsigned long long*) &cur[c & (kF - 1)], 1ull);
                const uint32_t w   = (c >> 10) | (key << 22);
                if (NT) __builtin_nontemporal_store(w, out + p);
                else out[p] = w;
            }
        }
    }
}

template <class K>
static float timeit(K launch, int reps = 5) {
    hipEvent_t a, b;
    (void) hipEventCreate(&a);
    (void) hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 1; r++) {
        (void) hipEventRecord(a);
        launch();
        (void) hipEventRecord(b);
        (void) hipEventSynchronize(b);
        float ms;
        (void) hipEventElapsedTime(&ms, a, b);
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

__global__ void k_fill(uint2* S, uint64_t n) {  // pseudo-random keys (a multiplicative hash of the row)
    const uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    if (i < n) S[i] = make_uint2((uint32_t) (i * 0x9E3779B97F4A7C15ull >> 29), (uint32_t) i);
}

int main() {
    const uint64_t n = 1024000000ull, n2 = n / 2;
    uint2*    S;
    uint32_t *out, *hist, *gtab;
    uint64_t* off;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&S, n * 8));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&gtab, 128 * 4));
    std::vector<uint32_t> t(128);
    for (int i = 0; i < 128; i++) t[i] = (uint32_t) (0x9E3779B1u * (uint32_t) (i + 1)) ^ ((uint32_t) i << 7);
    CK(hipMemcpy(gtab, t.data(), 512, hipMemcpyHostToDevice));
    k_fill<<<(n + 255) / 256, 256>>>(S, n);
    CK(hipDeviceSynchronize());
    printf("two-pass S partition model: |S| = %llu (%.2f GB), F = %u, %d CUs\n", (unsigned long long) n, n * 8e-9, kF, cus);
    for (int wpc : {1, 2, 4}) {
        const uint32_t G = (uint32_t) cus * wpc;
        CK(hipMalloc(&hist, (size_t) G * kF * 4));
        CK(hipMalloc(&off, (size_t) G * kF * 8));
        const float th = timeit([&] { k_hist<4><<<G, 1024>>>((const uint4*) S, n2, gtab, hist); });
        const float ts = timeit([&] { k_scan<<<1, kF>>>(hist, G, off); });
        const float tp = timeit([&] { k_place<4, false><<<G, 1024>>>((const uint4*) S, n2, gtab, off, out); });
        const float tn = timeit([&] { k_place<4, true><<<G, 1024>>>((const uint4*) S, n2, gtab, off, out); });
        printf("G = %5u (%d per CU): hist %.3f ms (%.0f GB/s) | scan %.3f ms | place %.3f ms (%.0f GB/s), nt stores %.3f ms "
               "| two-pass total %.3f ms\n",
               G, wpc, th, n * 8 / (th * 1e6), ts, tp, n * 12 / (tp * 1e6), tn, th + ts + std::min(tp, tn));
        CK(hipFree(hist));
        CK(hipFree(off));
    }
    printf("(k_scatter_s, the one-pass LDS-staged kernel, takes 2.37-2.45 ms on these boxes: DESIGN.md s7)\n");
    return 0;
}
