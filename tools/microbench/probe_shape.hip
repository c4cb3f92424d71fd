// probe_shape.hip -- what k_probe's shape costs beyond its chunk gathers.
// The gather loop of chunk_pipe.hip (128-byte chunks through a random list, list entries two
// steps ahead, chunks one step ahead, 1024 threads per workgroup, one workgroup per CU, U chunk
// quads per thread per step), with k_probe's other parts added one at a time:
//   BAR   one workgroup barrier per step (k_probe's B1)
//   TEST  every word tests one bit of a 128 KiB LDS array at a random position (the slice test)
//   W     the step's survivors (a fraction of its words, 12 % like the north star) written as
//         16-byte stores: W=1 into the step's own region (k_probe: the item region of its input
//         chunks, i.e. sparse), W=2 appended to a per-workgroup dense stream
// Dev tool:  hipcc -O3 --offload-arch=gfx950 probe_shape.hip -o probe_shape && ./probe_shape
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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short) 0, (int) bytes, 0x00020000);
}

// W = 3: W = 2 into a ring of `ring` bytes shared by all workgroups (what the Infinity Cache
// absorbs when written data is overwritten soon); AUX: the stores' cache policy; BATCH: steps whose
// survivors are written together
template <int U, bool BAR, bool TEST, int W, int AUX = 0, int BATCH = 1>
__global__ __launch_bounds__(1024) void k_shape(v4u* pool, uint32_t* list,
                                                uint32_t n, uint32_t* __restrict__ out, uint32_t wfrac_q,
                                                uint32_t* sink) {
    extern __shared__ uint32_t lds[];  // 32768 words
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t b = blockIdx.x * per, e = min(n, b + per);
    if (b >= e) return;
    const uint32_t tid = threadIdx.x, cs = tid >> 3, l8 = tid & 7;
    if (TEST)
        for (uint32_t i = tid; i < 32768; i += 1024) lds[i] = (i * 2654435761u) & 0x10204081u;  // ~12 % bits
    __syncthreads();
    const uint32_t nst = (e - b + 128 * U - 1) / (128 * U);
    auto pos = [&](uint32_t s, int u) { return b + s * 128u * U + (uint32_t) u * 128u + cs; };
    uint32_t L0[U], L1[U];
    v4u      C[U];
#pragma unroll
    for (int u = 0; u < U; u++) L0[u] = list[min(pos(0, u), e - 1)];
#pragma unroll
    for (int u = 0; u < U; u++) L1[u] = list[min(pos(1, u), e - 1)];
#pragma unroll
    for (int u = 0; u < U; u++) C[u] = pool[(uint64_t) L0[u] * 8 + l8];
    uint32_t acc = 0;
    uint64_t dense = (uint64_t) b * 32;  // W = 2: this workgroup's stream (inside its own range)
    for (uint32_t s = 0; s < nst; s++) {
        v4u Cn[U];
#pragma unroll
        for (int u = 0; u < U; u++) Cn[u] = pool[(uint64_t) L1[u] * 8 + l8];
#pragma unroll
        for (int u = 0; u < U; u++) L0[u] = list[min(pos(s + 2, u), e - 1)];
        asm volatile("" ::: "memory");  // the loads stay issued here, a step ahead of their use
        uint32_t x = 0;
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (TEST) {
                x += (lds[C[u].x & 32767] >> (C[u].x >> 27)) & 1u;
                x += (lds[C[u].y & 32767] >> (C[u].y >> 27)) & 1u;
                x += (lds[C[u].z & 32767] >> (C[u].z >> 27)) & 1u;
                x += (lds[C[u].w & 32767] >> (C[u].w >> 27)) & 1u;
            } else {
                x ^= C[u].x ^ C[u].y ^ C[u].z ^ C[u].w;
            }
        }
        acc = acc * 31u + x;
        asm volatile("" : "+v"(acc));
        if (BAR) __syncthreads();
        if (W && (s % BATCH) == BATCH - 1) {
            // survivors of BATCH steps: wfrac_q / 1024 of their 4096 U words each, as whole quads
            const uint32_t words = (BATCH * 128u * U * 32u * wfrac_q) >> 10;
            uint64_t base = W == 1 ? (uint64_t) pos(s, 0) * 32 - cs * 32 : dense;
            if (W == 3) base = (blockIdx.x * 8192u + (dense & 0x3FFFFFu)) & ((64u << 20) / 4 - 1);
            const auto     r     = rsrc(out + base, words * 4);
            const v4u      v     = {x, acc, s, tid};
#pragma unroll
            for (int k = 0; k < (BATCH + 1) / 2; k++)
                __builtin_amdgcn_raw_buffer_store_b128(v, r, (tid + k * 1024) * 16, 0, AUX);
            dense += (words + 3) & ~3u;
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            C[u]  = Cn[u];
            L1[u] = L0[u];
        }
    }
    sink[blockIdx.x * 1024 + tid] = acc;
}

int main() {
    const uint32_t n = 32u << 20;  // chunks: 4 GiB
    v4u*      pool;
    uint32_t *list, *sink, *out;
    CK(hipMalloc(&pool, (size_t) n * 128));
    CK(hipMalloc(&out, (size_t) n * 128 + (1 << 20)));
    CK(hipMalloc(&list, (size_t) n * 4));
    CK(hipMalloc(&sink, 1024 * 1024 * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    {  // random words (the test's positions)
        std::vector<uint32_t> w((size_t) n * 32 / 64);
        std::mt19937 r(3);
        for (auto& v : w) v = r();
        for (int k = 0; k < 64; k++) CK(hipMemcpy((char*) pool + (size_t) k * w.size() * 4, w.data(), w.size() * 4, hipMemcpyHostToDevice));
    }
    std::vector<uint32_t> h(n);
    for (uint32_t i = 0; i < n; i++) h[i] = i;
    std::shuffle(h.begin(), h.end(), std::mt19937_64(7));
    CK(hipMemcpy(list, h.data(), (size_t) n * 4, hipMemcpyHostToDevice));
    hipEvent_t a, z;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&z));
    const uint32_t q12 = 123;  // 12 % survivors (/1024)
    struct V {
        const char* name;
        void (*k)(v4u*, uint32_t*, uint32_t, uint32_t*, uint32_t, uint32_t*);
        uint32_t q;
    } vs[] = {
        {"gathers (U=3)", k_shape<3, false, false, 0>, q12},
        {"+ barrier", k_shape<3, true, false, 0>, q12},
        {"+ LDS test", k_shape<3, false, true, 0>, q12},
        {"+ barrier + test", k_shape<3, true, true, 0>, q12},
        {"+ sparse writes 12%", k_shape<3, false, false, 1>, q12},
        {"+ dense writes 12%", k_shape<3, false, false, 2>, q12},
        {"+ bar+test+sparse W", k_shape<3, true, true, 1>, q12},
        {"+ bar+test+dense W", k_shape<3, true, true, 2>, q12},
        {"+ sparse W 6%", k_shape<3, false, false, 1>, q12 / 2},
        {"+ sparse W 9%", k_shape<3, false, false, 1>, q12 * 3 / 4},
        {"+ sparse W 24%", k_shape<3, false, false, 1>, q12 * 2},
        {"+ dense W nt", k_shape<3, false, false, 2, 2>, q12},
        {"+ dense W sc1", k_shape<3, false, false, 2, 16>, q12},
        {"+ dense W sc0sc1", k_shape<3, false, false, 2, 17>, q12},
        {"+ dense W batch 4", k_shape<3, false, false, 2, 0, 4>, q12},
        {"+ ring 64MB W", k_shape<3, false, false, 3>, q12},
        {"+ ring 64MB W nt", k_shape<3, false, false, 3, 2>, q12},
    };
    const int NV = sizeof(vs) / sizeof(vs[0]);
    std::vector<float> best(NV, 1e9f);
    for (int v = 0; v < NV; v++) CK(hipFuncSetAttribute((const void*) vs[v].k, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    for (int rep = 0; rep < 5; rep++)
        for (int v = 0; v < NV; v++) {
            float ms;
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(vs[v].k, dim3(cus), dim3(1024), 131072, 0, pool, list, n, out, vs[v].q, sink);
            CK(hipGetLastError());
            CK(hipEventRecord(z));
            CK(hipEventSynchronize(z));
            CK(hipEventElapsedTime(&ms, a, z));
            CK(hipDeviceSynchronize());
            best[v] = std::min(best[v], ms);
        }
    printf("probe shape: 4 GiB of 128-B chunks gathered through a random list, %d workgroups x 1024 threads\n", cus);
    printf("%-24s %8s %10s\n", "variant", "ms", "read TB/s");
    for (int v = 0; v < NV; v++)
        printf("%-24s %8.3f %10.2f\n", vs[v].name, best[v], (double) n * 132 / best[v] / 1e9);
    return 0;
}
