// rw_bw.hip -- read/write mix bandwidth on MI355X: read S tuples (8 B), write keys (4 B) --
// the traffic shape of the S partition pass, without the partitioning. Dev tool.
//   hipcc -O3 --offload-arch=gfx950 rw_bw.hip -o rw_bw && ./rw_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// each workgroup streams its own contiguous slice; U uint4 loads (2 tuples each) per thread per step
template <int U>
__global__ void k_rw(const uint4* __restrict__ in, uint2* __restrict__ out, uint64_t n4) {
    const uint64_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const uint64_t b = blockIdx.x * per, e = min(n4, b + per);
    for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t) blockDim.x * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * blockDim.x;
            v[u] = k < e ? in[k] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * blockDim.x;
            if (k < e) out[k] = make_uint2(v[u].x ^ 0x9e3779b9u, v[u].z ^ 0x9e3779b9u);
        }
    }
}

// read only
template <int U>
__global__ void k_r(const uint4* __restrict__ in, uint64_t n4, uint32_t* sink) {
    const uint64_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const uint64_t b = blockIdx.x * per, e = min(n4, b + per);
    uint32_t acc = 0;
    for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t) blockDim.x * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t k = i + (uint64_t) u * blockDim.x;
            v[u] = k < e ? in[k] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].z;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <class K>
static float timeit(K launch, int reps = 5) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    std::vector<float> t;
    for (int r = 0; r < reps + 1; r++) {
        hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (r) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const uint64_t nS = 1024000000ull, n4 = nS / 2;
    uint4* in; uint2* out; uint32_t* sink;
    CK(hipMalloc(&in, n4 * 16)); CK(hipMalloc(&out, n4 * 8)); CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 1, n4 * 16));
    const double rd = n4 * 16.0, wr = n4 * 8.0;
    for (int cfg = 0; cfg < 6; cfg++) {
        int grid = cfg < 3 ? 256 : 2048, thr = cfg < 3 ? 1024 : 256;
        int u = (cfg % 3 == 0) ? 1 : (cfg % 3 == 1) ? 4 : 8;
        float ms = timeit([&] {
            if (u == 1) k_rw<1><<<grid, thr>>>(in, out, n4);
            else if (u == 4) k_rw<4><<<grid, thr>>>(in, out, n4);
            else k_rw<8><<<grid, thr>>>(in, out, n4);
        });
        printf("rw   grid=%5d x %4d U=%d: %7.3f ms  %7.1f GB/s (read %.2f GB + write %.2f GB)\n", grid, thr, u, ms,
               (rd + wr) / ms / 1e6, rd / 1e9, wr / 1e9);
        float ms2 = timeit([&] {
            if (u == 1) k_r<1><<<grid, thr>>>(in, n4, sink);
            else if (u == 4) k_r<4><<<grid, thr>>>(in, n4, sink);
            else k_r<8><<<grid, thr>>>(in, n4, sink);
        });
        printf("read grid=%5d x %4d U=%d: %7.3f ms  %7.1f GB/s\n", grid, thr, u, ms2, rd / ms2 / 1e6);
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
