// mall_rt.hip -- can the S partition words' round trip stay in the 256 MiB Infinity Cache?
//  The S side moves S once (8.19 GB) and its 4-byte partition words twice
// (k_scatter_s writes 4.1 GB, k_probe gathers them back). Processed as windows of W bytes of words
// in a reused ring, window w's words might be re-read from the Infinity Cache instead of HBM. This
// models the windowed pipeline with the two kernels' access shapes:
//   writer (k_scatter_s): every workgroup streams its share of the window's S tuples (16-byte nt
//          loads, two tuples each) and writes one 4-byte word per tuple as 128-byte lines into its
//          own contiguous region of the ring (8 lanes x 16 B per line);
//   reader (k_probe): the window's 128-byte chunks gathered through a random list (8 lanes per
//          chunk, 8 chunk loads in flight per thread), optionally plus a reload of the 128 MiB
//          filter slices per window (every partition's slice is needed again by every window).
// For each W the whole S pass (1.024e9 tuples) runs as ceil(4.096 GB / W) windows; W = 4 GiB is
// today's unwindowed design. Times are HIP-event sums over the windows, best of 3.
//   hipcc -O3 --offload-arch=gfx950 mall_rt.hip -o mall_rt && ./mall_rt
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <random>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("err %s line %d\n", hipGetErrorString(e), __LINE__);                  \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short) 0, (int) bytes, 0x00020000);
}

// tuples [t0, t0 + nt) of S -> words into the ring: workgroup g's region is [g * reg, (g + 1) * reg)
// uint4s; each thread turns 4 tuples (two 16-byte loads) into one 16-byte store
template <int SAUX>  // cache policy of the word stores: 2 = nt (k_scatter_s), 0 = default
__global__ __launch_bounds__(1024) void k_writer(const uint4* __restrict__ S, uint64_t t0, uint64_t nt,
                                                 uint4* __restrict__ ring, uint64_t reg) {
    const uint64_t per = (nt / 4 + gridDim.x - 1) / gridDim.x;  // quads of tuples per workgroup
    const uint64_t b = blockIdx.x * per, e = std::min<uint64_t>(nt / 4, b + per);
    if (b >= e) return;
    // uniform descriptors (SGPRs), per-lane offsets: two 16-byte loads = 4 tuples in, one out
    const auto rin  = rsrc(S + (t0 / 2) + 2 * b, (uint32_t) ((e - b) * 32));
    const auto rout = rsrc(ring + blockIdx.x * reg, (uint32_t) (reg * 16));
    for (uint64_t i = b + threadIdx.x; i < e; i += 1024) {
        const uint32_t o = (uint32_t) (i - b);  // the region fills line by line (8 lanes per line)
        const v4u      x = __builtin_amdgcn_raw_buffer_load_b128(rin, o * 32, 0, 2);
        const v4u      y = __builtin_amdgcn_raw_buffer_load_b128(rin, o * 32 + 16, 0, 2);
        const v4u      w = {x.x * 0x9E3779B1u, x.z ^ 0x5bd1e995u, y.x + 7u, y.z};
        __builtin_amdgcn_raw_buffer_store_b128(w, rout, o * 16, 0, SAUX);
    }
}

// the window's chunks through a random list; slices != null: also stream this workgroup's share
// of the 128 MiB filter slices (the probe's per-window slice reload)
__global__ __launch_bounds__(1024) void k_reader(const uint4* __restrict__ ring, const uint32_t* __restrict__ list,
                                                 uint32_t n, const uint4* __restrict__ slices, uint64_t slice_u4,
                                                 uint32_t* sink) {
    constexpr int  U   = 8;
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t b = blockIdx.x * per, e = min(n, b + per);
    const uint32_t cs = threadIdx.x >> 3, l8 = threadIdx.x & 7;
    uint32_t       acc = 0;
    if (slices) {
        const uint64_t sp = slice_u4 / gridDim.x;
        for (uint64_t i = threadIdx.x; i < sp; i += 1024) {
            const uint4 v = slices[blockIdx.x * sp + i];
            acc ^= v.x ^ v.w;
        }
    }
    for (uint32_t i = b + cs; i < e; i += 128 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t k = i + u * 128;
            v[u] = k < e ? ring[(uint64_t) list[k] * 8 + l8] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint64_t nS      = 1024000000ull;        // tuples
    const uint64_t words_b = nS * 4;                // 4.096 GB of words
    const uint64_t slice_b = 128ull << 20;
    int            G       = 0;
    CK(hipDeviceGetAttribute(&G, hipDeviceAttributeMultiprocessorCount, 0));
    uint4 *S, *ring, *slices;
    uint32_t *list, *sink;
    const uint64_t ring_max = 4ull << 30;
    CK(hipMalloc(&S, nS * 8));
    CK(hipMalloc(&ring, ring_max + (uint64_t) G * 4096));
    CK(hipMalloc(&slices, slice_b));
    CK(hipMalloc(&list, (ring_max / 128) * 4));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(S, 3, nS * 8));
    CK(hipMemset(slices, 5, slice_b));
    hipEvent_t ev[3];
    for (auto& x : ev) CK(hipEventCreate(&x));
    std::mt19937_64 rng(11);
    printf("S = %llu tuples (8.19 GB) streamed once; words 4.096 GB written then gathered, in windows of W\n",
           (unsigned long long) nS);
    for (int saux : {2, 0}) {
    printf("word stores %s\n", saux ? "nt (as k_scatter_s)" : "default policy");
    printf("%10s %5s %11s %11s %13s %11s %11s\n", "W", "wins", "writer ms", "reader ms", "reader+slice", "total ms",
           "total+slice");
    for (uint64_t W : {64ull << 20, 128ull << 20, 192ull << 20, 256ull << 20, 512ull << 20, 1ull << 30, 4ull << 30}) {
        const uint64_t win_t  = W / 4;                       // tuples per window
        const uint32_t nwin   = (uint32_t) ((nS + win_t - 1) / win_t);
        const uint64_t reg    = (((W / 16 + G - 1) / G + 8) + 7) & ~7ull;  // uint4s per region (whole lines)
        // list: the window's chunks (W / 128 of them) in random order; regions hold reg * 16 bytes
        const uint32_t nch = (uint32_t) (W / 128);
        std::vector<uint32_t> h(nch);
        {
            std::vector<uint32_t> ids;
            ids.reserve(nch);
            const uint64_t chunks_per_reg = reg / 8;
            for (int g = 0; g < G && ids.size() < nch; g++)
                for (uint64_t c = 0; c < chunks_per_reg - 1 && ids.size() < nch; c++) ids.push_back((uint32_t) (g * chunks_per_reg + c));
            while (ids.size() < nch) ids.push_back(ids[ids.size() % 7]);
            std::shuffle(ids.begin(), ids.end(), rng);
            h = ids;
        }
        CK(hipMemcpy(list, h.data(), (size_t) nch * 4, hipMemcpyHostToDevice));
        float best[3] = {1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 3; rep++) {
            for (int withs = 0; withs < 2; withs++) {
                float tw = 0, tr = 0;
                for (uint32_t w = 0; w < nwin; w++) {
                    const uint64_t t0 = (uint64_t) w * win_t, nt = std::min(win_t, nS - t0);
                    float          a, b;
                    CK(hipEventRecord(ev[0]));
                    if (saux) k_writer<2><<<G, 1024>>>(S, t0, nt, ring, reg);
                    else k_writer<0><<<G, 1024>>>(S, t0, nt, ring, reg);
                    CK(hipEventRecord(ev[1]));
                    k_reader<<<G, 1024>>>(ring, list, (uint32_t) std::min<uint64_t>(nch, nt / 32), withs ? slices : nullptr,
                                          slice_b / 16, sink);
                    CK(hipEventRecord(ev[2]));
                    CK(hipEventSynchronize(ev[2]));
                    CK(hipEventElapsedTime(&a, ev[0], ev[1]));
                    CK(hipEventElapsedTime(&b, ev[1], ev[2]));
                    tw += a;
                    tr += b;
                }
                if (!withs) best[0] = std::min(best[0], tw);
                best[1 + withs] = std::min(best[1 + withs], tr);
            }
        }
        printf("%7llu MiB %5u %11.3f %11.3f %13.3f %11.3f %11.3f\n", (unsigned long long) (W >> 20), nwin, best[0],
               best[1], best[2], best[0] + best[1], best[0] + best[2]);
        fflush(stdout);
    }
    }
    return 0;
}
