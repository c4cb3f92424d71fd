// Primitive-rate microbenchmark for the bloom radix join design on MI355X (gfx950).
//
// Measures, at the north-star shape (|S| = 1024e6 8-byte tuples, 128 MiB bitmap):
//   stream    : read S once (uint4 = 2 tuples per lane)           -> HBM read roof
//   copy      : read 4 GB keys + write 4 GB                       -> read+write roof
//   probe_*   : read S + one random dword of a 128 MiB bitmap per key (blocked, k=1)
//               variants: crc via byte LDS tables, via nibble LDS tables, cheap mul hash
//               (isolates the random-lookup cost), nontemporal S loads
//   atomic    : 128e6 random atomicOr into the 128 MiB bitmap     -> bloom build rate
//   ldsprobe  : stream 4-byte keys + crc + LDS bit test           -> partition-first consumer
// Not part of the product; kept as design evidence (DESIGN.md "Primitive rates").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                    \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_),       \
                    __FILE__, __LINE__);                                            \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

static uint32_t crc_f(uint32_t x) {
    for (int i = 0; i < 32; i++) x = (x >> 1) ^ (0x82F63B78u & (0u - (x & 1u)));
    return x;
}

__device__ __forceinline__ uint32_t crapwow42(uint32_t key) {
    const uint32_t n = 0x5052acdbu;
    uint32_t h = 4u, k = 4u + 42u + n;
    uint64_t p = (uint64_t) key * n;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    p = (uint64_t) (h ^ (k + n)) * n;
    h ^= (uint32_t) p;
    k ^= (uint32_t) (p >> 32);
    return k ^ h;
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x85ebca6bu; x ^= x >> 13; x *= 0xc2b2ae35u; x ^= x >> 16;
    return x;
}

enum { CRC_BYTE = 0, CRC_NIB = 1, CRC_NONE = 2 };

template <int MODE>
__device__ __forceinline__ uint32_t crc42(uint32_t key, const uint32_t* tb, const uint32_t* tn) {
    uint32_t x = key ^ 42u;
    if (MODE == CRC_BYTE) {
        return tb[x & 0xff] ^ tb[256 + ((x >> 8) & 0xff)] ^ tb[512 + ((x >> 16) & 0xff)] ^
               tb[768 + (x >> 24)];
    } else if (MODE == CRC_NIB) {
        uint32_t r = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) r ^= tn[j * 16 + ((x >> (4 * j)) & 15)];
        return r;
    } else {
        return mix32(key);
    }
}

__global__ void k_init_tuples(uint2* t, uint64_t n, uint32_t salt) {
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n; i += stride) t[i] = make_uint2(mix32((uint32_t) i ^ salt) , (uint32_t) i);
}

__global__ void k_init_words(uint32_t* w, uint64_t n, uint32_t salt) {
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n; i += stride) w[i] = mix32((uint32_t) i * 2654435761u + salt) & mix32((uint32_t) i + salt);
}

__global__ void k_stream(const uint4* __restrict__ s, uint64_t n4, unsigned long long* out) {
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (; i < n4; i += stride) {
        uint4 v = s[i];
        acc ^= v.x + v.z;
    }
    if (acc == 0x12345678u) atomicAdd(out, 1ull);
}

__global__ void k_copy(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n4) {
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n4; i += stride) out[i] = in[i];
}

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k_probe(const uint4* __restrict__ s, uint64_t n4,
                                               const uint32_t* __restrict__ bitmap,
                                               uint32_t nblocks_mask, const uint32_t* gtb,
                                               const uint32_t* gtn, unsigned long long* out) {
    __shared__ uint32_t tb[1024];
    __shared__ uint32_t tn[128];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) tb[i] = gtb[i];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) tn[i] = gtn[i];
    __syncthreads();
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    uint32_t cnt = 0;
    for (; i < n4; i += stride) {
        uint4 v;
        if (NT) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 t = __builtin_nontemporal_load((const u32x4*) (s + i));
            v = make_uint4(t.x, t.y, t.z, t.w);
        } else {
            v = s[i];
        }
        uint32_t k0 = v.x, k1 = v.z;
        uint32_t b0 = crc42<MODE>(k0, tb, tn) & nblocks_mask;
        uint32_t b1 = crc42<MODE>(k1, tb, tn) & nblocks_mask;
        uint32_t h0 = crapwow42(k0) & 1023u, h1 = crapwow42(k1) & 1023u;
        uint32_t w0 = bitmap[b0 * 32u + (h0 >> 5)];
        uint32_t w1 = bitmap[b1 * 32u + (h1 >> 5)];
        cnt += (w0 >> (h0 & 31)) & 1u;
        cnt += (w1 >> (h1 & 31)) & 1u;
    }
    // wave reduce
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long) cnt);
}

__global__ __launch_bounds__(256) void k_atomic(const uint4* __restrict__ r, uint64_t n4,
                                                uint32_t* bitmap, uint32_t nblocks_mask,
                                                const uint32_t* gtb) {
    __shared__ uint32_t tb[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) tb[i] = gtb[i];
    __syncthreads();
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (; i < n4; i += stride) {
        uint4 v = r[i];
        uint32_t k0 = v.x, k1 = v.z;
        uint32_t b0 = crc42<CRC_BYTE>(k0, tb, nullptr) & nblocks_mask;
        uint32_t b1 = crc42<CRC_BYTE>(k1, tb, nullptr) & nblocks_mask;
        uint32_t h0 = crapwow42(k0) & 1023u, h1 = crapwow42(k1) & 1023u;
        atomicOr(bitmap + b0 * 32u + (h0 >> 5), 1u << (h0 & 31));
        atomicOr(bitmap + b1 * 32u + (h1 >> 5), 1u << (h1 & 31));
    }
}

// partition-first consumer model: 4-byte keys streamed, bit test in a 64 KB LDS slice
__global__ __launch_bounds__(256) void k_ldsprobe(const uint4* __restrict__ keys, uint64_t n4,
                                                  const uint32_t* gtn, unsigned long long* out) {
    __shared__ uint32_t tn[128];
    __shared__ uint32_t slice[16384];
    for (int i = threadIdx.x; i < 128; i += blockDim.x) tn[i] = gtn[i];
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) slice[i] = 0x01010101u * (i & 0xff);
    __syncthreads();
    uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    uint32_t cnt = 0;
    for (; i < n4; i += stride) {
        uint4 v = keys[i];
        uint32_t ks[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t b = crc42<CRC_NIB>(ks[j], nullptr, tn) >> 23;  // 512 blocks of 128 B
            uint32_t h = crapwow42(ks[j]) & 1023u;
            cnt += (slice[b * 32u + (h >> 5)] >> (h & 31)) & 1u;
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_down(cnt, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long) cnt);
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b)); }
    void start() { CHECK(hipEventRecord(a, 0)); }
    float stop() {
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
};

template <class F>
static void bench(const char* name, double bytes, double ops, int reps, F f) {
    Timer t;
    f();
    CHECK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < reps; r++) {
        t.start();
        f();
        v.push_back(t.stop());
    }
    std::sort(v.begin(), v.end());
    float med = v[v.size() / 2];
    printf("%-22s min %8.3f ms  med %8.3f ms  %8.1f GB/s  %8.2f Gop/s\n", name, v[0], med,
           bytes / v[0] / 1e6, ops / v[0] / 1e6);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint64_t NS = 1024000000ull, NR = 128000000ull;
    const uint64_t m_bits = 1ull << 30;
    const uint32_t nblocks = (uint32_t) (m_bits / 1024);
    int grid = argc > 1 ? atoi(argv[1]) : 2048;

    std::vector<uint32_t> tb(1024), tn(128);
    for (int j = 0; j < 4; j++)
        for (int v = 0; v < 256; v++) tb[j * 256 + v] = crc_f((uint32_t) v << (8 * j));
    for (int j = 0; j < 8; j++)
        for (int v = 0; v < 16; v++) tn[j * 16 + v] = crc_f((uint32_t) v << (4 * j));

    uint2 *S, *R;
    uint32_t *bitmap, *gtb, *gtn, *keys_out;
    unsigned long long* out;
    CHECK(hipMalloc(&S, NS * 8));
    CHECK(hipMalloc(&R, NR * 8));
    CHECK(hipMalloc(&bitmap, m_bits / 8));
    CHECK(hipMalloc(&keys_out, NS * 4));
    CHECK(hipMalloc(&gtb, 4096));
    CHECK(hipMalloc(&gtn, 512));
    CHECK(hipMalloc(&out, 8));
    CHECK(hipMemcpy(gtb, tb.data(), 4096, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(gtn, tn.data(), 512, hipMemcpyHostToDevice));
    k_init_tuples<<<4096, 256>>>(S, NS, 0x1234u);
    k_init_tuples<<<4096, 256>>>(R, NR, 0x9876u);
    k_init_words<<<4096, 256>>>(bitmap, m_bits / 32, 7u);
    CHECK(hipDeviceSynchronize());

    const uint64_t n4 = NS / 2;
    const double sbytes = NS * 8.0;
    printf("grid=%d blocks x 256 threads\n", grid);
    bench("stream S 8.19GB", sbytes, NS, 5, [&] { k_stream<<<grid, 256>>>((const uint4*) S, n4, out); });
    bench("copy 4.1GB+4.1GB", NS * 8.0, NS, 5, [&] {
        k_copy<<<grid, 256>>>((const uint4*) S, (uint4*) keys_out, NS / 4);
    });
    bench("probe crc=byte", sbytes, NS, 5, [&] {
        k_probe<CRC_BYTE, false><<<grid, 256>>>((const uint4*) S, n4, bitmap, nblocks - 1, gtb, gtn, out);
    });
    bench("probe crc=nibble", sbytes, NS, 5, [&] {
        k_probe<CRC_NIB, false><<<grid, 256>>>((const uint4*) S, n4, bitmap, nblocks - 1, gtb, gtn, out);
    });
    bench("probe crc=none(mul)", sbytes, NS, 5, [&] {
        k_probe<CRC_NONE, false><<<grid, 256>>>((const uint4*) S, n4, bitmap, nblocks - 1, gtb, gtn, out);
    });
    bench("probe crc=nibble nt", sbytes, NS, 5, [&] {
        k_probe<CRC_NIB, true><<<grid, 256>>>((const uint4*) S, n4, bitmap, nblocks - 1, gtb, gtn, out);
    });
    bench("probe 16M bitmap", sbytes, NS, 5, [&] {
        k_probe<CRC_NIB, false><<<grid, 256>>>((const uint4*) S, n4, bitmap, (nblocks >> 3) - 1, gtb, gtn, out);
    });
    bench("probe 1M bitmap", sbytes, NS, 5, [&] {
        k_probe<CRC_NIB, false><<<grid, 256>>>((const uint4*) S, n4, bitmap, (nblocks >> 7) - 1, gtb, gtn, out);
    });
    bench("atomicOr 128M", NR * 8.0, NR, 5, [&] {
        k_atomic<<<grid, 256>>>((const uint4*) R, NR / 2, bitmap, nblocks - 1, gtb);
    });
    bench("atomicOr 128M 16Mbm", NR * 8.0, NR, 5, [&] {
        k_atomic<<<grid, 256>>>((const uint4*) R, NR / 2, bitmap, (nblocks >> 3) - 1, gtb);
    });
    bench("ldsprobe 4.1GB keys", NS * 4.0, NS, 5, [&] {
        k_ldsprobe<<<grid, 256>>>((const uint4*) keys_out, NS / 4, gtn, out);
    });
    for (int g : {1024, 4096, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "probe nib grid=%d", g);
        bench(nm, sbytes, NS, 3, [&] {
            k_probe<CRC_NIB, false><<<g, 256>>>((const uint4*) S, n4, bitmap, nblocks - 1, gtb, gtn, out);
        });
        snprintf(nm, sizeof nm, "stream grid=%d", g);
        bench(nm, sbytes, NS, 3, [&] { k_stream<<<g, 256>>>((const uint4*) S, n4, out); });
    }
    CHECK(hipFree(S));
    CHECK(hipFree(R));
    CHECK(hipFree(bitmap));
    CHECK(hipFree(keys_out));
    printf("done\n");
    return 0;
}
