// Standalone HBM micro-benchmark for the streaming kernel shapes used by the xGMI all-reduce (copy / gather,
// 2..8-source reduce with 1 or 2 outputs). Used to pick the production kernel structure on MI355X:
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 csrc/tools/kbench.hip -o build/kbench && ./build/kbench [MiB]
// Prints one line per variant: effective HBM bandwidth (bytes read + written) / kernel time.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        hipError_t e_ = (x);                                                                                         \
        if (e_ != hipSuccess) {                                                                                      \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                                    \
            std::exit(1);                                                                                            \
        }                                                                                                            \
    } while (0)

constexpr int kB = 256;

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__device__ inline uint4 ntld(const uint4 *p) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ inline void ntst(uint4 v, uint4 *p) {
    const v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(p));
}

struct Srcs {
    const uint4 *p[8];
};

// ---- copy variants
__global__ __launch_bounds__(kB) void copy_gs4(uint4 *__restrict__ d, const uint4 *__restrict__ s, size_t n) {
    const size_t stride = size_t(gridDim.x) * kB;
    size_t i = size_t(blockIdx.x) * kB + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        uint4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
        d[i] = a;
        d[i + stride] = b;
        d[i + 2 * stride] = c;
        d[i + 3 * stride] = e;
    }
    for (; i < n; i += stride) d[i] = s[i];
}

__global__ __launch_bounds__(kB) void copy_gs4_nt(uint4 *__restrict__ d, const uint4 *__restrict__ s, size_t n) {
    const size_t stride = size_t(gridDim.x) * kB;
    size_t i = size_t(blockIdx.x) * kB + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        uint4 a = ntld(s + i), b = ntld(s + i + stride);
        uint4 c = ntld(s + i + 2 * stride), e = ntld(s + i + 3 * stride);
        ntst(a, d + i);
        ntst(b, d + i + stride);
        ntst(c, d + i + 2 * stride);
        ntst(e, d + i + 3 * stride);
    }
    for (; i < n; i += stride) ntst(ntld(s + i), d + i);
}

// each workgroup streams one contiguous chunk, 4 x 16 B per thread per iteration (4 KiB x 4 per WG step)
template<bool NT>
__global__ __launch_bounds__(kB) void copy_chunk(uint4 *__restrict__ d, const uint4 *__restrict__ s, size_t n) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = size_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
    size_t i = lo + threadIdx.x;
    for (; i + 3 * kB < hi; i += 4 * kB) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = NT ? ntld(s + i + u * kB) : s[i + u * kB];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (NT) ntst(v[u], d + i + u * kB);
            else d[i + u * kB] = v[u];
        }
    }
    for (; i < hi; i += kB) d[i] = s[i];
}

// ---- bf16 sum of nsrc sources -> 1 or 2 outputs
__device__ inline float bf2f(uint16_t v) { return __uint_as_float(uint32_t(v) << 16); }
__device__ inline uint16_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return uint16_t(u >> 16);
}
__device__ inline void acc8(float *a, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        a[2 * k] += __uint_as_float(w[k] << 16);
        a[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
    }
}
__device__ inline void ld8(float *a, uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        a[2 * k] = __uint_as_float(w[k] << 16);
        a[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
}
__device__ inline uint4 st8(const float *a) {
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = uint32_t(f2bf(a[2 * k])) | (uint32_t(f2bf(a[2 * k + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// production-like: grid-stride, 2 vectors per thread per iteration
__global__ __launch_bounds__(kB) void red_gs2(uint4 *__restrict__ d0, uint4 *__restrict__ d1, Srcs s, int ns, size_t n) {
    const size_t stride = size_t(gridDim.x) * kB;
    for (size_t i = size_t(blockIdx.x) * kB + threadIdx.x; i < n; i += 2 * stride) {
        const size_t j = i + stride < n ? i + stride : i;
        float a[8], b[8];
        ld8(a, s.p[0][i]);
        ld8(b, s.p[0][j]);
#pragma unroll 4
        for (int k = 1; k < ns; ++k) {
            const uint4 x = s.p[k][i], y = s.p[k][j];
            acc8(a, x);
            acc8(b, y);
        }
        const uint4 oa = st8(a), ob = st8(b);
        d0[i] = oa;
        if (d1) d1[i] = oa;
        if (j != i) {
            d0[j] = ob;
            if (d1) d1[j] = ob;
        }
    }
}

// contiguous chunk per WG, U vectors per thread in flight per source, all sources loaded before accumulation
template<int U, int NS, bool NT>
__global__ __launch_bounds__(kB) void red_chunk(uint4 *__restrict__ d0, uint4 *__restrict__ d1, Srcs s, size_t n) {
    const size_t per = ((n + gridDim.x - 1) / gridDim.x + kB - 1) / kB * kB;
    const size_t lo = size_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * kB < hi; i += U * kB) {
        uint4 v[NS][U];
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
            for (int u = 0; u < U; ++u) v[k][u] = NT ? ntld(s.p[k] + i + u * kB) : s.p[k][i + u * kB];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float a[8];
            ld8(a, v[0][u]);
#pragma unroll
            for (int k = 1; k < NS; ++k) acc8(a, v[k][u]);
            const uint4 o = st8(a);
            if (NT) {
                ntst(o, d0 + i + u * kB);
                if (d1) ntst(o, d1 + i + u * kB);
            } else {
                d0[i + u * kB] = o;
                if (d1) d1[i + u * kB] = o;
            }
        }
    }
    for (; i < hi; i += kB) {
        float a[8];
        ld8(a, s.p[0][i]);
        for (int k = 1; k < NS; ++k) acc8(a, s.p[k][i]);
        d0[i] = st8(a);
        if (d1) d1[i] = st8(a);
    }
}

template<typename F>
static float time_it(F &&launch, int iters = 10) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipGetLastError());
    return ms / iters;
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 512;
    const size_t bytes = mib << 20, n = bytes / 16;
    std::vector<uint4 *> src(8);
    for (auto &p : src) {
        CHECK(hipMalloc(&p, bytes));
        CHECK(hipMemset(p, 0x3f, bytes));
    }
    uint4 *d0, *d1;
    CHECK(hipMalloc(&d0, bytes));
    CHECK(hipMalloc(&d1, bytes));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto gbs = [&](double moved, float ms) { return moved / (ms * 1e-3) / 1e9; };
    std::printf("buffer %zu MiB, %d CUs\n", mib, cus);
    {
        float ms = time_it([&] { CHECK(hipMemcpyAsync(d0, src[0], bytes, hipMemcpyDeviceToDevice, nullptr)); });
        std::printf("copy  hipMemcpyAsync D2D              %8.3f ms %7.0f GB/s\n", ms, gbs(2.0 * bytes, ms));
    }
    for (int wpc : {2, 4, 8, 16}) {
        const int g = cus * wpc;
        float ms = time_it([&] { copy_gs4<<<g, kB>>>(d0, src[0], n); });
        std::printf("copy  gs4        grid %5d            %8.3f ms %7.0f GB/s\n", g, ms, gbs(2.0 * bytes, ms));
        ms = time_it([&] { copy_gs4_nt<<<g, kB>>>(d0, src[0], n); });
        std::printf("copy  gs4_nt     grid %5d            %8.3f ms %7.0f GB/s\n", g, ms, gbs(2.0 * bytes, ms));
        ms = time_it([&] { copy_chunk<false><<<g, kB>>>(d0, src[0], n); });
        std::printf("copy  chunk      grid %5d            %8.3f ms %7.0f GB/s\n", g, ms, gbs(2.0 * bytes, ms));
        ms = time_it([&] { copy_chunk<true><<<g, kB>>>(d0, src[0], n); });
        std::printf("copy  chunk_nt   grid %5d            %8.3f ms %7.0f GB/s\n", g, ms, gbs(2.0 * bytes, ms));
    }
    Srcs s{};
    for (int k = 0; k < 8; ++k) s.p[k] = src[k];
    for (int ns : {2, 8}) {
        // shard of 1/ns of the buffer per source, as in the two-shot reduce-scatter
        const size_t m = n / ns;
        for (int outs : {1, 2}) {
            const double moved = double(m) * 16 * (ns + outs);
            for (int wpc : {4, 8, 16}) {
                const int g = cus * wpc;
                float ms = time_it([&] { red_gs2<<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, ns, m); });
                std::printf("red%d->%d gs2        grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                if (ns == 2) {
                    ms = time_it([&] { red_chunk<4, 2, false><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk4     grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                    ms = time_it([&] { red_chunk<4, 2, true><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk4_nt  grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                    ms = time_it([&] { red_chunk<2, 2, false><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk2     grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                } else {
                    ms = time_it([&] { red_chunk<2, 8, false><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk2     grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                    ms = time_it([&] { red_chunk<1, 8, false><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk1     grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                    ms = time_it([&] { red_chunk<2, 8, true><<<g, kB>>>(d0, outs == 2 ? d1 : nullptr, s, m); });
                    std::printf("red%d->%d chunk2_nt  grid %5d          %8.3f ms %7.0f GB/s\n", ns, outs, g, ms, gbs(moved, ms));
                }
            }
        }
    }
    return 0;
}
