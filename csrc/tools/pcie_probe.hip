// PCIe (host <-> HBM) ceiling probe for the device TCP ring's staging hop, per mechanism:
//   * hipMemcpyAsync (copy engines / blit, as ROCclr chooses) D2H, H2D and both at once, on k streams
//   * zero-copy kernels: a kernel streaming reads from pinned host memory into HBM ("kread"), a kernel streaming
//     HBM into pinned host memory ("kwrite"), and both at once (duplex), with a chosen workgroup count
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 csrc/tools/pcie_probe.hip -o build/pcie_probe && ./build/pcie_probe [MiB]
// Prints one line per variant: GB/s (bytes crossing PCIe / wall time of the batch).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
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

// contiguous tile per workgroup, 4 x 16 B per thread in flight
__global__ __launch_bounds__(kB) void stream_copy(v4u *__restrict__ d, const v4u *__restrict__ s, size_t n16) {
    constexpr size_t kTile = size_t(kB) * 4;
    for (size_t t = blockIdx.x; t * kTile < n16; t += gridDim.x) {
        const size_t base = t * kTile + threadIdx.x;
        v4u v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (base + j * kB < n16) v[j] = __builtin_nontemporal_load(s + base + j * kB);
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (base + j * kB < n16) __builtin_nontemporal_store(v[j], d + base + j * kB);
    }
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256;
    const size_t n = mib << 20;
    constexpr int kMaxS = 8;
    void *h[2][kMaxS], *d[2][kMaxS];
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < kMaxS; ++i) {
            CHECK(hipHostMalloc(&h[k][i], n, hipHostMallocDefault));
            CHECK(hipMalloc(&d[k][i], n));
            std::memset(h[k][i], 1, n);
            CHECK(hipMemset(d[k][i], 2, n));
        }
    hipStream_t st[2 * kMaxS];
    for (auto &s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int reps = 4;

    // mode: 0 d2h, 1 h2d, 2 duplex; mech: 0 memcpy, 1 kernel
    auto run = [&](int mode, int mech, int ns, int grid) {
        auto issue = [&] {
            for (int i = 0; i < ns; ++i) {
                if (mode == 0 || mode == 2) {
                    if (mech == 0) CHECK(hipMemcpyAsync(h[0][i], d[0][i], n, hipMemcpyDeviceToHost, st[i]));
                    else hipLaunchKernelGGL(stream_copy, dim3(grid), dim3(kB), 0, st[i], (v4u *) h[0][i],
                                            (const v4u *) d[0][i], n / 16);
                }
                if (mode == 1 || mode == 2) {
                    if (mech == 0) CHECK(hipMemcpyAsync(d[1][i], h[1][i], n, hipMemcpyHostToDevice, st[kMaxS + i]));
                    else hipLaunchKernelGGL(stream_copy, dim3(grid), dim3(kB), 0, st[kMaxS + i], (v4u *) d[1][i],
                                            (const v4u *) h[1][i], n / 16);
                }
            }
        };
        issue();
        CHECK(hipDeviceSynchronize());
        const double t0 = now();
        for (int r = 0; r < reps; ++r) issue();
        CHECK(hipDeviceSynchronize());
        const double dt = now() - t0;
        const double bytes = double(reps) * ns * n * (mode == 2 ? 2 : 1);
        static const char *mn[] = {"d2h", "h2d", "duplex"};
        std::printf("%-7s %-6s streams %d grid %5d : %7.2f GB/s\n", mn[mode], mech ? "kernel" : "memcpy", ns,
                    mech ? grid : 0, bytes / dt / 1e9);
        std::fflush(stdout);
    };
    // pieces: the whole buffer as n/piece consecutive hipMemcpyAsync calls on ONE stream per direction (the device
    // ring's staging pattern), explicit kinds vs hipMemcpyDefault, default vs mapped|portable pinned memory
    void *hm[2];
    CHECK(hipHostMalloc(&hm[0], n, hipHostMallocPortable | hipHostMallocMapped));
    CHECK(hipHostMalloc(&hm[1], n, hipHostMallocPortable | hipHostMallocMapped));
    auto pieces = [&](int mode, size_t piece, bool dflt, bool mapped) {
        void *h0 = mapped ? hm[0] : h[0][0], *h1 = mapped ? hm[1] : h[1][0];
        auto issue = [&] {
            for (size_t off = 0; off < n; off += piece) {
                const size_t k = std::min(piece, n - off);
                if (mode == 0 || mode == 2)
                    CHECK(hipMemcpyAsync((char *) h0 + off, (char *) d[0][0] + off, k,
                                         dflt ? hipMemcpyDefault : hipMemcpyDeviceToHost, st[0]));
                if (mode == 1 || mode == 2)
                    CHECK(hipMemcpyAsync((char *) d[1][0] + off, (char *) h1 + off, k,
                                         dflt ? hipMemcpyDefault : hipMemcpyHostToDevice, st[kMaxS]));
            }
        };
        issue();
        CHECK(hipDeviceSynchronize());
        const double t0 = now();
        for (int r = 0; r < reps; ++r) issue();
        CHECK(hipDeviceSynchronize());
        const double dt = now() - t0;
        static const char *mn[] = {"d2h", "h2d", "duplex"};
        std::printf("%-7s pieces %5zu KiB %s %s : %7.2f GB/s\n", mn[mode], piece >> 10, dflt ? "default " : "explicit",
                    mapped ? "mapped " : "default", double(reps) * n * (mode == 2 ? 2 : 1) / dt / 1e9);
        std::fflush(stdout);
    };
    for (int mode = 0; mode < 3; ++mode)
        for (size_t piece : {size_t(1) << 20, size_t(4) << 20, size_t(16) << 20})
            for (int v = 0; v < 4; ++v) pieces(mode, piece, v & 1, v & 2);
    if (std::getenv("PIECES_ONLY")) return 0;
    for (int mode = 0; mode < 3; ++mode)
        for (int ns : {1, 4, 8}) run(mode, 0, ns, 0);
    for (int mode = 0; mode < 3; ++mode)
        for (int ns : {1, 4, 8})
            for (int grid : {64, 256, 1024}) run(mode, 1, ns, grid);
    // mixed: kernel writes D2H while memcpy does H2D (and vice versa)
    for (int ns : {1, 4}) {
        auto mixed = [&](bool kernel_d2h) {
            auto issue = [&] {
                for (int i = 0; i < ns; ++i) {
                    if (kernel_d2h) {
                        hipLaunchKernelGGL(stream_copy, dim3(256), dim3(kB), 0, st[i], (v4u *) h[0][i],
                                           (const v4u *) d[0][i], n / 16);
                        CHECK(hipMemcpyAsync(d[1][i], h[1][i], n, hipMemcpyHostToDevice, st[kMaxS + i]));
                    } else {
                        CHECK(hipMemcpyAsync(h[0][i], d[0][i], n, hipMemcpyDeviceToHost, st[i]));
                        hipLaunchKernelGGL(stream_copy, dim3(256), dim3(kB), 0, st[kMaxS + i], (v4u *) d[1][i],
                                           (const v4u *) h[1][i], n / 16);
                    }
                }
            };
            issue();
            CHECK(hipDeviceSynchronize());
            const double t0 = now();
            for (int r = 0; r < reps; ++r) issue();
            CHECK(hipDeviceSynchronize());
            const double dt = now() - t0;
            std::printf("duplex  mixed(%s) streams %d : %7.2f GB/s\n", kernel_d2h ? "kwrite+memcpy-h2d" : "memcpy-d2h+kread",
                        ns, double(reps) * ns * n * 2 / dt / 1e9);
            std::fflush(stdout);
        };
        mixed(true);
        mixed(false);
    }
    return 0;
}
