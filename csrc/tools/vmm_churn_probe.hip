// Is VMM memory (hipMemCreate + hipMemAddressReserve + hipMemMap) safe to unmap / free and re-create in a loop,
// the way IPC comm buffers come and go with communicators? Each round:
//   1. create + map a VMM buffer B of a varying size (the VA of a freed buffer is often handed out again)
//   2. fill B with a round-specific value with a kernel, and a hipMalloc'd canary C with a constant
//   3. verify B through a kernel (counted on the device) and through hipMemcpy to the host, and C on the host
//   4. keep up to `live` buffers, unmapping / freeing the oldest
// Any mismatch points at stale translations or aliasing after unmap/remap.
//   vmm_churn_probe [rounds=200] [live=3] [free_va=1]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <deque>
#include <set>
#include <vector>

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        hipError_t e_ = (x);                                                                                         \
        if (e_ != hipSuccess) {                                                                                      \
            std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));                         \
            std::exit(2);                                                                                            \
        }                                                                                                            \
    } while (0)

__global__ void k_fill(unsigned *p, size_t n, unsigned v) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = v;
}
__global__ void k_count(const unsigned *p, size_t n, unsigned v, unsigned long long *bad) {
    unsigned long long c = 0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        c += p[i] != v;
    if (c) atomicAdd(bad, c);
}

struct Buf {
    void *p;
    size_t size;
    hipMemGenericAllocationHandle_t h;
};

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 200;
    const size_t live = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 3;
    const bool free_va = argc > 3 ? std::atoi(argv[3]) != 0 : true;
    CHECK(hipSetDevice(0));
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    prop.requestedHandleType = hipMemHandleTypePosixFileDescriptor;
    size_t gran = 0, rec = 0;
    CHECK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    CHECK(hipMemGetAllocationGranularity(&rec, &prop, hipMemAllocationGranularityRecommended));
    std::printf("granularity min %zu recommended %zu, rounds %d, live %zu, free_va %d\n", gran, rec, rounds, live,
                int(free_va));
    const size_t sizes[] = {12000004, 1 << 20, 4194304 + 4096, 64u << 20, 2097152 * 3 + 8192, 3000001 * 2};
    unsigned long long *bad = nullptr;
    CHECK(hipMalloc(&bad, 8));
    const size_t cn = 8u << 20; // canary words
    unsigned *canary = nullptr;
    CHECK(hipMalloc(&canary, cn * 4));
    std::vector<unsigned> host;
    std::deque<Buf> bufs;
    std::set<void *> seen;
    int reused = 0, fails = 0;
    for (int r = 0; r < rounds; ++r) {
        const size_t want = sizes[r % 6];
        Buf b{nullptr, (want + gran - 1) / gran * gran, {}};
        CHECK(hipMemCreate(&b.h, b.size, &prop, 0));
        CHECK(hipMemAddressReserve(&b.p, b.size, gran, nullptr, 0));
        CHECK(hipMemMap(b.p, b.size, 0, b.h, 0));
        hipMemAccessDesc acc{};
        acc.location = prop.location;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        CHECK(hipMemSetAccess(b.p, b.size, &acc, 1));
        reused += seen.count(b.p) ? 1 : 0;
        seen.insert(b.p);
        const size_t n = b.size / 4;
        const unsigned v = 0x1000u + unsigned(r);
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, canary, cn, 0xC0FFEEu);
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, static_cast<unsigned *>(b.p), n, v);
        CHECK(hipMemset(bad, 0, 8));
        hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, static_cast<const unsigned *>(b.p), n, v, bad);
        CHECK(hipDeviceSynchronize());
        unsigned long long kbad = 0;
        CHECK(hipMemcpy(&kbad, bad, 8, hipMemcpyDeviceToHost));
        host.resize(n);
        CHECK(hipMemcpy(host.data(), b.p, n * 4, hipMemcpyDeviceToHost));
        size_t hbad = 0, first = n;
        for (size_t i = 0; i < n; ++i)
            if (host[i] != v) {
                if (first == n) first = i;
                ++hbad;
            }
        host.resize(cn);
        CHECK(hipMemcpy(host.data(), canary, cn * 4, hipMemcpyDeviceToHost));
        size_t cbad = 0;
        for (size_t i = 0; i < cn; ++i) cbad += host[i] != 0xC0FFEEu;
        // every live buffer still holds its own value
        size_t lbad = 0;
        for (size_t k = 0; k < bufs.size(); ++k) {
            const unsigned lv = 0x1000u + unsigned(r - int(bufs.size()) + int(k));
            CHECK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(k_count, dim3(1024), dim3(256), 0, 0, static_cast<const unsigned *>(bufs[k].p),
                               bufs[k].size / 4, lv, bad);
            unsigned long long x = 0;
            CHECK(hipMemcpy(&x, bad, 8, hipMemcpyDeviceToHost));
            lbad += x;
        }
        if (kbad || hbad || cbad || lbad) {
            ++fails;
            std::printf("round %d size %zu va %p: kernel-bad %llu host-bad %zu (first %zu) canary-bad %zu live-bad %zu\n",
                        r, b.size, b.p, kbad, hbad, first, cbad, lbad);
        }
        bufs.push_back(b);
        while (bufs.size() > live) {
            Buf o = bufs.front();
            bufs.pop_front();
            CHECK(hipMemUnmap(o.p, o.size));
            if (free_va) CHECK(hipMemAddressFree(o.p, o.size));
            CHECK(hipMemRelease(o.h));
        }
        hipLaunchKernelGGL(k_fill, dim3(1024), dim3(256), 0, 0, canary, cn, 0u); // churn the canary too
        CHECK(hipDeviceSynchronize());
    }
    std::printf("done: %d rounds, %d reused VAs, %d failing rounds\n", rounds, reused, fails);
    return fails ? 1 : 0;
}
