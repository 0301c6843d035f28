// Minimal reproducer for the round-5 SIGSEGV in the stream-ordered start path (profiles/r5/full2/crash.txt): no
// pccl code, only the HIP runtime calls that path made, from the same thread layout.
//
// The crashed build called hipStreamQuery(<caller's stream>) on the submitting thread (the idle-stream shortcut of
// pcclxAllReduceAsyncOnStream) while other peer threads of the process recorded readiness events on their own
// current stream (torch's default stream, handle 0), and collective worker threads created pooled streams / events
// and launched kernels on them. Modes (one per process, so a crash names its mode):
//   record     - Q threads: hipEventRecord(e, 0) + hipEventQuery (the path that remains in the library)
//   query_own  - Q threads: hipStreamQuery on a stream each thread created (the shortcut on a non-default stream)
//   query_null - Q threads: hipStreamQuery(0) (the shortcut on torch's default stream, as in the crashed test)
//   mixed_null - Q threads: a kernel on stream 0 (torch's default stream, where the test's backward ran), then
//                hipStreamQuery(0), hipEventRecord(e, 0) and hipEventQuery(e) - every call of the crashed path at once
// Every mode also runs C churn threads: hipStreamCreate, a small kernel, hipEventCreate / Record / Synchronize,
// hipEventDestroy, hipStreamDestroy in a loop. Prints one JSON line; a crash shows as the process's signal.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

__global__ void k_touch(float *p, int n) {
    const int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x);
    if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        const hipError_t e_ = (x);                                                                                   \
        if (e_ != hipSuccess && e_ != hipErrorNotReady) {                                                           \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));                                     \
            std::exit(2);                                                                                            \
        }                                                                                                            \
    } while (0)

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "record";
    const double seconds = argc > 2 ? std::atof(argv[2]) : 10.0;
    const int nq = argc > 3 ? std::atoi(argv[3]) : 8, nc = argc > 4 ? std::atoi(argv[4]) : 8;
    const bool record = std::strcmp(mode, "record") == 0, own = std::strcmp(mode, "query_own") == 0,
               null_q = std::strcmp(mode, "query_null") == 0, mixed = std::strcmp(mode, "mixed_null") == 0;
    if (!record && !own && !null_q && !mixed) {
        std::fprintf(stderr,
                     "usage: %s record|query_own|query_null|mixed_null [seconds] [query threads] [churn threads]\n",
                     argv[0]);
        return 1;
    }
    CHECK(hipSetDevice(0));
    float *buf = nullptr;
    const int n = 1 << 16;
    CHECK(hipMalloc(&buf, sizeof(float) * n * (nc + nq + 1)));
    CHECK(hipMemset(buf, 0, sizeof(float) * n * (nc + nq + 1)));
    CHECK(hipDeviceSynchronize());
    std::atomic<bool> stop{false};
    std::atomic<unsigned long long> q_iters{0}, c_iters{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nq; ++t)
        th.emplace_back([&, t] {
            CHECK(hipSetDevice(0));
            hipStream_t mine = nullptr;
            if (own) CHECK(hipStreamCreateWithFlags(&mine, hipStreamNonBlocking));
            hipEvent_t e = nullptr;
            CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            unsigned long long it = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                if (record) {
                    CHECK(hipEventRecord(e, nullptr));
                    while (hipEventQuery(e) == hipErrorNotReady) {
                    }
                } else if (mixed) {
                    float *p = buf + static_cast<size_t>(nc + 1 + t) * n;
                    hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, nullptr, p, n);
                    CHECK(hipStreamQuery(nullptr));
                    CHECK(hipEventRecord(e, nullptr));
                    CHECK(hipEventQuery(e));
                } else if (own) {
                    if (it % 64 == 0) hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, mine, buf, n);
                    CHECK(hipStreamQuery(mine));
                } else {
                    CHECK(hipStreamQuery(nullptr));
                }
                ++it;
            }
            (void)t;
            CHECK(hipEventDestroy(e));
            if (mine) {
                CHECK(hipStreamSynchronize(mine));
                CHECK(hipStreamDestroy(mine));
            }
            q_iters += it;
        });
    for (int t = 0; t < nc; ++t)
        th.emplace_back([&, t] {
            CHECK(hipSetDevice(0));
            float *p = buf + static_cast<size_t>(t + 1) * n;
            unsigned long long it = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                hipStream_t s = nullptr;
                hipEvent_t e = nullptr;
                CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
                CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, s, p, n);
                CHECK(hipEventRecord(e, s));
                CHECK(hipEventSynchronize(e));
                CHECK(hipEventDestroy(e));
                CHECK(hipStreamDestroy(s));
                ++it;
            }
            c_iters += it;
        });
    const auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
        std::fprintf(stderr, ".");
    }
    stop = true;
    for (auto &x : th) x.join();
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    std::printf("{\"mode\": \"%s\", \"seconds\": %.1f, \"query_threads\": %d, \"churn_threads\": %d, "
                "\"query_iters\": %llu, \"churn_iters\": %llu, \"crashed\": false}\n",
                mode, seconds, nq, nc, q_iters.load(), c_iters.load());
    return 0;
}
