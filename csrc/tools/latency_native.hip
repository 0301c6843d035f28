// Native small-op latency harness (no Python in the loop): P threaded peers of one process on device 0, each with
// its own communicator, all-reduce `bytes` of bf16 device memory `iters` times back to back (one tag per op). With
// PCCL_TRACE_OPS=1 the library prints the phase marks of every op on stderr; this prints one JSON line with the
// per-op wall time (max over the peers of each op) median / p90 and the rank-0 median.
//   latency_native <master_port> <peers> <bytes> <iters> [warmup=50] [ipc=1]
// Build: hipcc --offload-arch=gfx950 -O2 -std=c++20 -Iinclude csrc/tools/latency_native.hip -Lpccl_amd/lib -lpccl
#include <hip/hip_runtime.h>
#include <pccl.h>

#include <algorithm>
#include <atomic>
#include <barrier>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        const pcclResult_t r_ = (x);                                                                                 \
        if (r_ != pcclSuccess) {                                                                                     \
            std::fprintf(stderr, "%s failed: %d\n", #x, static_cast<int>(r_));                                      \
            std::exit(1);                                                                                            \
        }                                                                                                            \
    } while (0)

static ccoip_socket_address_t loopback(uint16_t port) {
    ccoip_socket_address_t a{};
    a.inet.protocol = inetIPv4;
    a.inet.ipv4.data[0] = 127;
    a.inet.ipv4.data[3] = 1;
    a.port = port;
    return a;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s master_port peers bytes iters [warmup] [ipc]\n", argv[0]);
        return 2;
    }
    const uint16_t port = static_cast<uint16_t>(std::atoi(argv[1]));
    const int P = std::atoi(argv[2]);
    const size_t bytes = std::strtoull(argv[3], nullptr, 10);
    const int iters = std::atoi(argv[4]);
    const int warmup = argc > 5 ? std::atoi(argv[5]) : 50;
    if (argc > 6 && std::atoi(argv[6]) == 0) setenv("PCCL_DISABLE_IPC", "1", 1);
    CHECK(pcclInit());
    pcclMasterInstance_t *master = nullptr;
    CHECK(pcclCreateMaster(loopback(port), &master));
    CHECK(pcclRunMaster(master));

    const size_t n = bytes / 2;
    std::vector<std::vector<double>> t(P, std::vector<double>(iters));
    std::barrier sync(P);
    std::atomic<int> world_ok{0};
    int ndev = 0;
    const bool gpu = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0; // else host buffers (CPU debugging)
    auto peer = [&](int r) {
        if (gpu && hipSetDevice(0) != hipSuccess) std::exit(3);
        pcclCommCreateParams_t params{};
        params.master_address = loopback(port);
        params.p2p_connection_pool_size = 1;
        params.internal_p2p_listen_port = static_cast<uint16_t>(port + 1 + 3 * r);
        params.internal_shared_state_listen_port = static_cast<uint16_t>(port + 2 + 3 * r);
        params.internal_benchmark_listen_port = static_cast<uint16_t>(port + 3 + 3 * r);
        pcclComm_t *comm = nullptr;
        CHECK(pcclCreateCommunicator(&params, &comm));
        CHECK(pcclConnect(comm));
        // like pccl_amd.utils.wait_for_world: check the world size first (an accepted peer must not start an
        // update-topology vote that the others, already complete, never join)
        for (int ws = 0;;) {
            CHECK(pcclGetAttribute(comm, PCCL_ATTRIBUTE_GLOBAL_WORLD_SIZE, &ws));
            if (ws >= P) break;
            bool pending = false;
            CHECK(pcclArePeersPending(comm, &pending));
            if (pending) CHECK(pcclUpdateTopology(comm));
            else std::this_thread::sleep_for(std::chrono::milliseconds(5));
        }
        ++world_ok;
        void *src = nullptr, *dst = nullptr;
        if (gpu) {
            if (hipMalloc(&src, std::max<size_t>(bytes, 256)) != hipSuccess ||
                hipMalloc(&dst, std::max<size_t>(bytes, 256)) != hipSuccess)
                std::exit(4);
            (void) hipMemset(src, 0, bytes);
            (void) hipDeviceSynchronize();
        } else {
            src = std::calloc(1, std::max<size_t>(bytes, 256));
            dst = std::calloc(1, std::max<size_t>(bytes, 256));
        }
        pcclReduceDescriptor_t d{};
        d.count = n;
        d.op = pcclSum;
        d.src_descriptor.datatype = pcclBFloat16;
        d.src_descriptor.distribution_hint = pcclDistributionNone;
        d.quantization_options.quantized_datatype = pcclBFloat16;
        d.quantization_options.algorithm = pcclQuantNone;
        pcclReduceInfo_t info{};
        sync.arrive_and_wait();
        for (int i = 0; i < warmup + iters; ++i) {
            d.tag = static_cast<uint64_t>(i);
            const auto t0 = std::chrono::steady_clock::now();
            CHECK(pcclAllReduce(src, dst, &d, comm, &info));
            const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (i >= warmup) t[r][i - warmup] = s;
        }
        int path = 0;
        CHECK(pcclGetAttribute(comm, PCCL_ATTRIBUTE_LAST_REDUCE_PATH, &path));
        if (r == 0) std::fprintf(stderr, "path %d\n", path);
        sync.arrive_and_wait();
        CHECK(pcclDestroyCommunicator(comm));
        if (gpu) {
            (void) hipFree(src);
            (void) hipFree(dst);
        } else {
            std::free(src);
            std::free(dst);
        }
    };
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r) th.emplace_back(peer, r);
    for (auto &x : th) x.join();
    std::vector<double> mx(iters), r0 = t[0];
    for (int i = 0; i < iters; ++i)
        for (int r = 0; r < P; ++r) mx[i] = std::max(mx[i], t[r][i]);
    std::sort(mx.begin(), mx.end());
    std::sort(r0.begin(), r0.end());
    std::printf("{\"peers\": %d, \"bytes\": %zu, \"iters\": %d, \"median_us\": %.1f, \"p90_us\": %.1f, "
                "\"min_us\": %.1f, \"rank0_median_us\": %.1f}\n",
                P, bytes, iters, 1e6 * mx[iters / 2], 1e6 * mx[iters * 9 / 10], 1e6 * mx[0], 1e6 * r0[iters / 2]);
    CHECK(pcclInterruptMaster(master));
    CHECK(pcclMasterAwaitTermination(master));
    CHECK(pcclDestroyMaster(master));
    return 0;
}
