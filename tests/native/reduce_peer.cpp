// Native (C API) peer used by tests/test_native.py — the C++ counterpart of the reference's
// tests/basic_reduce_test and tests/concurrent_reduce_test, bounded and self-checking:
//   reduce_peer <master_port> <world> <steps> <num_ops> <elements> [pool] [max_in_flight]
// Every step: update topology (after the first), sync a shared state ("weights"), all-reduce `num_ops` tensors of
// ones with pcclAllReduceMultipleWithRetry (SUM, one tag each) and verify every element equals the world size.
#include <pccl.h>

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

int main(int argc, char **argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s port world steps num_ops elements [pool] [max_in_flight]\n", argv[0]);
        return 2;
    }
    const uint16_t port = static_cast<uint16_t>(std::atoi(argv[1]));
    const int world = std::atoi(argv[2]);
    const int steps = std::atoi(argv[3]);
    const size_t num_ops = std::strtoull(argv[4], nullptr, 10);
    const size_t n = std::strtoull(argv[5], nullptr, 10);
    const uint32_t pool = argc > 6 ? static_cast<uint32_t>(std::atoi(argv[6])) : 1;
    const int max_in_flight = argc > 7 ? std::atoi(argv[7]) : 8;

    CHECK(pcclInit());
    pcclCommCreateParams_t params{};
    params.master_address.inet.protocol = inetIPv4;
    params.master_address.inet.ipv4.data[0] = 127;
    params.master_address.inet.ipv4.data[3] = 1;
    params.master_address.port = port;
    params.peer_group = 0;
    params.p2p_connection_pool_size = pool;
    pcclComm_t *comm = nullptr;
    CHECK(pcclCreateCommunicator(&params, &comm));
    CHECK(pcclConnect(comm));

    std::vector<float> weights(n, 0.0f);
    std::vector<std::vector<float>> grads(num_ops, std::vector<float>(n));
    pcclTensorInfo_t info{};
    info.name = "weights";
    info.data = weights.data();
    info.count = n;
    info.datatype = pcclFloat;
    info.device_type = pcclDeviceCpu;
    info.allow_content_inequality = false;
    pcclSharedState_t state{};
    state.revision = 0;
    state.count = 1;
    state.infos = &info;

    int ws = 0, it = 0, done = 0, syncs = 0;
    while (done < steps) {
        if (it++ > 0) {
            bool pending = false;
            CHECK(pcclArePeersPending(comm, &pending));
            if (pending) CHECK(pcclUpdateTopology(comm));
        }
        CHECK(pcclGetAttribute(comm, PCCL_ATTRIBUTE_GLOBAL_WORLD_SIZE, &ws));
        if (ws < world) {
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
            continue;
        }
        pcclSharedStateSyncInfo_t sinfo{};
        CHECK(pcclSynchronizeSharedState(comm, &state, PCCL_SHARED_STATE_SYNC_STRATEGY_ENFORCE_POPULAR, &sinfo));
        if (++syncs > 1 && sinfo.rx_bytes != 0) {
            std::fprintf(stderr, "shared state drifted (rx %llu bytes)\n", static_cast<unsigned long long>(sinfo.rx_bytes));
            return 3;
        }
        std::vector<pcclReduceOpDescriptor_t> descs(num_ops);
        for (size_t j = 0; j < num_ops; ++j) {
            std::fill(grads[j].begin(), grads[j].end(), 1.0f);
            pcclReduceDescriptor_t d{};
            d.count = n;
            d.op = pcclSum;
            d.tag = j;
            d.src_descriptor.datatype = pcclFloat;
            d.src_descriptor.distribution_hint = pcclDistributionNone;
            d.quantization_options.quantized_datatype = pcclFloat;
            d.quantization_options.algorithm = pcclQuantNone;
            descs[j].sendbuf = grads[j].data();
            descs[j].recvbuf = grads[j].data();
            descs[j].descriptor = d;
        }
        pcclReduceInfo_t rinfo{};
        const auto t0 = std::chrono::steady_clock::now();
        CHECK(pcclAllReduceMultipleWithRetry(descs.data(), descs.size(), comm, &rinfo, max_in_flight));
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (size_t j = 0; j < num_ops; ++j)
            for (size_t k = 0; k < n; ++k)
                if (grads[j][k] != static_cast<float>(ws)) {
                    std::fprintf(stderr, "op %zu element %zu = %f, expected %d\n", j, k, grads[j][k], ws);
                    return 4;
                }
        for (size_t k = 0; k < n; ++k) weights[k] += 1.0f;
        ++state.revision;
        ++done;
        std::printf("{\"step\": %d, \"world\": %d, \"rx\": %llu, \"tx\": %llu, \"MBps\": %.1f}\n", done, ws,
                    static_cast<unsigned long long>(rinfo.rx_bytes), static_cast<unsigned long long>(rinfo.tx_bytes),
                    (rinfo.rx_bytes + rinfo.tx_bytes) / 1e6 / sec);
        std::fflush(stdout);
    }
    CHECK(pcclDestroyCommunicator(comm));
    return 0;
}
