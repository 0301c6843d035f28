// Threaded peers in the stream-ordered start path (pcclxAllReduce[Async]OnStream) on the host-emulated device backend
// (csrc/testing/hostdev_backend.cpp, PCCL_HIP_PLUGIN): the configuration of the round-5 SIGSEGV
// (profiles/r5/full2/crash.txt: two threaded peers of one process submitting stream-ordered ops concurrently, the
// caller's stream being the process-wide default stream) without a GPU, so that it runs under ThreadSanitizer.
//
//   stream_ordered_peers <peers> <iterations> <elements>
//
// Every peer thread: a "producer kernel" writes its input on a stream (the null stream, shared by every peer as
// torch's default stream is, or a stream of its own, alternating), then submits the all-reduce ordered after it on
// that stream - async or blocking, alternating - without synchronising the stream itself. The op must wait for the
// producer (which sleeps before it writes), so every result is the exact sum of the values written; the device ring
// runs over loopback TCP between the threads. Exit 0 and one JSON line on success.
#include <arpa/inet.h>
#include <dlfcn.h>
#include <netinet/in.h>
#include <pccl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

namespace {

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        const pcclResult_t r_ = (x);                                                                                 \
        if (r_ != pcclSuccess) {                                                                                     \
            std::fprintf(stderr, "%s failed: %d (line %d)\n", #x, static_cast<int>(r_), __LINE__);                  \
            std::exit(1);                                                                                            \
        }                                                                                                            \
    } while (0)

using FillFn = void (*)(void *, float *, size_t, float, unsigned);

ccoip_socket_address_t loopback(uint16_t port) {
    ccoip_socket_address_t a{};
    a.inet.protocol = inetIPv4;
    a.inet.ipv4.data[0] = 127;
    a.inet.ipv4.data[3] = 1;
    a.port = port;
    return a;
}

uint16_t free_port() {
    const int s = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    socklen_t len = sizeof(a);
    ::bind(s, reinterpret_cast<sockaddr *>(&a), sizeof(a));
    ::getsockname(s, reinterpret_cast<sockaddr *>(&a), &len);
    ::close(s);
    return ntohs(a.sin_port);
}

} // namespace

int main(int argc, char **argv) {
    const int peers = argc > 1 ? std::atoi(argv[1]) : 2;
    const int iters = argc > 2 ? std::atoi(argv[2]) : 20;
    const size_t n = argc > 3 ? std::strtoull(argv[3], nullptr, 10) : (1u << 20);
    const char *plugin = std::getenv("PCCL_HIP_PLUGIN");
    if (!plugin) {
        std::fprintf(stderr, "set PCCL_HIP_PLUGIN to libpccl_hostdev.so\n");
        return 2;
    }
    // the same object the library loads (dlopen of one path returns one handle): its fill entry point
    void *h = dlopen(plugin, RTLD_NOW);
    auto fill = h ? reinterpret_cast<FillFn>(dlsym(h, "pccl_hostdev_fill")) : nullptr;
    auto mk_stream = h ? reinterpret_cast<void *(*)()>(dlsym(h, "pccl_hostdev_create_stream")) : nullptr;
    if (!fill || !mk_stream) {
        std::fprintf(stderr, "not the host-emulated backend: %s\n", plugin);
        return 2;
    }
    CHECK(pcclInit());
    pcclMasterInstance_t *master = nullptr;
    const uint16_t master_port = free_port();
    CHECK(pcclCreateMaster(loopback(master_port), &master));
    CHECK(pcclRunMaster(master));

    std::atomic<int> bad{0}, done{0};
    std::vector<std::thread> th;
    for (int r = 0; r < peers; ++r)
        th.emplace_back([&, r] {
            pcclCommCreateParams_t params{};
            params.master_address = loopback(master_port);
            params.p2p_connection_pool_size = 2;
            pcclComm_t *comm = nullptr;
            CHECK(pcclCreateCommunicator(&params, &comm));
            CHECK(pcclConnect(comm));
            while (true) { // admit the others (every accepted peer votes on pending peers until the world is full)
                int ws = 0;
                CHECK(pcclGetAttribute(comm, PCCL_ATTRIBUTE_GLOBAL_WORLD_SIZE, &ws));
                if (ws >= peers) break;
                bool pending = false;
                CHECK(pcclArePeersPending(comm, &pending));
                if (pending) CHECK(pcclUpdateTopology(comm));
                else std::this_thread::sleep_for(std::chrono::milliseconds(5));
            }
            void *own = mk_stream();
            std::vector<float> x(n), y(n);
            for (int it = 0; it < iters; ++it) {
                void *stream = it % 2 ? own : nullptr; // the shared default stream, or a stream of this peer
                // producer: sleeps, then writes the input (the op must not read it before)
                fill(stream, x.data(), n, static_cast<float>(r + 1 + it), 2000);
                pcclReduceDescriptor_t d{};
                d.count = n;
                d.op = pcclSum;
                d.tag = static_cast<uint64_t>(it);
                d.src_descriptor.datatype = pcclFloat;
                d.quantization_options.quantized_datatype = pcclFloat;
                d.quantization_options.algorithm = pcclQuantNone;
                pcclReduceInfo_t info{};
                if (it % 4 < 2) {
                    pcclAsyncReduceOp_t op{};
                    CHECK(pcclxAllReduceAsyncOnStream(x.data(), y.data(), &d, comm, stream, &op));
                    CHECK(pcclAwaitAsyncReduce(&op, &info));
                } else {
                    CHECK(pcclxAllReduceOnStream(x.data(), y.data(), &d, comm, stream, &info));
                }
                float want = 0;
                for (int k = 0; k < peers; ++k) want += static_cast<float>(k + 1 + it);
                for (size_t i = 0; i < n; ++i)
                    if (y[i] != want) {
                        if (bad.fetch_add(1) < 5)
                            std::fprintf(stderr, "peer %d op %d: y[%zu] = %f, want %f\n", r, it, i, y[i], want);
                        break;
                    }
                int path = 0;
                CHECK(pcclGetAttribute(comm, PCCL_ATTRIBUTE_LAST_REDUCE_PATH, &path));
                if (path != 2) bad.fetch_add(1); // the device ring
            }
            done.fetch_add(1);
            CHECK(pcclDestroyCommunicator(comm));
        });
    for (auto &t : th) t.join();
    CHECK(pcclInterruptMaster(master));
    CHECK(pcclMasterAwaitTermination(master));
    CHECK(pcclDestroyMaster(master));
    std::printf("{\"peers\": %d, \"ops\": %d, \"elements\": %zu, \"bad\": %d}\n", peers, iters, n, bad.load());
    return bad.load() == 0 && done.load() == peers ? 0 : 3;
}
