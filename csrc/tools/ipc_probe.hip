// Probe of HIP IPC behaviour on the target box (informs the zero-copy design of the xGMI path):
//   ipc_probe export <dir>   allocates, exports base + interior pointers, times hipIpcGetMemHandle, writes handles,
//                            waits for <dir>/done
//   ipc_probe import <dir>   opens the handles, reports the returned addresses/offsets and reads the data back
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#define CHECK(x)                                                                                                     \
    do {                                                                                                             \
        hipError_t e_ = (x);                                                                                         \
        if (e_ != hipSuccess) {                                                                                      \
            std::printf("%s -> %s\n", #x, hipGetErrorString(e_));                                                   \
        }                                                                                                            \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void write_handle(const std::string &path, const hipIpcMemHandle_t &h, size_t offset) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char *>(&h), sizeof(h));
    f.write(reinterpret_cast<const char *>(&offset), sizeof(offset));
}

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const std::string mode = argv[1], dir = argv[2];
    const size_t bytes = 64ull << 20;
    if (mode == "export") {
        void *base = nullptr;
        CHECK(hipMalloc(&base, bytes));
        std::vector<uint32_t> host(bytes / 4);
        for (size_t i = 0; i < host.size(); ++i) host[i] = static_cast<uint32_t>(i);
        CHECK(hipMemcpy(base, host.data(), bytes, hipMemcpyHostToDevice));
        void *interior = static_cast<char *>(base) + (4 << 20);
        void *rb = nullptr;
        size_t rs = 0;
        CHECK(hipMemGetAddressRange(reinterpret_cast<hipDeviceptr_t *>(&rb), &rs, interior));
        std::printf("address range of interior: base %p (alloc %p) size %zu\n", rb, base, rs);
        hipIpcMemHandle_t hb{}, hi{}, hb2{};
        double t0 = now_us();
        CHECK(hipIpcGetMemHandle(&hb, base));
        double t1 = now_us();
        CHECK(hipIpcGetMemHandle(&hb2, base));
        double t2 = now_us();
        CHECK(hipIpcGetMemHandle(&hi, interior));
        double t3 = now_us();
        for (int i = 0; i < 100; ++i) CHECK(hipIpcGetMemHandle(&hb2, base));
        double t4 = now_us();
        std::printf("hipIpcGetMemHandle: first %.1f us, second %.1f us, interior %.1f us, 100x repeat avg %.2f us\n",
                    t1 - t0, t2 - t1, t3 - t2, (t4 - t3) / 100);
        std::printf("repeat handle identical: %d, interior handle == base handle: %d\n",
                    std::memcmp(&hb, &hb2, sizeof(hb)) == 0, std::memcmp(&hb, &hi, sizeof(hb)) == 0);
        write_handle(dir + "/base.h", hb, 0);
        write_handle(dir + "/interior.h", hi, 4 << 20);
        // free + realloc: same address? same handle?
        void *other = nullptr;
        CHECK(hipMalloc(&other, bytes));
        CHECK(hipFree(other));
        void *again = nullptr;
        CHECK(hipMalloc(&again, bytes));
        hipIpcMemHandle_t ha{};
        CHECK(hipIpcGetMemHandle(&ha, again));
        std::printf("realloc at %p (previous %p): handle differs from previous allocation's: %d\n", again, other,
                    std::memcmp(&ha, &hb, sizeof(ha)) != 0);
        std::ofstream(dir + "/ready") << "1";
        for (int i = 0; i < 600; ++i) {
            if (std::ifstream(dir + "/done").good()) break;
            std::this_thread::sleep_for(std::chrono::milliseconds(100));
        }
        return 0;
    }
    for (int i = 0; i < 600 && !std::ifstream(dir + "/ready").good(); ++i)
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
    for (const char *name : {"base.h", "interior.h"}) {
        std::ifstream f(dir + "/" + name, std::ios::binary);
        hipIpcMemHandle_t h{};
        size_t off = 0;
        f.read(reinterpret_cast<char *>(&h), sizeof(h));
        f.read(reinterpret_cast<char *>(&off), sizeof(off));
        void *p = nullptr;
        double t0 = now_us();
        CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        double t1 = now_us();
        uint32_t first = 0xffffffff;
        if (p) CHECK(hipMemcpy(&first, p, 4, hipMemcpyDeviceToHost));
        std::printf("open %s: %.1f us -> %p, first word %u (base word 0, interior word %zu)\n", name, t1 - t0, p, first,
                    off / 4);
        if (p) CHECK(hipIpcCloseMemHandle(p));
    }
    std::ofstream(dir + "/done") << "1";
    return 0;
}
