#include "device_backend.hpp"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../kernels/host_kernels.hpp"
#include "log.hpp"

namespace pccl {

static DeviceBackend *g_backend = nullptr;
static std::once_flag g_once;

static std::string own_dir() {
    Dl_info info{};
    if (dladdr(reinterpret_cast<void *>(&own_dir), &info) == 0 || info.dli_fname == nullptr) return ".";
    std::string p(info.dli_fname);
    const auto pos = p.rfind('/');
    return pos == std::string::npos ? "." : p.substr(0, pos);
}

static void load_backend() {
    if (env_flag("PCCL_DISABLE_HIP", false)) {
        LOG(INFO) << "HIP backend disabled by PCCL_DISABLE_HIP";
        return;
    }
    const char *override_path = std::getenv("PCCL_HIP_PLUGIN");
    const std::string path = override_path ? std::string(override_path) : own_dir() + "/libpccl_hip.so";
    void *h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (h == nullptr) {
        LOG(INFO) << "HIP plugin not loadable (" << path << "): " << dlerror();
        return;
    }
    using Factory = DeviceBackend *(*)();
    auto f = reinterpret_cast<Factory>(dlsym(h, "pccl_create_hip_backend"));
    if (f == nullptr) {
        LOG(WARN) << "HIP plugin lacks pccl_create_hip_backend";
        return;
    }
    g_backend = f();
    if (g_backend == nullptr) {
        LOG(INFO) << "HIP plugin loaded but no HIP device is available";
    } else {
        LOG(INFO) << "HIP backend active: " << g_backend->device_count() << " device(s)";
    }
}

DeviceBackend *device_backend() {
    std::call_once(g_once, load_backend);
    return g_backend;
}

bool device_backend_available() { return device_backend() != nullptr; }

bool event_wait_polling(DeviceBackend *be, DevEvent e) {
    unsigned us = 2;
    while (true) {
        const int r = be->event_query(e);
        if (r != 0) return r == 1;
        std::this_thread::sleep_for(std::chrono::microseconds(us));
        us = std::min(us * 2, 100u);
    }
}

uint32_t device_crc32c(DeviceBackend *be, const void *dev_ptr, size_t n, DevStream s, bool *ok) {
    constexpr size_t kChunk = 64, kTile = 256 * kChunk, kMaxPartials = 1024;
    static const std::vector<uint32_t> tables = [] { // 8 slicing tables + tile-shift table, 12 x 256 words
        std::vector<uint32_t> t(12 * 256);
        const uint32_t(*sl)[256] = kernels::crc32c_tables();
        for (int k = 0; k < 8; ++k)
            for (int b = 0; b < 256; ++b) t[k * 256 + b] = sl[k][b];
        const uint32_t m = kernels::crc32c_x8n(kTile);
        for (int k = 0; k < 4; ++k)
            for (uint32_t b = 0; b < 256; ++b) t[(8 + k) * 256 + b] = kernels::crc32c_gf_mul(m, b << (8 * k));
        return t;
    }();
    static const std::vector<uint32_t> levels = [] {
        std::vector<uint32_t> l(8);
        for (int k = 0; k < 8; ++k) l[k] = kernels::crc32c_x8n(kChunk << k);
        return l;
    }();
    if (ok) *ok = true;
    if (n == 0) return 0;
    const auto *p = static_cast<const uint8_t *>(dev_ptr);
    const size_t head = std::min(n, (16 - reinterpret_cast<uintptr_t>(p) % 16) % 16);
    const size_t n_tiles = (n - head) / kTile;
    const size_t main = n_tiles * kTile;
    const size_t tail = n - head - main;
    std::vector<uint8_t> edge(head + tail);
    bool good = true;
    if (head) good = be->memcpy_sync(edge.data(), p, head);
    if (good && tail) good = be->memcpy_sync(edge.data() + head, p + head + main, tail);
    uint32_t raw = kernels::crc32c_raw_update(0, edge.data(), head);
    if (good && n_tiles) {
        std::vector<uint32_t> part(kMaxPartials);
        size_t np = 0, tpw = 0;
        good = be->crc32c_tiles(p + head, n_tiles, tables.data(), levels.data(), part.data(), part.size(), np, tpw, s);
        uint32_t main_raw = 0;
        const uint32_t full = kernels::crc32c_x8n(tpw * kTile);
        for (size_t g = 0; good && g < np; ++g) {
            const size_t tiles = std::min(tpw, n_tiles - g * tpw);
            const uint32_t m = tiles == tpw ? full : kernels::crc32c_x8n(tiles * kTile);
            main_raw = kernels::crc32c_gf_mul(m, main_raw) ^ part[g];
        }
        raw = kernels::crc32c_shift(raw, main) ^ main_raw;
    }
    raw = kernels::crc32c_raw_update(raw, edge.data() + head, tail);
    if (!good && ok) *ok = false;
    return kernels::crc32c_finish(raw, n);
}

} // namespace pccl
