#include "device_backend.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <mutex>
#include <string>

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

} // namespace pccl
