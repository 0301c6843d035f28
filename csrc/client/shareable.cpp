#include "shareable.hpp"

#include <sys/types.h>
#include <unistd.h>

#include <iterator>
#include <map>
#include <mutex>

#include "../common/device_backend.hpp"
#include "../common/log.hpp"

namespace pccl::client::shareable {

namespace {
struct Alloc {
    size_t size = 0;
    int device = -1;
    uint64_t share_id = 0;
};
std::mutex g_mtx;
std::map<uintptr_t, Alloc> *g_allocs = new std::map<uintptr_t, Alloc>(); // never destroyed (static teardown order)
size_t g_bytes = 0;
} // namespace

void *alloc(size_t bytes, int device) {
    DeviceBackend *be = device_backend();
    if (!be) return nullptr;
    const int cur = be->current_device();
    if (device >= 0) be->set_device(device);
    else device = cur;
    int fd = -1;
    size_t size = 0;
    void *p = be->vmm_alloc(bytes, device, &fd, &size);
    if (cur >= 0 && cur != device) be->set_device(cur);
    if (!p) {
        LOG(ERR) << "shareable memory: VMM allocation of " << bytes << " bytes on device " << device << " failed";
        return nullptr;
    }
    const uint64_t id = VmmShare::instance().publish(fd);
    if (id == 0) {
        ::close(fd);
        be->vmm_free(p);
        LOG(ERR) << "shareable memory: cannot publish the allocation's fd";
        return nullptr;
    }
    std::lock_guard l(g_mtx);
    (*g_allocs)[reinterpret_cast<uintptr_t>(p)] = Alloc{size, device, id};
    g_bytes += size;
    return p;
}

void free(void *p) {
    Alloc a;
    {
        std::lock_guard l(g_mtx);
        auto it = g_allocs->find(reinterpret_cast<uintptr_t>(p));
        if (it == g_allocs->end()) return;
        a = it->second;
        g_bytes -= a.size;
        g_allocs->erase(it);
    }
    // peers that imported it keep their own reference until they unmap; new imports of this id fail from here on
    VmmShare::instance().retract(a.share_id);
    if (DeviceBackend *be = device_backend()) be->vmm_free(p);
}

bool lookup(const void *p, size_t bytes, Share &out) {
    const auto x = reinterpret_cast<uintptr_t>(p);
    std::lock_guard l(g_mtx);
    auto it = g_allocs->upper_bound(x);
    if (it == g_allocs->begin()) return false;
    --it;
    const uintptr_t base = it->first;
    const Alloc &a = it->second;
    if (x < base || x + bytes > base + a.size) return false;
    out.handle = VmmHandle{};
    out.handle.pid = static_cast<int32_t>(::getpid());
    out.handle.nonce = VmmShare::instance().nonce();
    out.handle.id = a.share_id;
    out.handle.size = a.size;
    out.offset = x - base;
    out.size = a.size;
    out.device = a.device;
    return true;
}

size_t live_allocations() {
    std::lock_guard l(g_mtx);
    return g_allocs->size();
}

size_t live_bytes() {
    std::lock_guard l(g_mtx);
    return g_bytes;
}

} // namespace pccl::client::shareable

// PyTorch pluggable-allocator entry points (torch.cuda.memory.CUDAPluggableAllocator): the stream argument is unused
// (VMM allocation is synchronous; the caching allocator orders reuse itself).
extern "C" __attribute__((visibility("default"))) void *pcclxShareableMalloc(ssize_t size, int device, void *stream) {
    (void)stream;
    return pccl::client::shareable::alloc(size > 0 ? static_cast<size_t>(size) : 1, device);
}

extern "C" __attribute__((visibility("default"))) void pcclxShareableFree(void *ptr, ssize_t size, int device,
                                                                          void *stream) {
    (void)size;
    (void)device;
    (void)stream;
    pccl::client::shareable::free(ptr);
}

extern "C" __attribute__((visibility("default"))) int pcclxShareableQuery(const void *p, size_t bytes,
                                                                          uint64_t *offset, size_t *alloc_size) {
    pccl::client::shareable::Share s;
    if (!pccl::client::shareable::lookup(p, bytes, s)) return 0;
    if (offset) *offset = s.offset;
    if (alloc_size) *alloc_size = s.size;
    return 1;
}

extern "C" __attribute__((visibility("default"))) size_t pcclxShareableLiveBytes() {
    return pccl::client::shareable::live_bytes();
}
