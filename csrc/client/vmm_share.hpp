// Hands the POSIX fds of this process's exported VMM allocations (DeviceBackend::vmm_alloc) to peer processes on the
// same host: one service thread per process on a Unix domain socket in the abstract namespace
// ("\0pccl-vmm-<pid>-<nonce>"), fds travel with SCM_RIGHTS. A peer asks for an allocation id and receives its own
// copy of the fd, imports it (DeviceBackend::vmm_import) and closes the copy. The per-process random nonce is part of
// the socket name and of every handle, so a handle of a dead process never resolves in a new process that happens to
// reuse its pid. Only callers with this process's uid are served, and allocation ids are 64-bit random capabilities
// known only to the ring's peers (the socket name itself is public in /proc/net/unix).
#pragma once

#include <cstdint>
#include <cstring>

namespace pccl::client {

// Layout of a VMM share inside the 64-byte IPC handle field of the arena (distinguished from a hipIpcMemHandle_t by
// the magic).
struct VmmHandle {
    static constexpr uint32_t kMagic = 0x4d4d5650; // "PVMM"
    uint32_t magic = kMagic;
    int32_t pid = 0;
    uint64_t nonce = 0;
    uint64_t id = 0;
    uint64_t size = 0; // allocation size (granularity-rounded)
    static bool decode(const uint8_t *handle, VmmHandle &out) {
        std::memcpy(&out, handle, sizeof(VmmHandle));
        return out.magic == kMagic;
    }
};
static_assert(sizeof(VmmHandle) <= 64, "VMM share handle must fit the IPC handle field");

class VmmShare {
public:
    static VmmShare &instance();
    uint64_t nonce() const { return nonce_; }
    // registers an exported fd (the service owns and eventually closes it); returns its id (0 on failure)
    uint64_t publish(int fd);
    void retract(uint64_t id);
    // asks process `pid` (with `nonce`) for allocation `id`; returns a new fd owned by the caller, or -1
    static int fetch(int pid, uint64_t nonce, uint64_t id, int timeout_ms = 5000);

private:
    VmmShare();
    bool start();
    void serve();
    uint64_t nonce_;
    int listen_fd_ = -1;
    bool started_ = false;
};

} // namespace pccl::client
