// ccoip_master: standalone master (coordinator) process (reference: ccoip_master/src/main.cpp).
// Usage: ccoip_master [--port P] [--ipv6]
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "pccl.h"

static pcclMasterInstance_t *g_master = nullptr;

static void on_signal(int) {
    if (g_master) pcclInterruptMaster(g_master);
}

int main(int argc, char **argv) {
    uint16_t port = 48148;
    bool v6 = false;
    for (int i = 1; i < argc; ++i) {
        if (std::strcmp(argv[i], "--port") == 0 && i + 1 < argc) port = static_cast<uint16_t>(std::atoi(argv[++i]));
        else if (std::strcmp(argv[i], "--ipv6") == 0) v6 = true;
        else {
            std::fprintf(stderr, "usage: %s [--port P] [--ipv6]\n", argv[0]);
            return 2;
        }
    }
    pcclInit();
    ccoip_socket_address_t addr{};
    addr.inet.protocol = v6 ? inetIPv6 : inetIPv4;
    addr.port = port;
    if (pcclCreateMaster(addr, &g_master) != pcclSuccess || pcclRunMaster(g_master) != pcclSuccess) {
        std::fprintf(stderr, "failed to start master on port %u\n", port);
        return 1;
    }
    std::signal(SIGINT, on_signal);
    std::signal(SIGTERM, on_signal);
    std::printf("ccoip_master listening on port %u\n", port);
    std::fflush(stdout);
    pcclMasterAwaitTermination(g_master);
    pcclDestroyMaster(g_master);
    return 0;
}
