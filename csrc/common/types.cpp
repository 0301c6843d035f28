#include "types.hpp"

#include <arpa/inet.h>
#include <atomic>
#include <csignal>
#include <dirent.h>
#include <execinfo.h>
#include <mutex>
#include <sys/syscall.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <thread>
#include <fcntl.h>
#include <random>
#include <string>
#include <unistd.h>
#include <vector>

namespace pccl {

const char *dtype_name(DType t) {
    switch (t) {
        case DType::U8: return "uint8";
        case DType::I8: return "int8";
        case DType::U16: return "uint16";
        case DType::U32: return "uint32";
        case DType::I16: return "int16";
        case DType::I32: return "int32";
        case DType::U64: return "uint64";
        case DType::I64: return "int64";
        case DType::F16: return "float16";
        case DType::BF16: return "bfloat16";
        case DType::F32: return "float32";
        case DType::F64: return "float64";
        case DType::F8E4M3: return "float8_e4m3";
        case DType::F8E5M2: return "float8_e5m2";
    }
    return "?";
}

std::string Uuid::str() const {
    char buf[40];
    int p = 0;
    for (size_t i = 0; i < 16; ++i) {
        if (i == 4 || i == 6 || i == 8 || i == 10) buf[p++] = '-';
        p += std::snprintf(buf + p, sizeof(buf) - p, "%02x", data[i]);
    }
    return std::string(buf, p);
}

Uuid Uuid::random() {
    // UUIDv4 from the kernel CSPRNG (fallback: random_device)
    Uuid u;
    bool ok = false;
    const int fd = ::open("/dev/urandom", O_RDONLY | O_CLOEXEC);
    if (fd >= 0) {
        ok = ::read(fd, u.data.data(), 16) == 16;
        ::close(fd);
    }
    if (!ok) {
        std::random_device rd;
        for (auto &b : u.data) b = static_cast<uint8_t>(rd());
    }
    u.data[6] = (u.data[6] & 0x0f) | 0x40;
    u.data[8] = (u.data[8] & 0x3f) | 0x80;
    return u;
}

std::string sockaddr_str(const SockAddr &a) {
    char buf[INET6_ADDRSTRLEN + 16];
    if (a.inet.protocol == inetIPv4) {
        inet_ntop(AF_INET, a.inet.ipv4.data, buf, sizeof(buf));
        return std::string(buf) + ":" + std::to_string(a.port);
    }
    inet_ntop(AF_INET6, a.inet.ipv6.data, buf, sizeof(buf));
    return "[" + std::string(buf) + "]:" + std::to_string(a.port);
}

bool sockaddr_equal(const SockAddr &a, const SockAddr &b) { return SockAddrKey::of(a) == SockAddrKey::of(b); }

bool sockaddr_is_loopback(const SockAddr &a) {
    if (a.inet.protocol == inetIPv4) return a.inet.ipv4.data[0] == 127;
    for (int i = 0; i < 15; ++i)
        if (a.inet.ipv6.data[i] != 0) return false;
    return a.inet.ipv6.data[15] == 1;
}

bool sockaddr_is_zero(const SockAddr &a) {
    if (a.port != 0) return false;
    if (a.inet.protocol == inetIPv4) {
        for (auto b : a.inet.ipv4.data)
            if (b) return false;
        return true;
    }
    for (auto b : a.inet.ipv6.data)
        if (b) return false;
    return true;
}

SockAddr make_sockaddr_v4(uint8_t a, uint8_t b, uint8_t c, uint8_t d, uint16_t port) {
    SockAddr s{};
    s.inet.protocol = inetIPv4;
    s.inet.ipv4.data[0] = a;
    s.inet.ipv4.data[1] = b;
    s.inet.ipv4.data[2] = c;
    s.inet.ipv4.data[3] = d;
    s.port = port;
    return s;
}

SockAddrKey SockAddrKey::of(const SockAddr &a) {
    SockAddrKey k;
    k.v4 = a.inet.protocol == inetIPv4;
    if (k.v4)
        std::memcpy(k.ip.data(), a.inet.ipv4.data, 4);
    else
        std::memcpy(k.ip.data(), a.inet.ipv6.data, 16);
    k.port = a.port;
    return k;
}

namespace {
struct FaultSpec {
    std::string point, phase;
    uint64_t seq = 0;
    size_t step = SIZE_MAX; // SIZE_MAX: any
    bool armed = false;
};
const FaultSpec &fault_spec() {
    static const FaultSpec s = [] {
        FaultSpec f;
        const char *e = std::getenv("PCCL_FAULT_INJECT");
        if (!e || !*e) return f;
        std::vector<std::string> parts;
        std::string cur;
        for (const char *p = e;; ++p) {
            if (*p == ':' || *p == 0) {
                parts.push_back(cur);
                cur.clear();
                if (*p == 0) break;
            } else {
                cur += *p;
            }
        }
        if (parts.size() < 2) return f;
        f.point = parts[0];
        f.seq = std::strtoull(parts[1].c_str(), nullptr, 10);
        if (parts.size() > 2 && !parts[2].empty()) f.step = std::strtoull(parts[2].c_str(), nullptr, 10);
        if (parts.size() > 3) f.phase = parts[3];
        f.armed = true;
        return f;
    }();
    return s;
}
} // namespace

bool fault_injection_armed() { return fault_spec().armed; }

void fault_point(const char *point, uint64_t seq, size_t step, const char *phase) {
    const FaultSpec &f = fault_spec();
    if (!f.armed || f.seq != seq || f.point != point) return;
    if (f.step != SIZE_MAX && f.step != step) return;
    if (!f.phase.empty() && (phase == nullptr || f.phase != phase)) return;
    // PCCL_FAULT_SIGNAL=STOP: the process stops instead of dying (SIGSTOP: sockets stay open, the kernel keeps
    // ACKing; the harness resumes it with SIGCONT), the failure mode keepalive never detects
    static const bool stop = [] {
        const char *e = std::getenv("PCCL_FAULT_SIGNAL");
        return e && (std::strcmp(e, "STOP") == 0 || std::strcmp(e, "SIGSTOP") == 0);
    }();
    const int sig = stop ? SIGSTOP : SIGKILL;
    // wall-clock time of the kill (harnesses time recovery from it: benchmarks/fault_tolerance.py)
    timespec now{};
    ::clock_gettime(CLOCK_REALTIME, &now);
    std::fprintf(stderr, "[pccl] fault injection: %s at %s seq %llu step %lld phase %s t=%lld.%06ld\n",
                 stop ? "SIGSTOP" : "SIGKILL", point, static_cast<unsigned long long>(seq),
                 step == SIZE_MAX ? -1ll : static_cast<long long>(step), phase ? phase : "-",
                 static_cast<long long>(now.tv_sec), now.tv_nsec / 1000);
    std::fflush(stderr);
    if (const char *d = std::getenv("PCCL_FAULT_INJECT_DELAY_MS")) // die a little later (the point's work goes on)
        std::thread([ms = std::atol(d), sig] {
            ::usleep(static_cast<useconds_t>(ms) * 1000);
            ::kill(::getpid(), sig);
        }).detach();
    else
        ::kill(::getpid(), sig);
}

void fault_stall(const char *point, uint64_t seq) {
    static const char *spec = std::getenv("PCCL_FAULT_STALL");
    if (!spec || !*spec) return;
    const char *c1 = std::strchr(spec, ':');
    if (!c1 || std::strncmp(spec, point, static_cast<size_t>(c1 - spec)) != 0 || point[c1 - spec] != 0) return;
    char *end = nullptr;
    const unsigned long long max_seq = std::strtoull(c1 + 1, &end, 10);
    if (!end || *end != ':' || seq > max_seq) return;
    ::usleep(static_cast<useconds_t>(std::atol(end + 1)) * 1000);
}

namespace {
const std::string &fault_delay_spec() {
    static const std::string spec = [] {
        const char *e = std::getenv("PCCL_FAULT_DELAY");
        return std::string(e ? e : "");
    }();
    return spec;
}
} // namespace

bool fault_delay_armed() { return !fault_delay_spec().empty(); }

void fault_delay(uint64_t tag) {
    const std::string &spec = fault_delay_spec();
    if (spec.empty()) return;
    long ms = -1, any_ms = -1;
    size_t pos = 0;
    while (pos < spec.size()) {
        const size_t end = std::min(spec.find(',', pos), spec.size());
        const std::string item = spec.substr(pos, end - pos);
        const size_t colon = item.find(':');
        if (colon != std::string::npos) {
            const long v = std::atol(item.c_str() + colon + 1);
            if (item.compare(0, colon, "*") == 0) any_ms = v;
            else if (std::strtoull(item.c_str(), nullptr, 10) == tag) ms = v;
        }
        pos = end + 1;
    }
    if (ms < 0) ms = any_ms;
    if (ms > 0) ::usleep(static_cast<useconds_t>(ms) * 1000);
}

namespace {
std::atomic<int> g_bt_pending{0};
void bt_handler(int) {
    void *frames[64];
    const int n = ::backtrace(frames, 64);
    char hdr[64];
    const int k = std::snprintf(hdr, sizeof(hdr), "[pccl] backtrace tid %ld:\n", static_cast<long>(::syscall(SYS_gettid)));
    if (k > 0) (void)!::write(2, hdr, static_cast<size_t>(k));
    ::backtrace_symbols_fd(frames, n, 2);
    if (g_bt_pending.fetch_add(1) == 0) { // the first thread to get the signal forwards it to every other thread
        DIR *d = ::opendir("/proc/self/task");
        if (d) {
            const long me = static_cast<long>(::syscall(SYS_gettid));
            while (dirent *e = ::readdir(d)) {
                const long tid = std::atol(e->d_name);
                if (tid > 0 && tid != me) ::syscall(SYS_tgkill, ::getpid(), tid, SIGUSR2);
            }
            ::closedir(d);
        }
    }
}
// fatal signals (PCCL_DEBUG_BACKTRACE_SIGNAL): the faulting thread's native frames, then the handler that was
// installed before (e.g. Python's faulthandler, which adds the Python stacks) or the default action
struct sigaction g_prev_fatal[32];
void fatal_handler(int sig, siginfo_t *info, void *uctx) {
    void *frames[64];
    const int n = ::backtrace(frames, 64);
    char hdr[96];
    const int k = std::snprintf(hdr, sizeof(hdr), "[pccl] fatal signal %d (addr %p) tid %ld:\n", sig,
                                info ? info->si_addr : nullptr, static_cast<long>(::syscall(SYS_gettid)));
    if (k > 0) (void)!::write(2, hdr, static_cast<size_t>(k));
    ::backtrace_symbols_fd(frames, n, 2);
    const struct sigaction &prev = g_prev_fatal[sig & 31];
    if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) {
        prev.sa_sigaction(sig, info, uctx);
    } else if (prev.sa_handler != SIG_DFL && prev.sa_handler != SIG_IGN && prev.sa_handler != nullptr) {
        prev.sa_handler(sig);
    } else {
        ::signal(sig, SIG_DFL);
        ::raise(sig);
    }
}
} // namespace

void install_debug_backtrace_signal() {
    static std::once_flag once;
    std::call_once(once, [] {
        if (!env_flag("PCCL_DEBUG_BACKTRACE_SIGNAL", false)) return;
        void *warm[2];
        (void)::backtrace(warm, 2); // loads the unwinder outside of signal context
        struct sigaction sa{};
        sa.sa_handler = bt_handler;
        sa.sa_flags = SA_RESTART;
        ::sigaction(SIGUSR2, &sa, nullptr);
        for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL}) {
            struct sigaction fa{};
            fa.sa_sigaction = fatal_handler;
            fa.sa_flags = SA_SIGINFO | SA_RESETHAND;
            ::sigaction(sig, &fa, &g_prev_fatal[sig & 31]);
        }
    });
}

size_t env_size(const char *name, size_t dflt) {
    const char *v = std::getenv(name);
    if (v == nullptr || *v == 0) return dflt;
    char *end = nullptr;
    const unsigned long long x = std::strtoull(v, &end, 10);
    if (end == v) return dflt;
    return static_cast<size_t>(x);
}

bool env_flag(const char *name, bool dflt) {
    const char *v = std::getenv(name);
    if (v == nullptr || *v == 0) return dflt;
    return !(v[0] == '0' || v[0] == 'f' || v[0] == 'F' || v[0] == 'n' || v[0] == 'N');
}

} // namespace pccl
