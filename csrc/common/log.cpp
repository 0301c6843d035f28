#include "log.hpp"

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <dlfcn.h>
#include <mutex>
#include <unistd.h>

namespace pccl {

static LogLevel parse_level() {
    const char *env = std::getenv("PCCL_LOG_LEVEL");
    if (env == nullptr) return LogLevel::ERR;
    struct {
        const char *name;
        LogLevel lvl;
    } table[] = {{"TRACE", LogLevel::TRACE}, {"DEBUG", LogLevel::DEBUG}, {"INFO", LogLevel::INFO},
                 {"WARN", LogLevel::WARN},   {"ERR", LogLevel::ERR},     {"ERROR", LogLevel::ERR},
                 {"FATAL", LogLevel::FATAL}, {"NONE", LogLevel::NONE}};
    for (const auto &e : table)
        if (std::strcmp(env, e.name) == 0) return e.lvl;
    return LogLevel::NONE; // unknown value disables logging (reference behavior)
}

static std::atomic<int> g_level{-1};

LogLevel current_log_level() {
    int v = g_level.load(std::memory_order_relaxed);
    if (v < 0) {
        v = static_cast<int>(parse_level());
        g_level.store(v, std::memory_order_relaxed);
    }
    return static_cast<LogLevel>(v);
}

void set_log_level(LogLevel level) { g_level.store(static_cast<int>(level)); }

LogLine::LogLine(LogLevel level, const char *file, int line) : level_(level) {
    static const char *names[] = {"TRACE", "DEBUG", "INFO", "WARN", "ERR", "FATAL", "BUG", "NONE"};
    const auto now = std::chrono::system_clock::now();
    const auto t = std::chrono::system_clock::to_time_t(now);
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(now.time_since_epoch()).count() % 1000;
    std::tm tm{};
    localtime_r(&t, &tm);
    char buf[64];
    std::strftime(buf, sizeof(buf), "%H:%M:%S", &tm);
    const char *base = std::strrchr(file, '/');
    stream_ << "[" << buf << "." << ms << "] [" << names[static_cast<int>(level)] << "] [pid " << getpid() << "] ["
            << (base ? base + 1 : file) << ":" << line << "] ";
}

LogLine::~LogLine() {
    static std::mutex mtx;
    stream_ << "\n";
    const std::string s = stream_.str();
    std::lock_guard lock(mtx);
    std::fwrite(s.data(), 1, s.size(), level_ >= LogLevel::WARN ? stderr : stdout);
    std::fflush(level_ >= LogLevel::WARN ? stderr : stdout);
}

} // namespace pccl

#include "trace.hpp"

namespace pccl {
bool trace_ops_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("PCCL_TRACE_OPS");
        return e != nullptr && e[0] != '\0' && e[0] != '0';
    }();
    return v;
}
const Roctx &roctx() {
    static const Roctx r = [] {
        Roctx x;
        const char *e = std::getenv("PCCL_ROCTX");
        if (e != nullptr && e[0] == '0') return x;
        void *h = nullptr;
        for (const char *lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                                "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"})
            if ((h = dlopen(lib, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (h == nullptr) return x;
        auto push = reinterpret_cast<int (*)(const char *)>(dlsym(h, "roctxRangePushA"));
        auto pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        auto mark = reinterpret_cast<void (*)(const char *)>(dlsym(h, "roctxMarkA"));
        if (push && pop && mark) {
            x.push = push;
            x.pop = pop;
            x.mark = mark;
        }
        return x;
    }();
    return r;
}
bool roctx_io_enabled() {
    static const bool v = [] {
        const char *e = std::getenv("PCCL_ROCTX_IO");
        return e != nullptr && e[0] == '1';
    }();
    return v;
}
OpTrace *&current_trace() {
    thread_local OpTrace *t = nullptr;
    return t;
}
} // namespace pccl
