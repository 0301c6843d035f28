// Per-op phase tracing (PCCL_TRACE_OPS=1): every collective prints one line with the time of each protocol /
// data-path phase since the op started, e.g.
//   [pccl-trace] tag 3 bytes 1073741824 path ipc ok commence 85us vote 140us copy_in 610us reduce 1402us ...
// Each op runs on its own thread, so the active trace is thread-local and the data paths just call trace_mark().
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

namespace pccl {

bool trace_ops_enabled();

struct OpTrace {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    std::vector<std::pair<const char *, double>> marks;
    void mark(const char *what) {
        marks.emplace_back(what, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::string str() const {
        std::string s;
        char buf[64];
        for (const auto &[k, us] : marks) {
            std::snprintf(buf, sizeof(buf), " %s %.0fus", k, us);
            s += buf;
        }
        return s;
    }
};

OpTrace *&current_trace();

// roctx ranges / markers for rocprofv3 (`--marker-trace`): the roctx library is dlopen'ed on first use (absent on
// CPU-only hosts: every call is then a no-op); PCCL_ROCTX=0 disables. Collectives and shared-state syncs are ranges,
// their protocol phases (the trace_mark points) are markers, so they line up with the kernels in a timeline.
struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
    void (*mark)(const char *) = nullptr;
};
const Roctx &roctx();

struct RoctxRange {
    bool on;
    explicit RoctxRange(const char *name) : on(roctx().push != nullptr) {
        if (on) roctx().push(name);
    }
    ~RoctxRange() {
        if (on) roctx().pop();
    }
    RoctxRange(const RoctxRange &) = delete;
    RoctxRange &operator=(const RoctxRange &) = delete;
};

// Per-frame I/O ranges (device-ring sends), only with PCCL_ROCTX_IO=1: thousands per large op, for timelines that
// show socket sends against copies and kernels (scripts/ring_overlap.py).
bool roctx_io_enabled();
struct RoctxIoRange {
    bool on;
    explicit RoctxIoRange(const char *name) : on(roctx_io_enabled() && roctx().push != nullptr) {
        if (on) roctx().push(name);
    }
    ~RoctxIoRange() {
        if (on) roctx().pop();
    }
    RoctxIoRange(const RoctxIoRange &) = delete;
    RoctxIoRange &operator=(const RoctxIoRange &) = delete;
};

inline void trace_mark(const char *what) {
    if (OpTrace *t = current_trace()) t->mark(what);
    if (const Roctx &r = roctx(); r.mark) r.mark(what);
}

} // namespace pccl
