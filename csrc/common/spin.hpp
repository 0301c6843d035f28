#pragma once
// Bounded busy-wait used before blocking on a condition variable in the latency-critical waits (master packets,
// P2P sink progress): a futex wake-up of a sleeping thread costs 10-50 us on a loaded host, several times the
// loopback round trip of a small collective. 50 us bound the spin per wait.
#include <sys/prctl.h>

#include <chrono>
#include <cstddef>

#include "types.hpp"

namespace pccl {

constexpr long spin_budget_us() { return 50; }

/// The short sleeps of the op threads (IPC barriers: 5 us) would otherwise round up to the default 50 us timer
/// slack; 1 us for the calling thread, once per thread.
inline void low_timer_slack() {
    static thread_local const bool done = [] { return prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0) == 0; }();
    (void)done;
}

/// Names the calling thread (at most 15 characters; shown in /proc/<pid>/task/*/comm): per-thread CPU accounting of
/// the ring (bench.py extra.cpu_by_thread) groups the process's threads by these names.
inline void name_thread(const char *name) { prctl(PR_SET_NAME, reinterpret_cast<unsigned long>(name), 0, 0, 0); }

/// Spins until pred() is true or the budget (us) is spent; returns pred()'s last value.
template <class Pred> inline bool spin_until(Pred &&pred, long budget = spin_budget_us()) {
    if (budget <= 0) return pred();
    const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(budget);
    for (unsigned i = 0;; ++i) {
        if (pred()) return true;
        if ((i & 63) == 63 && std::chrono::steady_clock::now() >= end) return pred();
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

} // namespace pccl
