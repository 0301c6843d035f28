// Bandwidth store + asymmetric TSP ring optimizer (replaces the reference's BandwidthStore and the absent libtsp;
// reference: ccoip/src/cpp/bandwidth_store.cpp, ccoip/src/cpp/topolgy_optimizer.cpp:6-182).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <map>
#include <optional>
#include <set>
#include <unordered_map>
#include <vector>

#include "../common/types.hpp"

namespace pccl::master {

struct BandwidthEntry {
    Uuid from, to;
};

class BandwidthStore {
public:
    bool register_peer(const Uuid &u);
    bool unregister_peer(const Uuid &u);
    bool store(const Uuid &from, const Uuid &to, double mbps);
    std::optional<double> get(const Uuid &from, const Uuid &to) const;
    std::vector<BandwidthEntry> missing_for(const Uuid &peer) const; // edges touching `peer` without a measurement
    bool fully_populated() const;
    size_t num_peers() const { return peers_.size(); }
    std::string dump() const;

private:
    std::set<Uuid> peers_;
    std::map<Uuid, std::map<Uuid, double>> bw_;
};

struct AtspResult {
    std::vector<int> tour;
    double cost = 0;
    bool optimal = false;
    bool ok = false;
};

// cost[i][j] < 0 means "no edge". Exact Held-Karp DP for n <= exact_limit (at most 20), otherwise randomised
// construction + iterated local search (Or-opt, or-3opt segment swap, 2-opt; double-bridge kicks) with `restarts`
// restarts inside `time_limit_ms`. A set `cancel` ends the search early (best tour so far). Deterministic for a given
// seed when the time budget does not bind.
AtspResult solve_atsp(const std::vector<std::vector<double>> &cost, int exact_limit, int time_limit_ms,
                      int restarts, uint64_t seed, const std::atomic<bool> *cancel = nullptr);

// Computes a ring order over `ring` using measured bandwidths (cost = 1000 / Mbit/s). `moonshot` widens the exact
// bound and search budget (the reference's "ImproveTopologyMoonshot").
bool optimize_ring(const BandwidthStore &store, std::vector<Uuid> &ring, bool moonshot, bool &is_optimal,
                   bool &improved, const std::atomic<bool> *cancel = nullptr);

// Bounded worker pool for the asynchronous (moonshot) optimizations, like the reference master's thread pool of 4
// threads with a queue of 64 (ccoip_master_handler.cpp:13-14): at most `threads` workers, at most `queue` waiting
// tasks (submit() returns false beyond that), one task per key (a group) queued or running at a time.
class OptimizerPool {
public:
    OptimizerPool(size_t threads, size_t queue) : max_threads_(threads), max_queue_(queue) {}
    ~OptimizerPool(); // cancels waiting tasks, joins the workers
    bool submit(uint64_t key, std::function<void()> fn);
    size_t thread_count();
    size_t pending();
    void stop();

private:
    void loop();
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::pair<uint64_t, std::function<void()>>> q_;
    std::set<uint64_t> active_; // keys queued or running
    std::vector<std::thread> threads_;
    size_t idle_ = 0;
    const size_t max_threads_, max_queue_;
    bool stop_ = false;
};

double ring_cost(const BandwidthStore &store, const std::vector<Uuid> &ring);

} // namespace pccl::master
