// Bandwidth store + asymmetric TSP ring optimizer (replaces the reference's BandwidthStore and the absent libtsp;
// reference: ccoip/src/cpp/bandwidth_store.cpp, ccoip/src/cpp/topolgy_optimizer.cpp:6-182).
#pragma once

#include <cstdint>
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

// cost[i][j] < 0 means "no edge". Exact Held-Karp DP for n <= exact_limit, otherwise randomized
// nearest-neighbour construction + Or-opt/2-opt/3-opt-segment-insertion local search with restarts until
// `time_limit_ms`. Deterministic for a given seed.
AtspResult solve_atsp(const std::vector<std::vector<double>> &cost, int exact_limit, int time_limit_ms,
                      int restarts, uint64_t seed);

// Computes a ring order over `ring` using measured bandwidths (cost = 1000 / Mbit/s). `moonshot` widens the exact
// bound and search budget (the reference's "ImproveTopologyMoonshot").
bool optimize_ring(const BandwidthStore &store, std::vector<Uuid> &ring, bool moonshot, bool &is_optimal,
                   bool &improved);

double ring_cost(const BandwidthStore &store, const std::vector<Uuid> &ring);

} // namespace pccl::master
