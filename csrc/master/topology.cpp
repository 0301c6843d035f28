#include "topology.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <random>
#include <sstream>

#include "../common/log.hpp"

namespace pccl::master {

bool BandwidthStore::register_peer(const Uuid &u) { return peers_.insert(u).second; }

bool BandwidthStore::unregister_peer(const Uuid &u) {
    if (!peers_.erase(u)) return false;
    bw_.erase(u);
    for (auto &[_, m] : bw_) m.erase(u);
    return true;
}

bool BandwidthStore::store(const Uuid &from, const Uuid &to, double mbps) {
    if (!peers_.count(from) || !peers_.count(to)) return false;
    bw_[from][to] = mbps;
    return true;
}

std::optional<double> BandwidthStore::get(const Uuid &from, const Uuid &to) const {
    auto it = bw_.find(from);
    if (it == bw_.end()) return std::nullopt;
    auto jt = it->second.find(to);
    if (jt == it->second.end()) return std::nullopt;
    return jt->second;
}

std::vector<BandwidthEntry> BandwidthStore::missing_for(const Uuid &peer) const {
    std::vector<BandwidthEntry> out;
    if (!peers_.count(peer)) return out;
    for (const auto &o : peers_) {
        if (o == peer) continue;
        if (!get(peer, o)) out.push_back({peer, o});
        if (!get(o, peer)) out.push_back({o, peer});
    }
    return out;
}

bool BandwidthStore::fully_populated() const {
    for (const auto &a : peers_)
        for (const auto &b : peers_)
            if (a != b && !get(a, b)) return false;
    return true;
}

std::string BandwidthStore::dump() const {
    std::ostringstream os;
    for (const auto &[from, m] : bw_)
        for (const auto &[to, v] : m) os << from.str() << " -> " << to.str() << ": " << v << " Mbit/s\n";
    return os.str();
}

// ---------------------------------------------------------------------------------------------------------------
// ATSP
// ---------------------------------------------------------------------------------------------------------------
static constexpr double kInf = std::numeric_limits<double>::infinity();

static double tour_cost(const std::vector<std::vector<double>> &c, const std::vector<int> &t) {
    double s = 0;
    for (size_t i = 0; i < t.size(); ++i) {
        const double e = c[t[i]][t[(i + 1) % t.size()]];
        if (e < 0) return kInf;
        s += e;
    }
    return s;
}

static AtspResult held_karp(const std::vector<std::vector<double>> &c) {
    const int n = static_cast<int>(c.size());
    AtspResult r;
    const size_t full = size_t(1) << (n - 1); // subsets of {1..n-1}
    std::vector<float> dp(full * n, std::numeric_limits<float>::infinity());
    std::vector<int8_t> parent(full * n, -1);
    auto W = [&](int i, int j) -> float { return c[i][j] < 0 ? std::numeric_limits<float>::infinity() : float(c[i][j]); };
    for (int j = 1; j < n; ++j) dp[(size_t(1) << (j - 1)) * n + j] = W(0, j);
    for (size_t S = 1; S < full; ++S) {
        for (int j = 1; j < n; ++j) {
            if (!(S & (size_t(1) << (j - 1)))) continue;
            const float cur = dp[S * n + j];
            if (!std::isfinite(cur)) continue;
            for (int k = 1; k < n; ++k) {
                if (S & (size_t(1) << (k - 1))) continue;
                const size_t S2 = S | (size_t(1) << (k - 1));
                const float v = cur + W(j, k);
                if (v < dp[S2 * n + k]) {
                    dp[S2 * n + k] = v;
                    parent[S2 * n + k] = static_cast<int8_t>(j);
                }
            }
        }
    }
    float best = std::numeric_limits<float>::infinity();
    int last = -1;
    for (int j = 1; j < n; ++j) {
        const float v = dp[(full - 1) * n + j] + W(j, 0);
        if (v < best) {
            best = v;
            last = j;
        }
    }
    if (last < 0 || !std::isfinite(best)) return r;
    std::vector<int> rev;
    size_t S = full - 1;
    int j = last;
    while (j > 0) {
        rev.push_back(j);
        const int p = parent[S * n + j];
        S &= ~(size_t(1) << (j - 1));
        j = p;
    }
    r.tour.push_back(0);
    for (auto it = rev.rbegin(); it != rev.rend(); ++it) r.tour.push_back(*it);
    r.cost = tour_cost(c, r.tour);
    r.optimal = true;
    r.ok = std::isfinite(r.cost);
    return r;
}

static bool improve_local(const std::vector<std::vector<double>> &c, std::vector<int> &t, double &cost) {
    const int n = static_cast<int>(t.size());
    bool any = false;
    bool improved = true;
    while (improved) {
        improved = false;
        // Or-opt: move a segment of length 1..3 to another position (orientation preserved — ATSP safe)
        for (int len = 1; len <= 3 && len < n - 1; ++len) {
            for (int i = 0; i < n && !improved; ++i) {
                std::vector<int> seg, rest;
                for (int k = 0; k < len; ++k) seg.push_back(t[(i + k) % n]);
                for (int k = len; k < n; ++k) rest.push_back(t[(i + k) % n]);
                for (size_t pos = 0; pos <= rest.size() && !improved; ++pos) {
                    std::vector<int> cand(rest.begin(), rest.begin() + static_cast<long>(pos));
                    cand.insert(cand.end(), seg.begin(), seg.end());
                    cand.insert(cand.end(), rest.begin() + static_cast<long>(pos), rest.end());
                    const double cc = tour_cost(c, cand);
                    if (cc + 1e-12 < cost) {
                        t = cand;
                        cost = cc;
                        improved = any = true;
                    }
                }
            }
        }
        // 2-opt (segment reversal; recomputes the full asymmetric cost)
        for (int i = 0; i < n - 1 && !improved; ++i) {
            for (int j = i + 2; j < n && !improved; ++j) {
                std::vector<int> cand = t;
                std::reverse(cand.begin() + i + 1, cand.begin() + j + 1);
                const double cc = tour_cost(c, cand);
                if (cc + 1e-12 < cost) {
                    t = cand;
                    cost = cc;
                    improved = any = true;
                }
            }
        }
    }
    return any;
}

AtspResult solve_atsp(const std::vector<std::vector<double>> &cost, int exact_limit, int time_limit_ms, int restarts,
                      uint64_t seed) {
    const int n = static_cast<int>(cost.size());
    AtspResult r;
    if (n == 0) return r;
    if (n == 1) {
        r.tour = {0};
        r.ok = r.optimal = true;
        return r;
    }
    if (n <= exact_limit && n <= 20) {
        r = held_karp(cost);
        if (r.ok) return r;
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::mt19937_64 rng(seed);
    AtspResult best;
    best.cost = kInf;
    for (int rs = 0; rs < std::max(1, restarts); ++rs) {
        // randomized nearest neighbour
        std::vector<int> t;
        std::vector<bool> used(n, false);
        int cur = static_cast<int>(rng() % n);
        t.push_back(cur);
        used[cur] = true;
        for (int k = 1; k < n; ++k) {
            int nxt = -1;
            double bc = kInf;
            for (int j = 0; j < n; ++j) {
                if (used[j] || cost[cur][j] < 0) continue;
                const double noise = rs == 0 ? 0 : (rng() % 1000) * 1e-6 * cost[cur][j];
                if (cost[cur][j] + noise < bc) {
                    bc = cost[cur][j] + noise;
                    nxt = j;
                }
            }
            if (nxt < 0) // no edge: pick any unused (infeasible edge; local search may repair)
                for (int j = 0; j < n; ++j)
                    if (!used[j]) {
                        nxt = j;
                        break;
                    }
            t.push_back(nxt);
            used[nxt] = true;
            cur = nxt;
        }
        double c = tour_cost(cost, t);
        improve_local(cost, t, c);
        if (c < best.cost) {
            best.tour = t;
            best.cost = c;
        }
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > time_limit_ms) break;
    }
    best.ok = std::isfinite(best.cost);
    best.optimal = false;
    return best;
}

double ring_cost(const BandwidthStore &store, const std::vector<Uuid> &ring) {
    double s = 0;
    for (size_t i = 0; i < ring.size(); ++i) {
        auto bw = store.get(ring[i], ring[(i + 1) % ring.size()]);
        if (!bw || *bw <= 0) return kInf;
        s += 1000.0 / *bw;
    }
    return s;
}

bool optimize_ring(const BandwidthStore &store, std::vector<Uuid> &ring, bool moonshot, bool &is_optimal,
                   bool &improved) {
    improved = false;
    is_optimal = false;
    const int n = static_cast<int>(ring.size());
    if (n <= 3) { // every cyclic order of <= 3 peers in one direction... still directional for n == 3
        if (n <= 2) {
            is_optimal = true;
            return true;
        }
    }
    std::vector<std::vector<double>> cost(n, std::vector<double>(n, -1.0));
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            if (i == j) continue;
            auto bw = store.get(ring[i], ring[j]);
            if (bw && *bw > 0) cost[i][j] = 1000.0 / *bw;
        }
    const AtspResult r = moonshot ? solve_atsp(cost, 18, 30000, 16, 42) : solve_atsp(cost, 10, 1000, 4, 42);
    if (!r.ok) {
        LOG(WARN) << "ATSP solver found no feasible tour; keeping current ring";
        return false;
    }
    std::vector<Uuid> out;
    for (int idx : r.tour) out.push_back(ring[idx]);
    const double before = ring_cost(store, ring);
    if (r.cost + 1e-9 < before || !std::isfinite(before)) {
        ring = out;
        improved = true;
    }
    is_optimal = r.optimal;
    LOG(INFO) << "Topology optimization: cost " << before << " -> " << r.cost << (r.optimal ? " (optimal)" : " (approx)");
    return true;
}

} // namespace pccl::master
