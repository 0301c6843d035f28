#include "topology.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <random>
#include <sstream>

#include "../common/log.hpp"
#include "../common/spin.hpp"

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

// ---- heuristic: iterated local search over ATSP-safe moves with O(1) move deltas
//
// The reference hands the ring to libtsp (exact up to 8 / 20 nodes, else 3-opt + tabu + ant-colony sampling with
// restarts; topolgy_optimizer.cpp:52-60,136-144). Here: randomised construction (nearest neighbour with noise, or a
// random tour), then a first-improvement local search over
//   * Or-opt: move a segment of 1..3 nodes elsewhere, orientation kept (pure ATSP move);
//   * or-3opt "segment swap": A S1 S2 B -> A S2 S1 B, the 3-opt reconnection that reverses nothing (pure ATSP move);
//   * 2-opt with reversal, priced exactly through forward / backward prefix sums of the current tour;
// and double-bridge kicks (A B C D -> A C B D, orientation-preserving) to leave local optima, accepting a kicked tour
// when it is no worse (iterated local search). Restarts and the time budget follow the caller's (reference) budgets.
namespace {

struct Tour {
    const std::vector<std::vector<double>> &c;
    std::vector<int> t;
    std::vector<double> fwd, bwd; // fwd[i] = sum c[t[k]][t[k+1]], bwd[i] = sum c[t[k+1]][t[k]], k < i
    explicit Tour(const std::vector<std::vector<double>> &cc, std::vector<int> tt) : c(cc), t(std::move(tt)) { rebuild(); }
    int n() const { return static_cast<int>(t.size()); }
    double w(int a, int b) const { return c[a][b] < 0 ? 1e18 : c[a][b]; } // missing edge: prohibitive, not fatal
    void rebuild() {
        const int N = n();
        fwd.assign(N, 0);
        bwd.assign(N, 0);
        for (int i = 1; i < N; ++i) {
            fwd[i] = fwd[i - 1] + w(t[i - 1], t[i]);
            bwd[i] = bwd[i - 1] + w(t[i], t[i - 1]);
        }
    }
    double cost() const {
        double s = 0;
        for (int i = 0; i < n(); ++i) s += w(t[i], t[(i + 1) % n()]);
        return s;
    }
    // internal cost of t[i..j] (i <= j) forward and reversed
    double inner_fwd(int i, int j) const { return fwd[j] - fwd[i]; }
    double inner_bwd(int i, int j) const { return bwd[j] - bwd[i]; }
};

// Or-opt: segment t[i..i+len-1] (not wrapping) moved between t[p] and t[p+1] (p outside the segment)
bool or_opt_pass(Tour &T) {
    const int N = T.n();
    auto &t = T.t;
    for (int len = 1; len <= 3 && len < N - 2; ++len) {
        for (int i = 0; i + len <= N; ++i) {
            const int j = i + len - 1;
            const int prev = t[(i - 1 + N) % N], next = t[(j + 1) % N];
            const double remove = T.w(prev, t[i]) + T.w(t[j], next) - T.w(prev, next);
            for (int p = 0; p < N; ++p) {
                if (p >= i - 1 && p <= j) continue; // inserting next to its own position changes nothing
                const int a = t[p], b = t[(p + 1) % N];
                if ((p + 1) % N >= i && (p + 1) % N <= j) continue;
                const double gain = remove - (T.w(a, t[i]) + T.w(t[j], b) - T.w(a, b));
                if (gain > 1e-9) {
                    std::vector<int> seg(t.begin() + i, t.begin() + j + 1), rest;
                    rest.reserve(N - len);
                    for (int k = 0; k < N; ++k)
                        if (k < i || k > j) rest.push_back(t[k]);
                    const int pos = static_cast<int>(std::find(rest.begin(), rest.end(), a) - rest.begin()) + 1;
                    rest.insert(rest.begin() + pos, seg.begin(), seg.end());
                    t = std::move(rest);
                    T.rebuild();
                    return true;
                }
            }
        }
    }
    return false;
}

// segment swap (or-3opt): t[0..i] S1=t[i+1..j] S2=t[j+1..k] t[k+1..] -> t[0..i] S2 S1 t[k+1..]
bool swap_pass(Tour &T) {
    const int N = T.n();
    auto &t = T.t;
    for (int i = 0; i < N - 2; ++i)
        for (int j = i + 1; j < N - 1; ++j)
            for (int k = j + 1; k < N; ++k) {
                const int a = t[i], s1 = t[i + 1], e1 = t[j], s2 = t[j + 1], e2 = t[k], b = t[(k + 1) % N];
                if (b == s1) continue; // S1 S2 cover the whole cycle after a
                const double gain = (T.w(a, s1) + T.w(e1, s2) + T.w(e2, b)) - (T.w(a, s2) + T.w(e2, s1) + T.w(e1, b));
                if (gain > 1e-9) {
                    std::rotate(t.begin() + i + 1, t.begin() + j + 1, t.begin() + k + 1);
                    T.rebuild();
                    return true;
                }
            }
    return false;
}

// 2-opt: reverse t[i+1..j]; the reversed inner edges change direction (priced through the prefix sums)
bool two_opt_pass(Tour &T) {
    const int N = T.n();
    auto &t = T.t;
    for (int i = 0; i < N - 2; ++i)
        for (int j = i + 2; j < N; ++j) {
            const int a = t[i], s = t[i + 1], e = t[j], b = t[(j + 1) % N];
            if (b == a) continue;
            const double before = T.w(a, s) + T.inner_fwd(i + 1, j) + T.w(e, b);
            const double after = T.w(a, e) + T.inner_bwd(i + 1, j) + T.w(s, b);
            if (before - after > 1e-9) {
                std::reverse(t.begin() + i + 1, t.begin() + j + 1);
                T.rebuild();
                return true;
            }
        }
    return false;
}

void local_search(Tour &T, const std::chrono::steady_clock::time_point &deadline, const std::atomic<bool> *cancel) {
    while (std::chrono::steady_clock::now() < deadline && !(cancel && cancel->load(std::memory_order_relaxed))) {
        if (or_opt_pass(T) || swap_pass(T) || two_opt_pass(T)) continue;
        break;
    }
}

std::vector<int> double_bridge(const std::vector<int> &t, std::mt19937_64 &rng) {
    const int N = static_cast<int>(t.size());
    std::vector<int> cut = {1 + static_cast<int>(rng() % (N - 1)), 1 + static_cast<int>(rng() % (N - 1)),
                            1 + static_cast<int>(rng() % (N - 1))};
    std::sort(cut.begin(), cut.end());
    std::vector<int> out(t.begin(), t.begin() + cut[0]);
    out.insert(out.end(), t.begin() + cut[1], t.begin() + cut[2]);
    out.insert(out.end(), t.begin() + cut[0], t.begin() + cut[1]);
    out.insert(out.end(), t.begin() + cut[2], t.end());
    return out;
}

std::vector<int> construct(const std::vector<std::vector<double>> &cost, std::mt19937_64 &rng, int variant) {
    const int n = static_cast<int>(cost.size());
    std::vector<int> t;
    if (variant % 3 == 2) { // random tour (libtsp's TSP_INIT_RANDOM_STRATEGY)
        t.resize(n);
        for (int i = 0; i < n; ++i) t[i] = i;
        std::shuffle(t.begin(), t.end(), rng);
        return t;
    }
    std::vector<bool> used(n, false);
    int cur = static_cast<int>(rng() % n);
    t.push_back(cur);
    used[cur] = true;
    for (int k = 1; k < n; ++k) { // nearest neighbour, noisy after the first restart
        int nxt = -1;
        double bc = kInf;
        for (int j = 0; j < n; ++j) {
            if (used[j] || cost[cur][j] < 0) continue;
            const double noise = variant == 0 ? 0 : (rng() % 1000) * 2e-4 * cost[cur][j];
            if (cost[cur][j] + noise < bc) {
                bc = cost[cur][j] + noise;
                nxt = j;
            }
        }
        if (nxt < 0)
            for (int j = 0; j < n; ++j)
                if (!used[j]) {
                    nxt = j;
                    break;
                }
        t.push_back(nxt);
        used[nxt] = true;
        cur = nxt;
    }
    return t;
}

} // namespace

AtspResult solve_atsp(const std::vector<std::vector<double>> &cost, int exact_limit, int time_limit_ms, int restarts,
                      uint64_t seed, const std::atomic<bool> *cancel) {
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
    const auto deadline = t0 + std::chrono::milliseconds(std::max(1, time_limit_ms));
    std::mt19937_64 rng(seed);
    AtspResult best;
    best.cost = kInf;
    const int R = std::max(1, restarts);
    // kicks per restart without improvement before moving on (the budget ends earlier on large instances)
    const int patience = std::max(50, 20 * n);
    for (int rs = 0; rs < R; ++rs) {
        Tour T(cost, construct(cost, rng, rs));
        // each restart gets an equal share of what is left of the budget
        const auto now = std::chrono::steady_clock::now();
        if (now >= deadline && best.ok) break;
        const auto share = (deadline - now) / (R - rs);
        const auto rs_deadline = now + share;
        local_search(T, rs_deadline, cancel);
        double cur = T.cost();
        std::vector<int> cur_t = T.t;
        if (n >= 8) {
            for (int k = 0, stale = 0; stale < patience && std::chrono::steady_clock::now() < rs_deadline &&
                                       !(cancel && cancel->load(std::memory_order_relaxed));
                 ++k) {
                Tour K(cost, double_bridge(cur_t, rng));
                local_search(K, rs_deadline, cancel);
                const double kc = K.cost();
                if (kc < cur - 1e-9) stale = 0;
                else ++stale;
                if (kc <= cur + 1e-12) {
                    cur = kc;
                    cur_t = K.t;
                }
            }
        }
        const double exact = tour_cost(cost, cur_t); // kInf if the tour uses a missing edge
        if (exact < best.cost || best.tour.empty()) {
            best.tour = cur_t;
            best.cost = exact;
            best.ok = std::isfinite(exact);
        }
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
                   bool &improved, const std::atomic<bool> *cancel) {
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
    // reference budgets (topolgy_optimizer.cpp:52-60 / 136-144): exact up to 8 / 20 nodes, 4 / 16 restarts,
    // 1 s / 30 s. The synchronous pass runs on the master's event loop, so it solves exactly up to 10 nodes
    // (Held-Karp at 10: ~1 ms) and otherwise stops its local search after 250 ms; the moonshot runs off-loop.
    const AtspResult r = moonshot ? solve_atsp(cost, 20, 30000, 16, 42, cancel)
                                  : solve_atsp(cost, 10, 250, 4, 42, cancel);
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

OptimizerPool::~OptimizerPool() { stop(); }

void OptimizerPool::stop() {
    std::vector<std::thread> ts;
    {
        std::lock_guard l(m_);
        stop_ = true;
        q_.clear();
        ts.swap(threads_);
    }
    cv_.notify_all();
    for (auto &t : ts)
        if (t.joinable()) t.join();
}

bool OptimizerPool::submit(uint64_t key, std::function<void()> fn) {
    std::lock_guard l(m_);
    if (stop_ || active_.count(key) || q_.size() >= max_queue_) return false;
    active_.insert(key);
    q_.emplace_back(key, std::move(fn));
    if (idle_ == 0 && threads_.size() < max_threads_) threads_.emplace_back([this] { loop(); });
    else cv_.notify_one();
    return true;
}

size_t OptimizerPool::thread_count() {
    std::lock_guard l(m_);
    return threads_.size();
}

size_t OptimizerPool::pending() {
    std::lock_guard l(m_);
    return active_.size();
}

void OptimizerPool::loop() {
    name_thread("pccl-tsp");
    std::unique_lock l(m_);
    while (true) {
        ++idle_;
        cv_.wait(l, [this] { return stop_ || !q_.empty(); });
        --idle_;
        if (stop_) return;
        auto [key, fn] = std::move(q_.front());
        q_.pop_front();
        l.unlock();
        fn();
        l.lock();
        active_.erase(key);
    }
}

} // namespace pccl::master
