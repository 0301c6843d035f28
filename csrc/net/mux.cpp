#include "mux.hpp"

#include "../common/trace.hpp"

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include "../common/log.hpp"
#include "../common/spin.hpp"
#include "socket.hpp"

namespace pccl::net {

size_t multiplex_chunk_size() {
    static const size_t v = env_size("PCCL_MULTIPLEX_CHUNK_SIZE", 16ull << 20);
    return v == 0 ? (16ull << 20) : v;
}

void mux_frame_header(uint8_t out[kMuxHeaderBytes], uint64_t payload, uint64_t tag, uint64_t ctr) {
    const uint64_t vals[3] = {payload + 16, tag, ctr};
    for (int v = 0; v < 3; ++v)
        for (int i = 0; i < 8; ++i) out[v * 8 + i] = static_cast<uint8_t>(vals[v] >> (8 * (7 - i)));
}

bool mux_parse_header(const uint8_t in[kMuxHeaderBytes], uint64_t &payload, uint64_t &tag, uint64_t &ctr) {
    uint64_t vals[3] = {0, 0, 0};
    for (int v = 0; v < 3; ++v)
        for (int i = 0; i < 8; ++i) vals[v] = (vals[v] << 8) | in[v * 8 + i];
    tag = vals[1];
    ctr = vals[2];
    if (vals[0] < 16 || vals[0] - 16 > kMuxMaxFrame) return false;
    payload = vals[0] - 16;
    return true;
}

const WanSim &wan_sim() {
    static const WanSim s = [] {
        WanSim w;
        const char *e = std::getenv("PCCL_SIM_WAN");
        if (!e || !*e) return w;
        double lat = 0, flow = 0, link = 0;
        const int n = std::sscanf(e, "%lf:%lf:%lf", &lat, &flow, &link);
        if (n >= 2 && flow > 0) {
            w.enabled = true;
            w.latency_s = lat / 1e3;
            w.flow_bps = flow * 1e6 / 8;
            w.link_bps = n >= 3 ? link * 1e6 / 8 : 0;
            LOG(WARN) << "WAN emulation on: " << lat << " ms one-way, " << flow << " Mbit/s per flow"
                      << (n >= 3 ? ", shared link " + std::to_string(link) + " Mbit/s" : std::string());
        }
        return w;
    }();
    return s;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// shared bottleneck link of all emulated flows of this process
static std::mutex g_link_mtx;
static double g_link_next_free = 0;

static void wan_shape(size_t n, double &flow_next_free, double &last_send) {
    const WanSim &w = wan_sim();
    double start = now_s();
    if (start - last_send > w.latency_s) start += w.latency_s; // new burst: pay the pipe latency once
    start = std::max(start, flow_next_free);
    double done = start + static_cast<double>(n) / w.flow_bps;
    if (w.link_bps > 0) {
        std::lock_guard l(g_link_mtx);
        const double lstart = std::max(start, g_link_next_free);
        g_link_next_free = lstart + static_cast<double>(n) / w.link_bps;
        done = std::max(done, g_link_next_free);
    }
    flow_next_free = done;
    const double wait = done - now_s();
    if (wait > 0) std::this_thread::sleep_for(std::chrono::duration<double>(wait));
    last_send = now_s();
}

MuxConn::MuxConn(int fd, Mode mode, const SockAddr &peer_addr)
    : fd_(fd), mode_(mode), peer_addr_(peer_addr),
      zerocopy_(mode == Mode::Tx && fd >= 0 && socket_zerocopy_on(fd)) {}

MuxConn::~MuxConn() {
    interrupt();
    join();
    if (fd_ >= 0) {
        ::close(fd_);
        fd_ = -1;
    }
}

bool MuxConn::start() {
    open_.store(true, std::memory_order_release);
    if (mode_ == Mode::Rx) rx_thread_ = std::thread([this] {
        name_thread("pccl-mux-rx");
        rx_loop();
    });
    return true;
}

void MuxConn::interrupt() {
    stop_ = true;
    if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
    open_.store(false, std::memory_order_release);
    {
        std::lock_guard l(mtx_);
    }
    cv_.notify_all();
}

void MuxConn::join() {
    if (rx_thread_.joinable()) rx_thread_.join();
    {
        std::lock_guard l(job_mtx_);
        jobs_stop_ = true;
    }
    job_cv_.notify_all();
    if (tx_job_thread_.joinable()) tx_job_thread_.join();
}

void MuxConn::post_send_job(std::function<void()> job) {
    std::lock_guard l(job_mtx_);
    jobs_.push_back(std::move(job));
    if (!tx_job_thread_.joinable() && !jobs_stop_) tx_job_thread_ = std::thread([this] {
            name_thread("pccl-mux-tx");
            tx_job_loop();
        });
    job_cv_.notify_one();
}

void MuxConn::tx_job_loop() {
    std::unique_lock l(job_mtx_);
    while (true) {
        job_cv_.wait(l, [this] { return jobs_stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return; // stopped and drained
        auto job = std::move(jobs_.front());
        jobs_.pop_front();
        l.unlock();
        job();
        l.lock();
    }
}

static int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

bool MuxConn::send_frame(uint64_t tag, uint64_t ctr, const void *data, size_t n) {
    if (!is_open()) return false;
    uint8_t hdr[kMuxHeaderBytes];
    mux_frame_header(hdr, n, tag, ctr);
    iovec iov[2] = {{hdr, 24}, {const_cast<void *>(data), n}};
    std::lock_guard lock(tx_mtx_);
    if (wan_sim().enabled) wan_shape(n + 24, sim_next_free_, sim_last_send_);
    // bulk frames from pinned staging buffers may go out as MSG_ZEROCOPY (socket.cpp: sendv_all_zerocopy)
    const bool zc = zerocopy_ && n >= (256u << 10);
    send_since_ns_.store(steady_ns(), std::memory_order_relaxed);
    const bool ok = zc ? sendv_all_zerocopy(fd_, iov, n ? 2 : 1, zc_next_id_) : sendv_all(fd_, iov, n ? 2 : 1);
    send_since_ns_.store(0, std::memory_order_relaxed);
    if (!ok) {
        open_.store(false, std::memory_order_release);
        return false;
    }
    tx_total_.fetch_add(n + kMuxHeaderBytes, std::memory_order_relaxed);
    return true;
}

std::chrono::nanoseconds MuxConn::send_blocked_for() const {
    const int64_t t = send_since_ns_.load(std::memory_order_relaxed);
    return std::chrono::nanoseconds(t == 0 ? 0 : std::max<int64_t>(0, steady_ns() - t));
}

size_t interrupt_blocked_senders(const std::vector<std::shared_ptr<MuxConn>> &conns, std::chrono::nanoseconds min_blocked) {
    size_t n = 0;
    for (const auto &c : conns) {
        if (!c || !c->is_open()) continue;
        const auto b = c->send_blocked_for();
        if (b.count() > 0 && b >= min_blocked) {
            LOG(WARN) << "MuxConn: send to " << sockaddr_str(c->peer_addr()) << " blocked for "
                      << std::chrono::duration_cast<std::chrono::milliseconds>(b).count()
                      << " ms in a failed op; interrupting the connection";
            c->interrupt();
            ++n;
        }
    }
    return n;
}

std::chrono::milliseconds sink_drain_grace() {
    static const auto v = std::chrono::milliseconds(env_size("PCCL_SINK_DRAIN_MS", 1000));
    return v;
}

bool MuxConn::read_into(uint8_t *dst, size_t n, Sink *progress_sink) {
    constexpr size_t kPiece = 4 << 20;
    size_t done = 0;
    while (done < n) {
        const size_t want = std::min(kPiece, n - done);
        const ssize_t k = ::recv(fd_, dst + done, want, 0);
        if (k < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        if (k == 0) return false;
        done += static_cast<size_t>(k);
        rx_total_.fetch_add(static_cast<uint64_t>(k), std::memory_order_relaxed);
        if (progress_sink != nullptr) {
            // seq_cst pairs with wait_sink (store wake_at, then re-read received): one of the two sides sees the
            // other's write, so a waiter is never left sleeping past its threshold
            const size_t now = progress_sink->received.fetch_add(static_cast<size_t>(k)) + static_cast<size_t>(k);
            if (now >= progress_sink->wake_at.load()) {
                {
                    std::lock_guard l(mtx_);
                }
                cv_.notify_all();
            }
        }
    }
    return true;
}

void MuxConn::rx_loop() {
    while (!stop_) {
        uint8_t hdr[kMuxHeaderBytes];
        if (!recv_all(fd_, hdr, kMuxHeaderBytes)) break;
        uint64_t len = 0, tag = 0, ctr = 0;
        if (!mux_parse_header(hdr, len, tag, ctr)) {
            // malformed / oversized frame: the stream cannot be re-synchronised, so the connection is closed (the
            // reference pops and silently drops a frame larger than the receive buffer, Appendix C #8)
            LOG(WARN) << "MuxConn: invalid frame header from " << sockaddr_str(peer_addr_) << "; closing";
            break;
        }
        // The frame's payload is a run of the tag's byte stream: it fills the tag's oldest sinks with room in FIFO
        // order and may straddle several of them (a sender's frame size need not match the receiver's sinks: a
        // reference peer frames a ring step in PCCL_MULTIPLEX_CHUNK_SIZE pieces of its own choosing). Whatever finds
        // no sink is queued and copied into the sinks posted later.
        size_t left = len;
        bool ok = true;
        while (ok && left > 0) {
            Sink *sink = nullptr;
            size_t offset = 0, take = 0;
            {
                std::lock_guard l(mtx_);
                // deliver directly only if nothing for this tag/ctr is still queued ahead of these bytes (FIFO)
                auto qit = queued_.find(tag);
                bool queued_ahead = false;
                if (qit != queued_.end())
                    for (const auto &f : qit->second)
                        if (f.ctr == ctr) queued_ahead = true;
                if (!queued_ahead) sink = sink_for_locked(tag, ctr);
                if (sink != nullptr) {
                    sink->busy = true;
                    offset = sink->received.load(std::memory_order_relaxed);
                    take = std::min(left, sink->capacity - offset);
                }
            }
            if (sink == nullptr) break;
            {
                RoctxIoRange io("recv");
                ok = read_into(sink->dst + offset, take, sink);
            }
            {
                std::lock_guard l(mtx_);
                sink->busy = false;
            }
            cv_.notify_all();
            left -= take;
        }
        if (!ok) break;
        if (left == 0) continue;
        std::vector<uint8_t> buf(left);
        if (!read_into(buf.data(), left, nullptr)) break;
        {
            std::lock_guard l(mtx_);
            auto it = sinks_.find(tag);
            const bool stale = it != sinks_.end() && !it->second.empty() && ctr < it->second.front()->ctr;
            if (!stale) { // (stale: a frame of an aborted earlier op with the same tag)
                queued_[tag].push_back(Frame{ctr, std::move(buf)});
                // a sink may have been posted while this frame was read: deliver now (keeps FIFO order)
                drain_queued_locked(tag, ctr);
            }
        }
        cv_.notify_all();
    }
    open_.store(false, std::memory_order_release);
    {
        std::lock_guard l(mtx_);
    }
    cv_.notify_all();
}

std::optional<std::vector<uint8_t>> MuxConn::recv_frame(uint64_t tag, uint64_t ctr, std::chrono::milliseconds timeout) {
    std::unique_lock l(mtx_);
    const auto deadline = std::chrono::steady_clock::now() + timeout;
    while (true) {
        auto it = queued_.find(tag);
        if (it != queued_.end()) {
            auto &q = it->second;
            while (!q.empty() && q.front().ctr < ctr) q.pop_front();
            if (!q.empty() && q.front().ctr == ctr) {
                auto data = std::move(q.front().data);
                if (q.front().off > 0) data.erase(data.begin(), data.begin() + static_cast<long>(q.front().off));
                q.pop_front();
                if (q.empty()) queued_.erase(it);
                return data;
            }
        }
        if (!is_open()) return std::nullopt;
        if (cv_.wait_until(l, deadline) == std::cv_status::timeout) {
            // re-check once
            auto it2 = queued_.find(tag);
            if (it2 != queued_.end() && !it2->second.empty() && it2->second.front().ctr == ctr) continue;
            return std::nullopt;
        }
    }
}

MuxConn::Sink *MuxConn::sink_for_locked(uint64_t tag, uint64_t ctr) {
    auto it = sinks_.find(tag);
    if (it == sinks_.end()) return nullptr;
    for (auto &s : it->second) {
        if (s->ctr != ctr) continue;
        const size_t have = s->received.load(std::memory_order_relaxed);
        if (have >= s->capacity) continue; // full: the bytes belong to a later sink
        return s->busy ? nullptr : s.get();
    }
    return nullptr;
}

void MuxConn::drain_queued_locked(uint64_t tag, uint64_t ctr) {
    auto it = queued_.find(tag);
    if (it == queued_.end()) return;
    auto &q = it->second;
    auto sk = sinks_.find(tag);
    if (sk != sinks_.end() && !sk->second.empty()) {
        const uint64_t cur = sk->second.front()->ctr;
        while (!q.empty() && q.front().ctr < cur) q.pop_front(); // stale frames of an aborted earlier op
    }
    while (!q.empty() && q.front().ctr == ctr) {
        Sink *s = sink_for_locked(tag, ctr);
        if (s == nullptr) break;
        Frame &f = q.front();
        const size_t have = s->received.load(std::memory_order_relaxed);
        const size_t take = std::min(f.data.size() - f.off, s->capacity - have);
        std::memcpy(s->dst + have, f.data.data() + f.off, take);
        s->received.store(have + take, std::memory_order_release);
        f.off += take;
        if (f.off == f.data.size()) q.pop_front();
    }
    if (q.empty()) queued_.erase(it);
}

MuxConn::SinkRef MuxConn::post_sink(uint64_t tag, uint64_t ctr, uint8_t *dst, size_t n) {
    std::lock_guard l(mtx_);
    auto s = std::make_shared<Sink>();
    s->ctr = ctr;
    s->dst = dst;
    s->capacity = n;
    auto &dq = sinks_[tag];
    // sinks of an older ctr left behind (an aborted op that never removed them) no longer receive anything
    while (!dq.empty() && dq.front()->ctr < ctr && !dq.front()->busy) dq.pop_front();
    dq.push_back(s);
    drain_queued_locked(tag, ctr);
    return s;
}

size_t MuxConn::sink_progress(uint64_t tag) {
    std::lock_guard l(mtx_);
    auto it = sinks_.find(tag);
    if (it == sinks_.end() || it->second.empty()) return 0;
    return it->second.front()->received.load(std::memory_order_acquire);
}

size_t MuxConn::wait_sink(uint64_t tag, size_t want, std::chrono::milliseconds timeout) {
    SinkRef s;
    {
        std::lock_guard l(mtx_);
        auto it = sinks_.find(tag);
        if (it == sinks_.end() || it->second.empty()) return 0;
        s = it->second.front();
    }
    return wait_sink(s, want, timeout);
}

size_t MuxConn::wait_sink(const SinkRef &sr, size_t want, std::chrono::milliseconds timeout) {
    if (!sr) return 0;
    Sink *sink = sr.get(); // kept alive by the caller's reference
    if (sink->received.load(std::memory_order_acquire) >= want || !is_open())
        return sink->received.load(std::memory_order_acquire);
    // spin briefly without the lock, then sleep on the condition variable with the waiter's threshold published
    spin_until([&] { return sink->received.load(std::memory_order_acquire) >= want || !is_open(); });
    std::unique_lock l(mtx_);
    const auto deadline = std::chrono::steady_clock::now() + timeout;
    while (true) {
        const size_t have = sink->received.load(std::memory_order_acquire);
        if (have >= want || !is_open()) return have;
        sink->wake_at.store(want);
        if (sink->received.load() >= want) continue;
        const bool timed_out = cv_.wait_until(l, deadline) == std::cv_status::timeout;
        sink->wake_at.store(SIZE_MAX);
        if (timed_out) return sink->received.load(std::memory_order_acquire);
    }
}

void MuxConn::remove_sink(uint64_t tag) {
    SinkRef s;
    {
        std::lock_guard l(mtx_);
        auto it = sinks_.find(tag);
        if (it == sinks_.end() || it->second.empty()) return;
        s = it->second.front();
    }
    remove_sink(tag, s);
}

void MuxConn::remove_sink(uint64_t tag, const SinkRef &s) {
    if (!s) return;
    std::unique_lock l(mtx_);
    const auto deadline = std::chrono::steady_clock::now() + sink_drain_grace();
    bool interrupted = false;
    while (s->busy) {
        cv_.wait_for(l, std::chrono::milliseconds(20));
        if (std::chrono::steady_clock::now() > deadline && !interrupted) {
            LOG(WARN) << "MuxConn: sink still being written after " << sink_drain_grace().count()
                      << " ms; interrupting connection";
            interrupted = true;
            if (fd_ >= 0) ::shutdown(fd_, SHUT_RDWR);
        }
    }
    auto it = sinks_.find(tag);
    if (it == sinks_.end()) return;
    auto &dq = it->second;
    for (auto d = dq.begin(); d != dq.end(); ++d)
        if (d->get() == s.get()) {
            dq.erase(d);
            break;
        }
    if (dq.empty()) sinks_.erase(it);
}

} // namespace pccl::net
