// Big-endian packet encoding (CCoIP wire format): integers big-endian, float/double bit-cast to
// big-endian u32/u64, bool = 1 byte, string = u64 length + bytes, uuid = 16 raw bytes,
// socket address = bool is_ipv4 + 4|16 address bytes + u16 port.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../common/types.hpp"

namespace pccl::proto {

class WBuf {
public:
    std::vector<uint8_t> data;

    void u8(uint8_t v) { data.push_back(v); }
    void boolean(bool v) { data.push_back(v ? 1 : 0); }
    void u16(uint16_t v) { put_be(v); }
    void u32(uint32_t v) { put_be(v); }
    void u64(uint64_t v) { put_be(v); }
    void i64(int64_t v) { put_be(static_cast<uint64_t>(v)); }
    void f32(float v) {
        uint32_t u;
        std::memcpy(&u, &v, 4);
        put_be(u);
    }
    void f64(double v) {
        uint64_t u;
        std::memcpy(&u, &v, 8);
        put_be(u);
    }
    void bytes(const void *p, size_t n) {
        const auto *b = static_cast<const uint8_t *>(p);
        data.insert(data.end(), b, b + n);
    }
    void str(const std::string &s) {
        u64(s.size());
        bytes(s.data(), s.size());
    }
    void uuid(const Uuid &u) { bytes(u.data.data(), 16); }
    void sockaddr(const SockAddr &a) {
        const bool v4 = a.inet.protocol == inetIPv4;
        boolean(v4);
        if (v4)
            bytes(a.inet.ipv4.data, 4);
        else
            bytes(a.inet.ipv6.data, 16);
        u16(a.port);
    }

private:
    template<typename T>
    void put_be(T v) {
        for (int i = static_cast<int>(sizeof(T)) - 1; i >= 0; --i) data.push_back(static_cast<uint8_t>(v >> (8 * i)));
    }
};

class RBuf {
public:
    RBuf(const uint8_t *p, size_t n) : p_(p), n_(n) {}

    bool ok() const { return ok_; }
    size_t remaining() const { return n_ - off_; }

    uint8_t u8() { return get_be<uint8_t>(); }
    bool boolean() { return get_be<uint8_t>() != 0; }
    uint16_t u16() { return get_be<uint16_t>(); }
    uint32_t u32() { return get_be<uint32_t>(); }
    uint64_t u64() { return get_be<uint64_t>(); }
    int64_t i64() { return static_cast<int64_t>(get_be<uint64_t>()); }
    float f32() {
        const uint32_t u = get_be<uint32_t>();
        float f;
        std::memcpy(&f, &u, 4);
        return f;
    }
    double f64() {
        const uint64_t u = get_be<uint64_t>();
        double f;
        std::memcpy(&f, &u, 8);
        return f;
    }
    bool bytes(void *dst, size_t n) {
        if (!need(n)) return false;
        std::memcpy(dst, p_ + off_, n);
        off_ += n;
        return true;
    }
    std::string str() {
        const uint64_t len = u64();
        if (!ok_ || !need(len)) return {};
        std::string s(reinterpret_cast<const char *>(p_ + off_), len);
        off_ += len;
        return s;
    }
    Uuid uuid() {
        Uuid u;
        bytes(u.data.data(), 16);
        return u;
    }
    SockAddr sockaddr() {
        SockAddr a{};
        if (boolean()) {
            a.inet.protocol = inetIPv4;
            bytes(a.inet.ipv4.data, 4);
        } else {
            a.inet.protocol = inetIPv6;
            bytes(a.inet.ipv6.data, 16);
        }
        a.port = u16();
        return a;
    }
    // Bounds check for "n elements" style counts (defends against hostile lengths)
    bool plausible_count(uint64_t n, size_t min_elem_bytes) {
        if (min_elem_bytes == 0) min_elem_bytes = 1;
        if (n > remaining() / min_elem_bytes) {
            ok_ = false;
            return false;
        }
        return true;
    }

private:
    bool need(size_t n) {
        if (!ok_ || n > n_ - off_) {
            ok_ = false;
            return false;
        }
        return true;
    }
    template<typename T>
    T get_be() {
        if (!need(sizeof(T))) return T{};
        T v = 0;
        for (size_t i = 0; i < sizeof(T); ++i) v = static_cast<T>((static_cast<uint64_t>(v) << 8) | p_[off_ + i]);
        off_ += sizeof(T);
        return v;
    }

    const uint8_t *p_;
    size_t n_;
    size_t off_ = 0;
    bool ok_ = true;
};

} // namespace pccl::proto
