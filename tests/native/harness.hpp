// Tiny self-registering test harness shared by the native test translation units (no gtest in the image).
#pragma once

#include <cstdio>
#include <functional>
#include <string>
#include <utility>
#include <vector>

inline std::vector<std::pair<std::string, std::function<void()>>> &registry() {
    static std::vector<std::pair<std::string, std::function<void()>>> r;
    return r;
}
inline int g_failures = 0;
#define TEST(name)                                                                                                   \
    static void name();                                                                                              \
    static const bool reg_##name = (registry().emplace_back(#name, name), true);                                     \
    static void name()
#define EXPECT(cond)                                                                                                 \
    do {                                                                                                             \
        if (!(cond)) {                                                                                               \
            std::fprintf(stderr, "  %s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond);                         \
            ++g_failures;                                                                                            \
        }                                                                                                            \
    } while (0)
