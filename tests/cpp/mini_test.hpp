// Minimal gtest-style harness (googletest is not available offline).
#pragma once
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace mini {
struct Case {
    const char* suite;
    const char* name;
    std::function<void()> fn;
    bool gpu;
};
inline std::vector<Case>& registry() {
    static std::vector<Case> r;
    return r;
}
inline int& failures() {
    static int f = 0;
    return f;
}
struct Reg {
    Reg(const char* s, const char* n, std::function<void()> f, bool gpu) { registry().push_back({s, n, f, gpu}); }
};
inline int run_all(int argc, char** argv) {
    bool gpu = true;
    for (int i = 1; i < argc; ++i)
        if (!std::strcmp(argv[i], "--cpu-only")) gpu = false;
    int ran = 0, failed = 0;
    for (auto& c : registry()) {
        if (c.gpu && !gpu) continue;
        int before = failures();
        c.fn();
        ++ran;
        bool ok = failures() == before;
        if (!ok) ++failed;
        std::printf("[%s] %s.%s\n", ok ? "  OK  " : " FAIL ", c.suite, c.name);
    }
    std::printf("%d tests, %d failed\n", ran, failed);
    return failed ? 1 : 0;
}
}  // namespace mini

#define MINI_CAT(a, b) a##b
#define MINI_TEST(suite, name, gpu)                                                              \
    static void MINI_CAT(suite##_, name)();                                                      \
    static mini::Reg MINI_CAT(reg_##suite##_, name)(#suite, #name, MINI_CAT(suite##_, name), gpu); \
    static void MINI_CAT(suite##_, name)()
#define TEST(suite, name) MINI_TEST(suite, name, false)
#define GPU_TEST(suite, name) MINI_TEST(suite, name, true)
#define MINI_FAIL(msg)                                                        \
    do {                                                                      \
        std::printf("  %s:%d: %s\n", __FILE__, __LINE__, std::string(msg).c_str()); \
        ++mini::failures();                                                   \
    } while (0)
#define EXPECT_TRUE(c) \
    do {               \
        if (!(c)) MINI_FAIL("expected true: " #c); \
    } while (0)
#define ASSERT_TRUE(c)                              \
    do {                                            \
        if (!(c)) {                                 \
            MINI_FAIL("assertion failed: " #c);     \
            return;                                 \
        }                                           \
    } while (0)
#define EXPECT_EQ(a, b) \
    do {                \
        if (!((a) == (b))) MINI_FAIL("expected equal: " #a " == " #b); \
    } while (0)
#define ASSERT_EQ(a, b)                                            \
    do {                                                           \
        if (!((a) == (b))) {                                       \
            MINI_FAIL("assertion failed: " #a " == " #b);          \
            return;                                                \
        }                                                          \
    } while (0)
#define EXPECT_NEAR(a, b, tol)                                                              \
    do {                                                                                    \
        double a_ = (a), b_ = (b);                                                          \
        if (!(std::fabs(a_ - b_) <= (tol)))                                                 \
            MINI_FAIL("expected near: " #a " = " + std::to_string(a_) + " vs " + std::to_string(b_)); \
    } while (0)
