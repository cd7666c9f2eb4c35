// Exhaustive check of orbx::glibc_sinf/cosf and orbx::glibc_logf
// (my_orb_slam2_amd/csrc/orbx_math.h) against the host glibc over every float in [lo, hi).
// Test infrastructure only.
// Usage: libm_port_check [lo] [hi] [stride]        sinf / cosf (stride 1 = exhaustive)
//        libm_port_check logf [lo_bits] [hi_bits]   logf over the float bit patterns [lo, hi)
#include "../../my_orb_slam2_amd/csrc/orbx_math.h"
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <atomic>
#include <string>
static int check_logf(uint32_t a, uint32_t b) {
    int nt = std::thread::hardware_concurrency(); if (nt < 1) nt = 1;
    std::atomic<unsigned long long> bad{0}, total{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t] {
        unsigned long long bl = 0, n = 0;
        for (uint64_t u = a + (uint64_t)t; u < b; u += (uint64_t)nt) {
            volatile float x = orbx::u2f((uint32_t)u);
            const float r = logf(x), p = orbx::glibc_logf(x);
            if (orbx::f2u(r) != orbx::f2u(p) && !(r != r && p != p)) {
                if (bl < 3) printf("logf mismatch %a: %a vs %a\n", (float)x, r, p);
                ++bl;
            }
            ++n;
        }
        bad += bl; total += n;
    });
    for (auto& x : th) x.join();
    printf("checked=%llu logf_mismatch=%llu\n", (unsigned long long)total, (unsigned long long)bad);
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "logf")
        return check_logf(argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 0) : 0u,
                          argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 0) : 0x80000000u);
    float lo = argc > 1 ? strtof(argv[1], nullptr) : 0.0f;
    float hi = argc > 2 ? strtof(argv[2], nullptr) : 6.2831855f;
    uint32_t stride = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 10) : 1;
    uint32_t a = orbx::f2u(lo), b = orbx::f2u(hi);
    int nt = std::thread::hardware_concurrency(); if (nt < 1) nt = 1;
    std::atomic<unsigned long long> bad_s{0}, bad_c{0}, total{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t] {
        unsigned long long bs = 0, bc = 0, n = 0;
        for (uint64_t u = a + (uint64_t)t * stride; u < b; u += (uint64_t)nt * stride) {
            float x = orbx::u2f((uint32_t)u);
            volatile float xs = x;
            float rs = sinf(xs), rc = cosf(xs);
            if (orbx::f2u(rs) != orbx::f2u(orbx::glibc_sinf(x))) { if (bs < 3) printf("sin mismatch %a\n", x); ++bs; }
            if (orbx::f2u(rc) != orbx::f2u(orbx::glibc_cosf(x))) { if (bc < 3) printf("cos mismatch %a\n", x); ++bc; }
            ++n;
        }
        bad_s += bs; bad_c += bc; total += n;
    });
    for (auto& x : th) x.join();
    printf("checked=%llu sin_mismatch=%llu cos_mismatch=%llu\n", (unsigned long long)total, (unsigned long long)bad_s, (unsigned long long)bad_c);
    return (bad_s || bad_c) ? 1 : 0;
}
