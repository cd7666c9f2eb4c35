// Exhaustive check of orbx::glibc_sinf/cosf (my_orb_slam2_amd/csrc/orbx_math.h) against the
// host glibc over every float in [lo, hi).  Test infrastructure only.
// Usage: libm_port_check [lo] [hi] [stride]   (stride 1 = exhaustive)
#include "../../my_orb_slam2_amd/csrc/orbx_math.h"
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
#include <atomic>
int main(int argc, char** argv) {
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
