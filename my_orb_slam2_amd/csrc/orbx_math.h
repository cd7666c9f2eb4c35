// orbx_math.h — bit-exact scalar primitives shared by host and gfx950 device code.
//
// The reference ORB path (src/ORBextractor.cc) calls three pieces of float arithmetic that
// live outside its own sources:
//   * glibc cosf/sinf           — src/ORBextractor.cc:113  (`(float)cos(angle)` on a float)
//   * OpenCV 3.2 cv::fastAtan2  — src/ORBextractor.cc:103
//   * OpenCV cvRound / cvFloor  — src/ORBextractor.cc:81,115,119-120
// A GPU has none of these, and the device libm is not glibc, so this header restates them.
//
// sinf/cosf: glibc 2.35 sysdeps/ieee754/flt-32 (s_sinf.c / s_cosf.c / sincosf.h /
// sincosf_data.c), the double-precision polynomial algorithm.  On x86-64 glibc dispatches
// by ifunc to a copy built with -mfma (`__sinf_fma`) on FMA-capable CPUs; that copy
// contracts every `a + b*c` of the polynomial and the range reduction into an fma.  The
// port below writes those fmas explicitly (ORBX_GLIBC_FMA=1, default) so the result does
// not depend on the compiler's contraction mode.  tests/test_libm_port.py checks the
// host build of this port against the real glibc over every float in [0, 2*pi).
//
// Everything here is compiled with -ffp-contract=off (host and device).
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define ORBX_HD __host__ __device__ __forceinline__
#else
#define ORBX_HD static inline
#endif

#define ORBX_GLIBC_FMA 1

namespace orbx {

ORBX_HD uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
ORBX_HD float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// a*b+c with the rounding the glibc FMA ifunc variant uses (one rounding), or the SSE2
// variant (two roundings).
ORBX_HD double glibc_madd(double a, double b, double c) {
    return fma(a, b, c);
}

// Polynomial coefficients, __sincosf_table[0] of glibc sincosf_data.c (!TOINT_INTRINSICS).
struct SinCosTab {
    double sign0, sign1, sign2, sign3;
    double hpi_inv, hpi;
    double c0, c1, c2, c3, c4;
    double s1, s2, s3;
};

ORBX_HD SinCosTab sincos_tab(int which) {
    SinCosTab t;
    t.sign0 = 1.0; t.sign1 = -1.0; t.sign2 = -1.0; t.sign3 = 1.0;
    t.hpi_inv = 0x1.45F306DC9C883p+23;
    t.hpi = 0x1.921FB54442D18p0;
    const double s = which ? -1.0 : 1.0;
    t.c0 = s * 0x1p0;
    t.c1 = s * -0x1.ffffffd0c621cp-2;
    t.c2 = s * 0x1.55553e1068f19p-5;
    t.c3 = s * -0x1.6c087e89a359dp-10;
    t.c4 = s * 0x1.99343027bf8c3p-16;
    t.s1 = -0x1.555545995a603p-3;
    t.s2 = 0x1.1107605230bc4p-7;
    t.s3 = -0x1.994eb3774cf24p-13;
    return t;
}

ORBX_HD uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// sinf_poly of glibc sincosf.h
ORBX_HD float glibc_sinf_poly(double x, double x2, const SinCosTab& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = glibc_madd(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = glibc_madd(x3, p.s1, x);
        return (float)glibc_madd(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = glibc_madd(x2, p.c4, p.c3);
        double c1 = glibc_madd(x2, p.c1, p.c0);
        double x6 = x4 * x2;
        double c = glibc_madd(x4, p.c2, c1);
        return (float)glibc_madd(x6, c2, c);
    }
}

// reduce_fast of glibc sincosf.h (scaled float->int conversion variant).
ORBX_HD double glibc_reduce_fast(double x, const SinCosTab& p, int* np) {
    double r = x * p.hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, p.hpi, x);
}

ORBX_HD double sign_of(const SinCosTab& p, int q) {
    q &= 3;
    return q == 0 ? p.sign0 : q == 1 ? p.sign1 : q == 2 ? p.sign2 : p.sign3;
}

// glibc sinf for |y| < 120 (the ORB path feeds angles in [0, 2*pi)).  Larger inputs use
// glibc's Payne-Hanek path, which the ORB path cannot reach; they return NaN here so a
// misuse is loud.
ORBX_HD float glibc_sinf(float y) {
    double x = y;
    SinCosTab p = sincos_tab(0);
    if (abstop12(y) < abstop12(0x1.921FB54442D18p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return glibc_sinf_poly(x, s, p, 0);
    } else if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = glibc_reduce_fast(x, p, &n);
        double s = sign_of(p, n);
        if (n & 2) p = sincos_tab(1);
        return glibc_sinf_poly(x * s, x * x, p, n);
    }
    return __builtin_nanf("");
}

ORBX_HD float glibc_cosf(float y) {
    double x = y;
    SinCosTab p = sincos_tab(0);
    if (abstop12(y) < abstop12(0x1.921FB54442D18p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return glibc_sinf_poly(x, x2, p, 1);
    } else if (abstop12(y) < abstop12(120.0f)) {
        int n;
        x = glibc_reduce_fast(x, p, &n);
        double s = sign_of(p, n);
        if (n & 2) p = sincos_tab(1);
        return glibc_sinf_poly(x * s, x * x, p, n ^ 1);
    }
    return __builtin_nanf("");
}

// OpenCV cvRound(float)/cvRound(double) on x86-64 SSE2: cvtss2si / cvtsd2si with the
// default MXCSR, i.e. round-half-to-even.
ORBX_HD int cv_round(float v) { return (int)rintf(v); }
ORBX_HD int cv_round_d(double v) { return (int)rint(v); }
ORBX_HD int cv_floor(float v) { return (int)floorf(v); }
ORBX_HD int cv_ceil(float v) { return (int)ceilf(v); }

// OpenCV 3.2 cv::fastAtan2 (core/src/mathfuncs.cpp): octant reduction + 7th-order odd
// polynomial in degrees, every operation a separate float rounding.
ORBX_HD float cv_fast_atan2(float y, float x) {
    const float k180pi = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k180pi;
    const float p3 = -0.3258083974640975f * k180pi;
    const float p5 = 0.1555786518463281f * k180pi;
    const float p7 = -0.04432655554792128f * k180pi;
    const float eps = (float)2.2204460492503131e-16;  // (float)DBL_EPSILON
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// logf: glibc 2.35 sysdeps/ieee754/flt-32 (e_logf.c, e_logf_data.c; LOGF_TABLE_BITS 4,
// LOGF_POLY_ORDER 4): log(x) = log1p(z/c - 1) + log(c) + k ln2 in double, one rounding to
// float.  MapPoint::PredictScale (src/MapPoint.cc:430-444) and Frame's mfLogScaleFactor
// (src/Frame.cc:82) call std::log on floats (TemplatedVocabulary.h:36 puts `using namespace
// std` in scope), i.e. logf.  This port equals the host glibc logf for every positive normal
// float, both with the polynomial's a*b+c contracted into fma (the __logf_fma ifunc variant)
// and without (tests/native/libm_port_check.cpp checks every one).
struct LogfEntry { double invc, logc; };
ORBX_HD LogfEntry logf_tab(int i) {
    switch (i) {
        case 0: return {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2};
        case 1: return {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2};
        case 2: return {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2};
        case 3: return {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3};
        case 4: return {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3};
        case 5: return {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3};
        case 6: return {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4};
        case 7: return {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4};
        case 8: return {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5};
        case 9: return {0x1p+0, 0x0p+0};
        case 10: return {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5};
        case 11: return {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4};
        case 12: return {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3};
        case 13: return {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3};
        case 14: return {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2};
        default: return {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2};
    }
}

ORBX_HD float glibc_logf(float x) {
    uint32_t ix = f2u(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        // x < 0x1p-126, inf or nan
        if (ix * 2 == 0) return -INFINITY;                 // log(+-0)
        if (ix == 0x7f800000u) return x;                   // log(inf)
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;   // x < 0 or nan
        ix = f2u(x * 0x1p23f);                             // subnormal: normalize
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> (23 - 4)) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const LogfEntry e = logf_tab(i);
    const double z = (double)u2f(iz);
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double r = z * e.invc - 1;
    const double y0 = e.logc + (double)k * Ln2;
    const double r2 = r * r;
    double y = A1 * r + A2;
    y = A0 * r2 + y;
    y = y * r2 + (y0 + r);
    return (float)y;
}

}  // namespace orbx
