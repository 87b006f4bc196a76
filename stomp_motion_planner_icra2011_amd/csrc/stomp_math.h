// stomp_math.h -- deterministic fp64 elementary functions and the Philox noise
// stream, evaluated identically on gfx950 and on the host.
//
// The reference reaches libm through KDL (sin/cos in Rotation::Rot2, from
// treefksolverjointposaxis_partial.cpp:125), policy_improvement.cpp:356 (exp) and
// boost::normal_distribution (multivariate_gaussian.h:91).  Device and host libm
// disagree in the last ulp, and a one-ulp change in a sphere position can flip a
// distance-field cell (stomp_collision_space.h:190) and change the optimisation
// path, so the engine pins these functions to fdlibm's reductions and minimax
// polynomials, one rounding per operation (build with -ffp-contract=off).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define STOMP_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define STOMP_HD static inline
#endif

namespace stomp {

STOMP_HD double bits_to_double(uint64_t u)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double((long long)u);
#else
    double x;
    __builtin_memcpy(&x, &u, 8);
    return x;
#endif
}

STOMP_HD uint64_t double_to_bits(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint64_t)__double_as_longlong(x);
#else
    uint64_t u;
    __builtin_memcpy(&u, &x, 8);
    return u;
#endif
}

// exp: x = k ln2 + r, |r| <= ln2/2, rational approximation of exp(r) (fdlibm e_exp.c)
STOMP_HD double det_exp(double x)
{
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
    const double invln2 = 1.44269504088896338700e+00;
    const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
                 P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
                 P5 = 4.13813679705723846039e-08;
    double kd = floor(x * invln2 + 0.5);
    int k = (int)kd;
    double hi = x - kd * ln2hi;
    double lo = kd * ln2lo;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    return y * bits_to_double((uint64_t)(k + 1023) << 52);
}

// log for positive normal x (fdlibm e_log.c)
STOMP_HD double det_log(double x)
{
    const double ln2hi = 6.93147180369123816490e-01, ln2lo = 1.90821492927058770002e-10;
    const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
                 L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    uint64_t u = double_to_bits(x);
    int k = (int)((u >> 52) & 0x7ff) - 1023;
    uint64_t m = u & 0x000fffffffffffffULL;
    uint64_t i = (m + 0x95f6400000000ULL) & 0x0010000000000000ULL;
    double xm = bits_to_double(m | (i ^ 0x3ff0000000000000ULL));
    k += (int)(i >> 52);
    double f = xm - 1.0;
    double s = f / (2.0 + f);
    double dk = (double)k;
    double z = s * s;
    double w = z * z;
    double t1 = w * (L2 + w * (L4 + w * L6));
    double t2 = z * (L1 + w * (L3 + w * (L5 + w * L7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    return dk * ln2hi - ((hfsq - (s * (hfsq + R) + dk * ln2lo)) - f);
}

// sin and cos together: Cody-Waite reduction by pi/2 (two-part constant), fdlibm kernels
STOMP_HD void det_sincos(double x, double* s, double* c)
{
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double kd = floor(x * invpio2 + 0.5);
    double y = (x - kd * pio2_1) - kd * pio2_1t;
    int n = ((int)kd) & 3;
    double z = y * y;
    double v = z * y;
    double rs = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    double ks = y + v * (S1 + z * rs);
    double rc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    double kc = w + (((1.0 - w) - hz) + z * rc);
    // quadrant n: (sin, cos) = (ks, kc), (kc, -ks), (-ks, -kc), (-kc, ks), as selects (a
    // divergent if-chain runs every path under exec masks when the waypoints' quadrants differ)
    const bool odd = (n & 1) != 0, neg = (n & 2) != 0;
    const double so = odd ? kc : ks;
    const double co = odd ? -ks : kc;
    *s = neg ? -so : so;
    *c = neg ? -co : co;
}

// atan: fdlibm s_atan.c (reduction about atan(0.5), atan(1), atan(1.5), atan(inf), hi/lo
// constants, odd/even minimax polynomial)
STOMP_HD double det_atan(double x)
{
    const double hi0 = 4.63647609000806093515e-01, hi1 = 7.85398163397448278999e-01,
                 hi2 = 9.82793723247329054082e-01, hi3 = 1.57079632679489655800e+00;
    const double lo0 = 2.26987774529616870924e-17, lo1 = 3.06161699786838301793e-17,
                 lo2 = 1.39033110312309984516e-17, lo3 = 6.12323399573676603587e-17;
    const double a0 = 3.33333333333329318027e-01, a1 = -1.99999999998764832476e-01,
                 a2 = 1.42857142725034663711e-01, a3 = -1.11111104054623557880e-01,
                 a4 = 9.09088713343650656196e-02, a5 = -7.69187620504482999495e-02,
                 a6 = 6.66107313738753120669e-02, a7 = -5.83357013379057348645e-02,
                 a8 = 4.97687799461593236017e-02, a9 = -3.65315727442169155270e-02,
                 a10 = 1.62858201153657823623e-02;
    const int hx = (int)(double_to_bits(x) >> 32);
    const int ix = hx & 0x7fffffff;
    if (ix >= 0x44100000) {
        if (x != x) return x + x;
        return hx > 0 ? hi3 + lo3 : -hi3 - lo3;
    }
    int id = -1;
    if (ix < 0x3fdc0000) {
        if (ix < 0x3e400000) return x;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (a0 + w * (a2 + w * (a4 + w * (a6 + w * (a8 + w * a10)))));
    const double s2 = w * (a1 + w * (a3 + w * (a5 + w * (a7 + w * a9))));
    if (id < 0) return x - x * (s1 + s2);
    const double hi = id == 0 ? hi0 : (id == 1 ? hi1 : (id == 2 ? hi2 : hi3));
    const double lo = id == 0 ? lo0 : (id == 1 ? lo1 : (id == 2 ? lo2 : lo3));
    const double r = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -r : r;
}

// atan2: fdlibm e_atan2.c
STOMP_HD double det_atan2(double y, double x)
{
    const double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
                 pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
    if (x != x || y != y) return x + y;
    const uint64_t ux = double_to_bits(x), uy = double_to_bits(y);
    const int hx = (int)(ux >> 32), hy = (int)(uy >> 32);
    const int ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const unsigned lx = (unsigned)ux, ly = (unsigned)uy;
    if (x == 1.0) return det_atan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | ly) == 0) return m <= 1 ? y : (m == 2 ? pi : -pi);
    if ((ix | lx) == 0) return hy < 0 ? -pi_o_2 : pi_o_2;
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000)
            return m == 0 ? pi_o_4 : (m == 1 ? -pi_o_4 : (m == 2 ? 3.0 * pi_o_4 : -3.0 * pi_o_4));
        return m == 0 ? 0.0 : (m == 1 ? -0.0 : (m == 2 ? pi : -pi));
    }
    if (iy == 0x7ff00000) return hy < 0 ? -pi_o_2 : pi_o_2;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = det_atan(fabs(y / x));
    if (m == 0) return z;
    if (m == 1) return -z;
    if (m == 2) return pi - (z - pi_lo);
    return (z - pi_lo) - pi;
}

// asin: fdlibm e_asin.c
STOMP_HD double det_asin(double x)
{
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
                 pio4_hi = 7.85398163397448278999e-01;
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05;
    const double qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const uint64_t u = double_to_bits(x);
    const int hx = (int)(u >> 32);
    const int ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (((ix - 0x3ff00000) | (unsigned)u) == 0) return x * pio2_hi + x * pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000) {
        if (ix < 0x3e400000) return x;
        const double t = x * x;
        const double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
        const double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
        const double w = p / q;
        return x + x * w;
    }
    const double w0 = 1.0 - fabs(x);
    double t = w0 * 0.5;
    double p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    double q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    const double s = sqrt(t);
    if (ix >= 0x3FEF3333) {
        const double w = p / q;
        t = pio2_hi - (2.0 * (s + s * w) - pio2_lo);
    } else {
        const double w = bits_to_double(double_to_bits(s) & 0xFFFFFFFF00000000ull);
        const double c = (t - w * w) / (s + w);
        const double r = p / q;
        p = 2.0 * s * r - (pio2_lo - 2.0 * c);
        q = pio4_hi - 2.0 * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

// Philox4x32-10 (Salmon et al., SC'11)
STOMP_HD void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                            uint32_t out[4])
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Normal pair p of the noise stream for (iteration, joint, rollout): Box-Muller on two
// 53-bit uniforms, u1 in (0,1], u2 in [0,1).  Replaces boost mt19937 + normal_distribution
// (multivariate_gaussian.h:83-94), which cannot be sharded across rollouts or devices.
STOMP_HD void normal_pair(uint64_t seed, int iteration, int joint, int rollout, int p, double* z0, double* z1)
{
    uint32_t o[4];
    philox4x32_10((uint32_t)p, (uint32_t)rollout, (uint32_t)joint, (uint32_t)iteration, (uint32_t)seed,
                  (uint32_t)(seed >> 32), o);
    uint64_t a = ((((uint64_t)o[0]) << 32) | o[1]) >> 11;
    uint64_t b = ((((uint64_t)o[2]) << 32) | o[3]) >> 11;
    const double two_m53 = 1.1102230246251565404236316680908203125e-16;
    double u1 = (double)(a + 1) * two_m53;
    double u2 = (double)b * two_m53;
    double r = sqrt(-2.0 * det_log(u1));
    double s, c;
    det_sincos(6.283185307179586476925286766559 * u2, &s, &c);
    *z0 = r * c;
    *z1 = r * s;
}

}  // namespace stomp
