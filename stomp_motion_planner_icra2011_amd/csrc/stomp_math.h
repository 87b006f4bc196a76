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
    double so, co;
    if (n == 0) { so = ks; co = kc; }
    else if (n == 1) { so = kc; co = -ks; }
    else if (n == 2) { so = -ks; co = -kc; }
    else { so = -kc; co = ks; }
    *s = so;
    *c = co;
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
