/*
 * oracle/dmath.h -- TEST INFRASTRUCTURE (CPU oracle). Not product code.
 *
 * Deterministic fp64 elementary functions used by the oracle.  The reference
 * calls libm (exp in policy_improvement.cpp:356, sin/cos inside KDL
 * Rotation::Rot2 reached from treefksolverjointposaxis_partial.cpp:125, log/
 * sqrt/cos/sin inside boost::normal_distribution reached from
 * multivariate_gaussian.h:91).  libm results differ in the last ulp between
 * glibc and the ROCm device library, and a one-ulp difference in a sphere
 * position can flip a voxel index (stomp_collision_space.h:190), so the build
 * pins the elementary functions to one published algorithm (fdlibm's
 * argument reductions and minimax polynomials, evaluated in the order written
 * here) and evaluates them identically on the host and on gfx950.  Accuracy
 * is <= 1 ulp on the ranges the path uses; tests/test_oracle_math.py checks
 * them against glibc.
 *
 * Every expression is written so that -ffp-contract=off gives one rounding per
 * operation.  Compile with -ffp-contract=off -fno-fast-math.
 */
#ifndef STOMP_ORACLE_DMATH_H
#define STOMP_ORACLE_DMATH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

static inline uint64_t dm_bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static inline double dm_from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

/* fdlibm e_exp.c constants */
#define DM_LN2_HI  6.93147180369123816490e-01
#define DM_LN2_LO  1.90821492927058770002e-10
#define DM_INVLN2  1.44269504088896338700e+00
#define DM_EP1  1.66666666666666019037e-01
#define DM_EP2 -2.77777777770155933842e-03
#define DM_EP3  6.61375632143793436117e-05
#define DM_EP4 -1.65339022054652515390e-06
#define DM_EP5  4.13813679705723846039e-08

/* exp(x) for |x| < 700 (the path only uses x in [-10, 0]). */
static inline double dm_exp(double x)
{
    double kd = floor(x * DM_INVLN2 + 0.5);
    int k = (int)kd;
    double hi = x - kd * DM_LN2_HI;
    double lo = kd * DM_LN2_LO;
    double r = hi - lo;
    double t = r * r;
    double c = r - t * (DM_EP1 + t * (DM_EP2 + t * (DM_EP3 + t * (DM_EP4 + t * DM_EP5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    /* scale by 2^k; k in [-1010, 1010] on every call site */
    return y * dm_from_bits((uint64_t)(k + 1023) << 52);
}

/* fdlibm e_log.c constants */
#define DM_LG1 6.666666666666735130e-01
#define DM_LG2 3.999999999940941908e-01
#define DM_LG3 2.857142874366239149e-01
#define DM_LG4 2.222219843214978396e-01
#define DM_LG5 1.818357216161805012e-01
#define DM_LG6 1.531383769920937332e-01
#define DM_LG7 1.479819860511658591e-01

/* log(x) for positive normal x (the path uses x in [2^-53, 1]). */
static inline double dm_log(double x)
{
    uint64_t u = dm_bits(x);
    int k = (int)((u >> 52) & 0x7ff) - 1023;
    uint64_t m = u & 0x000fffffffffffffULL;
    /* normalise mantissa into [sqrt(2)/2, sqrt(2)) */
    uint64_t i = (m + 0x95f6400000000ULL) & 0x0010000000000000ULL;
    double xm = dm_from_bits(m | (i ^ 0x3ff0000000000000ULL));
    k += (int)(i >> 52);
    double f = xm - 1.0;
    double s = f / (2.0 + f);
    double dk = (double)k;
    double z = s * s;
    double w = z * z;
    double t1 = w * (DM_LG2 + w * (DM_LG4 + w * DM_LG6));
    double t2 = z * (DM_LG1 + w * (DM_LG3 + w * (DM_LG5 + w * DM_LG7)));
    double R = t2 + t1;
    double hfsq = 0.5 * f * f;
    return dk * DM_LN2_HI - ((hfsq - (s * (hfsq + R) + dk * DM_LN2_LO)) - f);
}

/* fdlibm k_sin.c / k_cos.c constants */
#define DM_S1 -1.66666666666666324348e-01
#define DM_S2  8.33333333332248946124e-03
#define DM_S3 -1.98412698298579493134e-04
#define DM_S4  2.75573137070700676789e-06
#define DM_S5 -2.50507602534068634195e-08
#define DM_S6  1.58969099521155010221e-10
#define DM_C1  4.16666666666666019037e-02
#define DM_C2 -1.38888888888741095749e-03
#define DM_C3  2.48015872894767294178e-05
#define DM_C4 -2.75573143513906633035e-07
#define DM_C5  2.08757232129817482790e-09
#define DM_C6 -1.13596475577881948265e-11
#define DM_INVPIO2 6.36619772367581382433e-01
#define DM_PIO2_1  1.57079632673412561417e+00
#define DM_PIO2_1T 6.07710050650619224932e-11

static inline double dm_ksin(double x)
{
    double z = x * x;
    double v = z * x;
    double r = DM_S2 + z * (DM_S3 + z * (DM_S4 + z * (DM_S5 + z * DM_S6)));
    return x + v * (DM_S1 + z * r);
}

static inline double dm_kcos(double x)
{
    double z = x * x;
    double r = z * (DM_C1 + z * (DM_C2 + z * (DM_C3 + z * (DM_C4 + z * (DM_C5 + z * DM_C6)))));
    double hz = 0.5 * z;
    double w = 1.0 - hz;
    return w + (((1.0 - w) - hz) + z * r);
}

/* sin and cos together, |x| < 1e5 (joint angles and 2*pi*u). */
static inline void dm_sincos(double x, double* s, double* c)
{
    double kd = floor(x * DM_INVPIO2 + 0.5);
    double y = (x - kd * DM_PIO2_1) - kd * DM_PIO2_1T;
    int n = ((int)kd) & 3;
    double ks = dm_ksin(y);
    double kc = dm_kcos(y);
    switch (n) {
    case 0: *s = ks; *c = kc; break;
    case 1: *s = kc; *c = -ks; break;
    case 2: *s = -ks; *c = -kc; break;
    default: *s = -kc; *c = ks; break;
    }
}

#endif
