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

/* fdlibm s_atan.c: reduction to |x| < 7/16 about atan(0.5), atan(1), atan(1.5), atan(inf)
 * with hi/lo constants, then the odd/even minimax polynomial of degree 22. */
static const double dm_atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                   9.82793723247329054082e-01, 1.57079632679489655800e+00};
static const double dm_atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                   1.39033110312309984516e-17, 6.12323399573676603587e-17};
static const double dm_aT[11] = {3.33333333333329318027e-01, -1.99999999998764832476e-01,
                                 1.42857142725034663711e-01, -1.11111104054623557880e-01,
                                 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                 6.66107313738753120669e-02, -5.83357013379057348645e-02,
                                 4.97687799461593236017e-02, -3.65315727442169155270e-02,
                                 1.62858201153657823623e-02};

static inline double dm_atan(double x)
{
    const uint64_t u = dm_bits(x);
    const int32_t hx = (int32_t)(u >> 32);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {                 /* |x| >= 2^66 (or NaN) */
        if (x != x) return x + x;
        return hx > 0 ? dm_atanhi[3] + dm_atanlo[3] : -dm_atanhi[3] - dm_atanlo[3];
    }
    if (ix < 0x3fdc0000) {                  /* |x| < 0.4375 */
        if (ix < 0x3e400000) return x;      /* |x| < 2^-27 */
        id = -1;
    } else {
        x = fabs(x);
        if (ix < 0x3ff30000) {              /* |x| < 1.1875 */
            if (ix < 0x3fe60000) { id = 0; x = (2.0 * x - 1.0) / (2.0 + x); }
            else { id = 1; x = (x - 1.0) / (x + 1.0); }
        } else {
            if (ix < 0x40038000) { id = 2; x = (x - 1.5) / (1.0 + 1.5 * x); }
            else { id = 3; x = -1.0 / x; }
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (dm_aT[0] + w * (dm_aT[2] + w * (dm_aT[4] + w * (dm_aT[6] + w * (dm_aT[8] + w * dm_aT[10])))));
    const double s2 = w * (dm_aT[1] + w * (dm_aT[3] + w * (dm_aT[5] + w * (dm_aT[7] + w * dm_aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = dm_atanhi[id] - ((x * (s1 + s2) - dm_atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

/* fdlibm e_atan2.c */
#define DM_PI_O_4 7.8539816339744827900E-01
#define DM_PI_O_2 1.5707963267948965580E+00
#define DM_PI     3.1415926535897931160E+00
#define DM_PI_LO  1.2246467991473531772E-16

static inline double dm_atan2(double y, double x)
{
    if (x != x || y != y) return x + y;
    const uint64_t ux = dm_bits(x), uy = dm_bits(y);
    const int32_t hx = (int32_t)(ux >> 32), hy = (int32_t)(uy >> 32);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    const uint32_t lx = (uint32_t)ux, ly = (uint32_t)uy;
    if (x == 1.0) return dm_atan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);   /* 2 sign(x) + sign(y) */
    if ((iy | ly) == 0) {                                  /* y = +-0 */
        if (m <= 1) return y;
        return m == 2 ? DM_PI : -DM_PI;
    }
    if ((ix | lx) == 0) return hy < 0 ? -DM_PI_O_2 : DM_PI_O_2;
    if (ix == 0x7ff00000) {
        if (iy == 0x7ff00000) {
            switch (m) {
            case 0: return DM_PI_O_4;
            case 1: return -DM_PI_O_4;
            case 2: return 3.0 * DM_PI_O_4;
            default: return -3.0 * DM_PI_O_4;
            }
        }
        switch (m) {
        case 0: return 0.0;
        case 1: return -0.0;
        case 2: return DM_PI;
        default: return -DM_PI;
        }
    }
    if (iy == 0x7ff00000) return hy < 0 ? -DM_PI_O_2 : DM_PI_O_2;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = DM_PI_O_2 + 0.5 * DM_PI_LO;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = dm_atan(fabs(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return DM_PI - (z - DM_PI_LO);
    default: return (z - DM_PI_LO) - DM_PI;
    }
}

/* fdlibm e_asin.c */
static inline double dm_asin(double x)
{
    const double pio2_hi = 1.57079632679489655800e+00, pio2_lo = 6.12323399573676603587e-17,
                 pio4_hi = 7.85398163397448278999e-01;
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05;
    const double qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const uint64_t u = dm_bits(x);
    const int32_t hx = (int32_t)(u >> 32);
    const int32_t ix = hx & 0x7fffffff;
    double t, w, p, q, c, r, s;
    if (ix >= 0x3ff00000) {                 /* |x| >= 1 */
        if (((ix - 0x3ff00000) | (uint32_t)u) == 0) return x * pio2_hi + x * pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000) {                  /* |x| < 0.5 */
        if (ix < 0x3e400000) return x;
        t = x * x;
        p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
        q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
        w = p / q;
        return x + x * w;
    }
    w = 1.0 - fabs(x);
    t = w * 0.5;
    p = t * (pS0 + t * (pS1 + t * (pS2 + t * (pS3 + t * (pS4 + t * pS5)))));
    q = 1.0 + t * (qS1 + t * (qS2 + t * (qS3 + t * qS4)));
    s = sqrt(t);
    if (ix >= 0x3FEF3333) {                 /* |x| > 0.975 */
        w = p / q;
        t = pio2_hi - (2.0 * (s + s * w) - pio2_lo);
    } else {
        w = dm_from_bits(dm_bits(s) & 0xFFFFFFFF00000000ull);
        c = (t - w * w) / (s + w);
        r = p / q;
        p = 2.0 * s * r - (pio2_lo - 2.0 * c);
        q = pio4_hi - 2.0 * w;
        t = pio4_hi - (p - q);
    }
    return hx > 0 ? t : -t;
}

#endif
