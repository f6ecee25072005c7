/*
 * mp_jlmath.h — deterministic double-precision elementary functions.
 *
 * The reference (congkaishen/MotionPlanning) is pure Julia; its `sin`, `cos`,
 * `tan`, `atan`, `atan(y,x)`, `acos`, `asin` come from Julia's Base.Math, which
 * is a port of Sun's FDLIBM (the same algorithms as FreeBSD msun).  This header
 * restates those published FDLIBM algorithms once, as plain arithmetic, so that
 *
 *   - the HIP kernels (compiled by hipcc for gfx950, -ffp-contract=off) and
 *   - the CPU oracle   (compiled by gcc, -ffp-contract=off)
 *
 * evaluate the *same* operation sequence and therefore agree bit for bit.  That
 * is what makes the Hybrid A* discrete outputs (Encode indices, collision
 * booleans, pop order) comparable bit-exactly between GPU and CPU.
 *
 * Polynomial (Horner) steps use fused multiply-add, mirroring Julia's
 * `@horner` macro which expands to `muladd` (fused on FMA hardware).  Every
 * other operation is a separately rounded IEEE op; no contraction is allowed
 * anywhere else (both builds pass -ffp-contract=off).
 *
 * `exp` is Julia's own table-driven exp (base/special/exp.jl); `log` (only the
 * Box–Muller of the synthetic Philox noise, not a reference path) is FDLIBM's e_log.c.
 *
 * Accuracy vs glibc is checked in tests/test_jlmath.py (CPU) and the GPU
 * implementation is checked bit-exact against the CPU one in
 * tests/test_gpu_mppi.py::test_jlmath_bitexact.
 *
 * This header holds pure functions only; it is NOT the oracle (oracle/ is the
 * reference restatement, and it includes this header for its libm).
 */
#ifndef MP_JLMATH_H
#define MP_JLMATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define MPJ_FN __host__ __device__ static inline
#else
#define MPJ_FN static inline
#endif

typedef union { double d; uint64_t u; } mpj_du;

MPJ_FN uint32_t mpj_hi(double x) { mpj_du v; v.d = x; return (uint32_t)(v.u >> 32); }
MPJ_FN uint32_t mpj_lo(double x) { mpj_du v; v.d = x; return (uint32_t)(v.u & 0xffffffffu); }
MPJ_FN double mpj_from_words(uint32_t hi, uint32_t lo) {
  mpj_du v; v.u = ((uint64_t)hi << 32) | (uint64_t)lo; return v.d;
}
MPJ_FN double mpj_flip(double t, uint32_t signbit) { /* -t when signbit == 0x80000000 (exact negation) */
  return mpj_from_words(mpj_hi(t) ^ signbit, mpj_lo(t));
}

MPJ_FN double mpj_zero_lo(double x) { mpj_du v; v.d = x; v.u &= 0xffffffff00000000ull; return v.d; }
MPJ_FN double mpj_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
MPJ_FN double mpj_sqrt(double x) { return __builtin_sqrt(x); }
MPJ_FN double mpj_fabs(double x) { return __builtin_fabs(x); }
MPJ_FN int mpj_isnan(double x) { return x != x; }
/* Julia `round(::Float64)` = RoundNearest (ties to even) = rint in the default mode. */
MPJ_FN double mpj_round(double x) { return __builtin_rint(x); }
/* Julia `max` / `min` for Float64 (base/math.jl): NaN-propagating (C fmax/fmin drop a NaN operand)
 * and -0.0 < +0.0:  max(x, y) = ifelse((y > x) | (signbit(y) < signbit(x)), ifelse(isnan(x), x, y),
 * ifelse(isnan(y), y, x)), min with < and > swapped. */
MPJ_FN int mpj_signbit(double x) { return (int)(mpj_hi(x) >> 31); }
MPJ_FN double mpj_jmax(double x, double y) {
  const int ty = (y > x) | (mpj_signbit(y) < mpj_signbit(x));
  return ty ? (mpj_isnan(x) ? x : y) : (mpj_isnan(y) ? y : x);
}
MPJ_FN double mpj_jmin(double x, double y) {
  const int ty = (y < x) | (mpj_signbit(y) > mpj_signbit(x));
  return ty ? (mpj_isnan(x) ? x : y) : (mpj_isnan(y) ? y : x);
}

/* Repeated addition q_k = RN(q_{k-1} + c), k = 1..K (createActPath's heading recurrence and the running
 * sums of a straight segment, ReedsSheppsUtils.jl:440-466) in closed form.  When q_0, q_1 = RN(q_0 + c)
 * and q_0 + K·d (d = q_1 - q_0, exact) share sign and binade [2^e, 2^(e+1)), lie at least one ulp
 * u = 2^(e-52) inside it (two at the top), and q_0 + c is not a rounding tie, every step adds exactly d:
 * the real q_k + c equals q_{k+1} + err with the same TwoSum error |err| < u/2 on the same u-grid, so
 * q_k = q_0 + k·d = fma(k, d, q_0) (a representable multiple of u).  c == 0 is always closed: q_k = q_1
 * for k >= 1.  Returns 0 when the closed form does not apply (the caller adds serially). */
MPJ_FN int mpj_rep_add_ok(double q0, double c, int K, double* d) {
  const double q1 = q0 + c;
  *d = 0.0;
  if (c == 0.0) return 1;
  const double dd = q1 - q0;
  const double qK = mpj_fma((double)K, dd, q0);
  const uint32_t e0 = mpj_hi(q0) >> 20; /* sign + exponent */
  if ((mpj_hi(q1) >> 20) != e0 || (mpj_hi(qK) >> 20) != e0) return 0;
  const uint32_t ex = e0 & 0x7ffu;
  if (ex < 54u || ex >= 0x7ffu) return 0; /* zero, subnormal, tiny; Inf / NaN */
  const double lo = mpj_from_words(ex << 20, 0), u = mpj_from_words((ex - 52u) << 20, 0);
  const double hi = 2.0 * lo;
  const double a0 = mpj_fabs(q0), aK = mpj_fabs(qK);
  const double mn = a0 < aK ? a0 : aK, mx = a0 < aK ? aK : a0;
  if (!(mn >= lo + u) || !(mx <= hi - 2.0 * u)) return 0;
  const double bb = q1 - q0; /* TwoSum: the exact rounding error of q0 + c */
  const double err = (q0 - (q1 - bb)) + (c - bb);
  if (mpj_fabs(err) == 0.5 * u) return 0;
  *d = dd;
  return 1;
}

/* ---------------------------------------------------------------- sin/cos */
/* FDLIBM k_sin.c / k_cos.c (Julia base/special/trig.jl sin_kernel/cos_kernel). */
#define MPJ_S1 (-1.66666666666666324348e-01)
#define MPJ_S2 ( 8.33333333332248946124e-03)
#define MPJ_S3 (-1.98412698298579493134e-04)
#define MPJ_S4 ( 2.75573137070700676789e-06)
#define MPJ_S5 (-2.50507602534068634195e-08)
#define MPJ_S6 ( 1.58969099521155010221e-10)
#define MPJ_C1 ( 4.16666666666666019037e-02)
#define MPJ_C2 (-1.38888888888741095749e-03)
#define MPJ_C3 ( 2.48015872894767294178e-05)
#define MPJ_C4 (-2.75573143513906633035e-07)
#define MPJ_C5 ( 2.08757232129817482790e-09)
#define MPJ_C6 (-1.13596475577881948265e-11)

/* sin kernel on [-pi/4, pi/4]; lo != 0 form used after argument reduction. */
MPJ_FN double mpj_sin_k0(double x) {
  double z = x * x, w = z * z;
  double r = mpj_fma(z, mpj_fma(z, MPJ_S4, MPJ_S3), MPJ_S2) + z * w * mpj_fma(z, MPJ_S6, MPJ_S5);
  double v = z * x;
  return x + v * (MPJ_S1 + z * r);
}
MPJ_FN double mpj_sin_k(double x, double y) {
  double z = x * x, w = z * z;
  double r = mpj_fma(z, mpj_fma(z, MPJ_S4, MPJ_S3), MPJ_S2) + z * w * mpj_fma(z, MPJ_S6, MPJ_S5);
  double v = z * x;
  return x - ((z * (0.5 * y - v * r) - y) - v * MPJ_S1);
}
MPJ_FN double mpj_cos_k(double x, double y) {
  double z = x * x, w = z * z;
  double r = z * mpj_fma(z, mpj_fma(z, MPJ_C3, MPJ_C2), MPJ_C1) +
             w * w * mpj_fma(z, mpj_fma(z, MPJ_C6, MPJ_C5), MPJ_C4);
  double hz = 0.5 * z;
  double ww = 1.0 - hz;
  return ww + (((1.0 - ww) - hz) + (z * r - x * y));
}

/* Cody–Waite reduction by pi/2 (FDLIBM e_rem_pio2.c, Julia rem_pio2_kernel).
 * Valid for |x| < 2^20*pi/2; beyond that Julia switches to Payne–Hanek, which
 * no input of this hot path reaches (states are angles of a few radians). */
#define MPJ_PIO2_1  1.57079632673412561417e+00
#define MPJ_PIO2_1T 6.07710050650619224932e-11
#define MPJ_PIO2_2  6.07710050630396597660e-11
#define MPJ_PIO2_2T 2.02226624879595063154e-21
#define MPJ_PIO2_3  2.02226624871116645580e-21
#define MPJ_PIO2_3T 8.47842766036889956997e-32
#define MPJ_INVPIO2 6.36619772367581382433e-01

MPJ_FN int mpj_cw2c(double x, double fn, int n, double* y0, double* y1) {
  double z = x - fn * MPJ_PIO2_1;
  double a = z - fn * MPJ_PIO2_1T;
  *y0 = a;
  *y1 = (z - a) - fn * MPJ_PIO2_1T;
  return n;
}
MPJ_FN int mpj_cwext(double x, uint32_t xhp, double* y0, double* y1) {
  double fn = mpj_round(x * MPJ_INVPIO2);
  double r = mpj_fma(-fn, MPJ_PIO2_1, x);
  double w = fn * MPJ_PIO2_1T;
  int32_t j = (int32_t)(xhp >> 20);
  double a = r - w;
  int32_t i = j - (int32_t)((mpj_hi(a) >> 20) & 0x7ff);
  if (i > 16) {
    double t = r;
    w = fn * MPJ_PIO2_2;
    r = t - w;
    w = mpj_fma(fn, MPJ_PIO2_2T, -((t - r) - w));
    a = r - w;
    i = j - (int32_t)((mpj_hi(a) >> 20) & 0x7ff);
    if (i > 49) {
      t = r;
      w = fn * MPJ_PIO2_3;
      r = t - w;
      w = mpj_fma(fn, MPJ_PIO2_3T, -((t - r) - w));
      a = r - w;
    }
  }
  *y0 = a;
  *y1 = (r - a) - w;
  return (int)fn;
}
MPJ_FN int mpj_rem_pio2(double x, double* y0, double* y1) {
  uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  if (xhp <= 0x400f6a7au) {
    if ((xhp & 0xfffffu) == 0x921fbu) return mpj_cwext(x, xhp, y0, y1);
    if (xhp <= 0x4002d97cu)
      return x > 0.0 ? mpj_cw2c(x, 1.0, 1, y0, y1) : mpj_cw2c(x, -1.0, -1, y0, y1);
    return x > 0.0 ? mpj_cw2c(x, 2.0, 2, y0, y1) : mpj_cw2c(x, -2.0, -2, y0, y1);
  }
  if (xhp <= 0x401c463bu) {
    if (xhp <= 0x4015fdbcu) {
      if (xhp == 0x4012d97cu) return mpj_cwext(x, xhp, y0, y1);
      return x > 0.0 ? mpj_cw2c(x, 3.0, 3, y0, y1) : mpj_cw2c(x, -3.0, -3, y0, y1);
    }
    if (xhp == 0x401921fbu) return mpj_cwext(x, xhp, y0, y1);
    return x > 0.0 ? mpj_cw2c(x, 4.0, 4, y0, y1) : mpj_cw2c(x, -4.0, -4, y0, y1);
  }
  return mpj_cwext(x, xhp, y0, y1);
}

#define MPJ_PIO4 7.85398163397448278999e-01
/* sqrt(eps(Float64)) and sqrt(eps/2): Julia's small-argument cut-offs. */
#define MPJ_SQRT_EPS 1.4901161193847656e-08
#define MPJ_SQRT_HALF_EPS 1.0536712127723509e-08

MPJ_FN double mpj_sin(double x) {
  double ax = mpj_fabs(x);
  if (ax < MPJ_PIO4) {
    if (ax < MPJ_SQRT_EPS) return x;
    return mpj_sin_k0(x);
  }
  if (mpj_isnan(x) || ax == __builtin_inf()) return x - x;
  double y0, y1;
  int n = mpj_rem_pio2(x, &y0, &y1) & 3;
  if (n == 0) return mpj_sin_k(y0, y1);
  if (n == 1) return mpj_cos_k(y0, y1);
  if (n == 2) return -mpj_sin_k(y0, y1);
  return -mpj_cos_k(y0, y1);
}
MPJ_FN double mpj_cos(double x) {
  double ax = mpj_fabs(x);
  if (ax < MPJ_PIO4) {
    if (ax < MPJ_SQRT_HALF_EPS) return 1.0;
    return mpj_cos_k(x, 0.0);
  }
  if (mpj_isnan(x) || ax == __builtin_inf()) return x - x;
  double y0, y1;
  int n = mpj_rem_pio2(x, &y0, &y1) & 3;
  if (n == 0) return mpj_cos_k(y0, y1);
  if (n == 1) return -mpj_sin_k(y0, y1);
  if (n == 2) return -mpj_cos_k(y0, y1);
  return mpj_sin_k(y0, y1);
}
/* sin and cos sharing one reduction; bit-identical to mpj_sin / mpj_cos. */
MPJ_FN void mpj_sincos(double x, double* s, double* c) {
  double ax = mpj_fabs(x);
  if (ax < MPJ_PIO4) {
    *s = ax < MPJ_SQRT_EPS ? x : mpj_sin_k0(x);
    *c = ax < MPJ_SQRT_HALF_EPS ? 1.0 : mpj_cos_k(x, 0.0);
    return;
  }
  if (mpj_isnan(x) || ax == __builtin_inf()) { *s = x - x; *c = x - x; return; }
  double y0, y1;
  int n = mpj_rem_pio2(x, &y0, &y1) & 3;
  double sk = mpj_sin_k(y0, y1), ck = mpj_cos_k(y0, y1);
  if (n == 0) { *s = sk; *c = ck; }
  else if (n == 1) { *s = ck; *c = -sk; }
  else if (n == 2) { *s = -sk; *c = -ck; }
  else { *s = -ck; *c = sk; }
}

/* -------------------------------------------------------------------- tan */
/* FDLIBM k_tan.c / s_tan.c */
MPJ_FN double mpj_tan_k(double x, double y, int iy) {
  const double T0 = 3.33333333333334091986e-01, T1 = 1.33333333333201242699e-01,
               T2 = 5.39682539762260521377e-02, T3 = 2.18694882948595424599e-02,
               T4 = 8.86323982359930005737e-03, T5 = 3.59207910759131235356e-03,
               T6 = 1.45620945432529025516e-03, T7 = 5.88041240820264096874e-04,
               T8 = 2.46463134818469906812e-04, T9 = 7.81794442939557092300e-05,
               T10 = 7.14072491382608190305e-05, T11 = -1.85586374855275456654e-05,
               T12 = 2.59073051863633712884e-05, pio4lo = 3.06161699786838301793e-17;
  int32_t hx = (int32_t)mpj_hi(x);
  int32_t ix = hx & 0x7fffffff;
  double z, r, v, w, s;
  if (ix >= 0x3FE59428) {
    if (hx < 0) { x = -x; y = -y; }
    z = MPJ_PIO4 - x;
    w = pio4lo - y;
    x = z + w;
    y = 0.0;
  }
  z = x * x;
  w = z * z;
  r = mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T11, T9), T7), T5), T3), T1);
  v = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T12, T10), T8), T6), T4), T2);
  s = z * x;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  w = x + r;
  if (ix >= 0x3FE59428) {
    v = (double)iy;
    return (double)(1 - ((hx >> 30) & 2)) * (v - 2.0 * (x - (w * w / (w + v) - r)));
  }
  if (iy == 1) return w;
  {
    double a, t;
    z = mpj_zero_lo(w);
    v = r - (z - x);
    t = a = -1.0 / w;
    t = mpj_zero_lo(t);
    s = 1.0 + t * z;
    return t + a * (s + t * v);
  }
}
MPJ_FN double mpj_tan(double x) {
  uint32_t ix = mpj_hi(x) & 0x7fffffffu;
  if (ix <= 0x3fe921fbu) {
    if (ix < 0x3e400000u) return x;
    return mpj_tan_k(x, 0.0, 1);
  }
  if (ix >= 0x7ff00000u) return x - x;
  double y0, y1;
  int n = mpj_rem_pio2(x, &y0, &y1);
  return mpj_tan_k(y0, y1, 1 - ((n & 1) << 1));
}

/* ------------------------------------------------------------------- atan */
/* FDLIBM s_atan.c (Julia base/special/trig.jl atan).  The four reduction
 * branches are expressed as one division with selected constants; every
 * branch's expression is reproduced exactly (e.g. 1*x, 0+x are exact). */
MPJ_FN double mpj_atan(double x) {
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  uint32_t hx = mpj_hi(x);
  uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x44100000u) { /* |x| >= 2^66 */
    if (mpj_isnan(x)) return x + x;
    const double hi3 = 1.57079632679489655800e+00, lo3 = 6.12323399573676603587e-17;
    return (hx >> 31) ? -hi3 - lo3 : hi3 + lo3;
  }
  int id;
  double ax;
  double hi = 0.0, lo = 0.0;
  if (ix < 0x3fdc0000u) { /* |x| < 0.4375 */
    if (ix < 0x3e400000u) return x;
    id = -1;
    ax = x;
  } else {
    double a = mpj_fabs(x), na, nb, dc, dd;
    if (ix < 0x3ff30000u) {
      if (ix < 0x3fe60000u) { id = 0; na = 2.0; nb = 1.0; dc = 2.0; dd = 1.0;
        hi = 4.63647609000806093515e-01; lo = 2.26987774529616870924e-17; }
      else { id = 1; na = 1.0; nb = 1.0; dc = 1.0; dd = 1.0;
        hi = 7.85398163397448278999e-01; lo = 3.06161699786838301793e-17; }
    } else {
      if (ix < 0x40038000u) { id = 2; na = 1.0; nb = 1.5; dc = 1.0; dd = 1.5;
        hi = 9.82793723247329054082e-01; lo = 1.39033110312309984516e-17; }
      else { id = 3; na = 0.0; nb = 1.0; dc = 0.0; dd = 1.0;
        hi = 1.57079632679489655800e+00; lo = 6.12323399573676603587e-17; }
    }
    /* id0: (2x-1)/(2+x); id1: (x-1)/(1+x) [== (x-1)/(x+1)];
     * id2: (x-1.5)/(1+1.5x); id3: -1/x  ==  (0*x-1)/(0+1*x)   (x > 0) */
    ax = (na * a - nb) / (dc + dd * a);
  }
  double z = ax * ax;
  double w = z * z;
  double s1 = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT10, aT8), aT6), aT4), aT2), aT0);
  double s2 = w * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT9, aT7), aT5), aT3), aT1);
  if (id < 0) return ax - ax * (s1 + s2);
  double r = hi - ((ax * (s1 + s2) - lo) - ax);
  return (hx >> 31) ? -r : r;
}

/* FDLIBM e_atan2.c (Julia atan(y, x)). */
MPJ_FN double mpj_atan2(double y, double x) {
  const double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
               pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
  if (mpj_isnan(x) || mpj_isnan(y)) return x + y;
  uint32_t hx = mpj_hi(x), lx = mpj_lo(x), hy = mpj_hi(y), ly = mpj_lo(y);
  int32_t ix = (int32_t)(hx & 0x7fffffffu), iy = (int32_t)(hy & 0x7fffffffu);
  if (hx == 0x3ff00000u && lx == 0) return mpj_atan(y);
  int m = (int)(((hy >> 31) & 1) | ((hx >> 30) & 2));
  if ((iy | (int32_t)ly) == 0) {
    if (m == 0 || m == 1) return y;
    return m == 2 ? pi : -pi;
  }
  if ((ix | (int32_t)lx) == 0) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      if (m == 0) return pi_o_4;
      if (m == 1) return -pi_o_4;
      if (m == 2) return 3.0 * pi_o_4;
      return -3.0 * pi_o_4;
    }
    if (m == 0) return 0.0;
    if (m == 1) return -0.0;
    if (m == 2) return pi;
    return -pi;
  }
  if (iy == 0x7ff00000) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  int32_t k = (iy - ix) >> 20;
  double z;
  if (k > 60) { z = pi_o_2 + 0.5 * pi_lo; m &= 1; }
  else if ((hx >> 31) && k < -60) z = 0.0;
  else z = mpj_atan(mpj_fabs(y / x));
  if (m == 0) return z;
  if (m == 1) return -z;
  if (m == 2) return pi - (z - pi_lo);
  return (z - pi_lo) - pi;
}

/* ------------------------------------------------------------ asin / acos */
/* FDLIBM e_asin.c / e_acos.c; the rational R(t)=p/q as in Julia's arc_p/arc_q. */
MPJ_FN double mpj_arc_p(double t) {
  return t * mpj_fma(t, mpj_fma(t, mpj_fma(t, mpj_fma(t, mpj_fma(t,
             3.47933107596021167570e-05, 7.91534994289814532176e-04),
             -4.00555345006794114027e-02), 2.01212532134862925881e-01),
             -3.25565818622400915405e-01), 1.66666666666666657415e-01);
}
MPJ_FN double mpj_arc_q(double t) {
  return mpj_fma(t, mpj_fma(t, mpj_fma(t, mpj_fma(t,
             7.70381505559019352791e-02, -6.88283971605453293030e-01),
             2.02094576023350569471e+00), -2.40339491173441421878e+00), 1.0);
}
#define MPJ_PIO2_HI 1.57079632679489655800e+00
#define MPJ_PIO2_LO 6.12323399573676603587e-17
#define MPJ_PIO4_HI 7.85398163397448278999e-01
#define MPJ_PI 3.14159265358979311600e+00

MPJ_FN double mpj_asin(double x) {
  uint32_t hx = mpj_hi(x);
  uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x3ff00000u) {
    if (((ix - 0x3ff00000u) | mpj_lo(x)) == 0) return x * MPJ_PIO2_HI + x * MPJ_PIO2_LO;
    return (x - x) / (x - x); /* NaN: Julia throws DomainError here */
  }
  if (ix < 0x3fe00000u) {
    if (ix < 0x3e500000u) return x;
    double t = x * x;
    double w = mpj_arc_p(t) / mpj_arc_q(t);
    return x + x * w;
  }
  double w = 1.0 - mpj_fabs(x);
  double t = w * 0.5;
  double p = mpj_arc_p(t), q = mpj_arc_q(t);
  double s = mpj_sqrt(t);
  if (ix >= 0x3FEF3333u) {
    w = p / q;
    t = MPJ_PIO2_HI - (2.0 * (s + s * w) - MPJ_PIO2_LO);
  } else {
    double ww = mpj_zero_lo(s);
    double c = (t - ww * ww) / (s + ww);
    double r = p / q;
    p = 2.0 * s * r - (MPJ_PIO2_LO - 2.0 * c);
    q = MPJ_PIO4_HI - 2.0 * ww;
    t = MPJ_PIO4_HI - (p - q);
  }
  return (hx >> 31) ? -t : t;
}
MPJ_FN double mpj_acos(double x) {
  uint32_t hx = mpj_hi(x);
  uint32_t ix = hx & 0x7fffffffu;
  if (ix >= 0x3ff00000u) {
    if (((ix - 0x3ff00000u) | mpj_lo(x)) == 0) return (hx >> 31) ? MPJ_PI + 2.0 * MPJ_PIO2_LO : 0.0;
    return (x - x) / (x - x); /* NaN: Julia throws DomainError here */
  }
  if (ix < 0x3fe00000u) {
    if (ix <= 0x3c600000u) return MPJ_PIO2_HI + MPJ_PIO2_LO;
    double z = x * x;
    double r = mpj_arc_p(z) / mpj_arc_q(z);
    return MPJ_PIO2_HI - (x - (MPJ_PIO2_LO - x * r));
  }
  if (hx >> 31) {
    double z = (1.0 + x) * 0.5;
    double s = mpj_sqrt(z);
    double r = mpj_arc_p(z) / mpj_arc_q(z);
    double w = r * s - MPJ_PIO2_LO;
    return MPJ_PI - 2.0 * (s + w);
  }
  double z = (1.0 - x) * 0.5;
  double s = mpj_sqrt(z);
  double df = mpj_zero_lo(s);
  double c = (z - df * df) / (s + df);
  double r = mpj_arc_p(z) / mpj_arc_q(z);
  double w = r * s + c;
  return 2.0 * (df + w);
}

/* -------------------------------------------------------------- exp / log */
/* Julia >= 1.6 `exp(::Float64)` (base/special/exp.jl, exp_impl with base e): reduction
 * N = round(x * 256/ln2) by the 1.5*2^52 shift (muladd), r = x - N*ln2/256 in two fused steps
 * (Cody-Waite hi/lo), 2^(j/256) from the packed 256-entry table (hi part jU rounded down,
 * lo part jL from 12 packed bits; tools/gen_jl_exp_table.py regenerates it), expm1 on
 * |r| <= ln2/512 by the degree-4 minimax polynomial (evalpoly = nested muladd), and the result
 * 2^k * (jU + jU*p(r) + jL) assembled by an integer add into the exponent field.  Julia JITs
 * `muladd` to a fused multiply-add on FMA hardware (every x86-64 since Haswell, and gfx950),
 * so every muladd is mpj_fma here.  Max error ~0.52 ulp (tests/test_jlmath.py). */
static const uint64_t mpj_exp_jtab[256] = {
    0x0000000000000000ull, 0xaac00b1afa5abcbeull, 0x9b60163da9fb3335ull, 0xab502168143b0280ull,
    0xadc02c9a3e778060ull, 0x656037d42e11bbccull, 0xa7a04315e86e7f84ull, 0x84c04e5f72f654b1ull,
    0x8d7059b0d3158574ull, 0xa510650a0e3c1f88ull, 0xa8d0706b29ddf6ddull, 0x83207bd42b72a836ull,
    0x6180874518759bc8ull, 0xa4b092bdf66607dfull, 0x91409e3ecac6f383ull, 0x85d0a9c79b1f3919ull,
    0x98a0b5586cf9890full, 0x94f0c0f145e46c85ull, 0x9010cc922b7247f7ull, 0xa210d83b23395debull,
    0x4030e3ec32d3d1a2ull, 0xa5b0efa55fdfa9c4ull, 0xae40fb66affed31aull, 0x8d41073028d7233eull,
    0xa4911301d0125b50ull, 0xa1a11edbab5e2ab5ull, 0xaf712abdc06c31cbull, 0xae8136a814f204aaull,
    0xa661429aaea92ddfull, 0xa9114e95934f312dull, 0x82415a98c8a58e51ull, 0x58f166a45471c3c2ull,
    0xab9172b83c7d517aull, 0x70917ed48695bbc0ull, 0xa7718af9388c8de9ull, 0x94a1972658375d2full,
    0x8e51a35beb6fcb75ull, 0x97b1af99f8138a1cull, 0xa351bbe084045cd3ull, 0x9001c82f95281c6bull,
    0x9e01d4873168b9aaull, 0xa481e0e75eb44026ull, 0xa711ed5022fcd91cull, 0xa201f9c18438ce4cull,
    0x8dc2063b88628cd6ull, 0x935212be3578a819ull, 0x82a21f49917ddc96ull, 0x8d322bdda27912d1ull,
    0x99b2387a6e756238ull, 0x8ac2451ffb82140aull, 0x8ac251ce4fb2a63full, 0x93e25e85711ece75ull,
    0x82b26b4565e27cddull, 0x9e02780e341ddf29ull, 0xa2d284dfe1f56380ull, 0xab4291ba7591bb6full,
    0x86129e9df51fdee1ull, 0xa352ab8a66d10f12ull, 0xafb2b87fd0dad98full, 0xa572c57e39771b2eull,
    0x9002d285a6e4030bull, 0x9d12df961f641589ull, 0x71c2ecafa93e2f56ull, 0xaea2f9d24abd886aull,
    0x86f306fe0a31b715ull, 0x89531432edeeb2fdull, 0x8a932170fc4cd831ull, 0xa1d32eb83ba8ea31ull,
    0x93233c08b26416ffull, 0xab23496266e3fa2cull, 0xa92356c55f929ff0ull, 0xa8f36431a2de883aull,
    0xa4e371a7373aa9caull, 0xa3037f26231e7549ull, 0xa0b38cae6d05d865ull, 0xa3239a401b7140eeull,
    0xad43a7db34e59ff6ull, 0x9543b57fbfec6cf4ull, 0xa083c32dc313a8e4ull, 0x7fe3d0e544ede173ull,
    0x8ad3dea64c123422ull, 0xa943ec70df1c5174ull, 0xa413fa4504ac801bull, 0x8bd40822c367a024ull,
    0xaf04160a21f72e29ull, 0xa3d423fb27094689ull, 0xab8431f5d950a896ull, 0x88843ffa3f84b9d4ull,
    0x48944e086061892dull, 0xae745c2042a7d231ull, 0x9c946a41ed1d0057ull, 0xa1e4786d668b3236ull,
    0x73c486a2b5c13cd0ull, 0xab1494e1e192aed1ull, 0x99c4a32af0d7d3deull, 0xabb4b17dea6db7d6ull,
    0x7d44bfdad5362a27ull, 0x9054ce41b817c114ull, 0x98e4dcb299fddd0dull, 0xa564eb2d81d8abfeull,
    0xa5a4f9b2769d2ca6ull, 0x7a2508417f4531eeull, 0xa82516daa2cf6641ull, 0xac65257de83f4eeeull,
    0xabe5342b569d4f81ull, 0x879542e2f4f6ad27ull, 0xa8a551a4ca5d920eull, 0xa7856070dde910d1ull,
    0x99b56f4736b527daull, 0xa7a57e27dbe2c4ceull, 0x82958d12d497c7fdull, 0xa4059c0827ff07cbull,
    0x9635ab07dd485429ull, 0xa245ba11fba87a02ull, 0x3c45c9268a5946b7ull, 0xa195d84590998b92ull,
    0x9ba5e76f15ad2148ull, 0xa985f6a320dceb70ull, 0xa60605e1b976dc08ull, 0x9e46152ae6cdf6f4ull,
    0xa636247eb03a5584ull, 0x984633dd1d1929fdull, 0xa8e6434634ccc31full, 0xa28652b9febc8fb6ull,
    0xa226623882552224ull, 0xa85671c1c70833f5ull, 0x60368155d44ca973ull, 0x880690f4b19e9538ull,
    0xa216a09e667f3bccull, 0x7a36b052fa75173eull, 0xada6c012750bdabeull, 0x9c76cfdcddd47645ull,
    0xae46dfb23c651a2eull, 0xa7a6ef9298593ae4ull, 0xa9f6ff7df9519483ull, 0x59d70f7466f42e87ull,
    0xaba71f75e8ec5f73ull, 0xa6f72f8286ead089ull, 0xa7a73f9a48a58173ull, 0x90474fbd35d7cbfdull,
    0xa7e75feb564267c8ull, 0x9b777024b1ab6e09ull, 0x986780694fde5d3full, 0x934790b938ac1cf6ull,
    0xaaf7a11473eb0186ull, 0xa207b17b0976cfdaull, 0x9f17c1ed0130c132ull, 0x91b7d26a62ff86f0ull,
    0x7057e2f336cf4e62ull, 0xabe7f3878491c490ull, 0xa6c80427543e1a11ull, 0x946814d2add106d9ull,
    0xa1582589994cce12ull, 0x9998364c1eb941f7ull, 0xa9c8471a4623c7acull, 0xaf2857f4179f5b20ull,
    0xa01868d99b4492ecull, 0x85d879cad931a436ull, 0x99988ac7d98a6699ull, 0x9d589bd0a478580full,
    0x96e8ace5422aa0dbull, 0x9ec8be05bad61778ull, 0xade8cf3216b5448bull, 0xa478e06a5e0866d8ull,
    0x85c8f1ae99157736ull, 0x959902fed0282c8aull, 0xa119145b0b91ffc5ull, 0xab2925c353aa2fe1ull,
    0xae893737b0cdc5e4ull, 0xa88948b82b5f98e4ull, 0xad395a44cbc8520eull, 0xaf296bdd9a7670b2ull,
    0xa1797d829fde4e4full, 0x7ca98f33e47a22a2ull, 0xa749a0f170ca07b9ull, 0xa119b2bb4d53fe0cull,
    0x7c79c49182a3f090ull, 0xa579d674194bb8d4ull, 0x7829e86319e32323ull, 0xaad9fa5e8d07f29dull,
    0xa65a0c667b5de564ull, 0x9c6a1e7aed8eb8bbull, 0x963a309bec4a2d33ull, 0xa2aa42c980460ad7ull,
    0xa16a5503b23e255cull, 0x650a674a8af46052ull, 0x9bca799e1330b358ull, 0xa58a8bfe53c12e58ull,
    0x90fa9e6b5579fdbfull, 0x889ab0e521356ebaull, 0xa81ac36bbfd3f379ull, 0x97ead5ff3a3c2774ull,
    0x97aae89f995ad3adull, 0xa5aafb4ce622f2feull, 0xa21b0e07298db665ull, 0x94db20ce6c9a8952ull,
    0xaedb33a2b84f15faull, 0xac1b468415b749b0ull, 0xa1cb59728de55939ull, 0x92ab6c6e29f1c52aull,
    0xad5b7f76f2fb5e46ull, 0xa24b928cf22749e3ull, 0xa08ba5b030a10649ull, 0xafcbb8e0b79a6f1eull,
    0x823bcc1e904bc1d2ull, 0xafcbdf69c3f3a206ull, 0xa08bf2c25bd71e08ull, 0xa89c06286141b33cull,
    0x811c199bdd85529cull, 0xa48c2d1cd9fa652bull, 0x9b4c40ab5fffd07aull, 0x912c544778fafb22ull,
    0x928c67f12e57d14bull, 0xa86c7ba88988c932ull, 0x71ac8f6d9406e7b5ull, 0xaa0ca3405751c4daull,
    0x750cb720dcef9069ull, 0xac5ccb0f2e6d1674ull, 0xa88cdf0b555dc3f9ull, 0xa2fcf3155b5bab73ull,
    0xa1ad072d4a07897bull, 0x955d1b532b08c968ull, 0xa15d2f87080d89f1ull, 0x93dd43c8eacaa1d6ull,
    0x82ed5818dcfba487ull, 0x5fed6c76e862e6d3ull, 0xa77d80e316c98397ull, 0x9a0d955d71ff6075ull,
    0x9c2da9e603db3285ull, 0xa24dbe7cd63a8314ull, 0x92ddd321f301b460ull, 0xa1ade7d5641c0657ull,
    0xa72dfc97337b9b5eull, 0xadae11676b197d16ull, 0xa42e264614f5a128ull, 0xa30e3b333b16ee11ull,
    0x839e502ee78b3ff6ull, 0xaa7e653924676d75ull, 0x92de7a51fbc74c83ull, 0xa77e8f7977cdb73full,
    0xa0bea4afa2a490d9ull, 0x948eb9f4867cca6eull, 0xa1becf482d8e67f0ull, 0x91cee4aaa2188510ull,
    0x9dcefa1bee615a27ull, 0xa66f0f9c1cb64129ull, 0x93af252b376bba97ull, 0xacdf3ac948dd7273ull,
    0x99df50765b6e4540ull, 0x9faf6632798844f8ull, 0xa12f7bfdad9cbe13ull, 0xaeef91d802243c88ull,
    0x874fa7c1819e90d8ull, 0xacdfbdba3692d513ull, 0x62efd3c22b8f71f1ull, 0x74afe9d96b2a23d9ull};
MPJ_FN double mpj_exp(double x) {
  const double magic = 6.755399441055744e15; /* 1.5 * 2^52 */
  double nf = mpj_fma(x, 369.3299304675746, magic);
  mpj_du nb; nb.d = nf;
  const int32_t n = (int32_t)(uint32_t)nb.u;
  nf = nf - magic;
  double r = mpj_fma(nf, -0.002707606173999011, x);
  r = mpj_fma(nf, -6.327543041662719e-14, r);
  const int32_t k = n >> 8;
  const uint64_t j = mpj_exp_jtab[n & 255];
  mpj_du ju, jl;
  ju.u = 0x3FF0000000000000ull | (j & 0x000FFFFFFFFFFFFFull);
  jl.u = 0x3C00000000000000ull | (j >> 8);
  const double p = mpj_fma(r, mpj_fma(r, mpj_fma(r, 0.04166666857598777, 0.1666666857598779), 0.4999999999999997),
                           0.9999999999999912);
  mpj_du sp;
  sp.d = mpj_fma(ju.d, r * p, jl.d) + ju.d;
  if (!(__builtin_fabs(x) <= 708.3964185322641)) {
    if (x != x) return x;
    if (x >= 709.782712893384) return __builtin_inf();
    if (x <= -745.1332191019412) return 0.0;
    if (k <= -53) {
      mpj_du o; o.u = ((uint64_t)(int64_t)(k + 53) << 52) + sp.u;
      return o.d * 1.1102230246251565e-16; /* 0x1p-53 */
    }
  }
  mpj_du o; o.u = ((uint64_t)(int64_t)k << 52) + sp.u; /* Int64(k) << 52, wrapping add */
  return o.d;
}

/* FDLIBM e_exp.c (the round-1/2 exp; kept for tools/ilqr_ulp_sources.py and the accuracy tests) */
MPJ_FN double mpj_exp_fdlibm(double x) {
  const double o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02,
               ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  uint32_t hx = mpj_hi(x);
  int xsb = (int)(hx >> 31);
  hx &= 0x7fffffffu;
  double hi = 0.0, lo = 0.0;
  int k = 0;
  if (hx >= 0x40862E42u) {
    if (hx >= 0x7ff00000u) {
      if (mpj_isnan(x)) return x + x;
      return xsb == 0 ? x : 0.0;
    }
    if (x > o_threshold) return __builtin_inf();
    if (x < u_threshold) return 0.0;
  }
  if (hx > 0x3fd62e42u) {
    if (hx < 0x3FF0A2B2u) {
      hi = xsb ? x + ln2HI : x - ln2HI;
      lo = xsb ? -ln2LO : ln2LO;
      k = 1 - xsb - xsb;
    } else {
      k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
      double t = (double)k;
      hi = x - t * ln2HI;
      lo = t * ln2LO;
    }
    x = hi - lo;
  } else if (hx < 0x3e300000u) {
    return 1.0 + x;
  }
  double t = x * x;
  double twopk;
  if (k >= -1021) twopk = mpj_from_words(0x3ff00000u + ((uint32_t)k << 20), 0);
  else twopk = mpj_from_words(0x3ff00000u + ((uint32_t)(k + 1000) << 20), 0);
  double c = x - t * mpj_fma(t, mpj_fma(t, mpj_fma(t, mpj_fma(t, P5, P4), P3), P2), P1);
  if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
  double y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
  if (k >= -1021) {
    if (k == 1024) return y * 2.0 * 8.98846567431157953865e+307;
    return y * twopk;
  }
  return y * twopk * 9.33263618503218878990e-302; /* 2^-1000 */
}

/* FDLIBM e_log.c (used only for the Box–Muller noise of the Philox mode). */
MPJ_FN double mpj_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               two54 = 1.80143985094819840000e+16,
               Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int32_t hx = (int32_t)mpj_hi(x);
  uint32_t lx = mpj_lo(x);
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -__builtin_inf();
    if (hx < 0) return (x - x) / (x - x);
    k -= 54;
    x *= two54;
    hx = (int32_t)mpj_hi(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  x = mpj_from_words((uint32_t)(hx | (i ^ 0x3ff00000)), mpj_lo(x));
  k += (i >> 20);
  double f = x - 1.0;
  double dk;
  if ((0x000fffff & (2 + hx)) < 3) {
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    double R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  double s = f / (2.0 + f);
  dk = (double)k;
  double z = s * s;
  i = hx - 0x6147a;
  double w = z * z;
  int32_t j = 0x6b851 - hx;
  double t1 = w * mpj_fma(w, mpj_fma(w, Lg6, Lg4), Lg2);
  double t2 = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, Lg7, Lg5), Lg3), Lg1);
  i |= j;
  double R = t2 + t1;
  if (i > 0) {
    double hfsq = 0.5 * f * f;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  if (k == 0) return f - s * (f - R);
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}


/* ------------------------------------------------- branchless hot variants */
/* Bit-identical to mpj_atan / mpj_sin / mpj_cos / mpj_sincos (checked on CPU in
 * tests/test_jlmath.py and on the GPU in tests/test_gpu_mppi.py), written with
 * selects instead of branches so a wavefront whose lanes fall in different
 * argument ranges executes ONE straight-line instruction stream (no exec-mask
 * serialisation) and independent chains can be interleaved by the scheduler.
 * On the device MPJ_SEL is a forced v_cndmask pair (hipcc otherwise re-forms
 * branches from nested ternaries).  Arguments outside the fast range of sincos
 * take the exact routine through a wave-uniform branch. */
/* MPJ_LANE_SAFE (set by kernels whose callers run these routines under divergent control
 * flow, e.g. hastar.hip): no wave-level operations at all — per-lane slow-path branches and
 * plain selects — so the result never depends on which lanes are active. */
#if defined(__HIP_DEVICE_COMPILE__) && !defined(MPJ_LANE_SAFE)
#if defined(MPJ_COUNT_HOT_PATH)
#define MPJ_ANY(c) 0  /* instruction-count builds only (tools/isa_count.py): slow paths compiled out, */
#define MPJ_ANYG(c) 1 /* general paths of the optional wave-uniform fast paths kept                   */
#else
#define MPJ_ANY(c) __any((int)(c))  /* wave-uniform: some lane needs the exact slow path */
#define MPJ_ANYG(c) __any((int)(c)) /* wave-uniform: some lane needs the general path    */
#endif
__device__ __forceinline__ double mpj_sel(int c, double t, double f) {
  const unsigned long long m = __ballot(c);
  unsigned rl, rh;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(rl) : "v"(__double2loint(f)), "v"(__double2loint(t)), "s"(m));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(rh) : "v"(__double2hiint(f)), "v"(__double2hiint(t)), "s"(m));
  return __hiloint2double((int)rh, (int)rl);
}
#define MPJ_SEL(c, t, f) mpj_sel((int)(c), (t), (f))
#else
#define MPJ_ANY(c) (c)
#define MPJ_ANYG(c) (c)
#define MPJ_SEL(c, t, f) ((c) ? (t) : (f))
#endif

MPJ_FN double mpj_atan_bl(double x) {
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const uint32_t hx = mpj_hi(x);
  const uint32_t ix = hx & 0x7fffffffu;
  const int small = ix < 0x3fdc0000u, c0 = ix < 0x3fe60000u, c1 = ix < 0x3ff30000u, c2 = ix < 0x40038000u;
  const int id2 = c2 && !c1;
  /* (na*a - nb) / (na + nb*a): id -1 -> x/1, 0 -> (2x-1)/(2+x), 1 -> (x-1)/(1+x),
   * 2 -> (x-1.5)/(1+1.5x), 3 -> -1/x == (0*x-1)/(0+1*x).  NaN propagates. */
  const double a = mpj_fabs(x); /* the odd polynomial makes the |x| < 0.4375 path sign-symmetric */
  const double na = small ? 1.0 : (c0 ? 2.0 : (c2 ? 1.0 : 0.0));
  const double nb = small ? 0.0 : (id2 ? 1.5 : 1.0);
  const double hi = small ? 0.0 : (c0 ? 4.63647609000806093515e-01 : (c1 ?
                    7.85398163397448278999e-01 : (c2 ? 9.82793723247329054082e-01 : 1.57079632679489655800e+00)));
  const double lo = small ? 0.0 : (c0 ? 2.26987774529616870924e-17 : (c1 ?
                    3.06161699786838301793e-17 : (c2 ? 1.39033110312309984516e-17 : 6.12323399573676603587e-17)));
  const double ax = (na * a - nb) / (na + nb * a);
  const double z = ax * ax;
  const double w = z * z;
  const double s1 = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT10, aT8), aT6), aT4), aT2), aT0);
  const double s2 = w * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT9, aT7), aT5), aT3), aT1);
  /* id -1: x - x*s == -((x*s - 0) - x) == hi - ((x*s - lo) - x) with hi = lo = 0 */
  const double r = hi - ((ax * (s1 + s2) - lo) - ax);
  const double rs = mpj_flip(r, hx & 0x80000000u);
  /* |x| >= 2^66 (incl. ±Inf, where 0*Inf would be NaN): atanhi[3] + atanlo[3] */
  const double big = 1.57079632679489655800e+00 + 6.12323399573676603587e-17;
  const double rb = MPJ_SEL(ix >= 0x44100000u && x == x, MPJ_SEL(hx >> 31, -big, big), rs);
  return MPJ_SEL(ix < 0x3e400000u, x, rb);
}

/* atan_bl with the range constants {na, nb, hi, lo} fetched from a 5-row table indexed by
 * the FDLIBM range (0: |x| < 0.4375, 1..4: the four reductions) instead of select trees —
 * on the device the table lives in LDS (mpj_atan_tab_init fills it).  Same operations on
 * the same operands as mpj_atan_bl / mpj_atan, so the same bits. */
MPJ_FN void mpj_atan_tab_init(double* tab) {
  const double t[20] = {1.0, 0.0, 0.0, 0.0,
                        2.0, 1.0, 4.63647609000806093515e-01, 2.26987774529616870924e-17,
                        1.0, 1.0, 7.85398163397448278999e-01, 3.06161699786838301793e-17,
                        1.0, 1.5, 9.82793723247329054082e-01, 1.39033110312309984516e-17,
                        0.0, 1.0, 1.57079632679489655800e+00, 6.12323399573676603587e-17};
  for (int i = 0; i < 20; i++) tab[i] = t[i];
}
MPJ_FN double mpj_atan_tab(double x, const double* tab) {
  const double aT0 = 3.33333333333329318027e-01, aT1 = -1.99999999998764832476e-01,
               aT2 = 1.42857142725034663711e-01, aT3 = -1.11111104054623557880e-01,
               aT4 = 9.09088713343650656196e-02, aT5 = -7.69187620504482999495e-02,
               aT6 = 6.66107313738753120669e-02, aT7 = -5.83357013379057348645e-02,
               aT8 = 4.97687799461593236017e-02, aT9 = -3.65315727442169155270e-02,
               aT10 = 1.62858201153657823623e-02;
  const uint32_t hx = mpj_hi(x);
  const uint32_t ix = hx & 0x7fffffffu;
  const int id = (ix >= 0x3fdc0000u) + (ix >= 0x3fe60000u) + (ix >= 0x3ff30000u) + (ix >= 0x40038000u);
  const double a = mpj_fabs(x);
  const double* t = tab + 4 * id;
  const double na = t[0], nb = t[1], hi = t[2], lo = t[3];
  const double ax = (na * a - nb) / (na + nb * a);
  const double z = ax * ax;
  const double w = z * z;
  const double s1 = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT10, aT8), aT6), aT4), aT2), aT0);
  const double s2 = w * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, aT9, aT7), aT5), aT3), aT1);
  const double r = hi - ((ax * (s1 + s2) - lo) - ax);
  /* FDLIBM's |x| < 2^-27 case needs no select here: with id 0 (ax = a) the polynomial term is
   * below half an ulp of a, so r == a exactly and the flip returns x (±0 and subnormals
   * included; tests/test_jlmath.py).  |x| >= 2^66 keeps a select (±Inf would give 0·Inf), taken
   * before the sign flip: FDLIBM's -atanhi[3] - atanlo[3] is exactly -(atanhi[3] + atanlo[3]). */
  const double big = 1.57079632679489655800e+00 + 6.12323399573676603587e-17;
  return mpj_flip(MPJ_SEL(ix >= 0x44100000u && x == x, big, r), hx & 0x80000000u);
}

/* mpj_atan2 with the branch-free atan core (bit-identical: mpj_atan_bl == mpj_atan). */
MPJ_FN double mpj_atan2_bl(double y, double x) {
  const double pi_o_4 = 7.8539816339744827900E-01, pi_o_2 = 1.5707963267948965580E+00,
               pi = 3.1415926535897931160E+00, pi_lo = 1.2246467991473531772E-16;
  if (mpj_isnan(x) || mpj_isnan(y)) return x + y;
  uint32_t hx = mpj_hi(x), lx = mpj_lo(x), hy = mpj_hi(y), ly = mpj_lo(y);
  int32_t ix = (int32_t)(hx & 0x7fffffffu), iy = (int32_t)(hy & 0x7fffffffu);
  if (hx == 0x3ff00000u && lx == 0) return mpj_atan_bl(y);
  int m = (int)(((hy >> 31) & 1) | ((hx >> 30) & 2));
  if ((iy | (int32_t)ly) == 0) {
    if (m == 0 || m == 1) return y;
    return m == 2 ? pi : -pi;
  }
  if ((ix | (int32_t)lx) == 0) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  if (ix == 0x7ff00000) {
    if (iy == 0x7ff00000) {
      if (m == 0) return pi_o_4;
      if (m == 1) return -pi_o_4;
      if (m == 2) return 3.0 * pi_o_4;
      return -3.0 * pi_o_4;
    }
    if (m == 0) return 0.0;
    if (m == 1) return -0.0;
    if (m == 2) return pi;
    return -pi;
  }
  if (iy == 0x7ff00000) return (hy >> 31) ? -pi_o_2 : pi_o_2;
  int32_t k = (iy - ix) >> 20;
  double z;
  if (k > 60) { z = pi_o_2 + 0.5 * pi_lo; m &= 1; }
  else if ((hx >> 31) && k < -60) z = 0.0;
  else z = mpj_atan_bl(mpj_fabs(y / x));
  if (m == 0) return z;
  if (m == 1) return -z;
  if (m == 2) return pi - (z - pi_lo);
  return (z - pi_lo) - pi;
}

/* sin and cos for |x| <= ~9π/4 as straight-line code (cw2c reduction, n in {0, ±1..±4}).
 * mpj_sincos_fast never branches: lanes outside the fast range set *bad and get garbage; the
 * caller re-evaluates with the exact routine (mpj_sincos_bl does so per call, the iLQR kernels
 * per trajectory). */
MPJ_FN void mpj_sincos_fast(double x, double* so, double* co, int* bad) {
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  const double ax = mpj_fabs(x);
  const int small = ax < MPJ_PIO4;
  /* exact-path cases: |x| > ~9π/4, NaN/Inf, or the cwext points near kπ/2 (e_rem_pio2.c) */
  const int ext = (xhp <= 0x400f6a7au && (xhp & 0xfffffu) == 0x921fbu) || xhp == 0x4012d97cu || xhp == 0x401921fbu;
  *bad |= xhp > 0x401c463bu || (!small && ext);
  /* |n| = 1..4 by range (e_rem_pio2.c), Cody–Waite with fn = ±|n| */
  const int na = 1 + (xhp > 0x4002d97cu) + (xhp > 0x400f6a7au) + (xhp > 0x4015fdbcu);
  const int ni = x > 0.0 ? na : -na;
  double y0, y1;
  mpj_cw2c(x, (double)ni, 0, &y0, &y1);
  /* one sin and one cos kernel: the |x| < π/4 path is sin_k0(x) / cos_k(x, 0), the
   * reduced path sin_k(y0, y1) / cos_k(y0, y1); both share z, w, r, v of their argument */
  const double xa = MPJ_SEL(small, x, y0), ya = MPJ_SEL(small, 0.0, y1);
  const double z = xa * xa, w = z * z;
  const double r = mpj_fma(z, mpj_fma(z, MPJ_S4, MPJ_S3), MPJ_S2) + z * w * mpj_fma(z, MPJ_S6, MPJ_S5);
  const double v = z * xa;
  const double sk0 = xa + v * (MPJ_S1 + z * r);                          /* mpj_sin_k0(x) */
  const double sk = xa - ((z * (0.5 * ya - v * r) - ya) - v * MPJ_S1);   /* mpj_sin_k(y0, y1) */
  const double ck = mpj_cos_k(xa, ya);
  const double s0 = MPJ_SEL(ax < MPJ_SQRT_EPS, x, sk0);
  const double c0 = MPJ_SEL(ax < MPJ_SQRT_HALF_EPS, 1.0, ck);
  /* n&3: 0 -> (s, c), 1 -> (c, -s), 2 -> (-s, -c), 3 -> (-c, s) */
  const int n = ni & 3;
  const double ts = MPJ_SEL(n & 1, ck, sk), tc = MPJ_SEL(n & 1, sk, ck);
  const double sr = mpj_flip(ts, (uint32_t)(n & 2) << 30);
  const double cr = mpj_flip(tc, (uint32_t)((n + 1) & 2) << 30);
  *so = MPJ_SEL(small, s0, sr);
  *co = MPJ_SEL(small, c0, cr);
}
/* sin and cos for every finite |x| < 2^20·π/2 as straight-line code: the cw2c reduction of
 * mpj_sincos_fast and, selected per lane, the 3-stage Cody–Waite reduction mpj_cwext uses for
 * |x| > 9π/4 and next to kπ/2 (its two data-dependent stage tests become selects).  NaN/Inf
 * and larger |x| set *bad. */
MPJ_FN void mpj_sincos_wide(double x, double* so, double* co, int* bad) {
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  const double ax = mpj_fabs(x);
  const int small = ax < MPJ_PIO4;
  *bad |= xhp >= 0x413921fbu;
  const int med = (xhp <= 0x400f6a7au && (xhp & 0xfffffu) == 0x921fbu) || xhp == 0x4012d97cu ||
                  xhp == 0x401921fbu || xhp > 0x401c463bu;
  /* cw2c: |n| = 1..4 by range */
  const int na = 1 + (xhp > 0x4002d97cu) + (xhp > 0x400f6a7au) + (xhp > 0x4015fdbcu);
  const int ni = x > 0.0 ? na : -na;
  double c0, c1;
  mpj_cw2c(x, (double)ni, 0, &c0, &c1);
  /* cwext, straight line (bad lanes: the conversion below is clamped by the select) */
  const double fn = mpj_round(MPJ_SEL(xhp >= 0x413921fbu, 0.0, x) * MPJ_INVPIO2);
  const int32_t j = (int32_t)(xhp >> 20);
  const double r1 = mpj_fma(-fn, MPJ_PIO2_1, x), w1 = fn * MPJ_PIO2_1T, a1 = r1 - w1;
  const int32_t i1 = j - (int32_t)((mpj_hi(a1) >> 20) & 0x7ff);
  const double w2a = fn * MPJ_PIO2_2, r2 = r1 - w2a;
  const double w2 = mpj_fma(fn, MPJ_PIO2_2T, -((r1 - r2) - w2a)), a2 = r2 - w2;
  const int32_t i2 = j - (int32_t)((mpj_hi(a2) >> 20) & 0x7ff);
  const double w3a = fn * MPJ_PIO2_3, r3 = r2 - w3a;
  const double w3 = mpj_fma(fn, MPJ_PIO2_3T, -((r2 - r3) - w3a)), a3 = r3 - w3;
  const int s2 = i1 > 16, s3 = s2 && i2 > 49;
  const double er = MPJ_SEL(s3, r3, MPJ_SEL(s2, r2, r1)), ew = MPJ_SEL(s3, w3, MPJ_SEL(s2, w2, w1));
  const double ea = MPJ_SEL(s3, a3, MPJ_SEL(s2, a2, a1));
  const double y0 = MPJ_SEL(med, ea, c0), y1 = MPJ_SEL(med, (er - ea) - ew, c1);
  const int nr = med ? (int)fn : ni;
  const double xa = MPJ_SEL(small, x, y0), ya = MPJ_SEL(small, 0.0, y1);
  const double z = xa * xa, w = z * z;
  const double r = mpj_fma(z, mpj_fma(z, MPJ_S4, MPJ_S3), MPJ_S2) + z * w * mpj_fma(z, MPJ_S6, MPJ_S5);
  const double v = z * xa;
  const double sk0 = xa + v * (MPJ_S1 + z * r);
  const double sk = xa - ((z * (0.5 * ya - v * r) - ya) - v * MPJ_S1);
  const double ck = mpj_cos_k(xa, ya);
  const double s0 = MPJ_SEL(ax < MPJ_SQRT_EPS, x, sk0);
  const double cc0 = MPJ_SEL(ax < MPJ_SQRT_HALF_EPS, 1.0, ck);
  const int n = nr & 3;
  const double ts = MPJ_SEL(n & 1, ck, sk), tc = MPJ_SEL(n & 1, sk, ck);
  const double sr = mpj_flip(ts, (uint32_t)(n & 2) << 30);
  const double cr = mpj_flip(tc, (uint32_t)((n + 1) & 2) << 30);
  *so = MPJ_SEL(small, s0, sr);
  *co = MPJ_SEL(small, cc0, cr);
}
MPJ_FN void mpj_sincos_bl(double x, double* so, double* co) {
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  const int ext = (xhp <= 0x400f6a7au && (xhp & 0xfffffu) == 0x921fbu) || xhp == 0x4012d97cu || xhp == 0x401921fbu;
  if (MPJ_ANY(xhp > 0x401c463bu || (!(mpj_fabs(x) < MPJ_PIO4) && ext))) {
    mpj_sincos(x, so, co);
    return;
  }
  int bad = 0;
  mpj_sincos_fast(x, so, co, &bad);
}

/* sin only, same fast range. */
MPJ_FN double mpj_sin_bl(double x) {
  double s, c;
  mpj_sincos_bl(x, &s, &c);
  return s;
}

/* sin for |x| <= 3π/4 as straight-line code (the tyre model's sin(C·atan(…)), C = 1.3,
 * vehicledynamics.jl:35-38, never leaves |x| < 1.3·π/2): below π/4 FDLIBM's sin_k0(x), above it
 * the reduction by n = ±1 and ±cos_k(y0, y1) — mpj_sin's own operations on that range, without
 * the sin_k / n = ±2..4 lanes of mpj_sincos_fast.  Larger |x|, NaN/Inf and the cwext points next
 * to ±π/2 take mpj_sin (wave-uniform on the device). */
MPJ_FN double mpj_sin_34(double x) {
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  const double ax = mpj_fabs(x);
  const int small = ax < MPJ_PIO4;
  if (MPJ_ANY(xhp > 0x4002d97cu || (!small && (xhp & 0xfffffu) == 0x921fbu))) return mpj_sin(x);
  double y0, y1;
  mpj_cw2c(x, x > 0.0 ? 1.0 : -1.0, 0, &y0, &y1);
  const double xa = MPJ_SEL(small, x, y0), ya = MPJ_SEL(small, 0.0, y1);
  const double z = xa * xa, w = z * z;
  const double r = mpj_fma(z, mpj_fma(z, MPJ_S4, MPJ_S3), MPJ_S2) + z * w * mpj_fma(z, MPJ_S6, MPJ_S5);
  const double v = z * xa;
  const double sk0 = xa + v * (MPJ_S1 + z * r); /* mpj_sin_k0(x) */
  const double ck = mpj_cos_k(xa, ya);           /* n = 1: cos_k; n = -1 (& 3 = 3): -cos_k */
  return MPJ_SEL(small, MPJ_SEL(ax < MPJ_SQRT_EPS, x, sk0), mpj_flip(ck, mpj_hi(x) & 0x80000000u));
}

/* log for the Box–Muller draws, FDLIBM e_log.c as one basic block: its four result forms are two
 * (the k == 0 forms are the k != 0 ones with dk = 0: 0·ln2_hi - (a - f) == f - a and
 * b ± 0·ln2_lo == b exactly, the result of a normal x != 1 being nonzero), selected by FDLIBM's
 * i > 0 test.  Zero, negative, subnormal, Inf/NaN and the |f| < 2^-20 case take mpj_log
 * (wave-uniform on the device). */
MPJ_FN double mpj_log_bl(double x) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
               Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  const int32_t hx0 = (int32_t)mpj_hi(x);
  const int32_t hm = hx0 & 0x000fffff;
  if (MPJ_ANY(hx0 < 0x00100000 || hx0 >= 0x7ff00000 || (0x000fffff & (2 + hm)) < 3)) return mpj_log(x);
  const int32_t i0 = (hm + 0x95f64) & 0x100000;
  const int32_t k = (hx0 >> 20) - 1023 + (i0 >> 20);
  const double f = mpj_from_words((uint32_t)(hm | (i0 ^ 0x3ff00000)), mpj_lo(x)) - 1.0;
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * mpj_fma(w, mpj_fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, Lg7, Lg5), Lg3), Lg1);
  const int32_t i = (hm - 0x6147a) | (0x6b851 - hm);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double rp = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  const double rn = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
  return MPJ_SEL(i > 0, rp, rn);
}

/* tan for |x| <= π/4 as one basic block (FDLIBM k_tan.c with iy = 1, both the |x| < 0.6744
 * and the reflected |x| >= 0.6744 forms, selected); larger |x|, NaN and Inf take mpj_tan. */
MPJ_FN double mpj_tan_fast(double x, int* bad) {
  const double T0 = 3.33333333333334091986e-01, T1 = 1.33333333333201242699e-01,
               T2 = 5.39682539762260521377e-02, T3 = 2.18694882948595424599e-02,
               T4 = 8.86323982359930005737e-03, T5 = 3.59207910759131235356e-03,
               T6 = 1.45620945432529025516e-03, T7 = 5.88041240820264096874e-04,
               T8 = 2.46463134818469906812e-04, T9 = 7.81794442939557092300e-05,
               T10 = 7.14072491382608190305e-05, T11 = -1.85586374855275456654e-05,
               T12 = 2.59073051863633712884e-05, pio4lo = 3.06161699786838301793e-17;
  const int32_t hx = (int32_t)mpj_hi(x);
  const int32_t ix = hx & 0x7fffffff;
  *bad |= ix > 0x3fe921fb;
  const int big = ix >= 0x3FE59428;
  const int neg = hx < 0;
  const double xn = MPJ_SEL(neg, -x, x), yn = MPJ_SEL(neg, -0.0, 0.0);
  const double xb = (MPJ_PIO4 - xn) + (pio4lo - yn);
  const double xx = MPJ_SEL(big, xb, x);
  const double y = 0.0;
  const double z = xx * xx;
  const double w = z * z;
  double r = mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T11, T9), T7), T5), T3), T1);
  const double v = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T12, T10), T8), T6), T4), T2);
  const double s = z * xx;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  const double ww = xx + r;
  const double rb = (double)(1 - ((hx >> 30) & 2)) * (1.0 - 2.0 * (xx - (ww * ww / (ww + 1.0) - r)));
  return MPJ_SEL(ix < 0x3e400000, x, MPJ_SEL(big, rb, ww));
}

/* e_rem_pio2.c for finite |x| < 2^20·π/2 as straight-line code: the cw2c reduction (|n| =
 * 1..4 by range) and, selected per lane, the 3-stage Cody–Waite mpj_cwext uses beyond 9π/4
 * and next to kπ/2 (its two stage tests become selects).  Returns n; equals mpj_rem_pio2 bit
 * for bit on that range (the caller flags larger |x|, NaN and Inf). */
MPJ_FN int mpj_rem_pio2_sl(double x, double* y0, double* y1) {
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  const int med = (xhp <= 0x400f6a7au && (xhp & 0xfffffu) == 0x921fbu) || xhp == 0x4012d97cu ||
                  xhp == 0x401921fbu || xhp > 0x401c463bu;
  const int na = 1 + (xhp > 0x4002d97cu) + (xhp > 0x400f6a7au) + (xhp > 0x4015fdbcu);
  const int ni = x > 0.0 ? na : -na;
  double c0, c1;
  mpj_cw2c(x, (double)ni, 0, &c0, &c1);
  const double fn = mpj_round(MPJ_SEL(xhp >= 0x413921fbu, 0.0, x) * MPJ_INVPIO2);
  const int32_t j = (int32_t)(xhp >> 20);
  const double r1 = mpj_fma(-fn, MPJ_PIO2_1, x), w1 = fn * MPJ_PIO2_1T, a1 = r1 - w1;
  const int32_t i1 = j - (int32_t)((mpj_hi(a1) >> 20) & 0x7ff);
  const double w2a = fn * MPJ_PIO2_2, r2 = r1 - w2a;
  const double w2 = mpj_fma(fn, MPJ_PIO2_2T, -((r1 - r2) - w2a)), a2 = r2 - w2;
  const int32_t i2 = j - (int32_t)((mpj_hi(a2) >> 20) & 0x7ff);
  const double w3a = fn * MPJ_PIO2_3, r3 = r2 - w3a;
  const double w3 = mpj_fma(fn, MPJ_PIO2_3T, -((r2 - r3) - w3a)), a3 = r3 - w3;
  const int s2 = i1 > 16, s3 = s2 && i2 > 49;
  const double er = MPJ_SEL(s3, r3, MPJ_SEL(s2, r2, r1)), ew = MPJ_SEL(s3, w3, MPJ_SEL(s2, w2, w1));
  const double ea = MPJ_SEL(s3, a3, MPJ_SEL(s2, a2, a1));
  *y0 = MPJ_SEL(med, ea, c0);
  *y1 = MPJ_SEL(med, (er - ea) - ew, c1);
  return med ? (int)fn : ni;
}

/* tan for every finite |x| < 2^20·π/2 as one basic block: mpj_rem_pio2_sl, then k_tan.c with
 * all three result forms (|x| >= 0.6744 reflection, iy = 1, and the iy = -1 -1/tan form with
 * its zero-low-word correction) evaluated and selected.  |x| <= π/4 takes k_tan(x, 0, 1) as
 * s_tan.c does.  NaN, Inf and larger |x| set *bad. */
MPJ_FN double mpj_tan_wide(double x, int* bad) {
  const double T0 = 3.33333333333334091986e-01, T1 = 1.33333333333201242699e-01,
               T2 = 5.39682539762260521377e-02, T3 = 2.18694882948595424599e-02,
               T4 = 8.86323982359930005737e-03, T5 = 3.59207910759131235356e-03,
               T6 = 1.45620945432529025516e-03, T7 = 5.88041240820264096874e-04,
               T8 = 2.46463134818469906812e-04, T9 = 7.81794442939557092300e-05,
               T10 = 7.14072491382608190305e-05, T11 = -1.85586374855275456654e-05,
               T12 = 2.59073051863633712884e-05, pio4lo = 3.06161699786838301793e-17;
  const uint32_t xhp = mpj_hi(x) & 0x7fffffffu;
  *bad |= xhp >= 0x413921fbu;
  const int small = xhp <= 0x3fe921fbu;
  double r0, r1;
  const int n = mpj_rem_pio2_sl(MPJ_SEL(small, 0.0, x), &r0, &r1);
  const double xa = MPJ_SEL(small, x, r0), ya = MPJ_SEL(small, 0.0, r1);
  const int iy = small ? 1 : 1 - ((n & 1) << 1);
  /* k_tan(xa, ya, iy) */
  const int32_t hx = (int32_t)mpj_hi(xa);
  const int32_t ix = hx & 0x7fffffff;
  const int big = ix >= 0x3FE59428;
  const int neg = hx < 0;
  const double xn = MPJ_SEL(neg, -xa, xa), yn = MPJ_SEL(neg, -ya, ya);
  const double xb = (MPJ_PIO4 - xn) + (pio4lo - yn);
  const double xx = MPJ_SEL(big, xb, xa), y = MPJ_SEL(big, 0.0, ya);
  const double z = xx * xx;
  const double w = z * z;
  double r = mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T11, T9), T7), T5), T3), T1);
  const double v = z * mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, mpj_fma(w, T12, T10), T8), T6), T4), T2);
  const double s = z * xx;
  r = y + z * (s * (r + v) + y);
  r += T0 * s;
  const double ww = xx + r;
  const double vy = (double)iy;
  const double rb = (double)(1 - ((hx >> 30) & 2)) * (vy - 2.0 * (xx - (ww * ww / (ww + vy) - r)));
  /* iy == -1, |xa| < 0.6744: -1/(x+r) with the zero-low-word correction */
  const double zl = mpj_zero_lo(ww);
  const double vl = r - (zl - xx);
  const double a = -1.0 / ww;
  const double t = mpj_zero_lo(a);
  const double sl = 1.0 + t * zl;
  const double rm = t + a * (sl + t * vl);
  const double res = MPJ_SEL(big, rb, MPJ_SEL(iy == 1, ww, rm));
  return MPJ_SEL(xhp < 0x3e400000u, x, res);
}

MPJ_FN double mpj_tan_bl(double x) {
  if (MPJ_ANY((mpj_hi(x) & 0x7fffffffu) > 0x3fe921fbu)) return mpj_tan(x);
  int bad = 0;
  return mpj_tan_fast(x, &bad);
}

/* atan2 as one basic block for finite y, x, not both zero (FDLIBM e_atan2.c: the y == 0,
 * x == 0 and |exponent difference| > 60 cases are selects around the general case; x == 1
 * gives atan(y) == ±atan(|y|) there too); NaN/Inf/(0, 0) set *bad. */
MPJ_FN double mpj_atan2_fast(double y, double x, int* bad) {
  const double pi_o_2 = 1.5707963267948965580E+00, pi = 3.1415926535897931160E+00,
               pi_lo = 1.2246467991473531772E-16;
  const uint32_t hx = mpj_hi(x), lx = mpj_lo(x), hy = mpj_hi(y), ly = mpj_lo(y);
  const int32_t ix = (int32_t)(hx & 0x7fffffffu), iy = (int32_t)(hy & 0x7fffffffu);
  const int xz = (ix | (int32_t)lx) == 0, yz = (iy | (int32_t)ly) == 0;
  *bad |= ix >= 0x7ff00000 || iy >= 0x7ff00000 || (xz && yz);
  const int32_t k = (iy - ix) >> 20;
  const int mq = (int)(((hy >> 31) & 1) | ((hx >> 30) & 2));
  const int kbig = k > 60, ksmall = (hx >> 31) && k < -60;
  const int m = kbig ? (mq & 1) : mq;
  const double za = mpj_atan_bl(mpj_fabs(y / x));
  const double z = MPJ_SEL(kbig, pi_o_2 + 0.5 * pi_lo, MPJ_SEL(ksmall, 0.0, za));
  const double zl = z - pi_lo;
  const double r01 = mpj_flip(z, (uint32_t)(m & 1) << 31);
  const double r2 = pi - zl, r3 = zl - pi;
  const double rg = MPJ_SEL(m & 2, MPJ_SEL(m & 1, r3, r2), r01);
  /* y == 0: m 0/1 -> y, 2 -> pi, 3 -> -pi;  x == 0: ±pi/2 by the sign of y */
  const double ry = MPJ_SEL(mq & 2, MPJ_SEL(mq & 1, -pi, pi), y);
  const double rx = MPJ_SEL(hy >> 31, -pi_o_2, pi_o_2);
  return MPJ_SEL(yz, ry, MPJ_SEL(xz, rx, rg));
}
MPJ_FN double mpj_atan2_sel(double y, double x) {
  int bad = 0;
  const double r = mpj_atan2_fast(y, x, &bad);
  if (MPJ_ANY(bad)) return mpj_atan2(y, x);
  return r;
}

/* ----------------------------------------------------------- Julia idioms */
/* Julia `mod(x, y)` for floats (base/floatfuncs.jl): rem, then sign fix. */
MPJ_FN double mpj_jlmod(double x, double y) {
  double r = __builtin_fmod(x, y);
  if (r == 0.0) return __builtin_copysign(r, y);
  if ((r > 0.0) != (y > 0.0)) return r + y;
  return r;
}
#define MPJ_TWO_PI 6.283185307179586
/* modπ, PathPlanning/ReedsSheppsCurves/src/ReedsSheppsUtils.jl:32-46 */
MPJ_FN double mpj_modpi(double a) {
  if (a >= -MPJ_PI && a <= MPJ_PI) return a;
  a = mpj_jlmod(a, MPJ_TWO_PI);
  if (a < -MPJ_PI) a = a + MPJ_TWO_PI;
  else if (a > MPJ_PI) a = a - MPJ_TWO_PI;
  return a;
}
/* mpj_modpi without the fmod loop: for |a| < 4π, fmod(a, 2π) is a or a ∓ 2π exactly
 * (Sterbenz), the rest is selects; |a| >= 4π and NaN take mpj_modpi (wave-uniform). */
MPJ_FN double mpj_modpi_bl(double a) {
  const double aa = mpj_fabs(a);
  if (MPJ_ANY(!(aa < 2 * MPJ_TWO_PI))) return mpj_modpi(a);
  double r = MPJ_SEL(aa >= MPJ_TWO_PI, a - __builtin_copysign(MPJ_TWO_PI, a), a);
  r = MPJ_SEL(r == 0.0, 0.0, r);          /* copysign(0, 2π) */
  r = MPJ_SEL(r < 0.0, r + MPJ_TWO_PI, r); /* Julia mod: result in [0, 2π] */
  r = MPJ_SEL(r > MPJ_PI, r - MPJ_TWO_PI, r);
  return MPJ_SEL(aa <= MPJ_PI, a, r);
}
/* Julia isless(a, b) for Float64: NaN sorts last, -0.0 < 0.0. */
MPJ_FN int mpj_isless(double a, double b) {
  if (mpj_isnan(a)) return 0;
  if (mpj_isnan(b)) return 1;
  if (a < b) return 1;
  if (a == b) return (mpj_hi(a) >> 31) > (mpj_hi(b) >> 31);
  return 0;
}

/* ------------------------------------------------ LinearAlgebra.pinv (2x2) */
/* Julia's `pinv(A::Matrix{Float64})` (stdlib LinearAlgebra dense.jl) for a 2x2 A, the path both
 * `pinv(Quu)` (ILQR.jl:61,63) and cubic_fit's `pinv(A)` (hybrid_astar_utils.jl:107-109) take:
 *   isdiag(A)  -> B = diag(abs(x) > tol ? inv(x) : 0), tol = 2eps * max|diag|, off-diagonal +0.0;
 *   otherwise  -> svd(A) = LAPACK dgesdd(JOBZ='S'), tol = 2eps * max(S), Sinv = S > tol ? inv(S) : 0,
 *                 pinv = Vt' * (Diagonal(Sinv) * U')  (matmul2x2!: a*b + c*d, no FMA).
 * dgesdd on a 2x2 (M < MNTHR = 3) is its path 5: dgebd2 (one Householder reflector H1 from dlarfg
 * on column 1, applied to column 2 by dlarf; the row and last-column reflectors are identities,
 * n = 1), dbdsdc -> dlasdq -> dbdsqr on the 2x2 upper bidiagonal [d1 e1; 0 d2] (split when
 * |e1| <= thresh, otherwise one dlasv2 and two drot on the identity), singular values made
 * non-negative and sorted decreasing, then dormbr applies H1 to U.  The BLAS level-1/2 calls inside
 * (dgemv, dger) round as the OpenBLAS kernels do: dgemv's w = C(1,j)*1 + C(2,j)*v2 rounds the
 * product and the sum separately, dger's C(2,j) += (-tau*w_j)*v2 is one fused multiply-add.
 * Pinned bit for bit against numpy's gesdd (OpenBLAS 0.3.29) on >= 1e5 random, near-singular,
 * triangular, orthogonal-column and scaled 2x2 matrices (tests/test_jlmath.py).
 * Domain: max|A_ij| in [6.7e-139, 1.5e138] or A == 0 (dgesdd rescales outside it; not restated),
 * finite entries (Julia's svd throws on NaN/Inf). */
MPJ_FN double mpj_fsign(double a, double b) { return __builtin_copysign(__builtin_fabs(a), b); } /* Fortran SIGN */

/* LAPACK DLASV2: SVD of the upper triangular [f g; 0 h]. */
MPJ_FN void mpj_lasv2(double f, double g, double h, double* ssmin, double* ssmax, double* snr, double* csr,
                      double* snl, double* csl) {
  const double eps = 1.1102230246251565e-16; /* DLAMCH('EPS') */
  double ft = f, fa = __builtin_fabs(f), ht = h, ha = __builtin_fabs(h);
  int pmax = 1;
  const int swap = ha > fa;
  if (swap) {
    pmax = 3;
    double t = ft; ft = ht; ht = t;
    t = fa; fa = ha; ha = t;
  }
  const double gt = g, ga = __builtin_fabs(g);
  double clt, crt, slt, srt, smin, smax;
  if (ga == 0.0) {
    smin = ha; smax = fa; clt = 1.0; crt = 1.0; slt = 0.0; srt = 0.0;
  } else {
    int gasmal = 1;
    if (ga > fa) {
      pmax = 2;
      if (fa / ga < eps) {
        gasmal = 0;
        smax = ga;
        smin = ha > 1.0 ? fa / (ga / ha) : (fa / ga) * ha;
        clt = 1.0; slt = ht / gt; srt = 1.0; crt = ft / gt;
      }
    }
    if (gasmal) {
      const double d = fa - ha;
      double l = d == fa ? 1.0 : d / fa;
      const double m = gt / ft;
      double t = 2.0 - l;
      const double mm = m * m, tt = t * t;
      const double s = mpj_sqrt(tt + mm);
      const double r = l == 0.0 ? __builtin_fabs(m) : mpj_sqrt(l * l + mm);
      const double a = 0.5 * (s + r);
      smin = ha / a;
      smax = fa * a;
      if (mm == 0.0) {
        if (l == 0.0) t = mpj_fsign(2.0, ft) * mpj_fsign(1.0, gt);
        else t = gt / mpj_fsign(d, ft) + m / t;
      } else {
        t = (m / (s + t) + m / (r + l)) * (1.0 + a);
      }
      l = mpj_sqrt(t * t + 4.0);
      crt = 2.0 / l;
      srt = t / l;
      clt = (crt + srt * m) / a;
      slt = (ht / ft) * srt / a;
    }
  }
  if (swap) { *csl = srt; *snl = crt; *csr = slt; *snr = clt; }
  else { *csl = clt; *snl = slt; *csr = crt; *snr = srt; }
  double tsign;
  if (pmax == 1) tsign = mpj_fsign(1.0, *csr) * mpj_fsign(1.0, *csl) * mpj_fsign(1.0, f);
  else if (pmax == 2) tsign = mpj_fsign(1.0, *snr) * mpj_fsign(1.0, *csl) * mpj_fsign(1.0, g);
  else tsign = mpj_fsign(1.0, *snr) * mpj_fsign(1.0, *snl) * mpj_fsign(1.0, h);
  *ssmax = mpj_fsign(smax, tsign);
  *ssmin = mpj_fsign(smin, tsign * mpj_fsign(1.0, f) * mpj_fsign(1.0, h));
}

/* dlarf('Left') of H = I - tau [1; v2][1 v2] on one column [c1; c2] already known to be inside
 * dlarf's iladlc range: lastv = 1 when v2 == 0 (row 2 untouched), else w = c1*1 + c2*v2
 * (dgemv('T'), separately rounded), c1 += (-tau*w)*1, c2 = fma(-tau*w, v2, c2) (dger). */
MPJ_FN void mpj_larf2(double tau, double v2, double* c1, double* c2) {
  if (v2 != 0.0) {
    const double tw = -tau * (*c1 + *c2 * v2);
    *c1 = *c1 + tw;
    *c2 = mpj_fma(tw, v2, *c2);
  } else {
    *c1 = *c1 + (-tau * *c1);
  }
}

/* svd(A) of a row-major 2x2 through dgesdd path 5 (above): U, VT row-major, S decreasing. */
MPJ_FN void mpj_svd2(const double* A, double* U, double* S, double* VT) {
  const double a11 = A[0], a12 = A[1], a21 = A[2], a22 = A[3];
  /* dgebd2, i = 1: dlarfg(2, a11, a21) -> beta, tau, v = [1, v2]; dlarf('L') on column 2 */
  double tau = 0.0, v2 = 0.0, d1 = a11, e1 = a12, d2 = a22;
  const double xnorm = __builtin_fabs(a21); /* dnrm2 of one entry */
  if (xnorm != 0.0) {
    const double aa = __builtin_fabs(a11);
    const double w = aa > xnorm ? aa : xnorm, z = aa > xnorm ? xnorm : aa; /* dlapy2 */
    const double q = z / w;
    const double py = z == 0.0 ? w : w * mpj_sqrt(1.0 + q * q);
    const double beta = -mpj_fsign(py, a11);
    tau = (beta - a11) / beta;
    v2 = a21 * (1.0 / (a11 - beta));
    d1 = beta;
    if (a12 != 0.0 || (v2 != 0.0 && a22 != 0.0)) mpj_larf2(tau, v2, &e1, &d2); /* column 2 (iladlc) */
  }
  /* dbdsqr on [d1 e1; 0 d2] with VT = U = I */
  double vt[4] = {1.0, 0.0, 0.0, 1.0}, ub[4] = {1.0, 0.0, 0.0, 1.0}, d[2];
  const double unfl = 2.2250738585072014e-308, tol = 1.0958066990042004e-14; /* TOLMUL*EPS, TOLMUL = EPS^(-1/8) */
  double sminoa = __builtin_fabs(d1);
  if (sminoa != 0.0) {
    const double mu = __builtin_fabs(d2) * (sminoa / (sminoa + __builtin_fabs(e1)));
    sminoa = mu < sminoa ? mu : sminoa;
  }
  sminoa = sminoa / 1.4142135623730951;
  const double th0 = tol * sminoa, th1 = 6.0 * (2.0 * (2.0 * unfl));
  const double thresh = th0 > th1 ? th0 : th1;
  if (__builtin_fabs(e1) <= thresh) {
    d[0] = d1; d[1] = d2;
  } else {
    double smin, smax, snr, csr, snl, csl;
    mpj_lasv2(d1, e1, d2, &smin, &smax, &snr, &csr, &snl, &csl);
    d[0] = smax; d[1] = smin;
    /* drot(VT rows 1, 2; csr, snr) and drot(U columns 1, 2; csl, snl) on the identity */
    for (int c = 0; c < 2; c++) {
      const double x = vt[c], y = vt[2 + c];
      vt[c] = csr * x + snr * y;
      vt[2 + c] = csr * y - snr * x;
    }
    for (int r = 0; r < 2; r++) {
      const double x = ub[2 * r], y = ub[2 * r + 1];
      ub[2 * r] = csl * x + snl * y;
      ub[2 * r + 1] = csl * y - snl * x;
    }
  }
  for (int i = 0; i < 2; i++)
    if (d[i] < 0.0) {
      d[i] = -d[i];
      vt[2 * i] = vt[2 * i] * -1.0;
      vt[2 * i + 1] = vt[2 * i + 1] * -1.0;
    }
  if (!(d[1] <= d[0])) { /* sort decreasing (ties keep the order) */
    double t = d[0]; d[0] = d[1]; d[1] = t;
    t = vt[0]; vt[0] = vt[2]; vt[2] = t;
    t = vt[1]; vt[1] = vt[3]; vt[3] = t;
    t = ub[0]; ub[0] = ub[1]; ub[1] = t;
    t = ub[2]; ub[2] = ub[3]; ub[3] = t;
  }
  /* dormbr('Q','L','N'): U = H1 * Ub (dorm2r -> dlarf on both columns) */
  for (int i = 0; i < 4; i++) U[i] = ub[i];
  if (tau != 0.0) {
    const int lastv = v2 != 0.0 ? 2 : 1;
    /* iladlc: the last column with a non-zero in rows 1..lastv; columns past it are untouched */
    const int nz1 = U[1] != 0.0 || (lastv == 2 && U[3] != 0.0);
    const int nz0 = U[0] != 0.0 || (lastv == 2 && U[2] != 0.0);
    const int lastc = nz1 ? 2 : (nz0 ? 1 : 0);
    for (int j = 0; j < lastc; j++) mpj_larf2(tau, v2, &U[j], &U[2 + j]);
  }
  S[0] = d[0]; S[1] = d[1];
  for (int i = 0; i < 4; i++) VT[i] = vt[i];
}

/* Julia `pinv(x::Number)`: inv(x) when finite, else zero. */
MPJ_FN double mpj_pinv_scalar(double x) {
  const double xi = 1.0 / x;
  return (xi - xi == 0.0) ? xi : 0.0;
}

/* pinv(M) for a row-major 2x2 (see the block comment above); P row-major. */
MPJ_FN void mpj_pinv2(const double* M, double* P) {
  const double rtol = 4.440892098500626e-16; /* eps(Float64) * min(size(A)...) */
  if (M[1] == 0.0 && M[2] == 0.0) { /* isdiag */
    const double a0 = __builtin_fabs(M[0]), a3 = __builtin_fabs(M[3]);
    const double mx = a3 > a0 ? a3 : a0; /* maximum(abs, dA) */
    const double tol = rtol * mx;
    P[0] = a0 > tol ? mpj_pinv_scalar(M[0]) : 0.0;
    P[3] = a3 > tol ? mpj_pinv_scalar(M[3]) : 0.0;
    P[1] = 0.0;
    P[2] = 0.0;
    return;
  }
  double U[4], S[2], VT[4];
  mpj_svd2(M, U, S, VT);
  const double tol = rtol * S[0]; /* maximum(S): S is sorted decreasing */
  const double i0 = S[0] > tol ? mpj_pinv_scalar(S[0]) : 0.0;
  const double i1 = S[1] > tol ? mpj_pinv_scalar(S[1]) : 0.0;
  /* D = Diagonal(Sinv) * U':  D[k][j] = Sinv[k] * U[j][k] */
  const double D00 = i0 * U[0], D01 = i0 * U[2], D10 = i1 * U[1], D11 = i1 * U[3];
  /* Vt' * D (matmul2x2!, tA = 'T'): P[i][j] = VT[0][i]*D[0][j] + VT[1][i]*D[1][j] */
  P[0] = VT[0] * D00 + VT[2] * D10;
  P[1] = VT[0] * D01 + VT[2] * D11;
  P[2] = VT[1] * D00 + VT[3] * D10;
  P[3] = VT[1] * D01 + VT[3] * D11;
}

#ifndef MPJ_PSEL /* the selects of mpj_pinv2_fast (A/B: plain ternaries) */
#define MPJ_PSEL(c, t, f) MPJ_SEL(c, t, f)
#endif
/* mpj_pinv2's general path as one basic block (the device's Riccati sweep, where the branchy
 * routine's ~20 uniform branches cost more than its divisions): every operation of mpj_pinv2 on the
 * path that a generic Quu takes -- not diagonal, a21 != 0 (a real reflector, v2 != 0), a12 != 0,
 * |e1| above dbdsqr's split threshold, dlasv2's gasmal branch with m*m != 0 -- with the swap, pmax,
 * sign-fix and cutoff decisions as selects.  Any lane off that path sets *rare; the caller then runs
 * mpj_pinv2 for it (mpj_pinv2_bl: wave-uniform on the device).  Same operations on the same
 * operands, so the same bits (tests/test_jlmath.py). */
MPJ_FN void mpj_pinv2_fast(const double* M, double* P, int* rare) {
  const double eps = 1.1102230246251565e-16, rtol = 4.440892098500626e-16;
  const double a11 = M[0], a12 = M[1], a21 = M[2], a22 = M[3];
  /* dgebd2: dlarfg(2, a11, a21) + dlarf on column 2 */
  const double xnorm = __builtin_fabs(a21), aa = __builtin_fabs(a11);
  const int big = aa > xnorm;
  const double w = MPJ_PSEL(big, aa, xnorm), z = MPJ_PSEL(big, xnorm, aa);
  const double q = z / w;
  const double py = MPJ_PSEL(z == 0.0, w, w * mpj_sqrt(1.0 + q * q));
  const double beta = -mpj_fsign(py, a11);
  const double tau = (beta - a11) / beta;
  const double v2 = a21 * (1.0 / (a11 - beta));
  const double d1 = beta;
  const double tw0 = -tau * (a12 + a22 * v2);
  const double e1 = a12 + tw0, d2 = mpj_fma(tw0, v2, a22);
  /* dbdsqr split test */
  const double unfl = 2.2250738585072014e-308, tol = 1.0958066990042004e-14;
  const double s0 = __builtin_fabs(d1);
  const double mu = __builtin_fabs(d2) * (s0 / (s0 + __builtin_fabs(e1)));
  const double sminoa = MPJ_PSEL(mu < s0, mu, s0) / 1.4142135623730951;
  const double th0 = tol * sminoa, th1 = 6.0 * (2.0 * (2.0 * unfl));
  const double thresh = MPJ_PSEL(th0 > th1, th0, th1);
  /* dlasv2(d1, e1, d2) */
  const double f = d1, g = e1, h = d2;
  const double fa0 = __builtin_fabs(f), ha0 = __builtin_fabs(h);
  const int swap = ha0 > fa0;
  const double ft = MPJ_PSEL(swap, h, f), ht = MPJ_PSEL(swap, f, h);
  const double fa = MPJ_PSEL(swap, ha0, fa0), ha = MPJ_PSEL(swap, fa0, ha0);
  const double gt = g, ga = __builtin_fabs(g);
  const int gbig = ga > fa;
  const double d = fa - ha;
  const double l0 = MPJ_PSEL(d == fa, 1.0, d / fa);
  const double m = gt / ft;
  const double t0 = 2.0 - l0;
  const double mm = m * m, tt = t0 * t0;
  const double s = mpj_sqrt(tt + mm);
  const double r = MPJ_PSEL(l0 == 0.0, __builtin_fabs(m), mpj_sqrt(l0 * l0 + mm));
  const double a = 0.5 * (s + r);
  const double smin = ha / a, smax = fa * a;
  const double t = (m / (s + t0) + m / (r + l0)) * (1.0 + a);
  const double l = mpj_sqrt(t * t + 4.0);
  const double crt = 2.0 / l, srt = t / l;
  const double clt = (crt + srt * m) / a;
  const double slt = (ht / ft) * srt / a;
  const double csl = MPJ_PSEL(swap, srt, clt), snl = MPJ_PSEL(swap, crt, slt);
  const double csr = MPJ_PSEL(swap, slt, crt), snr = MPJ_PSEL(swap, clt, srt);
  const double ts1 = mpj_fsign(1.0, csr) * mpj_fsign(1.0, csl) * mpj_fsign(1.0, f);
  const double ts2 = mpj_fsign(1.0, snr) * mpj_fsign(1.0, csl) * mpj_fsign(1.0, g);
  const double ts3 = mpj_fsign(1.0, snr) * mpj_fsign(1.0, snl) * mpj_fsign(1.0, h);
  const double tsign = MPJ_PSEL(gbig, ts2, MPJ_PSEL(swap, ts3, ts1));
  const double dd0 = mpj_fsign(smax, tsign);
  const double dd1 = mpj_fsign(smin, tsign * mpj_fsign(1.0, f) * mpj_fsign(1.0, h));
  *rare |= (a12 == 0.0) | (a21 == 0.0) | (v2 == 0.0) | !(__builtin_fabs(e1) > thresh) | (gbig && fa / ga < eps) |
           (mm == 0.0);
  /* drot on the identity */
  const double vt0 = csr * 1.0 + snr * 0.0, vt1 = csr * 0.0 + snr * 1.0;
  const double vt2 = csr * 0.0 - snr * 1.0, vt3 = csr * 1.0 - snr * 0.0;
  const double ub0 = csl * 1.0 + snl * 0.0, ub1 = csl * 0.0 - snl * 1.0;
  const double ub2 = csl * 0.0 + snl * 1.0, ub3 = csl * 1.0 - snl * 0.0;
  *rare |= (ub1 == 0.0) & (ub3 == 0.0);
  /* sign fix (d >= 0) and the sort (never swaps here: |ssmin| <= |ssmax|).  The fixed values are
   * |dd0| = smax and |dd1| = smin exactly (both >= 0), so the reciprocals below start from smax and
   * smin without waiting for the sign decision. */
  const int n0 = dd0 < 0.0, n1 = dd1 < 0.0;
  const double S0 = smax, S1 = smin;
  *rare |= !(S1 <= S0) | !(S0 > 0.0);
  const double V0 = MPJ_PSEL(n0, vt0 * -1.0, vt0), V1 = MPJ_PSEL(n0, vt1 * -1.0, vt1);
  const double V2 = MPJ_PSEL(n1, vt2 * -1.0, vt2), V3 = MPJ_PSEL(n1, vt3 * -1.0, vt3);
  /* dormbr: U = H1 * Ub on both columns (lastv = 2, lastc = 2: column 2 of Ub is never zero) */
  const double twa = -tau * (ub0 + ub2 * v2), twb = -tau * (ub1 + ub3 * v2);
  const double U0 = ub0 + twa, U2 = mpj_fma(twa, v2, ub2);
  const double U1 = ub1 + twb, U3 = mpj_fma(twb, v2, ub3);
  /* pinv composition */
  const double ctol = rtol * S0;
  const double x0 = 1.0 / S0, x1 = 1.0 / S1;
  const double i0 = MPJ_PSEL(S0 > ctol && x0 - x0 == 0.0, x0, 0.0);
  const double i1 = MPJ_PSEL(S1 > ctol && x1 - x1 == 0.0, x1, 0.0);
  const double D00 = i0 * U0, D01 = i0 * U2, D10 = i1 * U1, D11 = i1 * U3;
  P[0] = V0 * D00 + V2 * D10;
  P[1] = V0 * D01 + V2 * D11;
  P[2] = V1 * D00 + V3 * D10;
  P[3] = V1 * D01 + V3 * D11;
}
MPJ_FN void mpj_pinv2_bl(const double* M, double* P) {
  int rare = 0;
  mpj_pinv2_fast(M, P, &rare);
  if (MPJ_ANY(rare)) mpj_pinv2(M, P);
}

#endif /* MP_JLMATH_H */
