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
 * `exp` and `log` are FDLIBM's e_exp.c / e_log.c (Julia >= 1.6 uses a
 * table-driven exp; results agree to <= 1 ulp, not bit-for-bit).
 *
 * Accuracy vs glibc is checked in tests/test_jlmath.py (CPU) and the GPU
 * implementation is checked bit-exact against the CPU one in
 * tests/test_gpu_parity.py::test_jlmath_bitexact.
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
/* FDLIBM e_exp.c */
MPJ_FN double mpj_exp(double x) {
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

/* exp for 2^-28 <= |x| < 704 as one basic block (FDLIBM e_exp.c with every branch a select):
 * the |x| < 1.5 ln2 reduction (hi = x ∓ ln2HI, lo = ±ln2LO, k = ±1) is the general one with
 * t = k = ±1 (x - (-1)·ln2HI == x + ln2HI exactly), and (x·c)/(c-2) == -((x·c)/(2-c)) exactly,
 * so one division serves both the k == 0 and the k != 0 result.  Other arguments (incl. NaN,
 * Inf, overflow/underflow, k <= -1022) take mpj_exp through a wave-uniform branch. */
MPJ_FN double mpj_exp_fast(double x, int* bad) {
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00,
               P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  const uint32_t hx0 = mpj_hi(x);
  const uint32_t hx = hx0 & 0x7fffffffu;
  *bad |= hx < 0x3e300000u || hx >= 0x40860000u;
  const int xsb = (int)(hx0 >> 31);
  const int red = hx > 0x3fd62e42u;
  const int kfar = (int)(invln2 * MPJ_SEL(hx >= 0x40860000u, 0.0, x) + (xsb ? -0.5 : 0.5)); /* no UB on bad lanes */
  const int k = red ? (hx < 0x3FF0A2B2u ? 1 - xsb - xsb : kfar) : 0;
  const double t = (double)k;
  const double hi = x - t * ln2HI, lo = t * ln2LO;
  const double xr = MPJ_SEL(red, hi - lo, x);
  const double tt = xr * xr;
  const double c = xr - tt * mpj_fma(tt, mpj_fma(tt, mpj_fma(tt, mpj_fma(tt, P5, P4), P3), P2), P1);
  const double q = (xr * c) / (2.0 - c);
  const double r0 = 1.0 - ((-q) - xr);
  const double y = 1.0 - ((lo - q) - hi);
  const double twopk = mpj_from_words(0x3ff00000u + ((uint32_t)k << 20), 0);
  return MPJ_SEL(k == 0, r0, y * twopk);
}
MPJ_FN double mpj_exp_bl(double x) {
  const uint32_t hx = mpj_hi(x) & 0x7fffffffu;
  if (MPJ_ANY(hx < 0x3e300000u || hx >= 0x40860000u)) return mpj_exp(x);
  int bad = 0;
  return mpj_exp_fast(x, &bad);
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

#endif /* MP_JLMATH_H */
